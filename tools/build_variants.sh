# Build A/B variants of the engine library: build_variants.sh NAME "-DFLAG=..." [NAME "-D..."]...
# -> tools/diaglib/libnpfn_NAME.so, each with the Makefile's recipe and EXTRA flags (in parallel)
set -e
cd "$(dirname "$0")/.."
mkdir -p tools/diaglib
pids=()
while [ $# -ge 2 ]; do
  make -s -C npe-pfn_amd OUT="$PWD/tools/diaglib/libnpfn_$1.so" OBJDIR="/tmp/npfn_variant_$1" EXTRA="$2" -j4 &
  pids+=($!)
  shift 2
done
for p in "${pids[@]}"; do wait $p; done
