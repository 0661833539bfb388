# Build A/B variants of the engine library: build_variants.sh NAME "-DFLAG=..." [NAME "-D..."]...
# -> tools/diaglib/libnpfn_NAME.so (run from anywhere; builds in parallel)
set -e
cd "$(dirname "$0")/../npe-pfn_amd"
FL="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -I../include -Icsrc -Wall -Wno-unused-function -mllvm -amdgpu-mfma-vgpr-form=1 -fno-slp-vectorize"
SRCS="csrc/npfn_kernels.hip csrc/npfn_rowk2.hip csrc/npfn_engine.hip csrc/npfn_support.hip"
pids=()
while [ $# -ge 2 ]; do
  /opt/rocm/bin/hipcc $FL $2 $SRCS -o ../tools/diaglib/libnpfn_$1.so -lrocsolver -lrocblas &
  pids+=($!)
  shift 2
done
for p in "${pids[@]}"; do wait $p; done
