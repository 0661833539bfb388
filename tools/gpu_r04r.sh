# round 4 r: k_fp_train_hash / k_fp_train_resolve kernel times at 10 000 context rows, current
# build and the previous one (tools/diaglib/libnpfn_base4.so)
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r04r}
mkdir -p $OUT
export TMPDIR=/tmp
for v in new base; do
  case $v in new) L=npe-pfn_amd/npe_pfn/_lib/libnpfn.so;; base) L=tools/diaglib/libnpfn_base4.so;; esac
  NPFN_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt_$v -o kt -- python3 tools/fp_bench.py 10000 4 3 > $OUT/run_$v.log 2>&1 || exit $?
  S=$(find $OUT/kt_$v -name '*kernel_stats.csv' | head -n 1); echo "== $v"; grep -E "fp_train" "$S" | cut -d, -f1-4 | cut -c1-140
done
