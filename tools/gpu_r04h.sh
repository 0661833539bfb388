# round 4 h: (1) Jacobi pairs from the round number, the one-barrier double-buffered kernel vs
# the two-barrier one (NPFN_SVJ_DB=0); (2) the train row kernel writes k and v straight into the
# K/V cache (k_kv_pack gone from the fused path).  Bitwise vs the previous build
# (tools/diaglib/libnpfn_head.so) for both Jacobi kernels, engine + wide-table suites, and the
# kernel times of all three under rocprofv3 on the same box
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r04h
mkdir -p $OUT
export TMPDIR=/tmp
A=npe-pfn_amd/npe_pfn/_lib/libnpfn.so
B=tools/diaglib/libnpfn_head.so
timeout -k 10 200 env NPFN_LIB=$A python -u tools/bitwise_ab.py $OUT/a.npz > $OUT/bit.log 2>&1 && \
timeout -k 10 200 env NPFN_LIB=$A NPFN_SVJ_DB=0 python -u tools/bitwise_ab.py $OUT/a0.npz >> $OUT/bit.log 2>&1 && \
timeout -k 10 200 env NPFN_LIB=$B python -u tools/bitwise_ab.py $OUT/b.npz >> $OUT/bit.log 2>&1
rc=$?
python tools/bitwise_ab.py --compare $OUT/a.npz $OUT/b.npz >> $OUT/bit.log 2>&1
python tools/bitwise_ab.py --compare $OUT/a0.npz $OUT/b.npz >> $OUT/bit.log 2>&1
grep -v amdgpu.ids $OUT/bit.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_tables.py -x -v --timeout 200 --timeout-method thread --durations=5 > $OUT/tests.log 2>&1
rc=$?
tail -5 $OUT/tests.log
[ $rc -ne 0 ] && exit $rc
for v in a0 b a; do
  case $v in a) L=$A; D=1;; a0) L=$A; D=0;; b) L=$B; D=1;; esac
  NPFN_LIB=$L NPFN_SVJ_DB=$D timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt_$v -o kt -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --profile-all > $OUT/bench_$v.json 2> $OUT/rocprof_$v.err || exit $?
done
for v in a a0 b; do
  echo "== $v"
  S=$(find $OUT/kt_$v -name '*kernel_stats.csv' | head -n 1); grep -E "svd_jacobi|kv_pack|k_row_layer" "$S" | cut -d, -f1-4 | cut -c1-150
done
