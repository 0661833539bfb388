# round 4 i: the train row kernel writes k and v into the K/V cache through the LDS image in
# contiguous 1 KB pieces (k_kv_pack gone from the fused path); Jacobi pairs from the round
# number.  Bitwise vs the previous build (tools/diaglib/libnpfn_head.so), engine + wide-table
# suites, and both libraries' kernel times under rocprofv3 on the same box (alternating)
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r04i
mkdir -p $OUT
export TMPDIR=/tmp
A=npe-pfn_amd/npe_pfn/_lib/libnpfn.so
B=tools/diaglib/libnpfn_head.so
timeout -k 10 200 env NPFN_LIB=$A python -u tools/bitwise_ab.py $OUT/a.npz > $OUT/bit.log 2>&1 && \
timeout -k 10 200 env NPFN_LIB=$B python -u tools/bitwise_ab.py $OUT/b.npz >> $OUT/bit.log 2>&1
rc=$?
python tools/bitwise_ab.py --compare $OUT/a.npz $OUT/b.npz >> $OUT/bit.log 2>&1
grep -v amdgpu.ids $OUT/bit.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_tables.py -x -v --timeout 200 --timeout-method thread --durations=5 > $OUT/tests.log 2>&1
rc=$?
tail -3 $OUT/tests.log
[ $rc -ne 0 ] && exit $rc
for v in a b a2 b2; do
  case $v in a*) L=$A;; b*) L=$B;; esac
  NPFN_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt_$v -o kt -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --profile-all > $OUT/bench_$v.json 2> $OUT/rocprof_$v.err || exit $?
done
echo profiled
