# round 4 g: one-barrier-per-round Jacobi (double-buffered A in LDS) for m <= 64 --
# bitwise vs the previous build (tools/diaglib/libnpfn_head.so), the preprocessing / table
# suites, kernel stats of the profiled c2 bench
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r04g
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
timeout -k 10 900 python -u -m pytest tests/test_gpu_preprocess.py tests/test_gpu_tables.py tests/test_gpu_classifier.py tests/test_gpu_fit_reuse.py -x -v --timeout 200 --timeout-method thread --durations=8 > $OUT/tests.log 2>&1 && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --profile-all > $OUT/bench_under_rocprof.json 2> $OUT/rocprof.err && \
timeout -k 10 300 python -u bench.py --config sc --steps 5 --warmup 2 > $OUT/bench_sc.json 2> $OUT/bench_sc.err
rc=$?
tail -12 $OUT/tests.log
S=$(find $OUT/kt -name '*kernel_stats.csv' | head -n 1); [ -n "$S" ] && grep -E "svd|power|target|quantile|fp_|build_params|views|col_stats|kv_pack" "$S" | cut -d, -f1-4 | cut -c1-150
head -c 300 $OUT/bench_sc.json
exit $rc
