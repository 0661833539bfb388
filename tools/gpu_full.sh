# Whole -m gpu suite, smoke, the c2 bench (default ensemble preprocessing) and a kernel-trace profile.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-full}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 && \
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > $OUT/bench_c2.json 2> $OUT/bench_c2.err && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --profile-all > $OUT/bench_under_rocprof.json 2> $OUT/rocprof.err
rc=$?
tail -n 3 $OUT/gpu_tests.log; cat $OUT/smoke.log
head -c 400 $OUT/bench_c2.json
exit $rc
