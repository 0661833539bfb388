# The -m gpu suite minus the files already run, smoke, then the c2 bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-rest}
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread --deselect tests/test_gpu_configs.py --deselect tests/test_gpu_multigpu.py --deselect tests/test_gpu_preprocess.py > $OUT/gpu_tests.log 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && \
timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 10 --warmup 3 > $OUT/bench_c2.json 2> $OUT/bench_c2.err
rc=$?
tail -n 3 $OUT/gpu_tests.log; cat $OUT/smoke.log
cat $OUT/bench_c2.json 2>/dev/null | head -c 300
exit $rc
