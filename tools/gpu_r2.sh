# Round-2 GPU check: the new config / multi-GPU tests first, then the whole -m gpu suite, then the c2 bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r2a}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_multigpu.py tests/test_gpu_configs.py -x -v --timeout 300 --timeout-method thread > $OUT/new_tests.log 2>&1 && \
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread --deselect tests/test_gpu_configs.py --deselect tests/test_gpu_multigpu.py > $OUT/gpu_tests.log 2>&1 && \
timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 10 --warmup 3 > $OUT/bench_c2.json 2> $OUT/bench_c2.err
rc=$?
tail -3 $OUT/new_tests.log $OUT/gpu_tests.log
cat $OUT/bench_c2.json 2>/dev/null | head -c 600
exit $rc
