# parity tests of the touched paths + a wall-clock A/B of up to three arms (ARMS="a b c")
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-ab3}
mkdir -p $OUT
timeout -k 10 700 python -u -m pytest ${TESTS:-tests/test_gpu_engine.py tests/test_gpu_multigpu.py tests/test_gpu_preprocess.py} -x -v --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 && \
timeout -k 10 600 python -u tools/ab_bench.py ${ROUNDS:-4} $ARMS > $OUT/ab.txt 2>&1
rc=$?
tail -3 $OUT/tests.log
cat $OUT/ab.txt
exit $rc
