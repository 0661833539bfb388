# tests (TESTS=...) then a wall-clock A/B of libraries (LIBS="a.so b.so", ROUNDS)
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-abt}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest ${TESTS:-tests/test_gpu_engine.py} -x -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?
tail -4 $OUT/tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u tools/ab_bench.py ${ROUNDS:-4} $LIBS > $OUT/ab.txt 2>&1
rc=$?
cat $OUT/ab.txt
exit $rc
