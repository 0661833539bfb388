# round 4 p: the SVD views at every Jacobi form against the oracle (new test)
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r04p
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_tables.py -k "svd_views" -x -v --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?
tail -12 $OUT/tests.log
exit $rc
