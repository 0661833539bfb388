# Round-4 closing check: the whole -m gpu suite and smoke on the committed tree
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-suite}
mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 && \
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
rc=$?
tail -n 3 $OUT/gpu_tests.log; cat $OUT/smoke.log
exit $rc
