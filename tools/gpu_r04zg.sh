# round 4 zg: the tree with NPFN_ROWK2_WIDEV on: the table tests (long rows), the engine and
# preprocessing parity tests, the c2 log-prob test, smoke
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r04zg
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_tables.py tests/test_gpu_engine.py tests/test_gpu_preprocess.py tests/test_gpu_c2_logprob.py tests/test_gpu_configs.py -x -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 && \
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
rc=$?
tail -n 3 $OUT/tests.log; cat $OUT/smoke.log
exit $rc
