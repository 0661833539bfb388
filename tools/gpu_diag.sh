# Engine parity tests, then the k_row_layer phase clocks (make stamps) on the c2 workload.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-diag}
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest ${TESTS:-tests/test_gpu_engine.py} -x -v --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 && \
timeout -k 10 300 python -u tools/diag_stamps.py > $OUT/stamps.txt 2>&1
rc=$?
tail -3 $OUT/tests.log
cat $OUT/stamps.txt
exit $rc
