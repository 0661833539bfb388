# A/B of the working-tree engine against a baseline library + parity tests
#   TESTS="tests/..." LIB_A=... LIB_B=... ROUNDS=6 bash tools/gpu_ab.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-ab}
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest ${TESTS:-tests/test_gpu_engine.py tests/test_gpu_classifier.py} -x -v --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 && \
timeout -k 10 400 python -u tools/ab.py ${ROUNDS:-6} ${LIB_A:-tools/diaglib/libnpfn_base.so} ${LIB_B:-npe-pfn_amd/npe_pfn/_lib/libnpfn.so} > $OUT/ab.txt 2>&1
rc=$?
tail -3 $OUT/tests.log
cat $OUT/ab.txt
exit $rc
