# Parity tests, then the wall-clock A/B of bench.py (tools/ab_bench.py) on one GPU
#   TESTS="tests/..." LIB_A=... LIB_B=... ROUNDS=3 bash tools/gpu_abb.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-abb}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_engine.py} -x -v --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 && \
timeout -k 10 500 python -u tools/ab_bench.py ${ROUNDS:-3} ${LIB_A:-tools/diaglib/libnpfn_head.so} ${LIB_B:-npe-pfn_amd/npe_pfn/_lib/libnpfn.so} > $OUT/ab.txt 2>&1
rc=$?
tail -3 $OUT/tests.log
cat $OUT/ab.txt
exit $rc
