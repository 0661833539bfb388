# A/B of the working-tree engine against a baseline library + engine parity tests
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab
timeout -k 10 300 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_classifier.py -x -v --timeout 120 --timeout-method thread > gpurun_out/ab/tests.log 2>&1 && \
timeout -k 10 400 python -u tools/ab.py 6 ${LIB_A:-tools/diaglib/libnpfn_base.so} ${LIB_B:-npe-pfn_amd/npe_pfn/_lib/libnpfn.so} > gpurun_out/ab/ab.txt 2>&1
rc=$?
tail -3 gpurun_out/ab/tests.log
cat gpurun_out/ab/ab.txt
exit $rc
