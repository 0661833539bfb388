# round 4 zc: the c2-size AR log-prob parity test (1 000-simulation context, ensemble, 10 steps)
# against the oracle's precomputed per-step densities (tests/golden/c2_logprob.npz)
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r04zc
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_c2_logprob.py -x -v -s --timeout 300 --timeout-method thread > $OUT/test.log 2>&1
rc=$?
grep -E "c2 AR|passed|failed|Error|assert" $OUT/test.log
exit $rc
