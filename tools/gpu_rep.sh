# repeated-row AR step 0: its parity tests, the estimator-parallel bitwise tests, c2 bench
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-rep}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_multigpu.py tests/test_gpu_posterior.py -x -v --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 && \
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err
rc=$?
tail -4 $OUT/tests.log
python -c "import json; d=json.load(open('$OUT/bench.json')); print(d['value'], d['ms_per_step']); print({k: (v['ms_per_step'], v['tflops']) for k, v in d['kernels'].items()})" 2>/dev/null
exit $rc
