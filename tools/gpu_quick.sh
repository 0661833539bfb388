# quick GPU check: engine parity tests + c2 bench (no CPU baseline)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/q
timeout -k 10 300 python -u -m pytest tests/test_gpu_engine.py -x -v --timeout 120 --timeout-method thread > gpurun_out/q/tests.log 2>&1 && \
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/q/bench.json 2> gpurun_out/q/bench.err
rc=$?
tail -4 gpurun_out/q/tests.log
python -c "import json; d=json.load(open('gpurun_out/q/bench.json')); print(d['value'], d['ms_per_step']); print({k: (v['ms_per_step'], v['tflops']) for k, v in d['kernels'].items()})" 2>/dev/null
exit $rc
