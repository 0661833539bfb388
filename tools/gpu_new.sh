# GPU check of the newest tests + engine parity + c2 bench (default and with preprocessing)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/n
timeout -k 10 400 python -u -m pytest tests/test_gpu_preprocess.py tests/test_gpu_engine.py -x -v --timeout 120 --timeout-method thread > gpurun_out/n/tests.log 2>&1 && \
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/n/bench.json 2> gpurun_out/n/bench.err && \
timeout -k 10 300 python -u bench.py --no-cpu-baseline --preprocessing quantile+power > gpurun_out/n/bench_pre.json 2> gpurun_out/n/bench_pre.err
rc=$?
tail -25 gpurun_out/n/tests.log
python -c "import json; d=json.load(open('gpurun_out/n/bench.json')); print(d['value'], d['ms_per_step'])" 2>/dev/null
python -c "import json; d=json.load(open('gpurun_out/n/bench_pre.json')); print(d['value'], d['ms_per_step'], d['config'])" 2>/dev/null
exit $rc
