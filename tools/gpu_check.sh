# GPU check of a set of test files (TESTS=...) + the c2 bench (no CPU baseline)
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-chk}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest ${TESTS:-tests/test_gpu_engine.py} -x -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 && \
timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 10 --warmup 3 > $OUT/bench.json 2> $OUT/bench.err
rc=$?
tail -5 $OUT/tests.log
python -c "import json; d=json.load(open('$OUT/bench.json')); print(d['value'], d['ms_per_step']); print({k: (round(v['ms_per_step'],2), round(v.get('tflops',0),1)) for k, v in d['kernels'].items()})" 2>/dev/null
exit $rc
