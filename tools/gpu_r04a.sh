# round 4: tabpfn-sized tables -- new table tests, the full -m gpu suite, a short c2 bench
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04a
timeout -k 10 600 python -u -m pytest tests/test_gpu_tables.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r04a/tables.log 2>&1
rc1=$?
tail -15 gpurun_out/r04a/tables.log
[ $rc1 -eq 124 -o $rc1 -eq 137 -o $rc1 -eq 134 -o $rc1 -eq 139 ] && exit $rc1
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread --deselect tests/test_gpu_tables.py > gpurun_out/r04a/gpu_all.log 2>&1
rc2=$?
tail -8 gpurun_out/r04a/gpu_all.log
[ $rc2 -eq 124 -o $rc2 -eq 137 -o $rc2 -eq 134 -o $rc2 -eq 139 ] && exit $rc2
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r04a/bench.json 2> gpurun_out/r04a/bench.err
rc3=$?
python -c "import json; d=json.load(open('gpurun_out/r04a/bench.json')); print(d['value'], d['ms_per_step']); print({k: (v['ms_per_step'], v['tflops']) for k, v in d['kernels'].items()})"
echo "rc $rc1 $rc2 $rc3"
