set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/s3
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/s3/gpu_tests.log 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s3/smoke.log 2>&1 && \
timeout -k 10 400 python -u bench.py > gpurun_out/s3/bench_c2.json 2> gpurun_out/s3/bench_c2.err
