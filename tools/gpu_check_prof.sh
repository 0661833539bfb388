# Parity tests touched by a kernel change, the c2 bench, and a kernel-trace profile of it.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-chk}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_preprocess.py tests/test_gpu_multigpu.py "tests/test_gpu_configs.py::test_c2_predict_matches_oracle" "tests/test_gpu_configs.py::test_c2_full_sample_properties_and_determinism" -x -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 && \
timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 10 --warmup 3 > $OUT/bench_c2.json 2> $OUT/bench_c2.err && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > $OUT/bench_under_rocprof.json 2> $OUT/rocprof.err
rc=$?
tail -n 3 $OUT/tests.log
head -c 300 $OUT/bench_c2.json
exit $rc
