# c2 bench (default ensemble) + kernel-trace stats of the same command
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-bench}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py ${BENCH_ARGS:---steps 10 --warmup 3} > $OUT/bench_c2.json 2> $OUT/bench_c2.err && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > $OUT/bench_under_rocprof.json 2> $OUT/rocprof.err
rc=$?
head -c 1500 $OUT/bench_c2.json
exit $rc
