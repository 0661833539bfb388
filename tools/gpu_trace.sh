# kernel trace (every dispatch with its start/end) of a short c2 bench: the timeline of one sample() call
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-trace}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- python3 bench.py --steps 2 --warmup 1 --prof-steps 1 --no-cpu-baseline > $OUT/bench.json 2> $OUT/rocprof.err
rc=$?
find $OUT -name "*.csv" | head
exit $rc
