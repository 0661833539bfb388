# kernel trace + HIP API trace of a short c2 bench: when the host issued each dispatch vs when it ran
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-trace_api}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace --output-format csv -d $OUT/kt -o kt -- python3 bench.py --steps 2 --warmup 1 --prof-steps 1 --no-cpu-baseline > $OUT/bench.json 2> $OUT/rocprof.err
rc=$?
find $OUT -name "*.csv" | head
exit $rc
