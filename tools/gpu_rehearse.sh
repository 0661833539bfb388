# Multi-process rehearsal of bench.py --gpus N on ONE GPU: gloo collectives (host copies), ranks share cuda:0.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-reh}
mkdir -p $OUT
export NPFN_DIST_BACKEND=gloo
timeout -k 10 300 python -u bench.py --gpus 2 --mode ep --steps 3 --warmup 1 --no-cpu-baseline > $OUT/ep2.json 2> $OUT/ep2.err && \
timeout -k 10 300 python -u bench.py --gpus 2 --mode rows --steps 3 --warmup 1 --no-cpu-baseline > $OUT/rows2.json 2> $OUT/rows2.err && \
timeout -k 10 300 python -u bench.py --gpus 4 --mode ep --config c3 --steps 2 --warmup 1 --no-cpu-baseline > $OUT/ep4_c3.json 2> $OUT/ep4_c3.err && \
timeout -k 10 300 python -u bench.py --gpus 2 --config c5 --obs 4 --steps 2 --warmup 1 --no-cpu-baseline > $OUT/c5_2.json 2> $OUT/c5_2.err
rc=$?
for f in $OUT/*.json; do echo $f; head -c 400 $f; echo; done
exit $rc
