# Multi-process rehearsal on ONE GPU (gloo collectives, ranks share cuda:0): strided
# estimator-parallel sampling == the 1-engine sample bit for bit at 2 and 4 ranks, and the
# 2-rank bench line with its identity / collective-bytes fields (timings are not scaling numbers)
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-reh}
mkdir -p $OUT
export NPFN_DIST_BACKEND=gloo
run() { timeout -k 10 400 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node $1 --master-addr 127.0.0.1 --master-port $((29500 + $1)) tools/rehearse_check.py $2 > $OUT/check_$1_$2.log 2>&1; }
run 2 2 && run 4 4 && \
timeout -k 10 300 python -u bench.py --gpus 2 --steps 2 --warmup 1 --no-cpu-baseline > $OUT/bench2.json 2> $OUT/bench2.err
rc=$?
grep -h "equal to" $OUT/check_*.log
tail -c 1500 $OUT/bench2.json
exit $rc
