# Multi-process rehearsal of the multi-GPU path on ONE GPU: gloo collectives (host copies), ranks share cuda:0.
# 1) strided estimator-parallel sampling == the 1-engine sample, bit for bit (2, 4 ranks; 8 ranks = EP4 x 2 row groups)
# 2) bench.py --gpus N lines (timings are NOT scaling numbers: the ranks share one GPU)
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-reh}
mkdir -p $OUT
export NPFN_DIST_BACKEND=gloo
run() { timeout -k 10 400 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node $1 --master-addr 127.0.0.1 --master-port $((29500 + $1)) tools/rehearse_check.py $2 > $OUT/check_$1_$2.log 2>&1; }
run 2 2 && run 4 4 && run 8 4 && \
timeout -k 10 400 python -u bench.py --gpus 8 --steps 2 --warmup 1 --no-cpu-baseline > $OUT/bench8.json 2> $OUT/bench8.err && \
timeout -k 10 300 python -u bench.py --gpus 2 --steps 2 --warmup 1 --no-cpu-baseline > $OUT/bench2.json 2> $OUT/bench2.err
rc=$?
grep -h "equal to" $OUT/check_*.log
for f in $OUT/bench*.json; do echo $f; head -c 700 $f; echo; done
exit $rc
