# multi-rank rehearsal on one GPU (gloo) + bench lines of the other BASELINE configs (c3, c5)
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-cfg}
mkdir -p $OUT
bash tools/gpu_rehearse.sh ${1:-cfg}/reh && \
timeout -k 10 300 python -u bench.py --config c3 --steps 5 --warmup 2 --prof-steps 2 --no-cpu-baseline > $OUT/bench_c3.json 2> $OUT/bench_c3.err && \
timeout -k 10 400 python -u bench.py --config c5 --steps 1 --warmup 1 --prof-steps 1 --no-cpu-baseline > $OUT/bench_c5.json 2> $OUT/bench_c5.err
rc=$?
for f in $OUT/bench_c*.json; do echo $f; head -c 400 $f; echo; done
exit $rc
