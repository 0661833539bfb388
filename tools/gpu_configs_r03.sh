# Bench lines of the other configs on the final round-3 tree: c3 (SLCP), c5 (64 observations,
# sample_batched) and nb (the notebook's published workload), plus the gloo rehearsal on one GPU.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-cfg3}
mkdir -p $OUT
timeout -k 10 300 python -u bench.py --config c3 --steps 5 --warmup 2 --prof-steps 2 --no-cpu-baseline > $OUT/bench_c3.json 2> $OUT/bench_c3.err && \
timeout -k 10 400 python -u bench.py --config c5 --steps 1 --warmup 1 --prof-steps 1 --no-cpu-baseline > $OUT/bench_c5.json 2> $OUT/bench_c5.err && \
timeout -k 10 400 python -u bench.py --config nb --steps 3 --warmup 1 > $OUT/bench_nb.json 2> $OUT/bench_nb.err && \
bash tools/gpu_rehearse.sh ${1:-cfg3}/reh
rc=$?
for f in $OUT/bench_*.json; do echo $f; head -c 600 $f; echo; done
exit $rc
