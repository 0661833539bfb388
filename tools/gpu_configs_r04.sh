# Round-4 evidence, part 2: the other configs' bench lines (c3, c5, the notebook's nb, the
# sampling_comparison notebook's sc, c4) on the same tree as tools/gpu_final_r04.sh.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-final}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --config c3 --steps 10 --warmup 3 --no-cpu-baseline > $OUT/bench_c3.json 2> $OUT/bench_c3.err && \
timeout -k 10 400 python -u bench.py --config c5 --steps 1 --warmup 1 --prof-steps 1 --no-cpu-baseline > $OUT/bench_c5.json 2> $OUT/bench_c5.err && \
timeout -k 10 300 python -u bench.py --config nb --steps 5 --warmup 2 > $OUT/bench_nb.json 2> $OUT/bench_nb.err && \
timeout -k 10 300 python -u bench.py --config sc --steps 5 --warmup 2 > $OUT/bench_sc.json 2> $OUT/bench_sc.err && \
timeout -k 10 400 python -u bench.py --config c4 --steps 3 --warmup 1 > $OUT/bench_c4.json 2> $OUT/bench_c4.err
rc=$?
for f in c3 c5 nb sc c4; do head -c 300 $OUT/bench_$f.json; echo; done
exit $rc
