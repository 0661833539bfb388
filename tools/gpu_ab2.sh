# wall-clock A/B of two builds at the c2 size and at a small per-call size (EXTRA2 bench args)
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-ab2}
mkdir -p $OUT
timeout -k 10 500 python -u tools/ab_bench.py ${ROUNDS:-4} $ARMS > $OUT/ab.txt 2>&1 && \
timeout -k 10 500 python -u tools/ab_bench.py ${ROUNDS:-4} $ARMS -- ${EXTRA2:---samples 1250} > $OUT/ab_small.txt 2>&1
rc=$?
cat $OUT/ab.txt; cat $OUT/ab_small.txt
exit $rc
