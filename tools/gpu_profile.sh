# Round-end profile of the default c2 bench: kernel stats, k_row_layer HBM traffic
# (separate FETCH/WRITE passes), then the bench line with CPU baseline using that traffic.
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-r01v7}
OUT=gpurun_out/prof_$TAG
bash profiles/run_profile.sh $TAG k_row_layer > gpurun_out/prof_$TAG.log 2>&1 || exit 1
F=$(find $OUT/pmc_fetch -name '*counter_collection.csv' | head -n 1)
W=$(find $OUT/pmc_write -name '*counter_collection.csv' | head -n 1)
python3 profiles/traffic.py "$F" "$W" k_row_layer profiles/traffic.json || exit 1
cp profiles/traffic.json $OUT/traffic_row_layer.json
S=$(find $OUT/kt -name '*kernel_stats.csv' | head -n 1)
cp "$S" $OUT/kernel_stats.csv
timeout -k 10 500 python3 -u bench.py > $OUT/bench_c2.json 2> $OUT/bench_c2.err || exit 1
cat $OUT/bench_c2.json
