# Host issue order of the AR side work: launch-window probe, bitwise vs the previous library,
# parity tests, and the c2 wall-clock A/B of the new order against the old one (same library,
# NPFN_LATE_SIDE=0 NPFN_PREP_AHEAD=-1) and the previous library.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-issue}
PREV=${PREV:-tools/diaglib/libnpfn_r03e.so}
NEW=npe-pfn_amd/npe_pfn/_lib/libnpfn.so
mkdir -p $OUT
timeout -k 10 240 python3 -u tools/launch_probe.py > $OUT/launch_probe.txt 2>&1 || { tail -20 $OUT/launch_probe.txt; exit 1; }
cat $OUT/launch_probe.txt
NPFN_LIB=$PWD/$PREV timeout -k 10 200 python -u tools/bitwise_ab.py $OUT/bw_prev.npz > $OUT/bw_prev.log 2>&1 || { tail -20 $OUT/bw_prev.log; exit 1; }
NPFN_LIB=$PWD/$NEW timeout -k 10 200 python -u tools/bitwise_ab.py $OUT/bw0.npz > $OUT/bw0.log 2>&1 || { tail -20 $OUT/bw0.log; exit 1; }
python tools/bitwise_ab.py --compare $OUT/bw_prev.npz $OUT/bw0.npz
NPFN_LIB=$PWD/$NEW timeout -k 10 700 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_posterior.py tests/test_gpu_sharding.py -x -q --timeout 300 --timeout-method thread > $OUT/tests0.log 2>&1 || { tail -30 $OUT/tests0.log; exit 1; }
echo "tests: $(tail -1 $OUT/tests0.log)"
timeout -k 10 900 python -u tools/ab_bench.py ${ROUNDS_BENCH:-3} $PREV $NEW "$NEW@NPFN_LATE_SIDE=0,NPFN_PREP_AHEAD=-1" > $OUT/ab.txt 2>&1
rc=$?
tail -5 $OUT/ab.txt
exit $rc
