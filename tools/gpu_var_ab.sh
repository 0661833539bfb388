# Engine variants ($VARIANTS, the in-tree library included by name) against $PREV: bitwise report,
# parity tests ($TESTS) on each variant, kernel and wall-clock A/B.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-var}
mkdir -p $OUT
NPFN_LIB=$PWD/$PREV timeout -k 10 200 python -u tools/bitwise_ab.py $OUT/bw_prev.npz > $OUT/bw_prev.log 2>&1 || { tail -20 $OUT/bw_prev.log; exit 1; }
i=0
for v in $VARIANTS; do
  NPFN_LIB=$PWD/$v timeout -k 10 200 python -u tools/bitwise_ab.py $OUT/bw$i.npz > $OUT/bw$i.log 2>&1 || { tail -20 $OUT/bw$i.log; exit 1; }
  echo "$v vs $PREV:"; python tools/bitwise_ab.py --compare $OUT/bw_prev.npz $OUT/bw$i.npz
  NPFN_LIB=$PWD/$v timeout -k 10 700 python -u -m pytest ${TESTS:-tests/test_gpu_engine.py tests/test_gpu_preprocess.py tests/test_gpu_posterior.py} -x -q --timeout 300 --timeout-method thread > $OUT/tests$i.log 2>&1 || { tail -30 $OUT/tests$i.log; exit 1; }
  echo "$v: $(tail -1 $OUT/tests$i.log)"
  i=$((i+1))
done
timeout -k 10 900 python -u tools/ab.py ${ROUNDS:-3} $PREV $VARIANTS > $OUT/ab_kernels.txt 2>&1 || { cat $OUT/ab_kernels.txt; exit 1; }
head -2 $OUT/ab_kernels.txt
timeout -k 10 900 python -u tools/ab_bench.py ${ROUNDS_BENCH:-3} $PREV $VARIANTS > $OUT/ab.txt 2>&1
rc=$?
tail -4 $OUT/ab.txt
exit $rc
