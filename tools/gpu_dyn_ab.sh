# Row-kernel variants against the previous library ($PREV): the in-tree library (dynamic tile
# schedule; NPFN_ROWK_STATIC=1 = static) and the diagnostic builds in $VARIANTS -- bitwise check
# of each against $PREV, engine + config tests on the in-tree library, kernel and wall A/B.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-dyn}
mkdir -p $OUT
L=npe-pfn_amd/npe_pfn/_lib/libnpfn.so
NPFN_LIB=$PWD/$PREV timeout -k 10 200 python -u tools/bitwise_ab.py $OUT/bw_prev.npz > $OUT/bw_prev.log 2>&1 || { tail -20 $OUT/bw_prev.log; exit 1; }
i=0
for arm in $L $L@NPFN_ROWK_STATIC=1 $VARIANTS; do
  path=${arm%%@*}; sets=""; [ "$arm" != "$path" ] && sets=${arm#*@}
  env $sets NPFN_LIB=$PWD/$path timeout -k 10 200 python -u tools/bitwise_ab.py $OUT/bw$i.npz > $OUT/bw$i.log 2>&1 || { tail -20 $OUT/bw$i.log; exit 1; }
  echo "$arm vs $PREV:"; python tools/bitwise_ab.py --compare $OUT/bw_prev.npz $OUT/bw$i.npz
  i=$((i+1))
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 900 python -u tools/ab.py ${ROUNDS:-3} $PREV $L $L@NPFN_ROWK_STATIC=1 $VARIANTS > $OUT/ab_kernels.txt 2>&1 || { cat $OUT/ab_kernels.txt; exit 1; }
head -2 $OUT/ab_kernels.txt
timeout -k 10 900 python -u tools/ab_bench.py ${ROUNDS_BENCH:-2} $PREV $L $L@NPFN_ROWK_STATIC=1 $VARIANTS > $OUT/ab.txt 2>&1
rc=$?
tail -6 $OUT/ab.txt
exit $rc
