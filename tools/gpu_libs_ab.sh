# bitwise check of each lib in LIBS against the first, the engine tests on each, then kernel and
# wall-clock A/B (same-arithmetic refactorings: scheduling, ring depth, stagger)
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-libsab}
mkdir -p $OUT
set -- $LIBS
REF=$1
i=0
for lib in $LIBS; do
  timeout -k 10 200 env NPFN_LIB=$PWD/$lib python -u tools/bitwise_ab.py $OUT/bw$i.npz > $OUT/bw$i.log 2>&1 || { tail -20 $OUT/bw$i.log; exit 1; }
  if [ $i -gt 0 ]; then echo "$(basename $lib) vs $(basename $REF):"; python tools/bitwise_ab.py --compare $OUT/bw0.npz $OUT/bw$i.npz; fi
  i=$((i+1))
done
for lib in $LIBS; do
  NPFN_LIB=$PWD/$lib timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_engine.py} -x -q --timeout 300 --timeout-method thread > $OUT/tests_$(basename $lib).log 2>&1 || { tail -30 $OUT/tests_$(basename $lib).log; exit 1; }
  echo "$lib: $(tail -1 $OUT/tests_$(basename $lib).log)"
done
timeout -k 10 900 python -u tools/ab.py ${ROUNDS:-3} $LIBS > $OUT/ab_kernels.txt 2>&1 || { cat $OUT/ab_kernels.txt; exit 1; }
head -${NK:-4} $OUT/ab_kernels.txt
timeout -k 10 900 python -u tools/ab_bench.py ${ROUNDS_BENCH:-3} $LIBS > $OUT/ab.txt 2>&1
rc=$?
tail -${NL:-4} $OUT/ab.txt
exit $rc
