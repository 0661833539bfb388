# item-attention variants: default-lib tests, the variant's engine tests, kernel A/B, wall A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-ia}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_preprocess.py tests/test_gpu_engine.py} -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for lib in $VARIANTS; do
  NPFN_LIB=$PWD/$lib timeout -k 10 600 python -u -m pytest tests/test_gpu_engine.py -x -q --timeout 300 --timeout-method thread > $OUT/tests_$(basename $lib).log 2>&1 || { tail -30 $OUT/tests_$(basename $lib).log; exit 1; }
  echo "$lib: $(tail -1 $OUT/tests_$(basename $lib).log)"
done
timeout -k 10 900 python -u tools/ab.py ${ROUNDS:-3} $LIBS > $OUT/ab_kernels.txt 2>&1 || { cat $OUT/ab_kernels.txt; exit 1; }
head -4 $OUT/ab_kernels.txt
timeout -k 10 900 python -u tools/ab_bench.py ${ROUNDS_BENCH:-3} $LIBS > $OUT/ab.txt 2>&1
rc=$?
tail -${NL:-4} $OUT/ab.txt
exit $rc
