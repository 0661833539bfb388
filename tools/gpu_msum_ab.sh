# Item-attention variant ($VAR) against the in-tree library: bitwise report, the parity suites
# that cover item attention on the variant, kernel and wall A/B.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-msum}
mkdir -p $OUT
L=npe-pfn_amd/npe_pfn/_lib/libnpfn.so
timeout -k 10 200 python -u tools/bitwise_ab.py $OUT/bw0.npz > $OUT/bw0.log 2>&1 || { tail -20 $OUT/bw0.log; exit 1; }
NPFN_LIB=$PWD/$VAR timeout -k 10 200 python -u tools/bitwise_ab.py $OUT/bw1.npz > $OUT/bw1.log 2>&1 || { tail -20 $OUT/bw1.log; exit 1; }
echo "$VAR vs in-tree:"; python tools/bitwise_ab.py --compare $OUT/bw0.npz $OUT/bw1.npz
NPFN_LIB=$PWD/$VAR timeout -k 10 700 python -u -m pytest ${TESTS:-tests/test_gpu_engine.py tests/test_gpu_preprocess.py tests/test_gpu_configs.py tests/test_gpu_posterior.py} -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 900 python -u tools/ab.py ${ROUNDS:-3} $L $VAR > $OUT/ab_kernels.txt 2>&1 || { cat $OUT/ab_kernels.txt; exit 1; }
head -3 $OUT/ab_kernels.txt
timeout -k 10 900 python -u tools/ab_bench.py ${ROUNDS_BENCH:-3} $L $VAR > $OUT/ab.txt 2>&1
rc=$?
tail -2 $OUT/ab.txt
exit $rc
