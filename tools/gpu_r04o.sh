# round 4 o: the encoder applied inside the layer-0 row-kernel launch from 16 bytes of inputs per
# token (k_encode_in) instead of k_encode's 768-byte fp32 rows: bitwise vs the current build,
# engine / configs / classifier suites, per-kernel times (tools/ab.py) and c2 wall-clock A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r04o
mkdir -p $OUT
D=tools/diaglib
timeout -k 10 200 env NPFN_LIB=$D/libnpfn_encin.so python -u tools/bitwise_ab.py $OUT/a.npz > $OUT/bit.log 2>&1 && \
timeout -k 10 200 env NPFN_LIB=$D/libnpfn_base4.so python -u tools/bitwise_ab.py $OUT/b.npz >> $OUT/bit.log 2>&1
rc=$?
python tools/bitwise_ab.py --compare $OUT/a.npz $OUT/b.npz >> $OUT/bit.log 2>&1
grep -v amdgpu.ids $OUT/bit.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 700 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_classifier.py tests/test_gpu_configs.py -x -v --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?
tail -3 $OUT/tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u tools/ab.py 3 $D/libnpfn_base4.so $D/libnpfn_encin.so > $OUT/ab.txt 2>&1
rc=$?
grep -E "k_encode|k_row_layer|k_item" $OUT/ab.txt
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u tools/ab_bench.py 3 $D/libnpfn_base4.so $D/libnpfn_encin.so > $OUT/ab_bench.txt 2>&1
rc=$?
tail -3 $OUT/ab_bench.txt
exit $rc
