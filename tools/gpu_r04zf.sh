# round 4 zf: value-image writes of the feature attention widened to 16 bytes (NPFN_ROWK2_WIDEV=1,
# permlane16 pairs): bitwise vs the current build, per-kernel times, c2 A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r04zf
mkdir -p $OUT
D=tools/diaglib
timeout -k 10 200 env NPFN_LIB=$D/libnpfn_widev.so python -u tools/bitwise_ab.py $OUT/a.npz > $OUT/bit.log 2>&1 && \
timeout -k 10 200 env NPFN_LIB=$D/libnpfn_base9.so python -u tools/bitwise_ab.py $OUT/b.npz >> $OUT/bit.log 2>&1
rc=$?
python tools/bitwise_ab.py --compare $OUT/a.npz $OUT/b.npz >> $OUT/bit.log 2>&1
grep -v amdgpu.ids $OUT/bit.log | tail -4
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u tools/ab.py 3 $D/libnpfn_base9.so $D/libnpfn_widev.so > $OUT/ab.txt 2>&1
rc=$?
grep -E "k_row_layer|k_item|k_kv_pack" $OUT/ab.txt
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u tools/ab_bench.py 3 $D/libnpfn_base9.so $D/libnpfn_widev.so > $OUT/ab_bench.txt 2>&1
rc=$?
tail -3 $OUT/ab_bench.txt
exit $rc
