# round 4 z: k_kv_pack with the v tile transposed through LDS (16-byte loads instead of 8
# scattered 2-byte ones per output chunk): bitwise vs the current build, per-kernel times, c2 A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r04z
mkdir -p $OUT
D=tools/diaglib
timeout -k 10 200 env NPFN_LIB=$D/libnpfn_kvp.so python -u tools/bitwise_ab.py $OUT/a.npz > $OUT/bit.log 2>&1 && \
timeout -k 10 200 env NPFN_LIB=$D/libnpfn_base5.so python -u tools/bitwise_ab.py $OUT/b.npz >> $OUT/bit.log 2>&1
rc=$?
python tools/bitwise_ab.py --compare $OUT/a.npz $OUT/b.npz >> $OUT/bit.log 2>&1
grep -v amdgpu.ids $OUT/bit.log | tail -4
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u tools/ab.py 3 $D/libnpfn_base5.so $D/libnpfn_kvp.so > $OUT/ab.txt 2>&1
rc=$?
grep -E "k_kv_pack|k_row_layer|k_item" $OUT/ab.txt
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u tools/ab_bench.py 3 $D/libnpfn_base5.so $D/libnpfn_kvp.so > $OUT/ab_bench.txt 2>&1
rc=$?
tail -3 $OUT/ab_bench.txt
exit $rc
