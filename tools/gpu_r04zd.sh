# round 4 zd: feature attention with two items interleaved per loop iteration
# (NPFN_ROWK2_FA2=1 every row-kernel instance, =3 the test side's post launches only):
# bitwise vs the current build, per-kernel times, c2 A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r04zd
mkdir -p $OUT
D=tools/diaglib
timeout -k 10 200 env NPFN_LIB=$D/libnpfn_fa2.so python -u tools/bitwise_ab.py $OUT/a.npz > $OUT/bit.log 2>&1 && \
timeout -k 10 200 env NPFN_LIB=$D/libnpfn_fa2t.so python -u tools/bitwise_ab.py $OUT/t.npz >> $OUT/bit.log 2>&1 && \
timeout -k 10 200 env NPFN_LIB=$D/libnpfn_base8.so python -u tools/bitwise_ab.py $OUT/b.npz >> $OUT/bit.log 2>&1
rc=$?
python tools/bitwise_ab.py --compare $OUT/a.npz $OUT/b.npz >> $OUT/bit.log 2>&1
python tools/bitwise_ab.py --compare $OUT/t.npz $OUT/b.npz >> $OUT/bit.log 2>&1
grep -v amdgpu.ids $OUT/bit.log | grep -E "equal|differ|max"
[ $rc -ne 0 ] && exit $rc
timeout -k 10 500 python -u tools/ab.py 3 $D/libnpfn_base8.so $D/libnpfn_fa2.so $D/libnpfn_fa2t.so > $OUT/ab.txt 2>&1
rc=$?
grep -E "k_row_layer|k_item|k_kv_pack" $OUT/ab.txt
[ $rc -ne 0 ] && exit $rc
timeout -k 10 800 python -u tools/ab_bench.py 3 $D/libnpfn_base8.so $D/libnpfn_fa2.so $D/libnpfn_fa2t.so > $OUT/ab_bench.txt 2>&1
rc=$?
tail -4 $OUT/ab_bench.txt
exit $rc
