# round 4 v: the residual stored block by block right after its LayerNorm (block 0's stores drain
# under block 1's LayerNorm) vs the current build: bitwise, per-kernel times, c2 wall-clock A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r04v
mkdir -p $OUT
D=tools/diaglib
timeout -k 10 200 env NPFN_LIB=$D/libnpfn_lnst.so python -u tools/bitwise_ab.py $OUT/a.npz > $OUT/bit.log 2>&1 && \
timeout -k 10 200 env NPFN_LIB=$D/libnpfn_base5.so python -u tools/bitwise_ab.py $OUT/b.npz >> $OUT/bit.log 2>&1
rc=$?
python tools/bitwise_ab.py --compare $OUT/a.npz $OUT/b.npz >> $OUT/bit.log 2>&1
grep -v amdgpu.ids $OUT/bit.log | tail -4
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u tools/ab.py 3 $D/libnpfn_base5.so $D/libnpfn_lnst.so > $OUT/ab.txt 2>&1
rc=$?
grep -E "k_row_layer|k_item" $OUT/ab.txt
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u tools/ab_bench.py 3 $D/libnpfn_base5.so $D/libnpfn_lnst.so > $OUT/ab_bench.txt 2>&1
rc=$?
tail -3 $OUT/ab_bench.txt
exit $rc
