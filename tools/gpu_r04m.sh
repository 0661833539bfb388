# round 4 m: the ensemble mix with the next estimators' logits loaded ahead (NPFN_MIX_PF = 2 / 4,
# and 2 without the hoisted translation entries) against the current build: bitwise check of the
# PF=2 build, per-kernel live times (tools/ab.py), c2 wall-clock A/B (tools/ab_bench.py)
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r04m
mkdir -p $OUT
D=tools/diaglib
timeout -k 10 200 env NPFN_LIB=$D/libnpfn_pf2.so python -u tools/bitwise_ab.py $OUT/a.npz > $OUT/bit.log 2>&1 && \
timeout -k 10 200 env NPFN_LIB=$D/libnpfn_base4.so python -u tools/bitwise_ab.py $OUT/b.npz >> $OUT/bit.log 2>&1
rc=$?
python tools/bitwise_ab.py --compare $OUT/a.npz $OUT/b.npz >> $OUT/bit.log 2>&1
grep -v amdgpu.ids $OUT/bit.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u tools/ab.py 3 $D/libnpfn_base4.so $D/libnpfn_pf2.so $D/libnpfn_pf4.so $D/libnpfn_pf2nh.so > $OUT/ab.txt 2>&1
rc=$?
grep -E "k_mix|k_row_layer|k_item" $OUT/ab.txt
[ $rc -ne 0 ] && exit $rc
timeout -k 10 700 python -u tools/ab_bench.py 2 $D/libnpfn_base4.so $D/libnpfn_pf2.so $D/libnpfn_pf4.so > $OUT/ab_bench.txt 2>&1
rc=$?
tail -4 $OUT/ab_bench.txt
exit $rc
