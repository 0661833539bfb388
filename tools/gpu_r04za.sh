# round 4 za: q/k/v and decoder-row stores widened to 16 bytes (v_permlane16_swap pairs of half
# rows): bitwise vs the current build, per-kernel times, c2 A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r04za
mkdir -p $OUT
D=tools/diaglib
timeout -k 10 200 env NPFN_LIB=$D/libnpfn_wideq.so python -u tools/bitwise_ab.py $OUT/a.npz > $OUT/bit.log 2>&1 && \
timeout -k 10 200 env NPFN_LIB=$D/libnpfn_base6.so python -u tools/bitwise_ab.py $OUT/b.npz >> $OUT/bit.log 2>&1
rc=$?
python tools/bitwise_ab.py --compare $OUT/a.npz $OUT/b.npz >> $OUT/bit.log 2>&1
grep -v amdgpu.ids $OUT/bit.log | tail -4
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u tools/ab.py 3 $D/libnpfn_base6.so $D/libnpfn_wideq.so > $OUT/ab.txt 2>&1
rc=$?
grep -E "k_row_layer|k_item|k_kv_pack" $OUT/ab.txt
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u tools/ab_bench.py 3 $D/libnpfn_base6.so $D/libnpfn_wideq.so > $OUT/ab_bench.txt 2>&1
rc=$?
tail -3 $OUT/ab_bench.txt
exit $rc
