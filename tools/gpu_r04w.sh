# round 4 w: how much of the ensemble mix is its block barriers -- per-kernel times of the
# current build and a timing build without the fast mix's barriers (wrong results)
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r04w2
mkdir -p $OUT
D=tools/diaglib
timeout -k 10 400 python -u tools/ab.py 3 $D/libnpfn_base5.so $D/libnpfn_mixnobar.so $D/libnpfn_mixcoal.so > $OUT/ab.txt 2>&1
rc=$?
grep -E "k_mix|k_row_layer" $OUT/ab.txt
exit $rc
