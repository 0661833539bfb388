# round 4 l: where the row kernel's residual stores go -- per-kernel live times (tools/ab.py,
# c2-like fit + predict) of the current build, a timing build with the residual in tile-slot order
# (1 KB contiguous per wave load / store instruction, NPFN_DIAG_TSL) and one without the test side's
# residual / q stores (NPFN_DIAG_NOSTORE); both diagnostic builds give wrong results
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r04l
mkdir -p $OUT
D=tools/diaglib
timeout -k 10 600 python -u tools/ab.py 3 $D/libnpfn_base4.so $D/libnpfn_tsl.so $D/libnpfn_nostore.so > $OUT/ab.txt 2>&1
rc=$?
cat $OUT/ab.txt
exit $rc
