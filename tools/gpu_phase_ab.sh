# Phase costs of k_row_layer (diagnostic builds without feature attention / LayerNorm / GELU)
# and layout variants, by per-kernel live timing of a c2-like fit + predict (tools/ab.py), then a
# wall-clock bench A/B of the candidate libraries (LIBS_BENCH).
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-phase}
mkdir -p $OUT
D=tools/diaglib
timeout -k 10 600 python -u tools/ab.py ${ROUNDS:-3} ${LIBS_PHASE:-$D/libnpfn_base3.so $D/libnpfn_NOATTN.so $D/libnpfn_NOLN.so $D/libnpfn_NOGELU.so} > $OUT/phase.txt 2>&1
rc=$?
cat $OUT/phase.txt
[ $rc -ne 0 ] && exit $rc
if [ -n "$LIBS_BENCH" ]; then
  timeout -k 10 900 python -u tools/ab_bench.py ${ROUNDS_BENCH:-3} $LIBS_BENCH > $OUT/ab.txt 2>&1
  rc=$?
  cat $OUT/ab.txt
fi
exit $rc
