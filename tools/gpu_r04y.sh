# round 4 y: does an early stop of the first pass (a wave whose every query's row sum passed
# 2^100 after the first 64-key step) pay under overflowing scores?  Diagnostic build with the
# stop inside the step loop (more registers: the normal-case cost shows too) vs the current
# build, c2 item-attention time at score scales 1 / 12 / 48 / 128
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r04y
mkdir -p $OUT
D=tools/diaglib
for v in base5 iaearly; do
  NPFN_LIB=$D/libnpfn_$v.so timeout -k 10 400 python -u tools/ia_stress.py 1 12 48 128 > $OUT/stress_$v.jsonl 2> $OUT/stress_$v.err || exit $?
  echo "== $v"; cat $OUT/stress_$v.jsonl
done
