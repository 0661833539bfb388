# Diagnostic kernel A/B (timing only): the default build vs half-width row-kernel fragment reads
# (NPFN_DIAG_HALFLDS, wrong results) vs scalar item-attention row sums (NPFN_IA_SSUM), then the
# default library's engine tests and a c2 bench line without the CPU baseline.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-diag}
mkdir -p $OUT
D=tools/diaglib
timeout -k 10 600 python -u tools/ab.py ${ROUNDS:-3} $D/libnpfn_base.so $D/libnpfn_HALFLDS.so $D/libnpfn_SSUM.so > $OUT/ab_kernels.txt 2>&1 || { cat $OUT/ab_kernels.txt; exit 1; }
head -4 $OUT/ab_kernels.txt
timeout -k 10 400 python -u -m pytest tests/test_gpu_engine.py -x -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err
rc=$?
head -c 300 $OUT/bench.json
exit $rc
