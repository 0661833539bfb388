# round 4 s: phase cycle counters of the fingerprint resolve (diagnostic build, NPFN_DIAG_FPCLK)
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r04s
mkdir -p $OUT
NPFN_LIB=tools/diaglib/libnpfn_fpclk.so timeout -k 10 200 python3 tools/fp_bench.py 10000 4 2 > $OUT/run.log 2>&1
rc=$?
grep -E "fpclk|ok" $OUT/run.log
exit $rc
