# wall-clock A/B on one GPU: repeated-row AR step 0 (default) vs every row (NPFN_NO_REPEATED=1)
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-abrep}
mkdir -p $OUT
L=npe-pfn_amd/npe_pfn/_lib/libnpfn.so
timeout -k 10 600 python -u tools/ab_bench.py ${ROUNDS:-4} $L "$L@NPFN_NO_REPEATED=1" > $OUT/ab.txt 2>&1
rc=$?
cat $OUT/ab.txt
exit $rc
