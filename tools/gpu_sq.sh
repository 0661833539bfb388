# SQ counters of one kernel on the predict workload (tools/prof_predict.py), one pass per group
#   bash tools/gpu_sq.sh TAG KERNEL_REGEX
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-sq}
KREGEX=${2:-k_row_layer}
OUT=gpurun_out/sq_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
i=0
for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU" \
           "SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
           "SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_MISC SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM SQ_WAVES"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --kernel-include-regex "$KREGEX" --output-format csv -d $OUT/p$i -o p -- \
    python3 tools/prof_predict.py 1 > $OUT/run_p$i.log 2>&1 || exit 1
done
python3 profiles/sq_summary.py $OUT "$KREGEX" > $OUT/summary.txt
cat $OUT/summary.txt
