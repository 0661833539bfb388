# Row-kernel diagnostics: phase stamps (make stamps), SQ counters of the working tree and the base library
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/rkd
timeout -k 10 300 python -u tools/diag_stamps.py > gpurun_out/rkd/stamps.txt 2>&1 && \
bash tools/gpu_sq.sh new k_row_layer > gpurun_out/rkd/sq_new.txt 2>&1 && \
NPFN_LIB=$PWD/tools/diaglib/libnpfn_base.so bash tools/gpu_sq.sh base k_row_layer > gpurun_out/rkd/sq_base.txt 2>&1
rc=$?
cat gpurun_out/rkd/stamps.txt
paste gpurun_out/rkd/sq_base.txt gpurun_out/rkd/sq_new.txt | cut -c1-160
exit $rc
