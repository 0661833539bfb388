# bitwise + wall-clock A/B of the working-tree engine against a baseline build (LIB_B), with
# the parity suites that cover the touched paths
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-bitab}
mkdir -p $OUT
A=npe-pfn_amd/npe_pfn/_lib/libnpfn.so
B=${LIB_B:-tools/diaglib/libnpfn_head.so}
timeout -k 10 200 env NPFN_LIB=$A python -u tools/bitwise_ab.py $OUT/a.npz > $OUT/bit.log 2>&1 && \
timeout -k 10 200 env NPFN_LIB=$B python -u tools/bitwise_ab.py $OUT/b.npz >> $OUT/bit.log 2>&1 && \
python tools/bitwise_ab.py --compare $OUT/a.npz $OUT/b.npz >> $OUT/bit.log 2>&1; rc0=$?
timeout -k 10 700 python -u -m pytest ${TESTS:-tests/test_gpu_engine.py tests/test_gpu_multigpu.py tests/test_gpu_preprocess.py} -x -v --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 && \
timeout -k 10 500 python -u tools/ab_bench.py ${ROUNDS:-4} $A $B > $OUT/ab.txt 2>&1
rc=$?
cat $OUT/bit.log | grep -v amdgpu.ids; tail -3 $OUT/tests.log; cat $OUT/ab.txt
exit $rc
