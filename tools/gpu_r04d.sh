# round 4 d: target-only last layer + conflict-free LDS images -- bitwise vs the r04b build,
# the touched parity suites, wall-clock A/B (new / no-swizzle / r04b), LDS bank-conflict counters
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r04d
mkdir -p $OUT
export TMPDIR=/tmp
A=npe-pfn_amd/npe_pfn/_lib/libnpfn.so
B=tools/diaglib/libnpfn_head.so
S=tools/diaglib/libnpfn_noswz.so
timeout -k 10 200 env NPFN_LIB=$A python -u tools/bitwise_ab.py $OUT/a.npz > $OUT/bit.log 2>&1 && \
timeout -k 10 200 env NPFN_LIB=$B python -u tools/bitwise_ab.py $OUT/b.npz >> $OUT/bit.log 2>&1 && \
timeout -k 10 200 env NPFN_LIB=$S python -u tools/bitwise_ab.py $OUT/s.npz >> $OUT/bit.log 2>&1
rc=$?
python tools/bitwise_ab.py --compare $OUT/a.npz $OUT/b.npz >> $OUT/bit.log 2>&1
python tools/bitwise_ab.py --compare $OUT/a.npz $OUT/s.npz >> $OUT/bit.log 2>&1
grep -v amdgpu.ids $OUT/bit.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_configs.py tests/test_gpu_multigpu.py tests/test_gpu_classifier.py tests/test_gpu_sharding.py tests/test_gpu_preprocess.py -x -v --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 && \
timeout -k 10 700 python -u tools/ab_bench.py 4 $A $S $B > $OUT/ab.txt 2>&1
rc=$?
tail -3 $OUT/tests.log; cat $OUT/ab.txt
[ $rc -ne 0 ] && exit $rc
for L in A B; do
  eval LIB=\$$L
  i=0
  for set in "SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" "SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM SQ_WAVES"; do
    i=$((i+1))
    NPFN_LIB=$LIB timeout -s KILL 120 rocprofv3 --pmc $set --kernel-include-regex k_row_layer --output-format csv -d $OUT/sq_$L/p$i -o p -- python3 tools/prof_predict.py 1 > $OUT/sq_${L}_p$i.log 2>&1 || exit 1
  done
  python3 profiles/sq_summary.py $OUT/sq_$L k_row_layer > $OUT/sq_$L.txt 2>&1
  echo "== $L"; cat $OUT/sq_$L.txt
done
