# round 4 q: train fingerprints with growing precomputed candidate counts and a 16-wave slow
# path (the last rows of a 10 000-row block), plus the new SVD-views test: bitwise vs the current
# build on the c2 harness, the preprocessing / table / classifier suites, c4 timing
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r04q
mkdir -p $OUT
D=tools/diaglib
timeout -k 10 200 env NPFN_LIB=$D/libnpfn_fp.so python -u tools/bitwise_ab.py $OUT/a.npz > $OUT/bit.log 2>&1 && \
timeout -k 10 200 env NPFN_LIB=$D/libnpfn_base4.so python -u tools/bitwise_ab.py $OUT/b.npz >> $OUT/bit.log 2>&1
rc=$?
python tools/bitwise_ab.py --compare $OUT/a.npz $OUT/b.npz >> $OUT/bit.log 2>&1
grep -v amdgpu.ids $OUT/bit.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u -m pytest tests/test_gpu_preprocess.py tests/test_gpu_tables.py tests/test_gpu_classifier.py -x -v --timeout 300 --timeout-method thread --durations=6 > $OUT/tests.log 2>&1
rc=$?
tail -10 $OUT/tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u bench.py --config c4 --steps 3 --warmup 1 > $OUT/bench_c4.json 2> $OUT/bench_c4.err
rc=$?
python -c "
import json; d=json.loads(open('$OUT/bench_c4.json').read().strip().splitlines()[-1])
print(d['value'], d['split_ms']); print(d['classifier_kernels'].get('k_fp_train'), d['regressor_kernels'].get('k_fp_train'))"
exit $rc
