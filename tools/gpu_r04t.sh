# round 4 t: train fingerprints -- candidate counts growing with the block position (~1e-3
# slow-row probability, up to 256 precomputed), the first 64 staged for wave 0's batches, the
# rest read by the block for a slow row, claims for the duplicate check: kernel times at 10 000
# rows (new vs previous build), bitwise on the c2 harness, fingerprint / table / classifier
# suites, c4
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r04t
mkdir -p $OUT
export TMPDIR=/tmp
D=tools/diaglib
for v in new base; do
  case $v in new) L=$D/libnpfn_fp.so;; base) L=$D/libnpfn_base4.so;; esac
  NPFN_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt_$v -o kt -- python3 tools/fp_bench.py 10000 4 3 > $OUT/run_$v.log 2>&1 || exit $?
done
python3 tools/kstats_cmp.py $OUT/kt_new=new $OUT/kt_base=base "--grep=fp_train" | cut -c1-130
timeout -k 10 200 env NPFN_LIB=$D/libnpfn_fp.so python -u tools/bitwise_ab.py $OUT/a.npz > $OUT/bit.log 2>&1 && \
timeout -k 10 200 env NPFN_LIB=$D/libnpfn_base4.so python -u tools/bitwise_ab.py $OUT/b.npz >> $OUT/bit.log 2>&1
rc=$?
python tools/bitwise_ab.py --compare $OUT/a.npz $OUT/b.npz >> $OUT/bit.log 2>&1
grep -v amdgpu.ids $OUT/bit.log | tail -4
[ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u -m pytest tests/test_gpu_preprocess.py tests/test_gpu_tables.py tests/test_gpu_classifier.py -x -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?
tail -3 $OUT/tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u bench.py --config c4 --steps 3 --warmup 1 > $OUT/bench_c4.json 2> $OUT/bench_c4.err
rc=$?
python -c "
import json; d=json.loads(open('$OUT/bench_c4.json').read().strip().splitlines()[-1])
print(d['value'], d['split_ms']); print(d['classifier_kernels'].get('k_fp_train'))"
exit $rc
