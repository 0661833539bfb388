# round 4 b: item-attention fallback (tests, stress sweep, c2 bench with fallback_frac), the
# sampling_comparison and c4 bench lines, the 2-rank gloo rehearsal line (SCALE identity fields)
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r04b
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_tables.py -x -v --timeout 300 --timeout-method thread --durations=15 > $OUT/tests.log 2>&1 && \
timeout -k 10 400 python -u tools/ia_stress.py 1 2 3 4 6 8 12 16 24 > $OUT/ia_stress.jsonl 2> $OUT/ia_stress.err && \
timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 10 --warmup 3 > $OUT/bench_c2.json 2> $OUT/bench_c2.err && \
timeout -k 10 300 python -u bench.py --config sc --steps 5 --warmup 2 > $OUT/bench_sc.json 2> $OUT/bench_sc.err && \
timeout -k 10 400 python -u bench.py --config c4 --steps 3 --warmup 1 > $OUT/bench_c4.json 2> $OUT/bench_c4.err && \
NPFN_DIST_BACKEND=gloo timeout -k 10 400 python -u bench.py --gpus 2 --steps 2 --warmup 1 --no-cpu-baseline > $OUT/bench_gloo2.json 2> $OUT/bench_gloo2.err
rc=$?
tail -22 $OUT/tests.log
cat $OUT/ia_stress.jsonl
python -c "
import json
for f in ['bench_c2','bench_sc','bench_c4','bench_gloo2']:
    try:
        d=json.load(open('$OUT/'+f+'.json'))
    except Exception as e:
        print(f, 'missing', e); continue
    print(f, d['value'], d['unit'], d.get('kernels',{}).get('k_item_attn'))
    if f=='bench_sc': print(d['per_N'])
    if f=='bench_c4': print(d['split_ms']); print(d['per_round_ms']); print(d['classifier_roofline'])
    if f=='bench_gloo2': print(json.dumps(d.get('per_rank',{}).get('identity')), d.get('per_rank',{}).get('collective_bytes_per_step'))
"
exit $rc
