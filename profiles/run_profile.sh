#!/bin/bash
# Profiling recipe (run on the GPU box from the repo root):
#   1. kernel trace + stats of the bench command (per-kernel average durations)
#   2. separate PMC passes for HBM traffic of the dominant kernel (FETCH_SIZE and
#      WRITE_SIZE cannot share a pass on gfx950 -- MI355X_MICROARCH.md §rocprofv3)
set -euo pipefail
TAG=${1:-r01}
KREGEX=${2:-k_item_attn}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- \
  python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --profile-all > $OUT/bench_under_rocprof.json
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$KREGEX" --output-format csv -d $OUT/pmc_fetch -o f -- \
  python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --profile-all > $OUT/bench_pmc_fetch.json
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$KREGEX" --output-format csv -d $OUT/pmc_write -o w -- \
  python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --profile-all > $OUT/bench_pmc_write.json
echo done
