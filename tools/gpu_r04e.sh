# round 4 e: wall-clock A/B of the LDS layout switches (NPFN_ROWK2_SWZ bits), the fallback
# stress sweep at larger scales, and rocprofv3 kernel stats of the profiled c2 bench
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r04e
mkdir -p $OUT
export TMPDIR=/tmp
D=tools/diaglib
timeout -k 10 900 python -u tools/ab_bench.py 3 npe-pfn_amd/npe_pfn/_lib/libnpfn.so $D/libnpfn_swz0.so $D/libnpfn_swz1.so $D/libnpfn_swz2.so $D/libnpfn_swz4.so > $OUT/ab_swz.txt 2>&1 && \
timeout -k 10 400 python -u tools/ia_stress.py 32 48 64 96 128 > $OUT/ia_stress2.jsonl 2> $OUT/ia_stress2.err && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --profile-all > $OUT/bench_under_rocprof.json 2> $OUT/rocprof.err
rc=$?
cat $OUT/ab_swz.txt | tail -6; cat $OUT/ia_stress2.jsonl
S=$(find $OUT/kt -name '*kernel_stats.csv' | head -n 1); [ -n "$S" ] && head -25 "$S" | cut -c1-160
exit $rc
