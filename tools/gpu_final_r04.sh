# Round-4 evidence: whole -m gpu suite, smoke, the c2 bench line (default ensemble, with its CPU
# baseline), rocprofv3 kernel stats of the
# profiled form, the PMC passes (FETCH_SIZE, WRITE_SIZE) of k_row_layer and a GRBM_GUI_ACTIVE
# pass for the effective clock of the two dominant kernels.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-final}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 && \
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && \
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 > $OUT/bench_c2.json 2> $OUT/bench_c2.err && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --profile-all > $OUT/bench_under_rocprof.json 2> $OUT/rocprof.err && \
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_row_layer --output-format csv -d $OUT/pmc_fetch -o f -- python3 bench.py --steps 1 --warmup 0 --prof-steps 1 --no-cpu-baseline --profile-all > $OUT/bench_pmc_fetch.json 2> $OUT/pmc_fetch.err && \
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex k_row_layer --output-format csv -d $OUT/pmc_write -o w -- python3 bench.py --steps 1 --warmup 0 --prof-steps 1 --no-cpu-baseline --profile-all > $OUT/bench_pmc_write.json 2> $OUT/pmc_write.err && \
timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE --kernel-trace --kernel-include-regex "k_row_layer|k_item_attn" --output-format csv -d $OUT/pmc_clock -o c -- python3 bench.py --steps 1 --warmup 0 --prof-steps 1 --no-cpu-baseline --profile-all > $OUT/bench_pmc_clock.json 2> $OUT/pmc_clock.err
rc=$?
tail -n 3 $OUT/gpu_tests.log; cat $OUT/smoke.log
head -c 400 $OUT/bench_c2.json; echo
C=$(find $OUT/pmc_clock -name '*counter_collection.csv' | head -n 1)
K=$(find $OUT/pmc_clock -name '*kernel_trace.csv' | head -n 1)
[ -n "$C" ] && python3 profiles/clock.py "$C" "$K" > $OUT/clock.txt 2>&1; cat $OUT/clock.txt 2>/dev/null
exit $rc
