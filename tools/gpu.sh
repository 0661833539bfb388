# One parameterised GPU launcher (replaces the per-experiment gpu_r0*.sh scripts of rounds 1-4).
#   gpurun -- 'bash tools/gpu.sh <out> <step> [<step> ...]'
# Every step runs under its own time limit; the steps are chained with && so the first failure
# (or fault, or time limit) ends the call.  Steps:
#   tests:<pytest args, comma-separated>   e.g. tests:tests/test_gpu_engine.py,tests/test_gpu_kwargs.py
#   suite                                   the whole -m gpu suite
#   smoke                                   __graft_entry__.smoke()
#   bench[:<bench.py args, comma-separated>] the bench line (default: c2 with the CPU baseline)
#   quick                                   c2 bench line without the CPU baseline
#   kstats[:<bench.py args>]                rocprofv3 --kernel-trace --stats of the profiled bench form
#   pmc:<COUNTER>[:<kernel regex>]          one rocprofv3 --pmc pass (one counter group per pass)
#   ab:<reps>:<libA>:<libB>[:<bench.py args>]  alternating same-GPU A/B of two library builds
#   rehearse                                2 / 4 torchrun ranks with gloo on the one GPU: the multi-rank
#                                           layouts equal the 1-engine sample bit for bit, + a 2-rank bench line
#   sq[:<kernel regex>]                     the SQ counter groups of tools/gpu_sq.sh (predict workload)
#   configs                                 the other configs' bench lines (c3, c5, nb, sc, c4)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:?usage: tools/gpu.sh <out> <step>...}
shift
mkdir -p "$OUT"
export TMPDIR=/tmp
PYT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
n=0
run_step() {
  local step="$1" kind arg
  kind="${step%%:*}"
  arg=""
  [ "$kind" != "$step" ] && arg="${step#*:}"
  n=$((n + 1))
  case "$kind" in
    tests) timeout -k 10 900 $PYT ${arg//,/ } > "$OUT/tests_$n.log" 2>&1; local rc=$?; tail -n 3 "$OUT/tests_$n.log"; return $rc ;;
    suite) timeout -k 10 1000 $PYT tests -m gpu > "$OUT/gpu_tests.log" 2>&1; local rc=$?; tail -n 3 "$OUT/gpu_tests.log"; return $rc ;;
    smoke) timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1; local rc=$?; cat "$OUT/smoke.log"; return $rc ;;
    bench) timeout -k 10 600 python -u bench.py ${arg//,/ } > "$OUT/bench_$n.json" 2> "$OUT/bench_$n.err"; local rc=$?; head -c 600 "$OUT/bench_$n.json"; echo; return $rc ;;
    quick) timeout -k 10 400 python -u bench.py --no-cpu-baseline ${arg//,/ } > "$OUT/quick_$n.json" 2> "$OUT/quick_$n.err"; local rc=$?
           python tools/kstats_line.py "$OUT/quick_$n.json"; return $rc ;;
    kstats) timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt_$n" -o kt -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --profile-all ${arg//,/ } > "$OUT/kstats_$n.json" 2> "$OUT/kstats_$n.err" ;;
    pmc) local ctr="${arg%%:*}" rx="k_row_layer"
         [ "$ctr" != "$arg" ] && rx="${arg#*:}"
         timeout -s KILL 300 rocprofv3 --pmc $ctr --kernel-include-regex "$rx" --output-format csv -d "$OUT/pmc_${n}_$ctr" -o p -- python3 bench.py --steps 1 --warmup 0 --prof-steps 1 --no-cpu-baseline --profile-all > "$OUT/pmc_${n}.json" 2> "$OUT/pmc_${n}.err" ;;
    ab) local reps="${arg%%:*}" rest="${arg#*:}"; local la="${rest%%:*}"; rest="${rest#*:}"; local lb="${rest%%:*}" bargs=""
        [ "$lb" != "$rest" ] && bargs="${rest#*:}"
        timeout -k 10 1000 python -u tools/ab_bench.py "$reps" "$la" "$lb" -- ${bargs//,/ } > "$OUT/ab_$n.txt" 2> "$OUT/ab_$n.err"; local rc=$?; tail -n 6 "$OUT/ab_$n.txt"; return $rc ;;
    rehearse) (export NPFN_DIST_BACKEND=gloo
               for r in 2 4; do
                 timeout -k 10 400 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node $r --master-addr 127.0.0.1 \
                   --master-port $((29500 + r)) tools/rehearse_check.py $r > "$OUT/rehearse_$r.log" 2>&1 || exit 1
               done
               timeout -k 10 300 python -u bench.py --gpus 2 --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/bench_gloo2.json" 2> "$OUT/bench_gloo2.err")
              local rc=$?; grep -h "equal to" "$OUT"/rehearse_*.log; return $rc ;;
    sq) bash tools/gpu_sq.sh "${OUT#gpurun_out/}_sq" "${arg:-k_row_layer}" ;;
    configs) for c in c3:10:3 c5:1:1 nb:5:2 sc:5:2 c4:3:1; do
               local cf="${c%%:*}" r="${c#*:}"; local st="${r%%:*}" wu="${r#*:}"
               timeout -k 10 400 python -u bench.py --config $cf --steps $st --warmup $wu --prof-steps 1 --no-cpu-baseline \
                 > "$OUT/bench_$cf.json" 2> "$OUT/bench_$cf.err" || return 1
               head -c 300 "$OUT/bench_$cf.json"; echo
             done ;;
    *) echo "unknown step $step"; return 2 ;;
  esac
}
for s in "$@"; do
  echo "== $s"
  run_step "$s" || { rc=$?; echo "step $s failed ($rc)"; exit $rc; }
done
