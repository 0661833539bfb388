"""Wall-clock A/B of engine builds on one GPU: alternating `bench.py` subprocesses
(NPFN_LIB=<lib>, no CPU baseline), median samples/s per library, and with NPFN_AB_KERNELS=1 the
median per-call time of the main kernels from a 2-step profiled pass of the same process.

usage: python tools/ab_bench.py rounds libA.so libB.so [-- extra bench.py args]
An arm may carry environment settings: lib.so@VAR=1,VAR2=x (same library, different switches).
"""
import json
import os
import statistics
import subprocess
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
KERNELS = ("k_row_layer", "k_item_attn", "k_mix_sample", "k_gemm<EPI_LOGIT>", "k_kv_pack", "k_encode")
args = sys.argv[1:]
extra = []
if "--" in args:
    i = args.index("--")
    args, extra = args[:i], args[i + 1:]
rounds, libs = int(args[0]), args[1:]
with_k = os.environ.get("NPFN_AB_KERNELS") == "1"
res = {l: [] for l in libs}
kres = {l: {k: [] for k in KERNELS} for l in libs}
for r in range(rounds):
    for lib in libs:
        path, _, sets = lib.partition("@")
        env = dict(os.environ, NPFN_LIB=os.path.abspath(path))
        env.update(kv.split("=", 1) for kv in sets.split(",") if kv)
        cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "5", "--warmup", "2", "--no-cpu-baseline",
               "--prof-steps", "2" if with_k else "0"] + extra
        out = subprocess.run(cmd, env=env, check=True, timeout=400, capture_output=True, text=True).stdout
        line = json.loads([l for l in out.splitlines() if l.startswith("{")][-1])
        res[lib].append(line["value"])
        ks = line.get("kernels") or {}
        for k in KERNELS:
            if k in ks:
                kres[lib][k].append(ks[k]["ms_per_step"])
        print(f"round {r} {os.path.basename(lib)}: {line['value']:.1f}" +
              ("  " + " ".join(f"{k}={ks[k]['ms_per_step']}" for k in KERNELS if k in ks) if with_k else ""),
              flush=True)
for lib in libs:
    print(f"{os.path.basename(lib):24s} median {statistics.median(res[lib]):10.1f}  all {res[lib]}")
    if with_k:
        print(" " * 26 + "  ".join(f"{k} {statistics.median(v):.2f}" for k, v in kres[lib].items() if v))
