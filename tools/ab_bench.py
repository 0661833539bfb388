"""Wall-clock A/B of engine builds on one GPU: alternating `bench.py` subprocesses
(NPFN_LIB=<lib>, no CPU baseline, no profiled pass), median samples/s per library.

usage: python tools/ab_bench.py rounds libA.so libB.so [-- extra bench.py args]
An arm may carry environment settings: lib.so@VAR=1,VAR2=x (same library, different switches).
"""
import json
import os
import statistics
import subprocess
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
args = sys.argv[1:]
extra = []
if "--" in args:
    i = args.index("--")
    args, extra = args[:i], args[i + 1:]
rounds, libs = int(args[0]), args[1:]
res = {l: [] for l in libs}
for r in range(rounds):
    for lib in libs:
        path, _, sets = lib.partition("@")
        env = dict(os.environ, NPFN_LIB=os.path.abspath(path))
        env.update(kv.split("=", 1) for kv in sets.split(",") if kv)
        cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "5", "--warmup", "2", "--no-cpu-baseline",
               "--prof-steps", "0"] + extra
        out = subprocess.run(cmd, env=env, check=True, timeout=400, capture_output=True, text=True).stdout
        line = [l for l in out.splitlines() if l.startswith("{")][-1]
        v = json.loads(line)["value"]
        res[lib].append(v)
        print(f"round {r} {os.path.basename(lib)}: {v:.1f}", flush=True)
for lib in libs:
    print(f"{os.path.basename(lib):24s} median {statistics.median(res[lib]):10.1f}  all {res[lib]}")
