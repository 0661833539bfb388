"""A/B of engine builds on one GPU: alternating subprocesses (NPFN_LIB=<lib>), medians per kernel.

usage: python tools/ab.py rounds libA.so libB.so[@VAR=1] [...]   -- c2-like predict (n=1000, F=15, 10k rows)
"""
import os, statistics, subprocess, sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
CHILD = r'''
import os, sys
sys.path.insert(0, os.path.join(sys.argv[1], "npe-pfn_amd"))
import numpy as np, torch
from npe_pfn.engine import Engine
from npe_pfn.weights import ModelConfig, synthetic_weights
cfg = ModelConfig(); w = synthetic_weights(cfg, 0)
e = Engine(cfg, w, device=torch.device("cuda", 0), random_state=0)
rng = np.random.default_rng(0)
X = torch.from_numpy(rng.normal(size=(1000, 15)).astype(np.float32)).cuda()
y = torch.from_numpy(rng.normal(size=1000).astype(np.float32)).cuda()
Xq = torch.from_numpy(rng.normal(size=(10000, 15)).astype(np.float32)).cuda()
e.fit(X, y); e.predict_logits(Xq); torch.cuda.synchronize()
e.prof_read(); e.prof_enable(True)
for _ in range(3):
    e.fit(X, y); e.predict_logits(Xq)
torch.cuda.synchronize(); e.prof_enable(False)
print(" ".join(f"{r['name']}={r['ms'] / 3:.3f}" for r in e.prof_read()), flush=True)
'''
rounds = int(sys.argv[1])
libs = sys.argv[2:]
res = {l: {} for l in libs}
for _ in range(rounds):
    for lib in libs:
        path, _, sets = lib.partition("@")  # an arm may carry switches: lib.so@VAR=1,VAR2=x
        env = dict(os.environ, NPFN_LIB=os.path.abspath(path))
        env.update(kv.split("=", 1) for kv in sets.split(",") if kv)
        out = subprocess.run([sys.executable, "-c", CHILD, ROOT], env=env, check=True, timeout=300,
                             capture_output=True, text=True).stdout.strip().splitlines()[-1]
        for kv in out.split():
            k, v = kv.rsplit("=", 1)
            res[lib].setdefault(k, []).append(float(v))
keys = sorted({k for l in libs for k in res[l]}, key=lambda k: -statistics.median(res[libs[0]].get(k, [0])))
for k in keys:
    print(f"{k:28s} " + "  ".join(f"{os.path.basename(l)}: {statistics.median(res[l][k]):8.3f} ms" for l in libs if k in res[l]))
