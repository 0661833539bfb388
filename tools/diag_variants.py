"""Diagnostic: k_row_layer time of diagnostic builds (NPFN_LIB=<lib>), c2-like shapes.

usage: python tools/diag_variants.py lib1.so lib2.so ...   (each run in its own process)
"""
import os, subprocess, sys

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
    e.predict_logits(Xq)
torch.cuda.synchronize(); e.prof_enable(False)
for r in e.prof_read():
    if r["name"] == "k_row_layer":
        print(f"{os.path.basename(os.environ['NPFN_LIB'])}: k_row_layer {r['ms'] / r['launches'] * 1e3:.1f} us/launch "
              f"({r['launches']} launches)", flush=True)
'''
for lib in sys.argv[1:]:
    env = dict(os.environ, NPFN_LIB=os.path.abspath(lib))
    subprocess.run([sys.executable, "-c", CHILD, ROOT], env=env, check=True, timeout=300)
