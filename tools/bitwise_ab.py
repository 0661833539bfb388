"""Bitwise comparison of two engine builds on the c2 shape (ensemble: two estimator groups).

usage: NPFN_LIB=<lib> python tools/bitwise_ab.py OUT.npz     (once per build)
       python tools/bitwise_ab.py --compare A.npz B.npz
Draws of npfn_ar_sample (10 AR dims, 2000 queries or NPFN_BW_ROWS), the teacher-forced log-probs and one
predict's logits; a refactoring that keeps the per-tile arithmetic must match bit for bit."""
import os
import sys

import numpy as np

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(ROOT, "npe-pfn_amd"))

if sys.argv[1] == "--compare":
    a, b = np.load(sys.argv[2]), np.load(sys.argv[3])
    ok = True
    for k in a.files:
        same = np.array_equal(a[k], b[k])
        ok &= same
        print(f"{k}: {'bitwise equal' if same else 'DIFFER, max |d| = %g' % np.abs(a[k] - b[k]).max()}")
    sys.exit(0 if ok else 1)

import torch

from npe_pfn.engine import Engine
from npe_pfn.tasks import gaussian_linear_task
from npe_pfn.weights import ModelConfig, synthetic_weights

cfg = ModelConfig()
w = synthetic_weights(cfg, seed=0)
dev = torch.device("cuda", 0)
theta, x, x_o = gaussian_linear_task(10, 1000, seed=0)
g = torch.Generator().manual_seed(1)
NQ = int(os.environ.get("NPFN_BW_ROWS", "2000"))  # query rows (>= 4096: the engine's two AR lanes)
xq = x_o.repeat(NQ, 1) + 0.05 * torch.randn(NQ, 10, generator=g)
eng = Engine(cfg, w, device=dev, random_state=0)
eng.set_preprocessing("ensemble")
if os.environ.get("NPFN_BW_TOKEN") == "1":  # per-step fit slots, as sample() runs (the two AR lanes need them)
    eng.set_fit_token(12345)
th, lp = eng.ar_sample(x, theta, xq, counter=0, with_log_prob=True)
lp2 = eng.ar_log_prob(x, theta, xq, th)
eng.fit(torch.cat([x, theta[:, :3]], 1), theta[:, 3])
logits = eng.predict_logits(torch.cat([xq, th[:, :3].cpu()], 1)[:500])
np.savez(sys.argv[1], theta=th.cpu().numpy(), lp=lp.cpu().numpy(), lp2=lp2.cpu().numpy(),
         logits=logits.cpu().numpy())
print("saved", sys.argv[1])
