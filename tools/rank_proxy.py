"""Per-rank compute of the 8-GPU c2 layout on one GPU: rank 0 of an EP group of 4 (estimator
set {0, 4}: one estimator of each ensemble pipeline) fits its estimators and runs the
test-side forward over its row group (5000 rows) for the 10 AR steps -- the work a rank does
between collectives.  Prints ms per sample() call (median of 5) for the build in NPFN_LIB.

usage: NPFN_LIB=<lib> python tools/rank_proxy.py [ep_size rows]"""
import os
import statistics
import sys
import time

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(ROOT, "npe-pfn_amd"))
import torch

from npe_pfn.engine import Engine
from npe_pfn.tasks import gaussian_linear_task
from npe_pfn.weights import ModelConfig, synthetic_weights

g = int(sys.argv[1]) if len(sys.argv) > 1 else 4
rows = int(sys.argv[2]) if len(sys.argv) > 2 else 5000
cfg = ModelConfig()
dev = torch.device("cuda", 0)
theta, x, x_o = gaussian_linear_task(10, 1000, seed=0)
theta, x = theta.to(dev), x.to(dev)
eng = Engine(cfg, synthetic_weights(cfg, seed=0), device=dev, random_state=0)
eng.set_preprocessing("ensemble")
eng.set_estimator_set(0, cfg.n_estimators // g, g)
gen = torch.Generator().manual_seed(0)
feat = (x_o.repeat(rows, 1) + 0.0).to(dev)
cols = [torch.randn(rows, 1, generator=gen).to(dev) for _ in range(theta.shape[1])]


def call(token):
    eng.set_fit_token(token)
    eng.ar_fit_begin(x, theta)
    f = feat
    for k in range(theta.shape[1]):
        eng.ar_fit_step(k)
        eng.forward_targets(f)
        f = torch.cat([f, cols[k]], 1)
    torch.cuda.synchronize()


times = []
for i in range(7):
    t0 = time.perf_counter()
    call(100 + i)
    times.append((time.perf_counter() - t0) * 1e3)
print(f"ep{g} rank 0, {rows} rows: {statistics.median(times[2:]):.2f} ms per call (all {[round(t, 1) for t in times]})")
