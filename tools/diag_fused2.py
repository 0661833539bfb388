"""Diagnostic 2: large N and the fused AR sampler on the bench's GL-10D data, fused vs per-sublayer."""
import os, sys, math
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "npe-pfn_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import numpy as np, torch
from npe_pfn.engine import Engine
from npe_pfn.weights import ModelConfig, synthetic_weights
from bench import gl_task

cfg = ModelConfig(); w = synthetic_weights(cfg, 0)
engs = {}
for flag in ("0", "1"):
    os.environ["NPFN_UNFUSED"] = flag
    engs[flag] = Engine(cfg, w, device=torch.device("cuda", 0), random_state=0)
rng = np.random.default_rng(0)
n, F, N = 1000, 19, 10000
X = rng.normal(size=(n, F)).astype(np.float32); y = rng.normal(size=n).astype(np.float32)
Xq = rng.normal(size=(N, F)).astype(np.float32)
out = {}
for flag, e in engs.items():
    e.fit(torch.from_numpy(X), torch.from_numpy(y))
    out[flag] = torch.softmax(e.predict_logits(torch.from_numpy(Xq)), -1).double().cpu().numpy()
bad = np.where(~np.isfinite(out["0"]).all(1))[0]
print("predict N=10000 C=11: nbad", len(bad), bad[:10], "tv", (0.5*np.abs(np.nan_to_num(out["0"])-out["1"]).sum(1)).max(), flush=True)
theta, x, x_o = gl_task(10, 1000, 0)
for N in (1000, 10000):
    xq = x_o.repeat(N, 1)
    res = {}
    for flag, e in engs.items():
        th, lp = e.ar_sample(x, theta, xq, counter=0, with_log_prob=True)
        res[flag] = th.cpu().numpy()
        nb = (~np.isfinite(res[flag])).any(1)
        print(f"ar_sample N={N} flag={flag} nonfinite_rows={nb.sum()} first={np.where(nb)[0][:5]} cols_bad={(~np.isfinite(res[flag])).sum(0)}", flush=True)
    d = np.abs(np.nan_to_num(res["0"]) - res["1"])
    print("  median |fused-unfused| per dim", np.median(d, 0).round(4), flush=True)
