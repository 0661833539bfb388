"""Diagnostic: fused (k_row_layer) vs per-sublayer path over context/feature/row shapes."""
import os, sys, itertools
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "npe-pfn_amd"))
import numpy as np, torch
from npe_pfn.engine import Engine
from npe_pfn.weights import ModelConfig, synthetic_weights

cfg = ModelConfig(); w = synthetic_weights(cfg, 0)
engs = {}
for flag in ("0", "1"):
    os.environ["NPFN_UNFUSED"] = flag
    engs[flag] = Engine(cfg, w, device=torch.device("cuda", 0), random_state=0)
rng = np.random.default_rng(0)
for n, F, N in [(1000, 10, 500), (1000, 12, 500), (1000, 19, 500), (200, 11, 300), (64, 9, 100), (1000, 10, 4000)]:
    X = rng.normal(size=(n, F)).astype(np.float32); y = rng.normal(size=n).astype(np.float32)
    Xq = rng.normal(size=(N, F)).astype(np.float32)
    out = {}
    for flag, e in engs.items():
        e.fit(torch.from_numpy(X), torch.from_numpy(y))
        lg = e.predict_logits(torch.from_numpy(Xq))
        out[flag] = torch.softmax(lg, -1).double().cpu().numpy()
    fin = {k: bool(np.isfinite(v).all()) for k, v in out.items()}
    bad_rows = np.where(~np.isfinite(out["0"]).all(1))[0]
    tv = 0.5 * np.abs(np.nan_to_num(out["0"]) - out["1"]).sum(1)
    print(f"n={n} F={F} C={(F+1)//2+1} N={N} finite={fin} tv_max={tv.max():.4f} bad_rows={bad_rows[:10]} nbad={len(bad_rows)}", flush=True)
