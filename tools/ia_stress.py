"""Item-attention fallback vs score scale on the c2 workload (round-4 brief item 2).

For each score multiplier (npfn_debug_item_attn_scale) one c2 sample((10000,)) call after a
warm-up: the share of query rows / blocks that took the online-softmax pass (device counters,
npfn_item_attn_fallback), k_item_attn's time per call (live HIP events) and the call's wall time.
Prints one JSON line per scale.  Usage: python tools/ia_stress.py [scales...]
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "npe-pfn_amd")]

import torch  # noqa: E402

from npe_pfn import TabPFN_Based_NPE_PFN  # noqa: E402
from npe_pfn.tasks import gaussian_linear_prior, gaussian_linear_task  # noqa: E402

scales = [float(a) for a in sys.argv[1:]] or [1, 2, 3, 4, 6, 8, 12, 16]
dev = torch.device("cuda", 0)
theta, x, x_o = (t.to(dev) for t in gaussian_linear_task(10, 1000, seed=0))
post = TabPFN_Based_NPE_PFN(prior=gaussian_linear_prior(10, device=dev), regressor_init_kwargs={"device": dev})
post.append_simulations(theta, x)
eng = post._model.engine
post.sample((10_000,), x=x_o)
for sc in scales:
    eng.debug_item_attn_scale(sc)
    post.sample((10_000,), x=x_o)  # warm-up at this scale
    eng.item_attn_fallback(reset=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(3):
        out = post.sample((10_000,), x=x_o)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / 3
    fb = eng.item_attn_fallback(reset=True)
    eng.prof_read()
    eng.prof_enable(True)
    post.sample((10_000,), x=x_o)
    eng.prof_enable(False)
    prof = {e["name"]: e["ms"] for e in eng.prof_read()}
    print(json.dumps({"scale": sc, "rows_fallback_frac": round(fb["fallback_frac"], 5),
                      "blocks_fallback_frac": round(fb["block_fallback_frac"], 5),
                      "rows_overflow": fb.get("rows_overflow"), "rows_underflow": fb.get("rows_underflow"),
                      "rows_padding": fb.get("rows_padding"), "rows": fb["rows"],
                      "ms_per_call": round(wall * 1e3, 2), "samples_per_s": round(10_000 / wall, 1),
                      "k_item_attn_ms": round(prof.get("k_item_attn", 0.0), 2),
                      "finite": bool(torch.isfinite(out).all())}), flush=True)
eng.debug_item_attn_scale(1.0)
