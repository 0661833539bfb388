"""Diagnostic 3: the bench flow (TabPFN_Based_NPE_PFN.sample on device) repeated, finiteness per call."""
import os, sys, math
ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(ROOT, "npe-pfn_amd")); sys.path.insert(0, ROOT)
import numpy as np, torch
from bench import gl_task
from npe_pfn import TabPFN_Based_NPE_PFN

dev = torch.device("cuda", 0)
theta, x, x_o = [t.to(dev) for t in gl_task(10, 1000, 0)]
prior = torch.distributions.Independent(torch.distributions.Normal(torch.zeros(10, device=dev), torch.full((10,), math.sqrt(0.1), device=dev)), 1)
for flag in (os.environ.get("FLAGS", "0,1").split(",")):
    os.environ["NPFN_UNFUSED"] = flag
    post = TabPFN_Based_NPE_PFN(prior=prior, regressor_init_kwargs={"random_state": 0, "device": dev})
    post.append_simulations(theta, x)
    for call in range(6):
        s = post.sample((10000,), x=x_o)
        torch.cuda.synchronize()
        bad = ~torch.isfinite(s)
        a = s.nan_to_num().abs()
        i = int(a.argmax()); r, d = divmod(i, a.shape[1])
        print(f"flag={flag} call={call} nonfinite={int(bad.sum())} absmax={float(a.max()):.3f} at row={r} dim={d} row={s[r].tolist()}", flush=True)
