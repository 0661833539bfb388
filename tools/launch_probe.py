"""Diagnostic (no profiler attached): does the HIP runtime hold the host back inside a launch?

A) 2048 tiny launches on one stream queued behind a long sleeping kernel: host time per
   block of 64 launches (a jump = the queue depth after which a launch waits for the GPU).
B) one c2-shaped npfn_ar_sample_repeated call (fresh fit token: the full fit runs): host time
   until the call returns vs the call's GPU time.
"""
import math
import os
import sys
import time

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(ROOT, "npe-pfn_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

dev = torch.device("cuda", 0)
x = torch.zeros(16, device=dev)
for _ in range(10):
    x.add_(1.0)
torch.cuda.synchronize()
for streams in (1, 3):
    ss = [torch.cuda.Stream() for _ in range(streams)]
    for s in ss:
        with torch.cuda.stream(s):
            torch.cuda._sleep(2_000_000_000 // 10)   # ~0.1 s at ~2 GHz
    marks = []
    t0 = time.perf_counter()
    for i in range(2048):
        with torch.cuda.stream(ss[i % streams]):
            x.add_(1.0)
        if (i + 1) % 128 == 0:
            marks.append((time.perf_counter() - t0) * 1e6)
    torch.cuda.synchronize()
    tot = (time.perf_counter() - t0) * 1e3
    d = [marks[0]] + [b - a for a, b in zip(marks, marks[1:])]
    print(f"A) {streams} stream(s): us per 128 launches: " + " ".join(f"{v:.0f}" for v in d) + f"; total {tot:.1f} ms")
    sys.stdout.flush()

from npe_pfn import TabPFN_Based_NPE_PFN  # noqa: E402
from npe_pfn.tasks import gaussian_linear_prior, gaussian_linear_task  # noqa: E402

theta, xs, x_o = [t.to(dev) for t in gaussian_linear_task(10, 1000, seed=0)]
post = TabPFN_Based_NPE_PFN(prior=gaussian_linear_prior(10, device=dev),
                            regressor_init_kwargs={"random_state": 0, "device": dev, "preprocessing": "ensemble"})
post.append_simulations(theta, xs)
post.sample((10_000,), x=x_o)
eng = post._model.engine
xq = x_o.reshape(1, -1).repeat(10_000, 1)
for it in range(4):
    eng.set_fit_token(1000 + it)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    eng.ar_sample(xs, theta, xq, counter=7, x_unique=x_o.reshape(1, -1))
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"B) ar_sample: host issue {1e3 * (t1 - t0):.1f} ms, until done {1e3 * (t2 - t0):.1f} ms")
