"""Launch-size probe: c2's sample() call with one accept/reject batch of N rows for several N
(max_sampling_batch_size = N), per-sample time of the call and of k_row_layer / k_item_attn from
the engine's HIP-event profiler.  If the per-sample kernel time falls as N grows, the fixed-size
part of a launch (its last partial wave of tiles: ~8 tiles per CU at c2) is a measurable cost.
usage: python tools/tail_probe.py N [N ...]"""
import os
import sys
import time

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(ROOT, "npe-pfn_amd"))
import torch

from npe_pfn import TabPFN_Based_NPE_PFN
from npe_pfn.tasks import gaussian_linear_prior, gaussian_linear_task

dev = torch.device("cuda", 0)
theta, x, x_o = gaussian_linear_task(10, 1000, seed=0)
post = TabPFN_Based_NPE_PFN(prior=gaussian_linear_prior(10, device=dev),
                            regressor_init_kwargs={"random_state": 0, "device": dev})
post.append_simulations(theta.to(dev), x.to(dev))
eng = post._model.engine
for n in [int(a) for a in sys.argv[1:]]:
    for _ in range(2):
        post.sample((n,), x=x_o.to(dev), max_sampling_batch_size=n)
    torch.cuda.synchronize()
    ts = []
    for _ in range(3):
        t0 = time.perf_counter()
        post.sample((n,), x=x_o.to(dev), max_sampling_batch_size=n)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    eng.prof_read()
    eng.prof_enable(True)
    post.sample((n,), x=x_o.to(dev), max_sampling_batch_size=n)
    torch.cuda.synchronize()
    eng.prof_enable(False)
    k = {e["name"]: e for e in eng.prof_read()}
    t = sorted(ts)[1]
    rk, ia = k.get("k_row_layer", {}), k.get("k_item_attn", {})
    print(f"N {n:6d}: {n / t:9.1f} samples/s  call {t * 1e3:8.2f} ms  "
          f"row {rk.get('ms', 0) / n * 1e3:7.3f} us/sample ({rk.get('launches', 0)} launches)  "
          f"item {ia.get('ms', 0) / n * 1e3:7.3f} us/sample", flush=True)
