"""Diagnostic: k_row_layer phase clock shares on the bench workload (NPFN_STAMPS=1)."""
import os, sys, math
os.environ["NPFN_STAMPS"] = "1"
os.environ.setdefault("NPFN_LIB", os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "npe-pfn_amd", "npe_pfn", "_lib", "libnpfn_stamps.so"))
ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(ROOT, "npe-pfn_amd")); sys.path.insert(0, ROOT)
import torch
from bench import gl_task
from npe_pfn import TabPFN_Based_NPE_PFN

dev = torch.device("cuda", 0)
theta, x, x_o = [t.to(dev) for t in gl_task(10, 1000, 0)]
prior = torch.distributions.Independent(torch.distributions.Normal(torch.zeros(10, device=dev), torch.full((10,), math.sqrt(0.1), device=dev)), 1)
post = TabPFN_Based_NPE_PFN(prior=prior, regressor_init_kwargs={"random_state": 0, "device": dev})
post.append_simulations(theta, x)
post.sample((10000,), x=x_o)
eng = post._model.engine
eng.rowk_stamps(reset=True)
post.sample((10000,), x=x_o)
st = eng.rowk_stamps(reset=True)
names = ["prologue", "chunks", "layernorm", "vmcnt_wait", "kv_epi", "feat_attn", "stores", "dma_issue", "bar_wait"]
tot = sum(st[:9]); tiles = st[15]
print(f"tiles={tiles} total_ticks={tot} ticks/tile={tot / max(tiles, 1):.0f} (s_memtime = 100 MHz)")
for n, v in zip(names, st[:9]):
    print(f"  {n:10s} {v / max(tiles, 1):10.0f} ticks/tile  {100.0 * v / max(tot, 1):5.1f}%")
