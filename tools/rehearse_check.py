"""Multi-rank rehearsal on ONE GPU (torchrun, gloo collectives): every rank runs
sample_estimator_parallel (strided EP groups x row groups, npe_pfn.distributed) of one
sample((N,)) call; rank 0 then draws the same call on a single engine and compares: equal
bit for bit for every layout.  Row groups > 1 draw the same Philox rows (the first accept/reject
batch of every row group sits at the unsharded rows; the GL prior never rejects here), and a
row's arithmetic does not depend on its slot in the row kernel's tiles (row-relative feature
attention, npfn_rowk2.hip feat_attn_rows), so where a row group starts changes nothing.
usage: torchrun --nproc-per-node G tools/rehearse_check.py EP_SIZE"""
import math
import os
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(ROOT, "npe-pfn_amd"))
import torch
import torch.distributed as dist

from npe_pfn import TabPFN_Based_NPE_PFN
from npe_pfn.distributed import sample_estimator_parallel
from npe_pfn.tasks import gaussian_linear_prior, gaussian_linear_task

ep = int(sys.argv[1])
dist.init_process_group("gloo")
rank = dist.get_rank()
torch.cuda.set_device(0)
dev = torch.device("cuda", 0)
theta, x, x_o = gaussian_linear_task(6, 500, seed=4)
N = 3001


def post():
    p = TabPFN_Based_NPE_PFN(prior=gaussian_linear_prior(6, device=dev),
                             regressor_init_kwargs={"random_state": 2, "device": dev})
    p.append_simulations(theta.to(dev), x.to(dev))
    return p


th, lp = sample_estimator_parallel(post(), x_o.to(dev), (N,), with_log_prob=True, ep_size=ep)
ok = torch.tensor([1], dtype=torch.int64)
if rank == 0:
    th_ref, lp_ref = post().sample((N,), x=x_o.to(dev), with_log_prob=True)
    same = torch.equal(th.cpu(), th_ref.cpu()) and torch.equal(lp.cpu(), lp_ref.cpu())
    print(f"world {dist.get_world_size()} ep {ep}: {tuple(th.shape)} equal to the 1-engine sample "
          f"(bitwise): {same}; "
          f"max |d theta| {(th.cpu() - th_ref.cpu()).abs().max().item():.3g}", flush=True)
    ok[0] = 1 if same else 0
dist.broadcast(ok, 0)
dist.destroy_process_group()
sys.exit(0 if int(ok[0]) else 1)
