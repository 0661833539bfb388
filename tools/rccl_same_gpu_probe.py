"""Probe: can two RCCL ranks share one GPU on this box?  (If so, the multi-GPU path can be
rehearsed on RCCL -- not only gloo -- on a one-GPU box.)  torchrun --nproc-per-node 2."""
import os
import torch
import torch.distributed as dist

rank = int(os.environ["RANK"])
torch.cuda.set_device(0)
dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
t = torch.full((4,), float(rank + 1), device="cuda")
dist.all_reduce(t)
x = torch.arange(8, dtype=torch.int32, device="cuda") + 100 * rank
y = torch.empty(8, dtype=torch.int32, device="cuda")
dist.all_to_all_single(y, x)
torch.cuda.synchronize()
print(f"rank {rank}: all_reduce {t.tolist()} all_to_all {y.tolist()}", flush=True)
dist.destroy_process_group()
