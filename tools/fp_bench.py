"""Train-fingerprint timing workload: ensemble fits of a regressor on N context rows (default
10 000, the c4 classifier's context size) -- run under rocprofv3 --kernel-trace --stats to see
k_fp_train_hash / k_fp_train_resolve.  usage: python tools/fp_bench.py [N] [F] [reps]"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "npe-pfn_amd"))
from npe_pfn.engine import Engine  # noqa: E402
from npe_pfn.weights import ModelConfig, synthetic_weights  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000
F = int(sys.argv[2]) if len(sys.argv) > 2 else 4
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
cfg = ModelConfig()
eng = Engine(cfg, synthetic_weights(cfg, 0), device=torch.device("cuda", 0), random_state=0)
rng = np.random.default_rng(0)
X = torch.from_numpy(rng.normal(size=(n, F)).astype(np.float32)).cuda()
y = torch.from_numpy(rng.normal(size=n).astype(np.float32)).cuda()
for _ in range(reps):
    eng.fit(X, y)
torch.cuda.synchronize()
print("ok", n, F, reps, flush=True)
