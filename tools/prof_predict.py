"""Profiling target: fit + predict of a c2-like table (n=1000, F=15, 10k query rows) on one
GPU, default preprocessing of the engine; for rocprofv3 --pmc passes (profiles/pmc_sq.sh)."""
import os, sys
ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(ROOT, "npe-pfn_amd"))
import numpy as np, torch
from npe_pfn.engine import Engine
from npe_pfn.weights import ModelConfig, synthetic_weights

cfg = ModelConfig()
w = synthetic_weights(cfg, 0)
e = Engine(cfg, w, device=torch.device("cuda", 0), random_state=0)
rng = np.random.default_rng(0)
X = torch.from_numpy(rng.normal(size=(1000, 15)).astype(np.float32)).cuda()
y = torch.from_numpy(rng.normal(size=1000).astype(np.float32)).cuda()
Xq = torch.from_numpy(rng.normal(size=(10000, 15)).astype(np.float32)).cuda()
for _ in range(int(sys.argv[1]) if len(sys.argv) > 1 else 2):
    e.fit(X, y)
    e.predict_logits(Xq)
torch.cuda.synchronize()
print("ok")
