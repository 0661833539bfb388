import sys, os
sys.path[:0] = [os.getcwd(), os.path.join(os.getcwd(), "npe-pfn_amd")]
import numpy as np, torch
from npe_pfn.engine import Engine
from npe_pfn.weights import ModelConfig, synthetic_weights
cfg = ModelConfig(); w = synthetic_weights(cfg, 0)
rng = np.random.default_rng(0)
X = torch.from_numpy(np.exp(rng.normal(size=(1000, 6))).astype(np.float32))
y = torch.from_numpy(rng.normal(size=1000).astype(np.float32))
Xq = torch.from_numpy(np.exp(rng.normal(size=(500, 6))).astype(np.float32))
outs = []
for i in range(3):
    e = Engine(cfg, w, device=torch.device("cuda", 0), random_state=1)
    e.set_preprocessing("quantile+power")
    e.fit(X, y)
    outs.append(e.predict_logits(Xq).cpu())
    del e
print("bitwise identical across engines:", all(torch.equal(outs[0], o) for o in outs[1:]))
assert all(torch.equal(outs[0], o) for o in outs[1:])
