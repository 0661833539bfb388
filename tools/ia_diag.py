"""Item-attention fallback diagnostics: x40 item q/k weights (tests/test_gpu_engine.py
test_item_attn_fallback_on_large_scores), NaN / inf counts of the auto and forced-online
passes for the library NPFN_LIB names (default: the in-tree build)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "npe-pfn_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from npe_pfn.engine import Engine  # noqa: E402
from npe_pfn.weights import ModelConfig, synthetic_weights  # noqa: E402

CFG = ModelConfig()
w = synthetic_weights(CFG, seed=0)
scale = float(sys.argv[1]) if len(sys.argv) > 1 else 40.0
for l in range(CFG.n_layers):
    w[f"l{l}.item_qkv"][: 2 * CFG.d_model] *= scale
eng = Engine(CFG, w, device=torch.device("cuda", 0), random_state=3)
rng = np.random.default_rng(5)
X = rng.normal(size=(200, 3)).astype(np.float32)
y = (X @ rng.normal(size=3) + 0.3 * rng.normal(size=200)).astype(np.float32)
Xq = rng.normal(size=(300, 3)).astype(np.float32)
eng.fit(torch.from_numpy(X), torch.from_numpy(y))
for onl in (False, True):
    eng.debug_item_attn_online(onl)
    lg = eng.predict_logits(torch.from_numpy(Xq)).cpu().numpy()
    print(f"lib={os.environ.get('NPFN_LIB', 'tree')} scale={scale} online={onl}: "
          f"nonfinite rows {int((~np.isfinite(lg).all(1)).sum())}/{lg.shape[0]}, "
          f"nan {int(np.isnan(lg).sum())}")
eng.debug_item_attn_online(False)
lg = eng.predict_logits(torch.from_numpy(Xq)).cpu().numpy()
lg2 = eng.predict_logits(torch.from_numpy(Xq)).cpu().numpy()
print("repeat equal:", np.array_equal(lg, lg2, equal_nan=True))
for a, b in ((0, 210), (0, 256), (0, 128), (42, 252)):
    ls = eng.predict_logits(torch.from_numpy(Xq[a:b])).cpu().numpy()
    ref = lg[a:b]
    fin = np.isfinite(ref) & np.isfinite(ls)
    rows = np.nonzero(~((ls == ref) | (np.isnan(ls) & np.isnan(ref))).all(1))[0]
    d = np.abs(ls - ref)[fin].max() if fin.any() else 0.0
    print(f"slice [{a}:{b}] differing rows {len(rows)} first {rows[:8] + a} max|d| finite {d:.3g} "
          f"inf-pattern equal {np.array_equal(np.isfinite(ls), np.isfinite(ref))}")
