"""GPU: a TabPFN-v2-format checkpoint drives the engine through ``model_path=``.

The checkpoint is the synthetic weight set written under the v2 key layout
(npe_pfn/checkpoint.py) with a non-trivial positional ``Linear``; the engine
loaded from it must (a) produce the same logits, bit for bit, as the engine
given the converted tensors directly and (b) match the CPU oracle on those
tensors (TV <= 0.02 per row against the bf16-emulating oracle, the tolerance of
test_gpu_engine.py).
"""
import numpy as np
import pytest
import torch

from npe_pfn.checkpoint import load_tabpfn_checkpoint, weights_to_tabpfn_state
from npe_pfn.tabpfn import TabPFNRegressor
from npe_pfn.weights import ModelConfig, synthetic_weights
from oracle.tabpfn_oracle import OracleTabPFN

pytestmark = pytest.mark.gpu


def test_ckpt_model_path_matches_oracle(tmp_path):
    cfg = ModelConfig()
    w = synthetic_weights(cfg, seed=11)
    rng = np.random.default_rng(0)
    W = (rng.standard_normal((cfg.d_model, cfg.d_model // 4)) * 0.3).astype(np.float32)
    b = (0.1 * rng.standard_normal(cfg.d_model)).astype(np.float32)
    sd = {k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in weights_to_tabpfn_state(w, cfg, pos_base=(W, b)).items()}
    path = str(tmp_path / "v2.ckpt")
    torch.save({"state_dict": sd, "config": {"emsize": 192, "nhead": 6, "nlayers": 12, "nhid_factor": 4,
                                             "features_per_group": 2}}, path)
    _, conv = load_tabpfn_checkpoint(path)

    X = rng.normal(size=(150, 4)).astype(np.float32)
    y = (X @ rng.normal(size=4) + 0.2 * rng.normal(size=150)).astype(np.float32)
    Xq = rng.normal(size=(70, 4)).astype(np.float32)
    outs = []
    for kw in ({"model_path": path}, {"weights": conv}):
        reg = TabPFNRegressor(random_state=5, device="cuda:0", **kw)
        reg.fit(torch.from_numpy(X), torch.from_numpy(y))
        outs.append(reg.predict(torch.from_numpy(Xq), output_type="full")["logits"].float().cpu())
    assert torch.equal(outs[0], outs[1])

    orc = OracleTabPFN(conv, cfg.n_estimators, cfg.softmax_temperature, seed=5, emulate_bf16=True,
                       preprocessing=3)  # the regressor's default: tabpfn's preprocessing ensemble
    orc.fit(X, y)
    p_ref = orc.predict_probs(Xq).astype(np.float64)
    p_gpu = torch.softmax(outs[0], -1).numpy().astype(np.float64)
    tv = 0.5 * np.abs(p_gpu - p_ref).sum(1)
    assert tv.max() <= 0.02, (tv.max(), tv.mean())
