"""c2 at its own context size, end to end through the fused AR log-prob path.

The Gaussian-linear 10D task with all 1 000 simulations as context, tabpfn's default
preprocessing ensemble, 10 autoregressive steps (F = 10 .. 19 features, up to 25 tokens
per estimator row): ``npfn_ar_log_prob`` (plain and the repeated-row form c2's x_o uses)
against the CPU oracle's per-step fit / predict / bar NLL loop (reference
npe_pfn.py:462-524), precomputed in tests/golden/c2_logprob.npz by
tests/golden/make_golden_c2_logprob.py (the oracle takes minutes at this size).

Tolerance on the 10-dimension sum: median |d| <= 0.05, 95th percentile <= 0.1, max <= 0.2
(measured on MI355X: 0.0044 / 0.011 / 0.017, profiles/r04/gputest_c2_logprob_r04zc.txt), i.e.
under 0.01 nats per dimension at the median against the bf16-emulating oracle.
"""
import os

import numpy as np
import pytest
import torch

from npe_pfn.weights import ModelConfig, synthetic_weights

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "c2_logprob.npz")


def test_c2_ar_log_prob_matches_oracle():
    from npe_pfn.engine import Engine

    g = np.load(GOLDEN)
    cfg = ModelConfig()
    eng = Engine(cfg, synthetic_weights(cfg, seed=0), device=torch.device("cuda", 0), random_state=2)
    eng.set_preprocessing("ensemble")
    args = [torch.from_numpy(g[k]) for k in ("x", "theta", "xq", "tq")]
    ref = g["steps"].sum(0)
    for kw in ({}, {"x_unique": torch.from_numpy(g["xq"][:1])}):
        lp = eng.ar_log_prob(*args, **kw).cpu().numpy()
        assert np.isfinite(lp).all()
        diff = np.abs(lp - ref)
        print(f"c2 AR log-prob ({'repeated' if kw else 'plain'}): |d| median {np.median(diff):.4f} "
              f"p95 {np.quantile(diff, 0.95):.4f} max {diff.max():.4f}; far-tail row {lp[-1]:.2f} vs {ref[-1]:.2f}")
        assert np.median(diff) <= 0.05 and np.quantile(diff, 0.95) <= 0.1 and diff.max() <= 0.2, (
            np.median(diff), np.quantile(diff, 0.95), diff.max())
