"""Observation sharding on the engine (SURVEY.md §8e, config c5 in miniature).

Two estimators that each sample one observation shard with the shard's Philox
row base (``_obs_offset`` -> ``npfn_ar_sample(row_base)``) reproduce the 1-GPU
``sample_batched`` of all observations bit for bit: every row draws the same
uniforms, and the forward is batch-invariant (a row's arithmetic does not depend
on where it sits in the row kernel's tile: npfn_rowk2.hip feat_attn_rows).
Without the row base the draws are unrelated (median |d theta| ~ 0.2).
"""
import pytest
import torch

from npe_pfn.tasks import gaussian_linear_prior, gaussian_linear_task

pytestmark = pytest.mark.gpu


def _post(theta, x, dev):
    from npe_pfn import NPE_PFN_Core

    p = NPE_PFN_Core(prior=gaussian_linear_prior(theta.shape[1], device=dev),
                     regressor_init_kwargs={"random_state": 11, "device": dev})
    p.append_simulations(theta.to(dev), x.to(dev))
    return p


def test_sharded_sample_batched_bitwise_equal():
    dev = torch.device("cuda", 0)
    theta, x, _ = gaussian_linear_task(3, 300, seed=5)
    x_obs = gaussian_linear_task(3, 5, seed=9)[1].to(dev)   # 5 observations
    full, lp_full = _post(theta, x, dev).sample_batched(x_obs, (64,), with_log_prob=True)
    parts, lps = [], []
    for a, b in ((0, 2), (2, 5)):
        p = _post(theta, x, dev)     # a fresh estimator per shard, like one per rank
        p._obs_offset = a
        th, lp = p.sample_batched(x_obs[a:b], (64,), with_log_prob=True)
        parts.append(th)
        lps.append(lp)
    assert torch.equal(torch.cat(parts), full), (torch.cat(parts) - full).abs().max()
    assert torch.equal(torch.cat(lps), lp_full), (torch.cat(lps) - lp_full).abs().max()
    # a shard without the row base draws other uniforms: unrelated samples
    p = _post(theta, x, dev)
    d0 = (p.sample_batched(x_obs[2:5], (64,)) - full[2:5]).abs().flatten()
    assert d0.median() > 0.02, d0.median()
