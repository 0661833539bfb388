"""The K11 / K10 restatement (oracle/support_oracle.py) against the reference's torch arithmetic.

CPU only.  The reference's resampling step (support_posterior.py:219-235) is
evaluated here with torch exactly as written there, and the restatement must
give the same ESS and the same pick distribution (its draw uses Philox
uniforms instead of torch's Categorical, so picks agree in distribution).
"""
import numpy as np
import pytest
import torch

from oracle.support_oracle import box_mask, log_ratios, sir_select


def _reference_step(lpr, lq, afn, k):
    """support_posterior.py:219-232 verbatim in torch (the arithmetic under test)."""
    lpr = lpr.clone()
    thr = torch.quantile(lq, afn)
    lpr[lq < thr] = -float("inf")
    lr = torch.nan_to_num(lpr - lq, -float("inf")).reshape(-1, k)
    probs = torch.exp(lr - torch.logsumexp(lr, dim=1, keepdim=True))
    return thr, lr, probs, 1.0 / torch.sum(probs**2, dim=1)


@pytest.mark.parametrize("k,afn", [(100, 0.0), (7, 0.2), (130, 0.5), (1, 0.1)])
def test_log_ratios_and_ess_match_reference(k, afn):
    g = torch.Generator().manual_seed(k)
    G = 40
    lq = torch.randn(G * k, generator=g) * 3
    lpr = torch.randn(G * k, generator=g)
    lpr[::11] = -float("inf")  # outside the prior's support
    thr, lr, probs, ess_ref = _reference_step(lpr, lq, afn, k)
    lw = log_ratios(lpr.numpy(), lq.numpy(), float(thr))
    np.testing.assert_array_equal(lw.reshape(-1, k), lr.numpy())
    pick, ess = sir_select(lpr.numpy(), lq.numpy(), float(thr), k, seed=3, counter=0)
    np.testing.assert_allclose(ess, ess_ref.numpy(), rtol=1e-5)
    assert pick.min() >= 0 and pick.max() < k
    # a pick never lands on a zero-probability proposal
    assert np.all(probs.numpy()[np.arange(G), pick] > 0)


def test_nan_to_num_edge_cases():
    # NaN (inf - inf) -> -inf; +inf -> FLT_MAX; -inf -> -FLT_MAX, as torch.nan_to_num(x, -inf)
    lpr = np.array([-np.inf, 1.0, -np.inf, 0.0], np.float32)
    lq = np.array([-np.inf, -np.inf, 0.0, np.nan], np.float32)
    ref = torch.nan_to_num(torch.from_numpy(lpr) - torch.from_numpy(lq), -float("inf")).numpy()
    np.testing.assert_array_equal(log_ratios(lpr, lq, -np.inf), ref)


def test_fully_truncated_group_is_uniform_like_the_reference():
    k = 10
    lq = np.linspace(-5, 5, 2 * k).astype(np.float32)
    lpr = np.zeros(2 * k, np.float32)
    thr = 0.5  # group 0 lies entirely below the threshold
    _, _, probs, ess_ref = _reference_step(torch.from_numpy(lpr), torch.from_numpy(lq), 0.0, k)
    # the reference's own quantile is min(lq); restate with the fixed threshold instead
    lw = torch.from_numpy(log_ratios(lpr, lq, thr)).reshape(-1, k)
    p = torch.exp(lw - torch.logsumexp(lw, dim=1, keepdim=True))
    _, ess = sir_select(lpr, lq, thr, k, seed=1, counter=0)
    np.testing.assert_allclose(ess, (1.0 / (p**2).sum(1)).numpy(), rtol=1e-6)
    assert ess[0] == pytest.approx(1.0 / k)  # all -FLT_MAX: torch's probs are all 1


def test_pick_distribution_matches_categorical():
    k, reps = 6, 6000
    with np.errstate(divide="ignore"):
        logits = np.log(np.array([0.05, 0.3, 0.0, 0.15, 0.4, 0.1], np.float64)).astype(np.float32)
    lq = np.zeros(k * reps, np.float32)
    lpr = np.tile(logits, reps)
    pick, _ = sir_select(lpr, lq, -np.inf, k, seed=11, counter=2)
    freq = np.bincount(pick, minlength=k) / reps
    p = np.exp(logits.astype(np.float64))
    p /= p.sum()
    assert freq[2] == 0.0
    np.testing.assert_allclose(freq, p, atol=4 * np.sqrt(0.25 / reps))


def test_box_mask_matches_reference_expression():
    g = torch.Generator().manual_seed(0)
    s = torch.randn(1000, 3, generator=g)
    lo, hi = torch.tensor([-1.0, -0.5, -2.0]), torch.tensor([1.0, 0.5, 0.0])
    ref = torch.all((s >= lo) & (s <= hi), dim=1).numpy()
    np.testing.assert_array_equal(box_mask(s.numpy(), lo.numpy(), hi.numpy()), ref)
