"""GPU parity of the support kernels (K9-K12) through the C-ABI.

* K11 ``npfn_sir_select`` vs oracle/support_oracle.sir_select on the same
  inputs and Philox stream: ESS within rtol 1e-5 (fp32 exp / fp64 sums on both
  sides), picks identical except where u * sum lands within rounding of a CDF
  step (allowed: <= 0.2 % of groups), gathered rows bit-exact for the pick;
* K9 mask + K10 ordered compaction vs torch boolean indexing: bit-exact;
* K12 standardized-Euclidean filter vs the reference-generated golden
  (tests/golden/filters.npz): bit-exact selection;
* PosteriorSupport (rejection and SIR) end to end on the engine, shaped like
  the reference's tests/test_support_posterior.py (sizes reduced).
"""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from oracle.support_oracle import box_mask, sir_select as oracle_sir

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda", 0)


def _sir_case(G, k, seed, afn=0.1, nan_every=0):
    g = torch.Generator().manual_seed(seed)
    lq = torch.randn(G * k, generator=g) * 4
    lpr = torch.randn(G * k, generator=g)
    lpr[::13] = -float("inf")
    if nan_every:
        lq[::nan_every] = -float("inf")
        lpr[::nan_every] = -float("inf")  # -inf - -inf = NaN -> -inf ratio
    thr = torch.quantile(lq[torch.isfinite(lq)], afn)
    th = torch.randn(G * k, 3, generator=g)
    return th, lpr, lq, thr


@pytest.mark.parametrize("G,k", [(1000, 100), (257, 7), (64, 300), (50, 1), (33, 64), (20, 4096)])
def test_sir_select_matches_oracle(G, k):
    from npe_pfn.support_posterior import sir_select

    th, lpr, lq, thr = _sir_case(G, k, seed=G + k, nan_every=17 if k > 1 else 0)
    sel, pick, ess = sir_select(th.to(DEV), lpr.to(DEV), lq.to(DEV), thr.to(DEV), k, seed=99, counter=5)
    ref_pick, ref_ess = oracle_sir(lpr.numpy(), lq.numpy(), float(thr), k, seed=99, counter=5)
    pick, ess, sel = pick.cpu().numpy(), ess.cpu().numpy(), sel.cpu().numpy()
    np.testing.assert_allclose(ess, ref_ess, rtol=1e-5)
    mism = np.count_nonzero(pick != ref_pick)
    assert mism <= max(1, G // 500), (mism, G)
    np.testing.assert_array_equal(sel, th.numpy().reshape(G, k, 3)[np.arange(G), pick])


def test_sir_select_degenerate_groups():
    from npe_pfn.support_posterior import sir_select

    k = 10
    lq = torch.linspace(-5, 5, 3 * k)
    lpr = torch.zeros(3 * k)
    lpr[2 * k:] = float("nan")  # group 2: every ratio NaN -> -inf -> NaN probabilities in torch
    thr = torch.tensor(-4.0)  # group 0 partly, group 1 not truncated
    thr_all = torch.tensor(0.5)  # group 0 fully truncated: uniform like the reference
    th = torch.arange(3 * k * 2, dtype=torch.float32).reshape(3 * k, 2)
    for t in (thr, thr_all):
        _, pick, ess = sir_select(th.to(DEV), lpr.to(DEV), lq.to(DEV), t.to(DEV), k, seed=1)
        rp, re = oracle_sir(lpr.numpy(), lq.numpy(), float(t), k, seed=1, counter=0)
        np.testing.assert_allclose(ess.cpu().numpy()[:2], re[:2], rtol=1e-5)
        assert np.isnan(ess.cpu().numpy()[2]) and np.isnan(re[2])
        np.testing.assert_array_equal(pick.cpu().numpy(), rp)


def test_box_compact_bit_exact():
    from npe_pfn.support_posterior import box_compact

    g = torch.Generator().manual_seed(4)
    for n, D in [(100_000, 3), (1_000, 1), (0, 2), (5_000, 10)]:
        s = torch.randn(n, D, generator=g)
        lo, hi = -torch.rand(D, generator=g), torch.rand(D, generator=g)
        got = box_compact(s.to(DEV), lo.to(DEV), hi.to(DEV)).cpu()
        ref = s[torch.from_numpy(box_mask(s.numpy(), lo.numpy(), hi.numpy()))]
        assert torch.equal(got, ref)


def test_prereject_with_bounds_on_device():
    from npe_pfn.support_posterior import prereject_with_bounds

    prior = torch.distributions.Independent(
        torch.distributions.Normal(torch.zeros(2, device=DEV), torch.ones(2, device=DEV)), 1)
    lo, hi = torch.tensor([-0.5, -1.0], device=DEV), torch.tensor([1.0, 0.2], device=DEV)
    torch.manual_seed(0)
    s, rate = prereject_with_bounds(prior, lo, hi, sampling_batch_size=5000, pre_sampling_batch_size=20_000)
    assert s.shape == (5000, 2) and s.is_cuda
    assert bool(((s >= lo) & (s <= hi)).all())
    assert 0.1 < rate < 0.3  # P(box) = 0.2902 * 0.4207 = 0.122 for N(0, 1)


def test_stdeuclid_filter_matches_golden():
    from npe_pfn.support_posterior import standardized_euclidean_filtering

    g = np.load(os.path.join(GOLDEN, "filters.npz"))
    t, x = standardized_euclidean_filtering(torch.from_numpy(g["obs"]).to(DEV), torch.from_numpy(g["theta"]).to(DEV),
                                            torch.from_numpy(g["x"]).to(DEV), 100)
    np.testing.assert_array_equal(t.cpu().numpy(), g["standardized_euclidean_filtering_theta"])
    np.testing.assert_array_equal(x.cpu().numpy(), g["standardized_euclidean_filtering_x"])


@pytest.mark.parametrize("method,n", [("rejection", 300), ("sir", 40)])
def test_posterior_support_on_engine(method, n):
    """Reference tests/test_support_posterior.py:14-70 at reduced sizes, on the GPU engine."""
    from npe_pfn.npe_pfn import TabPFN_Based_NPE_PFN
    from npe_pfn.support_posterior import PosteriorSupport

    torch.manual_seed(0)
    prior = torch.distributions.MultivariateNormal(torch.zeros(2, device=DEV), torch.eye(2, device=DEV))
    theta = prior.sample((1000,))
    x = theta + torch.randn_like(theta)
    post = TabPFN_Based_NPE_PFN(prior=prior, filter_type="standardized_euclidean_filtering",
                                regressor_init_kwargs={"random_state": 0, "device": DEV})
    post.append_simulations(theta, x)
    sup = PosteriorSupport(prior, post, torch.zeros(2, device=DEV), num_samples_to_estimate_support=2000,
                           batch_size_for_estimate_support=2000, allowed_false_negatives=0.001,
                           sampling_method=method, oversample_sir=10)
    out = sup.sample((n,), show_progress_bars=False, sampling_batch_size=1000,
                     **({"return_ess": True} if method == "sir" else {}))
    s = out[0] if method == "sir" else out
    assert s.shape == (n, 2)
    assert torch.isfinite(s).all()
    if method == "sir":
        ess = out[1]
        assert ess.shape == (((n + 99) // 100) * 100,)
        assert bool(((ess >= 1.0 - 1e-4) & (ess <= 10.0 + 1e-3)).all())
