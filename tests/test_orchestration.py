"""Host orchestration vs golden vectors produced by the REFERENCE's own Python.

tests/golden/make_golden.py ran the reference npe_pfn.py / accept_reject_sampler.py /
support_posterior.py (loaded by path) with the oracle as ``tabpfn.TabPFNRegressor``.
Here the build's own orchestration (npe-pfn_amd/npe_pfn) drives the same oracle:
identical call sequences and identical numbers are required (CPU, no GPU needed).
"""
import json
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from oracle.tabpfn_oracle import OracleClassifier, OracleRegressor


@pytest.fixture(scope="module", autouse=True)
def oracle_as_tabpfn():
    from npe_pfn.weights import ModelConfig, synthetic_weights, weights_digest
    import npe_pfn.npe_pfn as mod

    meta = json.load(open(os.path.join(GOLDEN, "meta.json")))
    cfg = ModelConfig(**meta["config"])  # the fixtures' table (256 positional rows; ModelConfig() extends it)
    w = synthetic_weights(cfg, seed=meta["weights_seed"])
    assert weights_digest(w, cfg) == meta["weights_digest"], "synthetic weight generator drifted from the fixtures"
    OracleRegressor.default_weights = w
    from npe_pfn.weights import synthetic_classifier_weights

    ccfg = ModelConfig(**meta["classifier_config"])
    cw = synthetic_classifier_weights(ccfg, seed=meta["classifier_weights_seed"])
    assert weights_digest(cw, ccfg) == meta["classifier_weights_digest"], "classifier weights drifted"
    OracleClassifier.default_weights = cw
    saved = mod.TabPFNRegressor, mod.TabPFNClassifier
    mod.TabPFNRegressor = OracleRegressor
    mod.TabPFNClassifier = OracleClassifier
    yield
    mod.TabPFNRegressor, mod.TabPFNClassifier = saved


def _g(name):
    return np.load(os.path.join(GOLDEN, f"{name}.npz"))


def _box(lo, hi):
    from npe_pfn.support_posterior import BoxUniform

    return BoxUniform(torch.as_tensor(lo), torch.as_tensor(hi))


def test_core_sample_and_log_prob_c1():
    from npe_pfn.npe_pfn import NPE_PFN_Core

    g = _g("c1")
    prior = torch.distributions.Independent(
        torch.distributions.Normal(torch.zeros(2), torch.full((2,), float(np.sqrt(0.1)))), 1)
    core = NPE_PFN_Core(prior=prior, regressor_init_kwargs={"random_state": int(g["random_state"])})
    core.append_simulations(torch.from_numpy(g["theta"]), torch.from_numpy(g["x"]))
    s, lp = core.sample((1000,), x=torch.from_numpy(g["x_o"]), with_log_prob=True)
    np.testing.assert_allclose(s.numpy(), g["samples"], rtol=2e-5, atol=2e-6)
    np.testing.assert_allclose(lp.numpy(), g["log_probs"], rtol=2e-5, atol=2e-5)
    lp_ar = core.log_prob(s[:200], torch.from_numpy(g["x_o"]))
    np.testing.assert_allclose(lp_ar.numpy(), g["log_prob_ar"], rtol=2e-5, atol=2e-5)
    assert [list(map(lambda v: list(v) if isinstance(v, tuple) else v, c)) for c in core._model.calls] == \
        json.loads(str(g["calls"]))


def test_filtered_estimator_sample():
    from npe_pfn.npe_pfn import TabPFN_Based_NPE_PFN

    g = _g("filt")
    prior = torch.distributions.Independent(
        torch.distributions.Normal(torch.zeros(3), torch.full((3,), float(np.sqrt(0.1)))), 1)
    post = TabPFN_Based_NPE_PFN(prior=prior, filter_type="standardized_euclidean_filtering", filter_context_size=64,
                                regressor_init_kwargs={"random_state": int(g["random_state"])})
    post.append_simulations(torch.from_numpy(g["theta"]), torch.from_numpy(g["x"]))
    s, lp = post.sample((200,), x=torch.from_numpy(g["x_o"]), with_log_prob=True)
    np.testing.assert_allclose(s.numpy(), g["samples"], rtol=2e-5, atol=2e-6)
    np.testing.assert_allclose(lp.numpy(), g["log_probs"], rtol=2e-5, atol=2e-5)


def test_box_prior_rejection_loop():
    from npe_pfn.npe_pfn import NPE_PFN_Core

    g = _g("box")
    core = NPE_PFN_Core(prior=_box(g["low"], g["high"]), regressor_init_kwargs={"random_state": int(g["random_state"])})
    core.append_simulations(torch.from_numpy(g["theta"]), torch.from_numpy(g["x"]))
    s = core.sample((300,), x=torch.from_numpy(g["x_o"]), max_sampling_batch_size=250)
    np.testing.assert_allclose(s.numpy(), g["samples"], rtol=2e-5, atol=2e-6)
    calls = [[c[0], list(c[1]), c[2] if not isinstance(c[2], tuple) else list(c[2])] for c in core._model.calls]
    assert calls == json.loads(str(g["calls"]))


def test_sample_batched_with_rejection():
    from npe_pfn.npe_pfn import NPE_PFN_Core

    g = _g("batched")
    core = NPE_PFN_Core(prior=_box([-1.0, -1.0], [1.0, 1.0]),
                        regressor_init_kwargs={"random_state": int(g["random_state"])})
    core.append_simulations(torch.from_numpy(g["theta"]), torch.from_numpy(g["x"]))
    s, lp = core.sample_batched(torch.from_numpy(g["x_o"]), (40,), with_log_prob=True)
    np.testing.assert_allclose(s.numpy(), g["samples"], rtol=2e-5, atol=2e-6)
    np.testing.assert_allclose(lp.numpy(), g["log_probs"], rtol=2e-5, atol=2e-5)


@pytest.mark.parametrize("name", ["no_filtering", "latest_filtering", "random_filtering",
                                  "standardized_euclidean_filtering"])
def test_filters(name):
    from npe_pfn.support_posterior import get_filtering_method

    g = _g("filters")
    torch.manual_seed(1234)
    t, x = get_filtering_method(name)(torch.from_numpy(g["obs"]), torch.from_numpy(g["theta"]),
                                      torch.from_numpy(g["x"]), 100)
    np.testing.assert_array_equal(t.numpy(), g[name + "_theta"])
    np.testing.assert_array_equal(x.numpy(), g[name + "_x"])


def test_accept_reject_recurrence():
    from npe_pfn.accept_reject_sampler import accept_reject_sample

    g = _g("accrej")
    state = {"i": 0}

    def proposal(bs, **kw):
        state["i"] += 1
        gg = torch.Generator().manual_seed(100 + state["i"])
        c = torch.rand(bs, 2, generator=gg)
        return c, c.sum(1)

    trace = []

    def acc(c):
        trace.append(c.shape[0])
        return c[:, 0] < 0.3

    s, lps, rate = accept_reject_sample(proposal, acc, num_samples=700, max_sampling_batch_size=1000)
    assert trace == list(g["batch_trace"])
    np.testing.assert_array_equal(s.numpy(), g["samples"])
    np.testing.assert_array_equal(lps.numpy(), g["log_probs"])
    assert rate == float(g["rate"])


def test_max_iter_fallback_appends_unfiltered():
    from npe_pfn.accept_reject_sampler import accept_reject_sample

    def proposal(bs, **kw):
        return torch.ones(bs, 1), None

    s, lps, rate = accept_reject_sample(proposal, lambda c: torch.zeros(c.shape[0], dtype=torch.bool), 50,
                                        max_sampling_batch_size=20, max_iter_rejection=2)
    assert s.shape == (20, 1) and lps is None and rate == pytest.approx(20 / 60)  # reference :89


def test_sample_rejects_multiple_observations():
    from npe_pfn.npe_pfn import NPE_PFN_Core

    core = NPE_PFN_Core(prior=None)
    core.append_simulations(torch.randn(10, 2), torch.randn(10, 2))
    with pytest.raises(ValueError, match="batchsize == 1"):
        core.sample((5,), x=torch.randn(2, 2))


def test_pickling_drops_and_rebuilds_estimator():
    import pickle

    from npe_pfn.npe_pfn import NPE_PFN_Core

    core = NPE_PFN_Core(prior=None, regressor_init_kwargs={"random_state": 4})
    core.append_simulations(torch.randn(10, 2), torch.randn(10, 3))
    core2 = pickle.loads(pickle.dumps(core))
    assert core2._model is not None and core2._model is not core._model
    assert torch.equal(core2._theta_train, core._theta_train)


def test_ratio_based_log_prob():
    """DensityRatioWrapper orchestration (reference npe_pfn.py:526-704) with the oracle classifier."""
    from npe_pfn.npe_pfn import NPE_PFN_Core

    g = _g("ratio")
    prior = torch.distributions.Independent(
        torch.distributions.Normal(torch.zeros(2), torch.full((2,), float(np.sqrt(0.1)))), 1)
    core = NPE_PFN_Core(prior=prior, regressor_init_kwargs={"random_state": int(g["random_state"])},
                        classifier_init_kwargs={"random_state": int(g["clf_random_state"])})
    core.append_simulations(torch.from_numpy(g["theta"]), torch.from_numpy(g["x"]))
    th_q = torch.from_numpy(g["theta_q"])
    x_o = torch.from_numpy(g["x_o"])
    torch.manual_seed(int(g["torch_seed"]))
    lp = core.log_prob(th_q, x_o, mode="ratio_based", num_posterior_samples=100)
    lp2 = core.log_prob(th_q[:10], x_o, mode="ratio_based", num_posterior_samples=100)
    wrap = core._model_classifier
    np.testing.assert_allclose(wrap._padded_dim_min.numpy(), g["pad_min"], rtol=1e-6, atol=1e-6)
    np.testing.assert_allclose(wrap._padded_dim_max.numpy(), g["pad_max"], rtol=1e-6, atol=1e-6)
    np.testing.assert_allclose(lp.numpy(), g["log_prob"], rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(lp2.numpy(), g["log_prob_reuse"], rtol=1e-5, atol=1e-5)
    calls = [[c[0]] + [list(v) for v in c[1:]] for c in wrap._classifier.calls]
    assert calls == json.loads(str(g["clf_calls"]))  # one fit, reused for the second call


def test_class_permutation_is_a_permutation():
    from oracle.philox import class_permutation

    for e in range(8):
        for k in (2, 3, 10):
            p = class_permutation(5, e, k)
            assert sorted(p.tolist()) == list(range(k))
    assert any(class_permutation(5, e, 2)[0] == 1 for e in range(8))  # some estimators swap the labels


@pytest.mark.parametrize("method", ["rejection", "sir"])
def test_posterior_support_matches_reference(method):
    """PosteriorSupport (support_posterior.py:13-258) vs tests/golden/support.npz (make_golden_support.py)."""
    from npe_pfn.npe_pfn import TabPFN_Based_NPE_PFN
    from npe_pfn.support_posterior import PosteriorSupport

    g = _g("support")
    prior = torch.distributions.Independent(
        torch.distributions.Normal(torch.zeros(2), torch.full((2,), float(np.sqrt(0.1)))), 1)
    post = TabPFN_Based_NPE_PFN(prior=prior, regressor_init_kwargs={"random_state": int(g["random_state"])})
    post.append_simulations(torch.from_numpy(g["theta"]), torch.from_numpy(g["x"]))
    x_o = torch.from_numpy(g["x_o"])
    if method == "rejection":
        torch.manual_seed(2024)
        sup = PosteriorSupport(prior, post, x_o, num_samples_to_estimate_support=200,
                               batch_size_for_estimate_support=200, allowed_false_negatives=0.05,
                               sampling_method="rejection")
        s, rate = sup.sample((150,), show_progress_bars=False, sampling_batch_size=100, return_acceptance_rate=True)
        np.testing.assert_allclose(float(sup.thr), float(g["rej_thr"]), rtol=1e-5)
        np.testing.assert_allclose(s.numpy(), g["rej_samples"], rtol=2e-5, atol=2e-6)
        assert rate == pytest.approx(float(g["rej_rate"]))
        calls = json.loads(str(g["rej_calls"]))
    else:
        torch.manual_seed(77)
        sup = PosteriorSupport(prior, post, x_o, allowed_false_negatives=0.05, sampling_method="sir",
                               oversample_sir=10)
        s, ess = sup.sample((25,), show_progress_bars=False, sampling_batch_size=100, return_ess=True)
        np.testing.assert_allclose(s.numpy(), g["sir_samples"], rtol=2e-5, atol=2e-6)
        np.testing.assert_allclose(ess.numpy(), g["sir_ess"], rtol=1e-4)
        calls = json.loads(str(g["sir_calls"]))
    got = [[c[0], list(c[1]), c[2] if not isinstance(c[2], tuple) else list(c[2])] for c in post._model.calls]
    assert got == calls


def test_sample_batched_per_observation_quota_and_order(monkeypatch):
    """Vectorised per-observation rejection (reference npe_pfn.py:360-410): each observation
    keeps its first accepted draws in order across rounds; an observation that never fills
    fails as the reference's final torch.stack does."""
    from npe_pfn.npe_pfn import NPE_PFN_Core

    core = NPE_PFN_Core(prior=_box([-1.0], [1.0]))
    rounds = []

    def fake(x, n, with_log_prob=False, eps=1e-15):
        r = len(rounds)
        rounds.append(n)
        th = torch.full((x.shape[0], n, 1), 5.0)               # out of support by default
        th[0, ::2, 0] = torch.arange(0, n, 2) / 100.0 + r        # obs 0: every other draw accepted in round 0
        th[0, ::2, 0] = torch.where(th[0, ::2, 0] < 1.0, th[0, ::2, 0], torch.tensor(5.0))
        if r >= 1:
            th[1, :3, 0] = torch.tensor([0.1, 0.2, 0.3]) * r     # obs 1: three per round from round 1
        lp = th[..., 0] * 10
        return th, lp

    monkeypatch.setattr(core, "_sample_batched", fake)
    with pytest.raises(RuntimeError, match="fewer than"):
        core.sample_batched(torch.zeros(2, 1), (4,), with_log_prob=True)
    assert len(rounds) == 10 and rounds[0] == 6

    rounds.clear()

    def fake2(x, n, with_log_prob=False, eps=1e-15):
        r = len(rounds)
        rounds.append(n)
        th = torch.full((x.shape[0], n, 1), 5.0)
        th[0, :, 0] = torch.linspace(-0.9, 0.9, n)               # obs 0 fills in round 0
        th[1, r::4, 0] = 0.01 * (r + 1)                          # obs 1: sparse acceptances per round
        return th, th[..., 0] * 10

    monkeypatch.setattr(core, "_sample_batched", fake2)
    s, lp = core.sample_batched(torch.zeros(2, 1), (4,), with_log_prob=True)
    assert s.shape == (2, 4, 1) and lp.shape == (2, 4)
    np.testing.assert_allclose(s[0, :, 0].numpy(), torch.linspace(-0.9, 0.9, 6)[:4].numpy())
    np.testing.assert_allclose(s[1, :, 0].numpy(), [0.01, 0.01, 0.02, 0.02])   # round 0 then round 1, in order
    np.testing.assert_allclose(lp.numpy(), s[..., 0].numpy() * 10)


def test_tsnpe_round_loop_matches_reference():
    """c4's orchestration: the repo's run_tsnpe_pfn (own ``simulate`` in place of sbi's
    simulate_for_sbi) against tests/golden/tsnpe.npz, made by the REFERENCE's tsnpe_pfn.py
    (make_golden_tsnpe.py): same rounds, same simulations, same SIR proposals, same final
    posterior draws, with the same (small) oracle estimator and torch seeds."""
    import sys

    sys.path.insert(0, GOLDEN)
    from make_golden_tsnpe import TSNPE_KW, TINY, simulator

    from npe_pfn import run_tsnpe_pfn
    from npe_pfn.support_posterior import BoxUniform
    from npe_pfn.weights import ModelConfig, synthetic_weights

    g = _g("tsnpe")
    prior = BoxUniform(torch.full((2,), float(g["low"])), torch.full((2,), float(g["high"])))
    x_o = torch.from_numpy(g["x_o"])
    rk = {"random_state": 9, "preprocessing": "none", "weights": synthetic_weights(ModelConfig(**TINY), seed=3)}
    torch.manual_seed(123)
    post = run_tsnpe_pfn(simulator, prior, x_o, regressor_init_kwargs=rk, **TSNPE_KW)
    np.testing.assert_array_equal(post._theta_train.numpy(), g["theta"])
    np.testing.assert_array_equal(post._x_train.numpy(), g["x"])
    torch.manual_seed(321)
    s = post.sample((300,), x=x_o)
    np.testing.assert_allclose(s.numpy(), g["samples"], rtol=2e-5, atol=2e-6)
