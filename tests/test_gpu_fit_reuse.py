"""Per-step fit slots under fit tokens (npfn_set_fit_token, npfn_ar_fit_begin / _step): a slot
filled under another token, context or estimator set must never be taken for this call's fit.

The reference refits at every step of every call (npe_pfn.py:135-140); the engine keeps a
step's fit only while the token, the context shape, the preprocessing mode and the estimator
set are unchanged.  Each case compares the stepwise path's target tokens with a fresh
engine that fits the same context with npfn_fit -- bit for bit."""
import pytest
import torch

from npe_pfn.tasks import gaussian_linear_task
from npe_pfn.weights import ModelConfig, synthetic_weights

pytestmark = pytest.mark.gpu

CFG = ModelConfig()
DEV = torch.device("cuda", 0)


@pytest.fixture(scope="module")
def weights():
    return synthetic_weights(CFG, seed=0)


def _fresh_tokens(weights, x, theta, k, xq, est_set=None):
    from npe_pfn.engine import Engine

    e = Engine(CFG, weights, device=DEV, random_state=3)
    if est_set is not None:
        e.set_estimator_set(*est_set)
    joint = torch.cat([x, theta], 1)
    dx = x.shape[1]
    e.fit(joint[:, : dx + k], joint[:, dx + k])
    return e.forward_targets(torch.cat([xq, theta[: xq.shape[0], :k]], 1))


def _step_tokens(e, x, theta, k, xq):
    e.ar_fit_begin(x, theta)
    for j in range(k + 1):
        e.ar_fit_step(j)
    return e.forward_targets(torch.cat([xq, theta[: xq.shape[0], :k]], 1))


def test_single_dim_new_token_new_context_refits(weights):
    """dim_theta = 1 (no piping): the second token's context differs, so its step-0 fit must be
    recomputed, not read from the slot the first token filled."""
    from npe_pfn.engine import Engine

    thA, xA, _ = gaussian_linear_task(1, 200, seed=1)
    thB, xB, _ = gaussian_linear_task(1, 200, seed=2)
    xA, thA, xB, thB = (t.to(DEV) for t in (xA, thA, xB, thB))
    xq = xB[:50]
    e = Engine(CFG, weights, device=DEV, random_state=3)
    e.set_fit_token(101)
    _step_tokens(e, xA, thA, 0, xq)
    e.set_fit_token(102)
    got = _step_tokens(e, xB, thB, 0, xq)
    e.set_fit_token(0)
    assert torch.equal(got, _fresh_tokens(weights, xB, thB, 0, xq))


def test_estimator_set_change_between_tokens_refits(weights):
    """A new estimator set between two tokens on the same context: the slots hold the old set's
    per-estimator layout and must be refitted."""
    from npe_pfn.engine import Engine

    th, x, _ = gaussian_linear_task(3, 250, seed=4)
    th, x = th.to(DEV), x.to(DEV)
    xq = x[:40]
    e = Engine(CFG, weights, device=DEV, random_state=3)
    e.set_fit_token(201)
    e.set_estimator_set(0, 4, 2)
    _step_tokens(e, x, th, 2, xq)
    e.set_fit_token(202)
    e.set_estimator_set(1, 4, 2)
    got = _step_tokens(e, x, th, 2, xq)
    e.set_fit_token(0)
    assert torch.equal(got, _fresh_tokens(weights, x, th, 2, xq, est_set=(1, 4, 2)))


def test_same_token_reuses_and_matches(weights):
    """Two passes under ONE token on one context: the second reuses every slot and gives the
    same tokens as the first and as a fresh fit."""
    from npe_pfn.engine import Engine

    th, x, _ = gaussian_linear_task(2, 180, seed=6)
    th, x = th.to(DEV), x.to(DEV)
    xq = x[:30]
    e = Engine(CFG, weights, device=DEV, random_state=3)
    e.set_fit_token(301)
    a = _step_tokens(e, x, th, 1, xq)
    b = _step_tokens(e, x, th, 1, xq)
    e.set_fit_token(0)
    assert torch.equal(a, b)
    assert torch.equal(a, _fresh_tokens(weights, x, th, 1, xq))
