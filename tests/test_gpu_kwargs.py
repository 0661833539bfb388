"""GPU parity of tabpfn's ``average_before_softmax=True`` (npfn_set_average_before_softmax) against
the oracle's restatement (oracle/tabpfn_oracle.py, checked against its definition on the CPU in
tests/test_kwargs.py).  The reference forwards the kwarg unchanged through regressor_init_kwargs /
classifier_init_kwargs (/root/reference/npe_pfn/npe_pfn.py:45-48, 610).

Tolerances as tests/test_gpu_engine.py / test_gpu_classifier.py: predictive bars TV <= 0.02 per row
against the bf16-emulating oracle (default ensemble preprocessing, so the border-translated
estimators take part); class probabilities max |dp| <= 0.01; the fused AR sampler's draws within 1 %
of 10 sigma at the median of the oracle loop's, same uniforms.
"""
import numpy as np
import pytest
import torch

from npe_pfn.weights import ModelConfig, classifier_config, synthetic_classifier_weights, synthetic_weights
from oracle.philox import uniforms
from oracle.tabpfn_oracle import OracleTabPFN, bar_sample

pytestmark = pytest.mark.gpu

CFG = ModelConfig()
DEV = torch.device("cuda", 0)


@pytest.fixture(scope="module")
def weights():
    return synthetic_weights(CFG, seed=0)


def _table(n, F, N, seed):
    rng = np.random.default_rng(seed)
    X = rng.normal(size=(n, F)).astype(np.float32)
    y = np.exp(X[:, 0] + 0.4 * rng.normal(size=n)).astype(np.float32)   # skewed target: translated estimators
    Xq = rng.normal(size=(N, F)).astype(np.float32)
    return X, y, Xq


@pytest.mark.parametrize("n,F,N", [(300, 4, 90), (120, 2, 50)])
def test_regressor_average_before_softmax_matches_oracle(weights, n, F, N):
    from npe_pfn.engine import Engine

    X, y, Xq = _table(n, F, N, seed=n + F)
    eng = Engine(CFG, weights, device=DEV, random_state=4)
    eng.fit(torch.from_numpy(X), torch.from_numpy(y))
    p_mean = torch.softmax(eng.predict_logits(torch.from_numpy(Xq)), -1).double().cpu().numpy()
    eng.set_average_before_softmax(True)
    p_geo = torch.softmax(eng.predict_logits(torch.from_numpy(Xq)), -1).double().cpu().numpy()
    orc = OracleTabPFN(weights, CFG.n_estimators, CFG.softmax_temperature, seed=4, emulate_bf16=True,
                       preprocessing=3, average_before_softmax=True)
    orc.fit(X, y)
    assert any(es.target_tf for es in orc.state.estimators)
    p_ref = orc.predict_probs(Xq).astype(np.float64)
    tv = 0.5 * np.abs(p_geo - p_ref).sum(1)
    assert tv.max() <= 0.02, (tv.max(), tv.mean())
    tv_mean = 0.5 * np.abs(p_mean - p_ref).sum(1)
    assert tv_mean.mean() > 2 * tv.mean(), (tv_mean.mean(), tv.mean())   # the switch is live
    eng.set_average_before_softmax(False)
    p_back = torch.softmax(eng.predict_logits(torch.from_numpy(Xq)), -1).double().cpu().numpy()
    assert np.array_equal(p_back, p_mean)


def test_regressor_average_before_softmax_ar_sample(weights):
    """The fused sampler mixes with the same switch (k_mix_sample / k_mix_prob + k_group_sample):
    draws within 1 % of 10 sigma (median) of the oracle loop with the same uniforms, and the
    repeated-row step 0 equal to the plain path bit for bit."""
    from npe_pfn.engine import Engine

    rng = np.random.default_rng(8)
    n, dx, dth, N = 200, 3, 2, 64
    th = rng.normal(size=(n, dth)).astype(np.float32)
    x = (th @ rng.normal(size=(dth, dx)) + 0.2 * rng.normal(size=(n, dx))).astype(np.float32)
    x[:, 0] = np.exp(x[:, 0])
    xq = np.repeat(x[:1], N, 0)
    eng = Engine(CFG, weights, device=DEV, random_state=6)
    eng.set_average_before_softmax(True)
    theta, _ = eng.ar_sample(torch.from_numpy(x), torch.from_numpy(th), torch.from_numpy(xq), counter=2)
    theta_rep, _ = eng.ar_sample(torch.from_numpy(x), torch.from_numpy(th), torch.from_numpy(xq), counter=2,
                                 x_unique=torch.from_numpy(x[:1]))
    assert torch.equal(theta, theta_rep)
    theta = theta.cpu().numpy()
    orc = OracleTabPFN(weights, CFG.n_estimators, CFG.softmax_temperature, seed=6, emulate_bf16=True,
                       preprocessing=3, average_before_softmax=True)
    joint = np.concatenate([x, th], 1)
    feats = xq.copy()
    for k in range(dth):
        orc.fit(joint[:, : dx + k], joint[:, dx + k])
        p = orc.predict_probs(feats)
        sk = bar_sample(np.log(np.maximum(p, 1e-38)), orc.borders(), uniforms(6, 2 + k, N))
        span = np.std(joint[:, dx + k]) * 10
        assert np.median(np.abs(theta[:, k] - sk)) <= 0.01 * span, k
        feats = np.concatenate([feats, theta[:, k: k + 1]], 1)


def test_classifier_average_before_softmax_and_balance(weights):
    from npe_pfn.tabpfn import TabPFNClassifier

    ccfg = classifier_config()
    cw = synthetic_classifier_weights(ccfg, seed=1)
    rng = np.random.default_rng(3)
    X = rng.normal(size=(160, 3)).astype(np.float32)
    y = (X @ np.array([1.0, -0.5, 0.3]) > 0.6).astype(np.int64)    # unbalanced classes
    Xq = rng.normal(size=(70, 3)).astype(np.float32)
    clf = TabPFNClassifier(weights=cw, device=DEV, random_state=4, preprocessing="none",
                           average_before_softmax=True)
    clf.fit(torch.from_numpy(X), torch.from_numpy(y))
    p = clf.predict_proba(torch.from_numpy(Xq))
    orc = OracleTabPFN(cw, ccfg.n_estimators, ccfg.softmax_temperature, seed=4, emulate_bf16=True,
                       average_before_softmax=True)
    orc.fit_classes(X, y, 2)
    assert np.abs(p - orc.predict_proba(Xq)).max() <= 0.01
    bal = TabPFNClassifier(weights=cw, device=DEV, random_state=4, preprocessing="none", balance_probabilities=True)
    bal.fit(torch.from_numpy(X), torch.from_numpy(y))
    pb = bal.predict_proba(torch.from_numpy(Xq))
    orc0 = OracleTabPFN(cw, ccfg.n_estimators, ccfg.softmax_temperature, seed=4, emulate_bf16=True)
    orc0.fit_classes(X, y, 2)
    q = orc0.predict_proba(Xq) / (np.bincount(y) / len(y))
    q /= q.sum(1, keepdims=True)
    assert np.abs(pb - q).max() <= 0.01
