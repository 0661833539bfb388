"""tabpfn keyword arguments the reference forwards unchanged (regressor_init_kwargs /
classifier_init_kwargs, /root/reference/npe_pfn/npe_pfn.py:45-48, 610): each is honoured,
refused, or a true no-op (npe_pfn/tabpfn.py, INTEGRATION.md "tabpfn keyword arguments").
CPU only: the estimator objects create their engine lazily, so construction needs no GPU; the
oracle's average_before_softmax mix is checked against its definition on a small model.
"""
import warnings

import numpy as np
import pytest
import torch

from npe_pfn.tabpfn import TabPFNClassifier, TabPFNRegressor


@pytest.mark.parametrize("cls", [TabPFNRegressor, TabPFNClassifier])
def test_average_before_softmax_is_honoured(cls):
    assert cls().average_before_softmax is False
    assert cls(average_before_softmax=True).average_before_softmax is True


@pytest.mark.parametrize("cls", [TabPFNRegressor, TabPFNClassifier])
def test_inference_precision(cls):
    for ok in ("auto", "autocast"):
        assert cls(inference_precision=ok).inference_precision == ok
    for bad in (torch.float32, torch.float64, torch.bfloat16, "fp32"):
        with pytest.raises(ValueError, match="bf16 MFMA"):
            cls(inference_precision=bad)


@pytest.mark.parametrize("cls", [TabPFNRegressor, TabPFNClassifier])
def test_result_changing_kwargs_only_at_their_defaults(cls):
    cls(categorical_features_indices=None, differentiable_input=False, inference_config=None)
    for kw in ({"categorical_features_indices": [0]}, {"differentiable_input": True},
               {"inference_config": {"FEATURE_SHIFT_METHOD": None}}):
        with pytest.raises(ValueError, match="not supported"):
            cls(**kw)


@pytest.mark.parametrize("cls", [TabPFNRegressor, TabPFNClassifier])
def test_noop_kwargs_warn_and_unknown_raise(cls):
    for kw in ({"fit_mode": "low_memory"}, {"memory_saving_mode": True}, {"n_jobs": 4},
               {"n_preprocessing_jobs": 2}):
        with pytest.warns(UserWarning, match="ignoring"):
            cls(**kw)
    with warnings.catch_warnings():
        warnings.simplefilter("error")
        cls(average_before_softmax=False, inference_precision="auto")  # honoured: no warning
    with pytest.raises(TypeError):
        cls(not_a_tabpfn_kwarg=1)


def test_balance_probabilities_classifier_only():
    assert TabPFNClassifier(balance_probabilities=True).balance_probabilities is True
    with pytest.raises(TypeError):
        TabPFNRegressor(balance_probabilities=True)


def _small_oracle(avg, classifier=False):
    from npe_pfn.weights import ModelConfig, classifier_config, synthetic_classifier_weights, synthetic_weights
    from oracle.tabpfn_oracle import OracleTabPFN

    if classifier:
        import dataclasses

        cfg = dataclasses.replace(classifier_config(4, 0.9), n_layers=2)
        w = synthetic_classifier_weights(cfg, seed=1)
    else:
        cfg = ModelConfig(n_layers=2, n_bars=64, n_estimators=4)
        w = synthetic_weights(cfg, seed=0)
    return OracleTabPFN(w, cfg.n_estimators, cfg.softmax_temperature, seed=5, average_before_softmax=avg,
                        preprocessing=3)


def test_oracle_average_before_softmax_regressor():
    """softmax(mean_e log q_e) of the estimators' (border-translated) probabilities q_e, with the
    ensemble preprocessing so translated estimators take part."""
    from oracle.tabpfn_oracle import softmax, translate_probs

    rng = np.random.default_rng(0)
    X = rng.normal(size=(60, 3)).astype(np.float32)
    y = np.exp(X[:, 0] + 0.3 * rng.normal(size=60)).astype(np.float32)   # skewed: target transform bites
    Xq = rng.normal(size=(9, 3)).astype(np.float32)
    orc = _small_oracle(True)
    orc.fit(X, y)
    p_geo, lg = orc.predict_probs(Xq, return_estimator_logits=True)
    st = orc.state
    logs = []
    for e, es in enumerate(st.estimators):
        l = lg[e] * np.float32(1 / orc.T)
        if es.target_tf:
            idx, share, flag, cancel = st.trans
            q = translate_probs(softmax(np.where(cancel[None], np.float32(-np.inf), l), -1), idx, share, flag)
        else:
            q = softmax(l, -1)
        with np.errstate(divide="ignore"):
            logs.append(np.log(q.astype(np.float64)))
    assert any(es.target_tf for es in st.estimators)
    z = np.mean(logs, 0)
    want = np.exp(z - z.max(1, keepdims=True))
    want /= want.sum(1, keepdims=True)
    np.testing.assert_allclose(p_geo, want, rtol=1e-5, atol=1e-9)
    assert np.allclose(p_geo.sum(1), 1.0, atol=1e-5)
    orc_mean = _small_oracle(False)
    orc_mean.fit(X, y)
    assert np.abs(orc_mean.predict_probs(Xq) - p_geo).sum(1).max() > 1e-4   # the switch does something


def test_oracle_average_before_softmax_classifier():
    """tabpfn's classifier form: the estimators' (un-permuted) class logits / T averaged, then one
    softmax."""
    rng = np.random.default_rng(1)
    X = rng.normal(size=(50, 2)).astype(np.float32)
    y = (X[:, 0] > 0).astype(np.int64)
    Xq = rng.normal(size=(7, 2)).astype(np.float32)
    orc = _small_oracle(True, classifier=True)
    orc.fit_classes(X, y, 2)
    p = orc.predict_proba(Xq)
    lg = orc._estimator_logits(Xq)
    z = np.mean([lg[e][:, orc.state.cperm[e]].astype(np.float64) / orc.T for e in range(orc.E)], 0)
    want = np.exp(z - z.max(1, keepdims=True))
    want /= want.sum(1, keepdims=True)
    np.testing.assert_allclose(p, want, rtol=1e-5, atol=1e-7)
