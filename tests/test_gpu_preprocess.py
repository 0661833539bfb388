"""GPU parity of the preprocessing modes (npfn_set_preprocessing(h, 1 | 2 | 3)).

k_quantile_fit / k_power_fit / k_svd_fit / the SHA-256 fingerprints / the target
transform + border translation (k_target_tf, k_mix_*) against the oracle with
``preprocessing=1 | 2 | 3`` (oracle/preprocess_oracle.py, itself pinned to sklearn's
QuantileTransformer / PowerTransformer / TruncatedSVD and to hashlib in
tests/test_preprocess_oracle.py).  Tolerances are those of
test_gpu_engine.py: TV <= 0.02 per row against the bf16-emulating oracle; the fused
AR sampler's draws within 1 % of 10 sigma at the median.
"""
import numpy as np
import pytest
import torch

from npe_pfn.weights import ModelConfig, synthetic_weights
from oracle.philox import uniforms
from oracle.tabpfn_oracle import OracleTabPFN, bar_sample

pytestmark = pytest.mark.gpu

CFG = ModelConfig()


@pytest.fixture(scope="module")
def weights():
    return synthetic_weights(CFG, seed=0)


def _table(n, F, N, seed):
    rng = np.random.default_rng(seed)
    X = rng.normal(size=(n, F)).astype(np.float32)
    X[:, 0] = np.exp(2.0 * X[:, 0])                          # heavy right tail: the transform matters
    X[:, 1] = rng.integers(0, 5, size=n).astype(np.float32)   # ties -> repeated quantiles
    y = (np.log(X[:, 0]) + X[:, 1] + 0.3 * rng.normal(size=n)).astype(np.float32)
    Xq = rng.normal(size=(N, F)).astype(np.float32)
    Xq[:, 0] = np.exp(2.5 * Xq[:, 0])                        # values beyond the train range too
    Xq[:, 1] = rng.integers(-1, 7, size=N).astype(np.float32)
    Xq[3, 2] = np.nan                                         # NaN indicator path
    return X, y, Xq


MODES = {"quantile": 1, "quantile+power": 2, "ensemble": 3}


@pytest.mark.parametrize("mode", list(MODES))
@pytest.mark.parametrize("n,F,N", [(300, 4, 90), (1000, 3, 64), (57, 5, 33)])
def test_preprocessed_predict_matches_oracle(weights, n, F, N, mode):
    from npe_pfn.engine import Engine

    X, y, Xq = _table(n, F, N, seed=n + F)
    eng = Engine(CFG, weights, device=torch.device("cuda", 0), random_state=4)
    out = {}
    for m in ("none", mode):
        eng.set_preprocessing(m)
        eng.fit(torch.from_numpy(X), torch.from_numpy(y))
        out[m] = torch.softmax(eng.predict_logits(torch.from_numpy(Xq)), -1).double().cpu().numpy()
    orc = OracleTabPFN(weights, CFG.n_estimators, CFG.softmax_temperature, seed=4, emulate_bf16=True,
                       preprocessing=MODES[mode])
    orc.fit(X, y)
    p_ref = orc.predict_probs(Xq).astype(np.float64)
    tv = 0.5 * np.abs(out[mode] - p_ref).sum(1)
    assert tv.max() <= 0.02, (tv.max(), tv.mean())
    # the mode is live: without it the prediction sits much further from the quantile oracle
    tv_none = 0.5 * np.abs(out["none"] - p_ref).sum(1)
    assert tv_none.mean() > max(3 * tv.mean(), 0.005), (tv_none.mean(), tv.mean())


@pytest.mark.parametrize("mode", list(MODES))
def test_preprocessed_ar_sample_matches_oracle_loop(weights, mode):
    from npe_pfn.engine import Engine

    rng = np.random.default_rng(8)
    n, dx, dth, N = 200, 3, 2, 64
    th = rng.normal(size=(n, dth)).astype(np.float32)
    x = np.exp(th @ rng.normal(size=(dth, dx)) + 0.2 * rng.normal(size=(n, dx))).astype(np.float32)
    xq = np.repeat(x[:1], N, 0)
    eng = Engine(CFG, weights, device=torch.device("cuda", 0), random_state=6)
    eng.set_preprocessing(mode)
    theta, _ = eng.ar_sample(torch.from_numpy(x), torch.from_numpy(th), torch.from_numpy(xq), counter=2)
    theta = theta.cpu().numpy()
    orc = OracleTabPFN(weights, CFG.n_estimators, CFG.softmax_temperature, seed=6, emulate_bf16=True,
                       preprocessing=MODES[mode])
    joint = np.concatenate([x, th], 1)
    feats = xq.copy()
    for k in range(dth):
        orc.fit(joint[:, : dx + k], joint[:, dx + k])
        p = orc.predict_probs(feats)
        sk = bar_sample(np.log(np.maximum(p, 1e-38)), orc.borders(), uniforms(6, 2 + k, N))
        feats = np.concatenate([feats, theta[:, k: k + 1]], 1)
        span = np.std(joint[:, dx + k]) * 10
        diff = np.abs(theta[:, k] - sk)
        assert np.median(diff) <= 0.01 * span, (k, np.median(diff))


def test_quantile_mode_rejects_oversized_context(weights):
    """sklearn's QuantileTransformer refuses n_quantiles = n // 5 > subsample = 10 000; the same
    ValueError before the engine is called (contexts up to 50 004 rows fit on the subsample)."""
    from npe_pfn.engine import Engine

    eng = Engine(CFG, weights, device=torch.device("cuda", 0), random_state=0)
    eng.set_preprocessing("quantile")
    X = torch.zeros(50_005, 2)
    with pytest.raises(ValueError, match="10001 quantiles and 10000 samples"):
        eng.fit(X, torch.zeros(50_005))
    with pytest.raises(ValueError):
        eng.set_preprocessing("power")


@pytest.mark.parametrize("mode", ["none"] + list(MODES))
def test_ar_log_prob_matches_oracle(weights, mode):
    """Fused npfn_ar_log_prob (teacher-forced sum over dims, reference npe_pfn.py:462-524,
    -inf -> log(eps) per dim) vs the oracle's fit/predict/NLL loop; tolerance as the
    posterior log-prob test: median |d| <= 0.05, 95th percentile <= 0.25."""
    from npe_pfn.engine import Engine
    from oracle.tabpfn_oracle import bar_nll

    rng = np.random.default_rng(21)
    n, dx, dth, N = 150, 3, 2, 80
    th = rng.normal(size=(n, dth)).astype(np.float32)
    x = np.exp(0.5 * (th @ rng.normal(size=(dth, dx)))) + 0.1 * rng.normal(size=(n, dx))
    x = x.astype(np.float32)
    xq = np.repeat(x[:1], N, 0)
    tq = rng.normal(size=(N, dth)).astype(np.float32)
    tq[0] = 40.0                                   # far tail: half-normal end bars
    eng = Engine(CFG, weights, device=torch.device("cuda", 0), random_state=2)
    eng.set_preprocessing(mode)  # "none" included: the engine's default is the ensemble
    lp = eng.ar_log_prob(torch.from_numpy(x), torch.from_numpy(th), torch.from_numpy(xq),
                         torch.from_numpy(tq)).cpu().numpy()
    orc = OracleTabPFN(weights, CFG.n_estimators, CFG.softmax_temperature, seed=2, emulate_bf16=True,
                       preprocessing=0 if mode == "none" else MODES[mode])
    joint = np.concatenate([x, th], 1)
    test = np.concatenate([xq, tq], 1)
    ref = np.zeros(N)
    for k in range(dth):
        orc.fit(joint[:, : dx + k], joint[:, dx + k])
        p = orc.predict_probs(test[:, : dx + k])
        d = -bar_nll(np.log(np.maximum(p, 1e-38)), orc.borders(), tq[:, k])
        ref += np.where(np.isneginf(d), np.log(1e-15), d)
    assert np.isfinite(lp).all()
    diff = np.abs(lp - ref)
    assert np.median(diff) <= 0.05 and np.quantile(diff, 0.95) <= 0.25, (np.median(diff), np.quantile(diff, 0.95))
    # npfn_ar_log_prob_repeated: step 0 once for the one distinct query row (x_unique), whose
    # mixture is the repeated rows' own (batch-invariant forward); bitwise reproducible
    lp_rep = eng.ar_log_prob(torch.from_numpy(x), torch.from_numpy(th), torch.from_numpy(xq), torch.from_numpy(tq),
                             x_unique=torch.from_numpy(x[:1])).cpu().numpy()
    lp_rep2 = eng.ar_log_prob(torch.from_numpy(x), torch.from_numpy(th), torch.from_numpy(xq), torch.from_numpy(tq),
                              x_unique=torch.from_numpy(x[:1])).cpu().numpy()
    assert np.array_equal(lp_rep, lp_rep2)
    d_rep = np.abs(lp_rep - lp)
    assert np.median(d_rep) <= 1e-2 and np.quantile(d_rep, 0.95) <= 0.1, (np.median(d_rep), np.quantile(d_rep, 0.95))
    diff = np.abs(lp_rep - ref)
    assert np.median(diff) <= 0.05 and np.quantile(diff, 0.95) <= 0.25, (np.median(diff), np.quantile(diff, 0.95))


def test_fingerprints_bit_exact_vs_hashlib():
    """The device SHA-256 fingerprints (k_views_fp / k_fp_train_*) equal hashlib's on the same
    float64 bytes: predict with 0 layers is not needed -- the engine's fitted state is checked
    through the feature statistics it derives from them (mean of the fingerprint column)."""
    from npe_pfn.engine import Engine
    from oracle.preprocess_oracle import MODE_ENSEMBLE, fingerprint, fingerprint_salt
    from oracle.tabpfn_oracle import OracleTabPFN

    w = synthetic_weights(CFG, seed=0)
    rng = np.random.default_rng(5)
    X = rng.normal(size=(400, 3)).astype(np.float32)
    X[200:230] = X[7]           # duplicates: collision re-hashing on the train rows
    y = rng.normal(size=400).astype(np.float32)
    eng = Engine(CFG, w, device=torch.device("cuda", 0), random_state=3)
    eng.set_preprocessing("ensemble")
    eng.fit(torch.from_numpy(X), torch.from_numpy(y))
    views = eng.debug_views(400)
    orc = OracleTabPFN(w, CFG.n_estimators, CFG.softmax_temperature, seed=3, preprocessing=MODE_ENSEMBLE)
    st = orc.fit(X, y)
    F, k = 3, 1
    fp_off = 3 * F + k
    for e in range(CFG.n_estimators):
        ref = fingerprint(X, fingerprint_salt(3, e), train=True)
        np.testing.assert_array_equal(views[:, fp_off + e], ref)
    # the SVD and quantile columns agree with the oracle's features of estimator 0
    feats = orc._features(X, st, st.estimators[0], train=True)
    np.testing.assert_allclose(views[:, F:2 * F], feats[:, F:2 * F], atol=1e-6)
    np.testing.assert_allclose(views[:, 2 * F:2 * F + k], feats[:, 2 * F:2 * F + k], rtol=1e-4, atol=1e-5)
