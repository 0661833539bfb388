"""tabpfn-sized tables through the default (ensemble) preprocessing on the GPU.

* The reference's published timing workload (notebooks/sampling_comparison.ipynb:85-106:
  theta 2-D, x 50-D, 100 simulations, y = A theta + b + 0.1 noise) fits 50 and 51 features
  (npe_pfn.py:140-143): the widest estimator has 2 * 51 + 11 + 1 = 114 features, 58 tokens per
  row, and its SVD runs on a [102, 102] Gram matrix (the LDS Jacobi with V in the workspace).
* 128 features (2 * 128 + 13 + 1 = 270 features, 136 tokens per row at 120 rows, the long-row feature
  attention and the SVD of a [256, 256] Gram matrix in the workspace); 300 features under
  "none" (151 tokens).
* Contexts above 10 000 rows (``ignore_pretraining_limits=True``; sample_batched uses every
  simulation as context, npe_pfn.py:201-204): the preprocessed train table (views) at 20 000
  rows against the oracle -- the quantile fit on sklearn's 10 000-row subsample
  (k_qt_subsample: numpy's MT19937 shuffle), the Yeo-Johnson fit reading the column from
  global memory, the SVD, and the fingerprints with a fresh set of taken hashes every 10 000
  rows -- and a full sample_batched call.

Tolerances as tests/test_gpu_preprocess.py: TV <= 0.02 per row against the bf16-emulating
oracle; views: raw exact, quantile 1e-6, SVD rtol 1e-4, fingerprints bit-exact.
"""
import numpy as np
import pytest
import torch

from npe_pfn.weights import ModelConfig, synthetic_weights
from oracle.tabpfn_oracle import OracleTabPFN

pytestmark = pytest.mark.gpu

CFG = ModelConfig()
DEV = torch.device("cuda", 0)


@pytest.fixture(scope="module")
def weights():
    return synthetic_weights(CFG, seed=0)


def _sc_task(n=100, n_query=48, seed=42):
    """The notebook's model: theta ~ N(0, I_2), y = theta A^T + b + 0.1 noise (A [50, 2], b [50])."""
    g = torch.Generator().manual_seed(seed)
    A = torch.randn(50, 2, generator=g)
    b = torch.randn(50, generator=g)
    th = torch.randn(n + n_query, 2, generator=g)
    x = th @ A.T + b + 0.1 * torch.randn(n + n_query, 50, generator=g)
    return th[:n].numpy(), x[:n].numpy(), th[n:].numpy(), x[n:].numpy()


def _predict_tv(weights, X, y, Xq, mode, seed):
    from npe_pfn.engine import Engine

    eng = Engine(CFG, weights, device=DEV, random_state=seed, preprocessing=mode)
    eng.fit(torch.from_numpy(X), torch.from_numpy(y))
    p = torch.softmax(eng.predict_logits(torch.from_numpy(Xq)), -1).double().cpu().numpy()
    orc = OracleTabPFN(weights, CFG.n_estimators, CFG.softmax_temperature, seed=seed, emulate_bf16=True,
                       preprocessing=eng.PREPROCESSING_MODES[mode])
    orc.fit(X, y)
    p_ref = orc.predict_probs(Xq).astype(np.float64)
    return 0.5 * np.abs(p - p_ref).sum(1)


@pytest.mark.parametrize("k", [0, 1])
def test_sampling_comparison_shape_matches_oracle(weights, k):
    th, x, thq, xq = _sc_task()
    X = np.concatenate([x, th[:, :k]], 1).astype(np.float32)
    Xq = np.concatenate([xq, thq[:, :k]], 1).astype(np.float32)
    tv = _predict_tv(weights, X, th[:, k].astype(np.float32), Xq, "ensemble", seed=4)
    assert tv.max() <= 0.02, (tv.max(), tv.mean())


def test_sampling_comparison_ar_sample_matches_oracle_loop(weights):
    """The fused AR sampler on the notebook's call (10 draws for one observation, theta 2-D)."""
    from npe_pfn.engine import Engine
    from oracle.philox import uniforms
    from oracle.tabpfn_oracle import bar_sample

    th, x, thq, xq = _sc_task()
    N = 64
    q = np.repeat(xq[:1], N, 0).astype(np.float32)
    eng = Engine(CFG, weights, device=DEV, random_state=6)
    theta, _ = eng.ar_sample(torch.from_numpy(x), torch.from_numpy(th), torch.from_numpy(q), counter=0,
                             x_unique=torch.from_numpy(q[:1]))
    theta = theta.cpu().numpy()
    assert np.isfinite(theta).all()
    orc = OracleTabPFN(weights, CFG.n_estimators, CFG.softmax_temperature, seed=6, emulate_bf16=True, preprocessing=3)
    joint = np.concatenate([x, th], 1).astype(np.float32)
    feats = q
    for k in range(2):
        orc.fit(joint[:, : 50 + k], joint[:, 50 + k])
        p = orc.predict_probs(feats)
        ref = bar_sample(np.log(np.maximum(p, 1e-38)), orc.borders(), uniforms(6, k, N))
        span = np.std(joint[:, 50 + k]) * 10
        assert np.median(np.abs(theta[:, k] - ref)) <= 0.01 * span, (k, np.median(np.abs(theta[:, k] - ref)))
        feats = np.concatenate([feats, theta[:, k: k + 1]], 1)


@pytest.mark.parametrize("F,mode", [(128, "ensemble"), (300, "none")])
def test_wide_tables_long_rows_match_oracle(weights, F, mode):
    rng = np.random.default_rng(F)
    n, N = 120, 24  # the CPU oracle's size (C = 140 / 151 tokens per row)
    z = rng.normal(size=(n + N, 3))
    X = (z @ rng.normal(size=(3, F)) + 0.3 * rng.normal(size=(n + N, F))).astype(np.float32)
    y = (z[:n, 0] + 0.2 * rng.normal(size=n)).astype(np.float32)
    tv = _predict_tv(weights, X[:n], y, X[n:], mode, seed=3)
    assert tv.max() <= 0.02, (tv.max(), tv.mean())


def test_views_at_20k_context_rows_match_oracle(weights):
    from npe_pfn.engine import Engine
    from oracle.preprocess_oracle import (fingerprint, fingerprint_salt, quantile_fit, quantile_subsample,
                                          quantile_transform_vec, svd_components, svd_fit, svd_transform, yj_fit,
                                          power_transform_vec)

    rng = np.random.default_rng(20)
    n, F, seed = 20_000, 4, 5
    X = rng.normal(size=(n, F)).astype(np.float32)
    X[:, 0] = np.exp(X[:, 0])
    X[:, 1] = rng.integers(0, 50, size=n).astype(np.float32)      # ties; duplicate rows below
    X[15_000:15_040] = X[3]                                          # duplicates across the two hash blocks
    y = (X[:, 2] + 0.1 * rng.normal(size=n)).astype(np.float32)
    eng = Engine(CFG, weights, device=DEV, random_state=seed)        # ensemble
    eng.fit(torch.from_numpy(X), torch.from_numpy(y))
    views = eng.debug_views(n, 64)
    k = svd_components(n, F)
    assert views.shape == (n, 3 * F + k + CFG.n_estimators)
    np.testing.assert_array_equal(views[:, :F], X)
    sub = quantile_subsample(n, seed)
    assert sub is not None
    q = np.stack([quantile_transform_vec(X[:, j], quantile_fit(X[:, j], n, sub=sub)) for j in range(F)], 1)
    np.testing.assert_allclose(views[:, F:2 * F], q, rtol=0, atol=1e-6)
    Z = np.concatenate([X, q], 1).astype(np.float64)
    s = svd_transform(Z, *svd_fit(Z, k))
    np.testing.assert_allclose(views[:, 2 * F:2 * F + k], s, rtol=1e-4, atol=1e-4)
    pw = np.stack([power_transform_vec(X[:, j], yj_fit(X[:, j])) for j in range(F)], 1)
    np.testing.assert_allclose(views[:, 2 * F + k:3 * F + k], pw, rtol=1e-5, atol=1e-5)
    for e in (0, CFG.n_estimators - 1):
        ref = fingerprint(X, fingerprint_salt(seed, e), train=True)
        np.testing.assert_array_equal(views[:, 3 * F + k + e], ref)


@pytest.mark.parametrize("F", [3, 19, 24, 40, 70])
def test_svd_views_every_jacobi_form_match_oracle(weights, F):
    """The ensemble's TruncatedSVD columns at every Jacobi form of k_svd_jacobi (2F = m): A and V
    in LDS with one unit per thread (m <= 40: F = 3, 19), A and V in LDS with the unit loops
    (m = 48), A in LDS and V in the workspace (m = 80), both in the workspace (m = 140) -- against
    the oracle's svd_fit (sklearn-pinned) at rtol 1e-4."""
    from npe_pfn.engine import Engine
    from oracle.preprocess_oracle import quantile_fit, quantile_transform_vec, svd_components, svd_fit, svd_transform

    rng = np.random.default_rng(100 + F)
    n = 300
    z = rng.normal(size=(n, 4))
    X = (z @ rng.normal(size=(4, F)) + 0.5 * rng.normal(size=(n, F))).astype(np.float32)
    y = (z[:, 0] + 0.1 * rng.normal(size=n)).astype(np.float32)
    eng = Engine(CFG, weights, device=DEV, random_state=7)
    eng.fit(torch.from_numpy(X), torch.from_numpy(y))
    k = svd_components(n, F)
    views = eng.debug_views(n, 3 * F + k + CFG.n_estimators)
    assert views.shape == (n, 3 * F + k + CFG.n_estimators)
    q = np.stack([quantile_transform_vec(X[:, j], quantile_fit(X[:, j], n)) for j in range(F)], 1)
    Z = np.concatenate([X, q], 1).astype(np.float64)
    s = svd_transform(Z, *svd_fit(Z, k))
    np.testing.assert_allclose(views[:, 2 * F:2 * F + k], s, rtol=1e-4, atol=1e-4)


def test_sample_batched_20k_context_rows():
    """sample_batched with every one of 20 000 simulations as context (npe_pfn.py:201-204):
    refused as tabpfn refuses it without ignore_pretraining_limits, run with it."""
    from npe_pfn.npe_pfn import NPE_PFN_Core

    g = torch.Generator().manual_seed(1)
    n, dth, dx = 20_000, 3, 5
    theta = torch.randn(n, dth, generator=g)
    W = torch.randn(dx, dth, generator=g)
    x = theta @ W.T + 0.2 * torch.randn(n, dx, generator=g)
    xo = torch.randn(4, dth, generator=g) @ W.T
    prior = torch.distributions.Independent(torch.distributions.Normal(torch.zeros(dth), torch.ones(dth)), 1)
    m = NPE_PFN_Core(prior=prior, regressor_init_kwargs={"device": DEV})
    m.append_simulations(theta, x)
    with pytest.raises(ValueError, match="ignore_pretraining_limits"):
        m.sample_batched(xo, torch.Size([50]))
    draws = []
    for _ in range(2):  # two fresh models: the engine is deterministic
        m = NPE_PFN_Core(prior=prior, regressor_init_kwargs={"device": DEV, "ignore_pretraining_limits": True})
        m.append_simulations(theta, x)
        draws.append(m.sample_batched(xo, torch.Size([50])))
    assert draws[0].shape == (4, 50, dth)
    assert torch.isfinite(draws[0]).all()
    assert torch.equal(draws[0], draws[1])


def test_engine_caps_raise_value_errors(weights):
    """Past each cap: a ValueError naming it, before any C call; the C engine's own EINVAL
    backstop says the same when called directly."""
    import ctypes

    from npe_pfn.engine import Engine, _ptr

    eng = Engine(CFG, weights, device=DEV, random_state=0)
    msg = "SVD takes at most 1024 features past 512 context rows"
    with pytest.raises(ValueError, match=msg):
        eng.fit(torch.zeros(600, 1025), torch.zeros(600))
    with pytest.raises(ValueError, match="10001 quantiles"):
        eng.fit(torch.zeros(50_005, 2), torch.zeros(50_005))
    X = torch.randn(600, 1025, device=DEV)
    y = torch.randn(1000, device=DEV)
    rc = eng.lib.npfn_fit(eng.h, _ptr(X), 1025, _ptr(y), 1, 600, 1025, eng.stream)
    assert rc != 0 and msg.encode() in eng.lib.npfn_last_error()
    eng.set_preprocessing("none")
    with pytest.raises(ValueError, match="positional table holds 640 groups"):
        eng.fit(torch.zeros(100, 1281), torch.zeros(100))
    X = torch.randn(100, 1281, device=DEV)
    rc2 = eng.lib.npfn_fit(eng.h, _ptr(X), 1281, _ptr(y), 1, 100, 1281, eng.stream)
    assert rc2 != 0 and b"max_groups" in eng.lib.npfn_last_error()
    eng.fit(torch.randn(300, 200), torch.randn(300))  # 101 tokens: the fused path
    assert ctypes.c_int(rc).value != 0


@pytest.mark.parametrize("F,n", [(300, 100), (260, 99), (257, 512), (300, 1000), (257, 513)])
def test_svd_dual_views_match_oracle(weights, F, n):
    """Past 256 features (2F > kSvdMaxM) the SVD diagonalises the dual [n, n] matrix Y Y^T and maps
    its eigenvectors back (k_svd_colscale / k_svd_dual_gram / k_svd_jacobi / k_svd_dual_out) up to
    512 context rows, and the dense [2F, 2F] Gram matrix by rocSOLVER's dsyevd past that
    (k_svd_gram / k_svd_assemble / k_svd_select): the SVD columns of the views against the oracle's
    svd_fit (eigh of the [2F, 2F] Gram matrix, sklearn-pinned) at rtol 1e-4 -- an odd n (a zero
    padding row) and n = 512 (the Jacobi's workspace form) included."""
    from npe_pfn.engine import Engine
    from oracle.preprocess_oracle import quantile_fit, quantile_transform_vec, svd_components, svd_fit, svd_transform

    rng = np.random.default_rng(F + n)
    z = rng.normal(size=(n, 4))
    X = (z @ rng.normal(size=(4, F)) + 0.5 * rng.normal(size=(n, F))).astype(np.float32)
    y = (z[:, 0] + 0.1 * rng.normal(size=n)).astype(np.float32)
    eng = Engine(CFG, weights, device=DEV, random_state=7)
    eng.fit(torch.from_numpy(X), torch.from_numpy(y))
    k = svd_components(n, F)
    views = eng.debug_views(n, 3 * F + k + CFG.n_estimators)
    q = np.stack([quantile_transform_vec(X[:, j], quantile_fit(X[:, j], n)) for j in range(F)], 1)
    Z = np.concatenate([X, q], 1).astype(np.float64)
    s = svd_transform(Z, *svd_fit(Z, k))
    np.testing.assert_allclose(views[:, 2 * F:2 * F + k], s, rtol=1e-4, atol=1e-4)


def test_500_features_under_the_ensemble_match_oracle(weights):
    """tabpfn's maximum, 500 features, under the default ensemble at 100 context rows: the
    quantile + original + SVD estimators have 1012 features (507 tokens per row: the per-sublayer
    path with k_feat_attn_wide, the positional table past 256 groups, the dual SVD), the power +
    fingerprint estimators 501 (252 tokens: the fused row kernel) -- the 12-layer model's
    predictive distribution against the bf16-emulating oracle's (tests/golden/wide500.npz, made by
    tests/golden/make_golden_wide.py: ~28 min of CPU oracle), TV <= 0.02 per row.  The synthetic
    model averages its 507 tokens, so its rows differ by only TV ~0.002 and the TV bar alone would
    pass an engine that ignored the inputs: the rows' deviations from their mean distribution must
    also correlate >= 0.8 with the oracle's (r05q: TV 0.0008, correlation 0.89)."""
    import os

    from conftest import GOLDEN
    from npe_pfn.engine import Engine

    g = np.load(os.path.join(GOLDEN, "wide500.npz"))
    X, y, p_ref = g["X"], g["y"], g["probs"].astype(np.float64)
    n = y.shape[0]
    eng = Engine(CFG, weights, device=DEV, random_state=int(g["random_state"]), preprocessing="ensemble")
    eng.fit(torch.from_numpy(X[:n]), torch.from_numpy(y))
    p = torch.softmax(eng.predict_logits(torch.from_numpy(X[n:])), -1).double().cpu().numpy()
    tv = 0.5 * np.abs(p - p_ref).sum(1)
    # the rows' own differences (the synthetic model averages 507 tokens: its rows differ by TV ~0.002)
    d, d_ref = p - p.mean(0), p_ref - p_ref.mean(0)
    corr = float((d * d_ref).sum() / np.sqrt((d * d).sum() * (d_ref * d_ref).sum()))
    tv_rows = 0.5 * np.abs(p_ref[:, None] - p_ref[None]).sum(-1)[np.triu_indices(len(p_ref), 1)]
    print(f"500 features: TV to the oracle max {tv.max():.4f} mean {tv.mean():.4f}; oracle rows differ by TV "
          f"median {np.median(tv_rows):.4f}; correlation of the rows' deviations from their mean {corr:.3f}")
    assert tv.max() <= 0.02, (tv.max(), tv.mean())
    assert corr >= 0.8, corr


def test_500_features_ar_sample_is_deterministic_and_finite(weights):
    """The fused AR sampler over a 498-dim x and a 2-dim theta (the wide groups at every step):
    finite draws, bit for bit equal across two engines."""
    from npe_pfn.engine import Engine

    rng = np.random.default_rng(9)
    n, dx, N = 100, 498, 64
    th = rng.normal(size=(n, 2)).astype(np.float32)
    x = (th @ rng.normal(size=(2, dx)) + 0.3 * rng.normal(size=(n, dx))).astype(np.float32)
    q = np.repeat(x[:1], N, 0)
    out = []
    for _ in range(2):
        eng = Engine(CFG, weights, device=DEV, random_state=5)
        theta, lp = eng.ar_sample(torch.from_numpy(x), torch.from_numpy(th), torch.from_numpy(q), counter=0,
                                  x_unique=torch.from_numpy(q[:1]))
        out.append(theta.cpu().numpy())
    assert np.isfinite(out[0]).all()
    assert np.array_equal(out[0], out[1])


def test_300_features_at_1000_rows_ar_sample(weights):
    """The fused AR sampler over a 298-dim x at 1 000 context rows: every step's SVD takes the
    dsyevd form (2F > 512, n > 512) inside the side-stream fits and the quantile + original + SVD
    estimators run the per-sublayer path (352 tokens per row): finite draws, bit for bit equal
    across two engines (the dsyevd views themselves: test_svd_dual_views_match_oracle)."""
    from npe_pfn.engine import Engine

    rng = np.random.default_rng(13)
    n, dx, N = 1000, 298, 128
    th = rng.normal(size=(n, 2)).astype(np.float32)
    x = (th @ rng.normal(size=(2, dx)) + 0.3 * rng.normal(size=(n, dx))).astype(np.float32)
    q = np.repeat(x[:1], N, 0)
    out = []
    for _ in range(2):
        eng = Engine(CFG, weights, device=DEV, random_state=5)
        theta, _ = eng.ar_sample(torch.from_numpy(x), torch.from_numpy(th), torch.from_numpy(q), counter=0,
                                 x_unique=torch.from_numpy(q[:1]))
        out.append(theta.cpu().numpy())
    assert np.isfinite(out[0]).all()
    assert np.array_equal(out[0], out[1])
