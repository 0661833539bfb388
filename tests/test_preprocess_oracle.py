"""The quantile-transform restatement (oracle/preprocess_oracle.py) against sklearn's
QuantileTransformer, the implementation tabpfn's "quantile_uni" preprocessing calls [ext].

Tolerance: the restatement evaluates the same float64 arithmetic; outputs are
float32, compared at 1 ulp-scale (|d| <= 1e-6) and quantiles at rtol 1e-12.
"""
import numpy as np
import pytest
from sklearn.preprocessing import QuantileTransformer

from oracle.preprocess_oracle import (estimator_uses_quantile, n_quantiles_for, quantile_fit, quantile_transform,
                                      quantile_transform_vec)


def _cases():
    rng = np.random.default_rng(0)
    yield "normal", rng.normal(size=1000).astype(np.float32), rng.normal(size=300).astype(np.float32) * 1.5
    yield "ties", rng.integers(0, 7, size=400).astype(np.float32), np.arange(-1, 9, 0.25, dtype=np.float32)
    yield "tiny", np.array([0.5, -1.0, 2.0], np.float32), np.array([-2, -1, 0, 0.5, 1, 2, 3], np.float32)
    yield "constant", np.full(50, 3.0, np.float32), np.array([2.0, 3.0, 4.0], np.float32)
    col = rng.exponential(size=237).astype(np.float32)
    col[::17] = np.nan
    yield "nan", col, np.concatenate([col[:40], np.array([np.nan, 0.0, 100.0], np.float32)])
    yield "heavy", (rng.standard_t(1.5, size=2000) * 10).astype(np.float32), rng.normal(size=500).astype(np.float32) * 30


@pytest.mark.parametrize("name,col,xq", list(_cases()), ids=[c[0] for c in _cases()])
def test_quantile_transform_matches_sklearn(name, col, xq):
    n = col.shape[0]
    qt = QuantileTransformer(output_distribution="uniform", n_quantiles=max(n // 5, 2)).fit(col[:, None])
    q = quantile_fit(col, n)
    assert q.size == n_quantiles_for(n) == qt.n_quantiles_
    np.testing.assert_allclose(q, qt.quantiles_[:, 0], rtol=1e-12, atol=0)
    for x in (col, xq):
        ref = qt.transform(x[:, None])[:, 0]
        got = quantile_transform(x, q)
        np.testing.assert_array_equal(np.isnan(got), np.isnan(ref))
        np.testing.assert_allclose(got, ref, rtol=0, atol=1e-6, equal_nan=True)
        np.testing.assert_array_equal(quantile_transform_vec(x, q), got)


@pytest.mark.parametrize("name,col,xq", list(_cases()), ids=[c[0] for c in _cases()])
def test_coarse_quantile_transform_matches_sklearn(name, col, xq):
    """tabpfn's classifier ensemble uses "quantile_uni_coarse" = n_quantiles max(n // 10, 2) [ext]."""
    from oracle.preprocess_oracle import QUANTILE_DIV_COARSE

    n = col.shape[0]
    qt = QuantileTransformer(output_distribution="uniform", n_quantiles=max(n // 10, 2)).fit(col[:, None])
    q = quantile_fit(col, n, QUANTILE_DIV_COARSE)
    assert q.size == n_quantiles_for(n, QUANTILE_DIV_COARSE) == qt.n_quantiles_
    # numpy's percentile interpolation rounds one reference differently at rtol ~5e-9 here
    np.testing.assert_allclose(q, qt.quantiles_[:, 0], rtol=1e-8, atol=1e-12)
    for x in (col, xq):
        np.testing.assert_allclose(quantile_transform(x, q), qt.transform(x[:, None])[:, 0], rtol=0, atol=1e-6,
                                   equal_nan=True)


def test_classifier_ensemble_assignment():
    """The classifier's ensemble: coarse-quantile + original + SVD on the first half of the
    estimators, the original features on the second half, fingerprint on both, no target
    transform [ext: tabpfn generate_for_classification, restated]."""
    from oracle.preprocess_oracle import MODE_ENSEMBLE, T_QSVD, T_RFP, estimator_configs, n_features_of

    assert estimator_configs(MODE_ENSEMBLE, 8, classifier=True) == [(T_QSVD, False)] * 4 + [(T_RFP, False)] * 4
    assert estimator_configs(MODE_ENSEMBLE, 3, classifier=True) == [(T_QSVD, False), (T_RFP, False), (T_QSVD, False)]
    assert n_features_of(T_RFP, 5, 100) == 6


def test_even_estimators_only():
    assert [estimator_uses_quantile(e, 1) for e in range(4)] == [True, False, True, False]
    assert not any(estimator_uses_quantile(e, 0) for e in range(8))


def _power_cases():
    rng = np.random.default_rng(1)
    yield "lognormal", np.exp(rng.normal(size=800)).astype(np.float32)
    yield "normal", rng.normal(size=500).astype(np.float32) * 3
    yield "skew_neg", (-np.exp(0.7 * rng.normal(size=600)) + 0.5).astype(np.float32)
    yield "ties", rng.integers(0, 6, size=300).astype(np.float32)


@pytest.mark.parametrize("name,col", list(_power_cases()), ids=[c[0] for c in _power_cases()])
def test_power_fit_matches_sklearn(name, col):
    """lambda: at least as likely as sklearn's and within 2e-3 of it (scipy's Brent runs on
    the float32-evaluated, flat likelihood); the transform at sklearn's lambda within 1e-5
    relative (sklearn evaluates it in float32)."""
    from sklearn.preprocessing import PowerTransformer

    from oracle.preprocess_oracle import power_transform_vec, yj_fit, yj_neg_llf

    pt = PowerTransformer(method="yeo-johnson", standardize=False).fit(col[:, None])
    lam = yj_fit(col)
    ref = float(pt.lambdas_[0])
    x = col.astype(np.float64)
    # same optimum: our lambda is at least as likely as sklearn's, and close to it
    assert yj_neg_llf(x, lam) <= yj_neg_llf(x, ref) + 1e-6 * abs(yj_neg_llf(x, ref))
    assert abs(lam - ref) <= 2e-3, (lam, ref)
    got = power_transform_vec(col, ref)
    want = pt.transform(col[:, None])[:, 0]
    np.testing.assert_allclose(got, want, rtol=1e-5, atol=1e-6)


def test_power_constant_column_is_identity():
    from oracle.preprocess_oracle import yj_fit

    assert yj_fit(np.full(20, 2.5, np.float32)) == 1.0


# ---------------------------------------------------------------- ensemble mode
def test_svd_matches_sklearn_truncated_svd():
    """StandardScaler(with_mean=False) + TruncatedSVD(arpack) -- the "svd" global transformer
    [ext] -- against the restatement (Gram eigenvectors, svd_flip signs)."""
    from sklearn.decomposition import TruncatedSVD
    from sklearn.preprocessing import StandardScaler

    from oracle.preprocess_oracle import svd_components, svd_fit, svd_transform

    rng = np.random.default_rng(3)
    for n, F in ((1000, 10), (1000, 19), (200, 2), (64, 7)):
        X = rng.normal(size=(n, F)).astype(np.float32) @ rng.normal(size=(F, F)).astype(np.float32)
        Z = np.concatenate([X, rng.uniform(size=(n, F)).astype(np.float32)], 1).astype(np.float64)
        k = svd_components(n, F)
        sc = StandardScaler(with_mean=False).fit(Z)
        ts = TruncatedSVD(n_components=k, algorithm="arpack", random_state=0).fit(sc.transform(Z))
        scale, comps = svd_fit(Z, k)
        np.testing.assert_allclose(scale, sc.scale_, rtol=1e-12)
        np.testing.assert_allclose(comps, ts.components_, atol=1e-8)
        Zq = rng.normal(size=(50, 2 * F))
        np.testing.assert_allclose(svd_transform(Zq, scale, comps), ts.transform(sc.transform(Zq)),
                                   rtol=1e-5, atol=1e-5)
    assert svd_components(1000, 1) == 0 and svd_components(1000, 19) == 9 and svd_components(30, 19) == 4


def test_fingerprint_is_tabpfn_hash_with_train_collision_offsets():
    """sha256(row + salt) mod 10000 / 10000; duplicate train rows re-hash with +1, +2, ..."""
    import hashlib

    from oracle.preprocess_oracle import FP_BUCKETS, fingerprint, fingerprint_salt

    rng = np.random.default_rng(0)
    X = rng.normal(size=(300, 4)).astype(np.float32)
    X[100:110] = X[5]              # duplicate rows
    salt = fingerprint_salt(7, 2)
    assert 0 <= salt < 65536 and salt != fingerprint_salt(7, 3)
    h_test = fingerprint(X, salt, train=False)
    for i in (0, 5, 100, 299):
        want = int(hashlib.sha256((X[i].astype(np.float64) + salt).tobytes()).hexdigest(), 16) % FP_BUCKETS
        assert h_test[i] == np.float32(want / FP_BUCKETS)
    assert len(set(h_test[100:110].tolist())) == 1
    h_train = fingerprint(X, salt, train=True)
    assert len(set(np.round(h_train * FP_BUCKETS).astype(int).tolist())) == 300   # all distinct
    assert h_train[5] == h_test[5]   # first occurrence keeps its hash


def test_yeo_johnson_inverse_roundtrip():
    from oracle.preprocess_oracle import yeo_johnson, yeo_johnson_inverse

    x = np.linspace(-5, 5, 101)
    for lam in (-1.3, 0.0, 0.7, 1.0, 2.0, 2.6):
        np.testing.assert_allclose(yeo_johnson_inverse(yeo_johnson(x, lam), lam), x, atol=1e-9)


def test_translation_conserves_mass_and_is_identity_on_equal_borders():
    from oracle.preprocess_oracle import cancel_broken_borders, translate_probs, translation_table

    rng = np.random.default_rng(1)
    nb = 500
    to = np.sort(rng.normal(size=nb + 1)).astype(np.float32) * 3
    p = rng.dirichlet(np.ones(nb), size=20).astype(np.float32)
    idx, share, flag = translation_table(to, to)
    np.testing.assert_allclose(translate_probs(p, idx, share, flag), p, atol=2e-6)
    frm = np.sinh(to.astype(np.float64)).astype(np.float32)       # monotone, wider support
    q = translate_probs(p, *translation_table(frm, to))
    assert (q >= 0).all()
    np.testing.assert_allclose(q.sum(1), 1.0, atol=1e-5)
    b, cancel = cancel_broken_borders(np.array([np.nan, np.inf, -5.0, 1.0, 2.0, 5e3, np.nan]))
    np.testing.assert_array_equal(b, [-6.0, -5.0, -5.0, 1.0, 2.0, 2.0, 3.0])
    np.testing.assert_array_equal(cancel, [True, True, False, False, True, True])


def test_ensemble_config_assignment():
    from oracle.preprocess_oracle import MODE_ENSEMBLE, T_PFP, T_QSVD, estimator_configs, n_features_of

    cfg = estimator_configs(MODE_ENSEMBLE, 8)
    assert cfg == [(T_QSVD, False)] * 2 + [(T_QSVD, True)] * 2 + [(T_PFP, False)] * 2 + [(T_PFP, True)] * 2
    assert estimator_configs(MODE_ENSEMBLE, 2) == [(T_QSVD, False), (T_QSVD, True)]
    assert n_features_of(T_QSVD, 10, 1000) == 26 and n_features_of(T_PFP, 19, 1000) == 20


def test_oracle_ensemble_predicts_a_distribution():
    """End to end on the CPU: mode 3 fit + predict gives normalized bar probabilities, and the
    target-transformed estimators' translated mass sits where the raw estimators' does."""
    from npe_pfn.weights import ModelConfig, synthetic_weights
    from oracle.preprocess_oracle import MODE_ENSEMBLE
    from oracle.tabpfn_oracle import OracleTabPFN

    cfg = ModelConfig(n_layers=2)
    w = synthetic_weights(cfg, seed=0)
    rng = np.random.default_rng(0)
    X = rng.normal(size=(120, 3)).astype(np.float32)
    y = np.exp(X[:, 0] + 0.2 * rng.normal(size=120)).astype(np.float32)   # skewed target
    orc = OracleTabPFN(w, 8, 0.9, seed=1, preprocessing=MODE_ENSEMBLE)
    st = orc.fit(X, y)
    assert [es.n_feat for es in st.estimators] == [8, 8, 8, 8, 4, 4, 4, 4]
    assert st.ylam is not None and st.trans is not None
    p, lg = orc.predict_probs(X[:17], return_estimator_logits=True)
    assert p.shape == (17, cfg.n_bars) and np.isfinite(p).all()
    np.testing.assert_allclose(p.sum(1), 1.0, atol=1e-4)


@pytest.mark.parametrize("n,seed", [(10_001, 0), (20_000, 7), (65_536, 2**32 - 1)])
def test_subsample_restatement_is_numpys_shuffle(n, seed):
    """The engine's k_qt_subsample restated step by step (MT19937, masked rejection, the swaps
    for i >= 10 000 only) gives the same SET of rows as numpy's RandomState(seed).shuffle's
    first 10 000 -- what sklearn's resample(replace=False) takes."""
    from oracle.preprocess_oracle import mt19937_shuffle_head, quantile_subsample

    idx = np.arange(n)
    np.random.RandomState(seed).shuffle(idx)
    np.testing.assert_array_equal(mt19937_shuffle_head(n, seed), np.sort(idx[:10_000]))
    np.testing.assert_array_equal(np.sort(quantile_subsample(n, seed)), np.sort(idx[:10_000]))
    assert quantile_subsample(10_000, seed) is None


def test_quantile_fit_with_subsample_matches_sklearn():
    """Contexts above 10 000 rows: QuantileTransformer(random_state=seed) fits on its default
    subsample of 10 000 rows; n_quantiles still follows the full row count."""
    from oracle.preprocess_oracle import check_n_quantiles, quantile_subsample

    rng = np.random.default_rng(3)
    n = 23_456
    X = rng.normal(size=(n, 2)).astype(np.float32)
    X[::97, 1] = np.nan
    sub = quantile_subsample(n, 11)
    for j in range(2):
        q = quantile_fit(X[:, j], n, sub=sub)
        qt = QuantileTransformer(n_quantiles=max(n // 5, 2), random_state=11).fit(X[:, j:j + 1])
        # nanpercentile's interpolation rounds an odd reference differently (rtol ~2e-8), as in
        # test_coarse_quantile_transform_matches_sklearn
        np.testing.assert_allclose(q, qt.quantiles_[:, 0], rtol=1e-7, atol=1e-11)
    with pytest.raises(ValueError, match="cannot be greater than the number of samples"):
        check_n_quantiles(50_005)


def test_fingerprint_blocks_of_distinct_hashes(monkeypatch):
    """Train rows take distinct hashes within each block of FP_BLOCK rows (10 000: tabpfn's 10 000
    hash values hold no more); a duplicate of a row of an earlier block hashes afresh."""
    import oracle.preprocess_oracle as po

    monkeypatch.setattr(po, "FP_BLOCK", 5)
    X = np.zeros((12, 2), np.float32)      # twelve identical rows
    fp = po.fingerprint(X, 9, train=True)
    assert len(set(fp[:5].tolist())) == 5 and len(set(fp[5:10].tolist())) == 5
    np.testing.assert_array_equal(fp[:5], fp[5:10])
    np.testing.assert_array_equal(fp[10:], fp[:2])
