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
