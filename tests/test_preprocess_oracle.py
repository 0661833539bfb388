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
