"""CPU restatement of the per-estimator quantile feature transform (TEST INFRASTRUCTURE).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use this
module, as the checker of the engine's ``k_quantile_fit`` / ``k_encode``
transform (npe-pfn_amd/csrc/npfn_kernels.hip); the product never imports it.

What it restates.  TabPFN's regressor ensemble preprocesses the table per
estimator before the transformer [ext: tabpfn==2.2.1 ``PreprocessorConfig``
"quantile_uni" = ``sklearn.preprocessing.QuantileTransformer(
output_distribution="uniform", n_quantiles=max(n // 5, 2))``; SURVEY.md §8f
row 3].  The engine's ``preprocessing="quantile"`` mode applies that transform
to every even estimator (odd estimators keep the plain standardization), then
the usual train-statistics standardization of the transformed columns.

Pinning.  The transform is sklearn 1.7.2's (installed here), restated from its
source: ``_dense_fit`` (``np.nanpercentile`` at ``linspace(0, 1, n_q)``, then
``np.maximum.accumulate``) and ``_transform_col`` (the two-sided ``np.interp``
average, ``x == q[0] -> 0``, ``x == q[-1] -> 1``).  tests/test_preprocess_oracle.py
checks this restatement against ``QuantileTransformer`` itself on ties, NaNs,
constant and tiny columns.  Which estimators tabpfn assigns to which config, and
the features it appends (``append_original``, SVD, fingerprint) are [ext] and
not restated: the ensemble assignment is **parity unpinned**.
"""

from __future__ import annotations

import numpy as np

QUANTILE_DIV = 5  # n_quantiles = max(n // 5, 2) [ext: tabpfn "quantile_uni"]
MODE_NONE, MODE_QUANTILE = 0, 1


def n_quantiles_for(n_rows: int) -> int:
    """sklearn caps ``n_quantiles`` at the number of samples (``n_quantiles_``)."""
    return max(1, min(max(n_rows // QUANTILE_DIV, 2), n_rows))


def estimator_uses_quantile(e: int, mode: int) -> bool:
    return mode in (MODE_QUANTILE, 2) and e % 2 == 0   # 2 = MODE_QUANTILE_POWER


def references(nq: int) -> np.ndarray:
    return np.linspace(0.0, 1.0, nq, endpoint=True)


def quantile_fit(col: np.ndarray, n_rows: int) -> np.ndarray:
    """``QuantileTransformer._dense_fit`` for one column -> float64 quantiles [n_q].

    NaN/inf are excluded (``nanpercentile``; the engine feeds non-finite values
    through its NaN-indicator path instead).  An all-non-finite column gives an
    empty table (the column is then passed through untransformed)."""
    nq = n_quantiles_for(n_rows)
    v = np.sort(np.asarray(col, dtype=np.float64)[np.isfinite(col)])
    if v.size == 0:
        return np.zeros(0)
    q = np.percentile(v, references(nq) * 100.0)
    return np.maximum.accumulate(q)


def _interp(x: float, xp: np.ndarray, fp: np.ndarray) -> float:
    """numpy ``interp`` (arr_interp): j = last index with xp[j] <= x."""
    n = xp.size
    if x > xp[-1]:
        return fp[-1]
    if x < xp[0]:
        return fp[0]
    j = int(np.searchsorted(xp, x, side="right")) - 1
    if j == n - 1 or xp[j] == x:
        return fp[j]
    slope = (fp[j + 1] - fp[j]) / (xp[j + 1] - xp[j])
    return slope * (x - xp[j]) + fp[j]


def quantile_transform(x: np.ndarray, q: np.ndarray) -> np.ndarray:
    """``QuantileTransformer._transform_col`` (uniform output), float32 result."""
    x = np.asarray(x, dtype=np.float32)
    out = x.copy()
    if q.size == 0:
        return out
    r = references(q.size)
    qr, rr = -q[::-1], -r[::-1]
    for i, xv in np.ndenumerate(x):
        if not np.isfinite(xv):
            continue
        xd = float(xv)
        val = 0.5 * (_interp(xd, q, r) - _interp(-xd, qr, rr))
        if xd == q[-1]:
            val = 1.0
        if xd == q[0]:
            val = 0.0
        out[i] = np.float32(val)
    return out


def quantile_transform_vec(x: np.ndarray, q: np.ndarray) -> np.ndarray:
    """Vectorised form of :func:`quantile_transform` (same arithmetic, np.interp)."""
    x = np.asarray(x, dtype=np.float32)
    if q.size == 0:
        return x.copy()
    r = references(q.size)
    fin = np.isfinite(x)
    xd = x.astype(np.float64)
    val = 0.5 * (np.interp(xd, q, r) - np.interp(-xd, -q[::-1], -r[::-1]))
    val = np.where(xd == q[-1], 1.0, val)
    val = np.where(xd == q[0], 0.0, val)
    return np.where(fin, val.astype(np.float32), x)


# ------------------------------------------------------------- Yeo-Johnson power
# tabpfn's second regressor preprocessing config is a Yeo-Johnson power transform
# [ext: tabpfn "safepower" = sklearn PowerTransformer(method="yeo-johnson")
# + safeguards].  Restated here: the transform of sklearn's
# ``PowerTransformer._yeo_johnson_transform`` and the log-likelihood of its
# ``_yeo_johnson_optimize``; lambda = argmax of that likelihood found by a fixed
# search (grid on [-6, 6] step 1, then 40 golden-section steps on the two grid
# cells around the best node, final bracket 2 * 0.618^40 = 9e-9), the same search the device runs (k_power_fit).
# sklearn/scipy maximise the same likelihood with Brent; tests pin lambda and the
# transformed values against ``PowerTransformer`` itself.  The StandardScaler
# after the transform is affine and cancels in the engine's own train-statistics
# standardization, so it is not repeated.  MODE_QUANTILE_POWER applies the power
# transform to odd estimators (quantile on even ones).
MODE_QUANTILE_POWER = 2
YJ_GRID_LO, YJ_GRID_STEP, YJ_GRID_N, YJ_GOLDEN_STEPS = -6.0, 1.0, 13, 40
_EPS1 = float(np.spacing(1.0))


def estimator_uses_power(e: int, mode: int) -> bool:
    return mode == MODE_QUANTILE_POWER and e % 2 == 1


def yeo_johnson(x: np.ndarray, lam: float) -> np.ndarray:
    x = np.asarray(x, dtype=np.float64)
    out = np.zeros_like(x)
    pos = x >= 0
    if abs(lam) < _EPS1:
        out[pos] = np.log1p(x[pos])
    else:
        out[pos] = (np.power(x[pos] + 1.0, lam) - 1.0) / lam
    if abs(lam - 2.0) > _EPS1:
        out[~pos] = -(np.power(-x[~pos] + 1.0, 2.0 - lam) - 1.0) / (2.0 - lam)
    else:
        out[~pos] = -np.log1p(-x[~pos])
    return out


def yj_neg_llf(x: np.ndarray, lam: float) -> float:
    """-loglike of sklearn ``_yeo_johnson_optimize`` (population variance)."""
    t = yeo_johnson(x, lam)
    var = float(np.mean((t - t.mean()) ** 2))
    if not var >= np.finfo(np.float64).tiny:
        return np.inf
    return -(-x.size / 2.0 * np.log(var) + (lam - 1.0) * float((np.sign(x) * np.log1p(np.abs(x))).sum()))


def yj_fit(col: np.ndarray) -> float:
    """lambda for one column (finite values only); constant column -> 1 (identity), as sklearn."""
    x = np.asarray(col, dtype=np.float64)
    x = x[np.isfinite(x)]
    if x.size == 0 or np.ptp(x) == 0:
        return 1.0
    grid = YJ_GRID_LO + YJ_GRID_STEP * np.arange(YJ_GRID_N)
    f = np.array([yj_neg_llf(x, g) for g in grid])
    i = int(np.argmin(f))                      # first minimum
    a = grid[max(i - 1, 0)]
    b = grid[min(i + 1, YJ_GRID_N - 1)]
    r = (np.sqrt(5.0) - 1.0) / 2.0
    c, d = b - r * (b - a), a + r * (b - a)
    fc, fd = yj_neg_llf(x, c), yj_neg_llf(x, d)
    for _ in range(YJ_GOLDEN_STEPS):
        if fc <= fd:
            b, d, fd = d, c, fc
            c = b - r * (b - a)
            fc = yj_neg_llf(x, c)
        else:
            a, c, fc = c, d, fd
            d = a + r * (b - a)
            fd = yj_neg_llf(x, d)
    return 0.5 * (a + b)


def power_transform_vec(x: np.ndarray, lam: float) -> np.ndarray:
    """Per-value transform of a column (float32 out); non-finite values pass through."""
    x = np.asarray(x, dtype=np.float32)
    fin = np.isfinite(x)
    out = x.copy()
    out[fin] = yeo_johnson(x[fin].astype(np.float64), lam).astype(np.float32)
    return out
