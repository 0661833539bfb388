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
    return mode == MODE_QUANTILE and e % 2 == 0


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
