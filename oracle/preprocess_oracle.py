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
QUANTILE_DIV_COARSE = 10  # n_quantiles = max(n // 10, 2) [ext: tabpfn "quantile_uni_coarse", the classifier's]
MODE_NONE, MODE_QUANTILE = 0, 1


def n_quantiles_for(n_rows: int, div: int = QUANTILE_DIV) -> int:
    """sklearn caps ``n_quantiles`` at the number of samples (``n_quantiles_``)."""
    return max(1, min(max(n_rows // div, 2), n_rows))


def estimator_uses_quantile(e: int, mode: int) -> bool:
    return mode in (MODE_QUANTILE, 2) and e % 2 == 0   # 2 = MODE_QUANTILE_POWER


def references(nq: int) -> np.ndarray:
    return np.linspace(0.0, 1.0, nq, endpoint=True)


QUANTILE_SUBSAMPLE = 10_000  # sklearn QuantileTransformer's default ``subsample``


def check_n_quantiles(n_rows: int, div: int = QUANTILE_DIV) -> int:
    """``QuantileTransformer.fit``'s own check: n_quantiles may not exceed ``subsample``."""
    nq_req = max(n_rows // div, 2)
    if nq_req > QUANTILE_SUBSAMPLE:
        raise ValueError(f"The number of quantiles cannot be greater than the number of samples used. Got {nq_req} "
                         f"quantiles and {QUANTILE_SUBSAMPLE} samples.")
    return n_quantiles_for(n_rows, div)


def quantile_subsample(n_rows: int, seed: int):
    """Rows ``QuantileTransformer(random_state=seed)`` fits its quantiles on (sklearn 1.7.2
    ``_dense_fit``: ``resample(X, replace=False, n_samples=subsample, random_state=
    RandomState(seed))`` = the first ``subsample`` entries of ``RandomState(seed).shuffle(arange(n))``),
    or None when the context has at most ``subsample`` rows (every row is used)."""
    if n_rows <= QUANTILE_SUBSAMPLE:
        return None
    idx = np.arange(n_rows)
    np.random.RandomState(int(seed) & 0xFFFFFFFF).shuffle(idx)
    return idx[:QUANTILE_SUBSAMPLE]


def mt19937_shuffle_head(n_rows: int, seed: int, head: int = QUANTILE_SUBSAMPLE) -> np.ndarray:
    """The engine's k_qt_subsample restated step by step (pure Python; tests pin it to numpy):
    MT19937 with numpy's legacy integer seeding, twist and tempering; ``random_interval``'s
    masked rejection; Fisher-Yates swaps for i = n-1 .. head only (the later swaps permute the
    first ``head`` entries among themselves, so the SET of the first ``head`` entries is final).
    Returns that set, sorted."""
    mt = [0] * 624
    v = int(seed) & 0xFFFFFFFF
    for i in range(624):
        mt[i] = v
        v = (1812433253 * (v ^ (v >> 30)) + i + 1) & 0xFFFFFFFF
    state = {"pos": 624}

    def twist():
        for kk in range(624):
            y = (mt[kk] & 0x80000000) | (mt[(kk + 1) % 624] & 0x7FFFFFFF)
            mt[kk] = mt[(kk + 397) % 624] ^ (y >> 1) ^ (0x9908B0DF if y & 1 else 0)

    def next32():
        if state["pos"] == 624:
            twist()
            state["pos"] = 0
        y = mt[state["pos"]]
        state["pos"] += 1
        y ^= y >> 11
        y ^= (y << 7) & 0x9D2C5680
        y ^= (y << 15) & 0xEFC60000
        y ^= y >> 18
        return y & 0xFFFFFFFF

    arr = list(range(n_rows))
    for i in range(n_rows - 1, head - 1, -1):
        mask = i
        for sh in (1, 2, 4, 8, 16):
            mask |= mask >> sh
        while True:
            j = next32() & mask
            if j <= i:
                break
        arr[i], arr[j] = arr[j], arr[i]
    return np.sort(np.asarray(arr[:head]))


def quantile_fit(col: np.ndarray, n_rows: int, div: int = QUANTILE_DIV, sub=None) -> np.ndarray:
    """``QuantileTransformer._dense_fit`` for one column -> float64 quantiles [n_q].

    NaN/inf are excluded (``nanpercentile``; the engine feeds non-finite values
    through its NaN-indicator path instead).  An all-non-finite column gives an
    empty table (the column is then passed through untransformed).  ``sub``: the
    fit's row subsample (:func:`quantile_subsample`) when the context has more than
    ``QUANTILE_SUBSAMPLE`` rows; n_quantiles still follows the full row count, as
    sklearn's ``n_quantiles_``."""
    nq = check_n_quantiles(n_rows, div)
    col = np.asarray(col)
    if sub is not None:
        col = col[sub]
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


def yeo_johnson_inverse(t: np.ndarray, lam: float) -> np.ndarray:
    """Inverse of :func:`yeo_johnson` (sklearn ``PowerTransformer._yeo_johnson_inverse_transform``);
    values outside the transform's range come out non-finite."""
    t = np.asarray(t, dtype=np.float64)
    out = np.zeros_like(t)
    pos = t >= 0
    with np.errstate(all="ignore"):
        if abs(lam) < _EPS1:
            out[pos] = np.exp(t[pos]) - 1.0
        else:
            out[pos] = np.power(t[pos] * lam + 1.0, 1.0 / lam) - 1.0
        if abs(lam - 2.0) > _EPS1:
            out[~pos] = 1.0 - np.power(-(2.0 - lam) * t[~pos] + 1.0, 1.0 / (2.0 - lam))
        else:
            out[~pos] = 1.0 - np.exp(-t[~pos])
    return out


# ===================================================================== ensemble
# MODE_ENSEMBLE restates the default TabPFNRegressor preprocessing ensemble
# [ext: tabpfn==2.2.1, reached through TabPFNRegressor(**regressor_init_kwargs) at
# npe_pfn/npe_pfn.py:48; the package is not installed here, so everything below is
# **parity unpinned** against tabpfn itself -- each sklearn piece is pinned against
# sklearn in tests/test_preprocess_oracle.py]:
#
# * two feature configs x two target transforms, balanced over the estimators in
#   product order (``EnsembleConfig.generate_for_regression``): estimator e takes combo
#   e // (E // 4) (leftovers: combos in order), combos = [(Q, none), (Q, safepower),
#   (P, none), (P, safepower)];
# * Q = ``PreprocessorConfig("quantile_uni", append_original=True,
#   global_transformer_name="svd")``: features [original F | quantile F | SVD k] where
#   the SVD is ``StandardScaler(with_mean=False)`` + ``TruncatedSVD(n_components=
#   max(1, min(n // 10 + 1, F // 2)))`` on [original | quantile] (none when F < 2),
#   appended (``FeatureUnion(passthrough, svd)``);
# * P = ``PreprocessorConfig("safepower")``: the Yeo-Johnson transform of every column;
# * then ``AddFingerprintFeaturesStep``: one column = sha256(row bytes + salt) mod 10000
#   / 10000, train rows re-hashed with +1, +2, ... until unique; the hashed row here is
#   the raw float64-widened feature row (tabpfn hashes its transformed row; equal raw
#   rows give equal transformed rows, and no float pipeline reproduces sklearn's
#   float64 bytes, so the hash VALUES cannot match tabpfn's anyway);
# * then the per-estimator feature shuffle (oracle.philox.estimator_permutation);
# * target transform "safepower": y -> Yeo-Johnson(y) before the standardization; the
#   estimator's bar distribution is mapped back by translating its probabilities from
#   the inverse-transformed borders to the common ones (``translate_probs_across_borders``
#   with ``_cancel_nan_borders`` repair).
#
# The CLASSIFIER's ensemble (MODE_ENSEMBLE on a classifier fit) [ext: tabpfn 2.2.1
# TabPFNClassifier default, reached through TabPFNClassifier(**classifier_init_kwargs) at
# npe_pfn/npe_pfn.py:610; parity unpinned against tabpfn, each piece pinned as above]:
# * two feature configs balanced over the estimators (``generate_for_classification``):
#   estimator e takes config e // (E // 2) (leftovers: configs in order), configs =
#   [Qc, N];
# * Qc = ``PreprocessorConfig("quantile_uni_coarse", append_original=True,
#   global_transformer_name="svd")``: as Q above with n_quantiles = max(n // 10, 2);
# * N = ``PreprocessorConfig("none")``: the original features;
# * both + the fingerprint feature; no target transform (the class shuffle of
#   OracleTabPFN.fit_classes stays).
MODE_ENSEMBLE = 3
T_RAW, T_QUANT, T_POWER, T_QSVD, T_PFP, T_RFP = 0, 1, 2, 3, 4, 5
FP_SALT = 0xF1A6E4A7F1A6E4A7
FP_BUCKETS = 10000


def estimator_configs(mode: int, E: int, classifier: bool = False):
    """[(feature type, target transform?)] per estimator for a preprocessing mode."""
    if mode == MODE_ENSEMBLE and classifier:
        combos = [(T_QSVD, False), (T_RFP, False)]
        bc = E // len(combos)
        out = [combos[i // bc] for i in range(bc * len(combos))] if bc else []
        out += combos[: E - len(out)]
        return out
    if mode == MODE_ENSEMBLE:
        combos = [(T_QSVD, False), (T_QSVD, True), (T_PFP, False), (T_PFP, True)]
        bc = E // len(combos)
        out = [combos[i // bc] for i in range(bc * len(combos))] if bc else []
        out += combos[: E - len(out)]
        return out
    out = []
    for e in range(E):
        if mode in (MODE_QUANTILE, MODE_QUANTILE_POWER) and e % 2 == 0:
            out.append((T_QUANT, False))
        elif mode == MODE_QUANTILE_POWER:
            out.append((T_POWER, False))
        else:
            out.append((T_RAW, False))
    return out


def svd_components(n: int, F: int) -> int:
    """TruncatedSVD n_components of the "svd" global transformer; 0 = no SVD (F < 2)."""
    return 0 if F < 2 else max(1, min(n // 10 + 1, F // 2))


def n_features_of(ftype: int, F: int, n: int) -> int:
    if ftype == T_QSVD:
        return 2 * F + svd_components(n, F) + 1
    if ftype in (T_PFP, T_RFP):
        return F + 1
    return F


def svd_fit(Z: np.ndarray, k: int):
    """StandardScaler(with_mean=False) + TruncatedSVD(k) on Z [n, m] (float64).

    Returns (scale [m], components [k, m]): scale = population std (1 where 0, as
    sklearn's ``_handle_zeros_in_scale``), components = the top-k right singular
    vectors of Z / scale (eigenvectors of the Gram matrix, descending), each signed so
    that its largest-magnitude entry is positive (sklearn ``svd_flip``,
    ``u_based_decision=False``)."""
    Z = np.asarray(Z, dtype=np.float64)
    mu = Z.mean(0)
    scale = np.sqrt(((Z - mu) ** 2).mean(0))
    scale = np.where(scale < 10 * np.finfo(np.float64).eps, 1.0, scale)
    Y = Z / scale
    w, v = np.linalg.eigh(Y.T @ Y)
    order = np.argsort(-w, kind="stable")[:k]
    comps = v[:, order].T.copy()
    for c in range(k):
        j = int(np.argmax(np.abs(comps[c])))
        if comps[c, j] < 0:
            comps[c] = -comps[c]
    return scale, comps


def svd_transform(Z: np.ndarray, scale: np.ndarray, comps: np.ndarray) -> np.ndarray:
    """(Z / scale) @ components^T, float64 -> float32."""
    return ((np.asarray(Z, dtype=np.float64) / scale) @ comps.T).astype(np.float32)


def fingerprint_salt(seed: int, estimator: int) -> int:
    """The estimator's hash salt in [0, 2^16) (tabpfn draws it from the step's RNG [ext])."""
    from oracle.philox import splitmix64_next

    s = ((int(seed) & 0xFFFFFFFF) | ((estimator & 0xFFFF) << 32)) ^ FP_SALT
    _, out = splitmix64_next(s)
    return int(out % 65536)


def row_hash(row64: np.ndarray) -> int:
    """int(sha256(row bytes).hexdigest(), 16) % 10000 (tabpfn ``_float_hash_arr`` [ext])."""
    import hashlib

    return int(hashlib.sha256(np.ascontiguousarray(row64, dtype="<f8").tobytes()).hexdigest(), 16) % FP_BUCKETS


FP_BLOCK = 10000  # train rows per block of distinct hashes (the engine's kFpBlock)


def fingerprint(X: np.ndarray, salt: int, train: bool) -> np.ndarray:
    """Fingerprint column of rows X [R, F] (float32, widened to float64 before hashing).

    Test rows: hash(row + salt).  Train rows, in order: the first of hash(row + salt),
    hash(row + salt + 1), ... not taken by an earlier train row of the same block of
    ``FP_BLOCK`` rows.  tabpfn keeps one set of taken hashes for all train rows [ext]; with
    10 000 hash values its re-hash loop cannot end past 10 000 rows, so the engine and this
    restatement start the set afresh every 10 000 rows (identical to tabpfn below that)."""
    X64 = np.asarray(X, dtype=np.float32).astype(np.float64)
    out = np.empty(X64.shape[0], dtype=np.float32)
    seen = set()
    for i in range(X64.shape[0]):
        if i % FP_BLOCK == 0:
            seen = set()
        base = X64[i] + float(salt)
        h = row_hash(base)
        if train:
            add = 0
            while h in seen:
                add += 1
                h = row_hash(base + float(add))
            seen.add(h)
        out[i] = np.float32(h / FP_BUCKETS)
    return out


def cancel_broken_borders(b: np.ndarray):
    """tabpfn ``_cancel_nan_borders`` [ext]: broken = non-finite or |b| > 1e3; a broken run
    at the left end takes the first good border (and b[0] = b[1] - 1), at the right end
    the last good one (and b[-1] = b[-2] + 1); bars touching a broken border get no mass.
    Returns (repaired borders float64, cancel mask [nb] bool)."""
    b = np.asarray(b, dtype=np.float64).copy()
    with np.errstate(invalid="ignore"):
        broken = ~np.isfinite(b) | (b > 1e3) | (b < -1e3)
    if broken.all():
        raise ValueError("every translated border is broken")
    good = np.where(~broken)[0]
    lo, hi = good[0], good[-1]
    if lo > 0:
        b[:lo] = b[lo]
        b[0] = b[1] - 1.0
    if hi < b.size - 1:
        b[hi + 1:] = b[hi]
        b[-1] = b[-2] + 1.0
    return b, broken[1:] | broken[:-1]


def translation_table(frm: np.ndarray, to: np.ndarray):
    """Row-independent part of ``translate_probs_across_borders`` [ext]: for every target
    border, its source bucket, the share of that bucket left of it, and a flag
    (-1: at/below frm[0] -> cdf 0, +1: at/above frm[-1] -> cdf 1, 0: interpolate).
    Float32 like tabpfn's torch arithmetic."""
    frm = np.asarray(frm, dtype=np.float32)
    to = np.asarray(to, dtype=np.float32)
    nb = frm.size - 1
    idx = np.clip(np.searchsorted(frm, to, side="left") - 1, 0, nb - 1)
    w = (frm[1:] - frm[:-1]).astype(np.float32)
    with np.errstate(all="ignore"):
        share = np.clip((to - frm[idx]) / w[idx], np.float32(0), np.float32(1)).astype(np.float32)
    flag = np.where(to <= frm[0], -1, np.where(to >= frm[-1], 1, 0)).astype(np.int32)
    return idx.astype(np.int32), share, flag


def translate_probs(p: np.ndarray, idx: np.ndarray, share: np.ndarray, flag: np.ndarray) -> np.ndarray:
    """Probabilities p [R, nb] over the source bars -> [R, nb] over the target bars:
    cdf at every target border (exclusive cumsum + share of the bucket), first / last
    forced to 0 / 1, differences clamped at 0 (float32)."""
    p = np.asarray(p, dtype=np.float32)
    cum = (np.cumsum(p, axis=1, dtype=np.float32) - p).astype(np.float32)
    left = (cum[:, idx] + p[:, idx] * share[None, :]).astype(np.float32)
    left = np.where(flag[None, :] < 0, np.float32(0), np.where(flag[None, :] > 0, np.float32(1), left))
    left = np.clip(left, 0, 1)
    left[:, 0] = 0
    left[:, -1] = 1
    return np.maximum(left[:, 1:] - left[:, :-1], np.float32(0)).astype(np.float32)
