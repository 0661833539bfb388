"""ORACLE (test infrastructure only) -- CPU restatement of the TabPFN-v2 regressor path.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s cpu_baseline leg
may import this package; the product path (``npe-pfn_amd/``) never does.

PARITY STATUS: **parity unpinned** for the transformer forward and the bar
distribution.  The reference calls this arithmetic through the external
``tabpfn==2.2.1`` package (pinned at poetry.lock:4455-4464; call sites
npe_pfn/npe_pfn.py:140-151, 215-228, 502-512), which is not vendored under
/root/reference, is not installed here, and ships no golden vectors; its
weights download from the network.  This module restates the published
algorithm of that release [ext], as listed below, and is the build's own
specification of it.  The orchestration around it (npe_pfn.py, accept/reject,
filters) IS pinned: tests/golden/make_golden.py runs the reference's own
Python with this oracle plugged in as ``tabpfn.TabPFNRegressor``.

Algorithm restated (tabpfn 2.2.1, [ext] module names):

* ``TabPFNRegressor.fit``: target standardization y_z = (y - mean) / (std + 1e-20)
  (population std); per-estimator preprocessing -- here a feature shuffle only
  (``oracle.philox.estimator_permutation``).  The quantile/power/SVD transforms,
  fingerprint feature and target transforms of the full ensemble are NOT
  restated (documented reduction, SURVEY.md §7 hard part 1, §8f row 3).
* encoder (``model/encoders.py``): NaN/inf handling (value -> train mean,
  indicator -2 / +2 / +4), per-feature normalization with train-row mean and
  unbiased std, clip to +-100, group scaling sqrt(2 / used features), linear
  map [x_a, x_b, ind_a, ind_b] -> d without bias, plus a per-group
  ("subspace") positional embedding; the target column is its own token,
  encoded from [y_z, nan-indicator] (test rows: [mean(y_z), -2]).
* ``PerFeatureEncoderLayer`` x 12, post-norm: feature attention over the C
  tokens of a row -> LN; item attention where every row attends to the
  TRAIN rows of the same column (multiquery for the test set) -> LN;
  MLP (GELU, no bias) -> LN.  Attention scale 1/sqrt(32), no biases.
* decoder: Linear(d, 768) + GELU + Linear(768, 5000) on the target token of
  the test rows; per-estimator softmax(logits / 0.9); probabilities averaged
  over estimators; ``logits`` returned as log of that average.
* ``FullSupportBarDistribution`` with borders * std + mean: ``sample`` =
  inverse CDF with linear interpolation inside the bucket; ``__call__`` =
  NLL = -(log p_b - log w_b) with half-normal tails in the two end buckets.

``emulate_bf16=True`` rounds every tensor at the points where the HIP engine
stores bf16 (GEMM operands, attention q/k/v/outputs, MLP hidden), which gives a
tighter per-kernel check than the plain fp32 restatement.
"""

from __future__ import annotations

import math
import os
from concurrent.futures import ThreadPoolExecutor
from dataclasses import dataclass
from typing import Dict, List, Optional

import numpy as np

from oracle.philox import class_permutation, estimator_permutation, uniforms
from oracle.preprocess_oracle import (MODE_QUANTILE, MODE_QUANTILE_POWER, estimator_uses_power, estimator_uses_quantile,
                                      power_transform_vec, quantile_fit, quantile_transform_vec, yj_fit)

NAN_INDICATOR = -2.0
INF_INDICATOR = 2.0
NEG_INF_INDICATOR = 4.0
HALFNORMAL_MEDIAN = 0.6744897501960817  # HalfNormal(1).icdf(0.5) = sqrt(2) erfinv(0.5)


def n_threads() -> int:
    """Worker threads of the oracle (OMP_NUM_THREADS, else all visible cores)."""
    env = os.environ.get("NPFN_ORACLE_THREADS") or os.environ.get("OMP_NUM_THREADS")
    return max(1, int(env)) if env else max(1, os.cpu_count() or 1)


_POOL: Optional[ThreadPoolExecutor] = None
_CTL = None


def _pmap(fn, items):
    """Run fn over items on a thread pool (numpy releases the GIL in its kernels).

    BLAS is limited to one thread inside the pool so the pool owns the cores.
    """
    global _POOL, _CTL
    items = list(items)
    if len(items) <= 1 or n_threads() == 1:
        return [fn(i) for i in items]
    if _POOL is None:
        from threadpoolctl import ThreadpoolController

        _POOL = ThreadPoolExecutor(max_workers=n_threads())
        _CTL = ThreadpoolController()
    with _CTL.limit(limits=1, user_api="blas"):
        return list(_POOL.map(fn, items))


def _row_chunks(n: int, parts: int):
    step = max(1, -(-n // parts))
    return [(i, min(n, i + step)) for i in range(0, n, step)]


def bf16_round(a: np.ndarray) -> np.ndarray:
    """Round float32 to the nearest bf16 (ties to even), returned as float32."""
    a = np.ascontiguousarray(a, dtype=np.float32)
    u = a.view(np.uint32).astype(np.uint64)
    u = (u + 0x7FFF + ((u >> 16) & 1)) & 0xFFFF0000
    return u.astype(np.uint32).view(np.float32).reshape(a.shape)


def gelu(x: np.ndarray) -> np.ndarray:
    from scipy.special import erf

    x = np.asarray(x, dtype=np.float32)
    return (np.float32(0.5) * x * (np.float32(1.0) + erf(x * np.float32(0.7071067811865476)))).astype(np.float32)


def layer_norm(x: np.ndarray, g: np.ndarray, b: np.ndarray, eps: float = 1e-5) -> np.ndarray:
    x = np.asarray(x, dtype=np.float32)
    mu = x.mean(-1, keepdims=True, dtype=np.float64).astype(np.float32)
    xc = x - mu
    var = (xc * xc).mean(-1, keepdims=True, dtype=np.float64).astype(np.float32)
    return (xc * (np.float32(1.0) / np.sqrt(var + np.float32(eps))) * g + b).astype(np.float32)


def softmax(x: np.ndarray, axis: int = -1) -> np.ndarray:
    x = np.asarray(x, dtype=np.float32)
    m = x.max(axis=axis, keepdims=True)
    e = np.exp(x - m)
    return (e / e.sum(axis=axis, keepdims=True, dtype=np.float64).astype(np.float32)).astype(np.float32)


@dataclass
class EstimatorState:
    perm: np.ndarray       # [F] column order for this estimator
    mu: np.ndarray         # [F] train mean of permuted columns
    sd: np.ndarray         # [F] train std (ddof=1) of permuted columns
    gscale: np.ndarray     # [G] sqrt(fpg / used features in group)


@dataclass
class FitState:
    n_features: int
    n_groups: int
    y_mean: float
    y_std: float
    ybar_z: float
    estimators: List[EstimatorState]
    kv: List[np.ndarray]   # per layer: [E, n, C, 2, d] train K and V of the item attention
    n_classes: int = 0                     # > 0: classifier fit (fit_classes)
    cperm: Optional[np.ndarray] = None     # [E, K] per-estimator class permutation
    ybar_e: Optional[np.ndarray] = None    # [E] test-row target value per estimator


class OracleTabPFN:
    """numpy restatement of the v2 regressor forward (see module docstring)."""

    def __init__(self, weights: Dict[str, np.ndarray], n_estimators: int = 8,
                 softmax_temperature: float = 0.9, seed: int = 0,
                 emulate_bf16: bool = False, n_heads: int = 6, features_per_group: int = 2,
                 preprocessing: int = 0):
        self.w = {k: np.asarray(v, dtype=np.float32) for k, v in weights.items()}
        self.pre = int(preprocessing)   # 1: quantile on even estimators; 2: + Yeo-Johnson on odd ones
        self.plam: List[float] = []
        self.qtab: List[np.ndarray] = []
        self.E = int(n_estimators)
        self.T = float(softmax_temperature)
        self.seed = int(seed)
        self.emulate = bool(emulate_bf16)
        self.H = n_heads
        self.fpg = features_per_group
        self.d = self.w["enc_w"].shape[0]
        self.hd = self.d // self.H
        self.L = sum(1 for k in self.w if k.endswith(".feat_qkv"))
        self.nb = self.w["dec_b2"].shape[0]
        if self.emulate:
            for k in list(self.w):
                if any(k.endswith(s) for s in ("feat_qkv", "feat_out", "item_qkv", "item_out",
                                               "mlp_w1", "mlp_w2")) or k in ("dec_w1", "dec_w2"):
                    self.w[k] = bf16_round(self.w[k])
        self.state: Optional[FitState] = None

    # ---------------------------------------------------------------- helpers
    def _bf(self, a):
        return bf16_round(a) if self.emulate else np.asarray(a, dtype=np.float32)

    def _mm(self, a, wname):
        """a @ W^T with fp32 accumulation (operands rounded when emulating)."""
        a = self._bf(a)
        W = self.w[wname]
        out = np.ascontiguousarray(a, dtype=np.float32).reshape(-1, a.shape[-1]) @ W.T
        return out.astype(np.float32).reshape(a.shape[:-1] + (W.shape[0],))

    # -------------------------------------------------------------------- fit
    def fit(self, X: np.ndarray, y: np.ndarray) -> FitState:
        """Regressor fit (npe_pfn.py:140, 215, 502): standardized target token."""
        X = np.asarray(X, dtype=np.float32)
        y = np.asarray(y, dtype=np.float32).reshape(-1)
        assert y.shape[0] == X.shape[0]
        y64 = y.astype(np.float64)
        y_mean = float(np.float32(y64.mean()))
        y_std = float(np.float32(y64.std() + 1e-20))
        y_z = ((y - np.float32(y_mean)) / np.float32(y_std)).astype(np.float32)
        ybar_z = float(np.float32(y_z.astype(np.float64).mean()))
        st = self._fit_features(X, y_mean, y_std, ybar_z)
        return self._fit_forward(X, st, y_z)

    def fit_classes(self, X: np.ndarray, y: np.ndarray, n_classes: int) -> FitState:
        """Classifier fit (TabPFNClassifier.fit at npe_pfn.py:661) [ext: tabpfn 2.2.1].

        ``y`` holds label indices 0..K-1 (the host's label encoding).  Per
        estimator the labels are permuted (``class_permutation``, restating the
        ensemble's class shift "shuffle"), and the target token of a train row
        encodes [perm_e(y), 0]; a test row encodes [mean_train perm_e(y), -2]
        (the target encoder's NaN handling fills the train mean).
        """
        X = np.asarray(X, dtype=np.float32)
        yi = np.asarray(y).reshape(-1).astype(np.int64)
        assert yi.shape[0] == X.shape[0]
        K = int(n_classes)
        assert K >= 2 and yi.min() >= 0 and yi.max() < K
        cperm = np.stack([class_permutation(self.seed, e, K) for e in range(self.E)])  # [E, K]
        ty = cperm[:, yi].astype(np.float32)                                             # [E, n]
        ybar_e = (ty.astype(np.float64).sum(1) / yi.shape[0]).astype(np.float32)
        st = self._fit_features(X, 0.0, 1.0, 0.0)
        st.n_classes, st.cperm, st.ybar_e = K, cperm, ybar_e
        return self._fit_forward(X, st, ty)

    def _fit_features(self, X: np.ndarray, y_mean: float, y_std: float, ybar_z: float) -> FitState:
        n, F = X.shape
        fpg = self.fpg
        G = (F + fpg - 1) // fpg
        ests = []
        pre = (MODE_QUANTILE, MODE_QUANTILE_POWER)
        self.qtab = [quantile_fit(X[:, j], n) for j in range(F)] if self.pre in pre else []
        self.plam = [yj_fit(X[:, j]) for j in range(F)] if self.pre == MODE_QUANTILE_POWER else []
        Xt = self._views(X)
        for e in range(self.E):
            perm = estimator_permutation(self.seed, e, F)
            Xp = Xt[self._view_of(e)][:, perm].astype(np.float64)
            finite = np.isfinite(Xp)
            cnt = finite.sum(0)
            s1 = np.where(finite, Xp, 0.0).sum(0)
            mu = s1 / np.maximum(cnt, 1)
            dev = np.where(finite, Xp - mu, 0.0)
            sd = np.sqrt((dev**2).sum(0) / np.maximum(cnt - 1, 1))
            mx = np.where(finite, Xp, -np.inf).max(0)
            mn = np.where(finite, Xp, np.inf).min(0)
            used = (mx > mn).astype(np.int64)
            used_pad = np.zeros(G * fpg, dtype=np.int64)
            used_pad[:F] = used
            ug = used_pad.reshape(G, fpg).sum(1)
            gscale = np.sqrt(fpg / np.maximum(ug, 1)).astype(np.float32)
            ests.append(EstimatorState(perm, mu.astype(np.float32), sd.astype(np.float32), gscale))
        return FitState(F, G, y_mean, y_std, ybar_z, ests, [])

    def _views(self, X: np.ndarray) -> Dict[str, np.ndarray]:
        """The table as each estimator sees it: raw, quantile- or power-transformed per
        column with the train tables (k_encode's per-value transforms)."""
        X = np.asarray(X, dtype=np.float32)
        v = {"raw": X}
        if self.qtab:
            v["quantile"] = np.stack([quantile_transform_vec(X[:, j], self.qtab[j]) for j in range(X.shape[1])], 1)
        if self.plam:
            v["power"] = np.stack([power_transform_vec(X[:, j], self.plam[j]) for j in range(X.shape[1])], 1)
        return v

    def _view_of(self, e: int) -> str:
        if estimator_uses_quantile(e, self.pre):
            return "quantile"
        return "power" if estimator_uses_power(e, self.pre) else "raw"

    def _fit_forward(self, X: np.ndarray, st: FitState, train_y: np.ndarray) -> FitState:
        self.state = st
        # train-side forward: K/V cache per layer
        x = self._encode(X, st, train_y=train_y)
        st.kv = []
        for l in range(self.L):
            x = self._layer(x, l, st, train=True)
        return st

    # ----------------------------------------------------------------- encode
    def _encode(self, Xrows: np.ndarray, st: FitState, train_y: Optional[np.ndarray]) -> np.ndarray:
        """Token embeddings [E, R, C, d] (C = groups + target token)."""
        R = Xrows.shape[0]
        G, fpg, d = st.n_groups, self.fpg, self.d
        C = G + 1
        W = self.w["enc_w"]          # [d, 4]
        Wy = self.w["y_enc_w"]       # [d, 2]
        pe = self.w["pos_emb"]       # [Gmax, d]
        out = np.zeros((self.E, R, C, d), dtype=np.float32)
        Xt = self._views(Xrows)
        for e, es in enumerate(st.estimators):
            xp = Xt[self._view_of(e)][:, es.perm]
            isnan = np.isnan(xp)
            ispinf = np.isposinf(xp)
            isninf = np.isneginf(xp)
            ind = (isnan * NAN_INDICATOR + ispinf * INF_INDICATOR + isninf * NEG_INF_INDICATOR).astype(np.float32)
            v = np.where(isnan | ispinf | isninf, es.mu[None, :], xp).astype(np.float32)
            xn = np.clip((v - es.mu) / (es.sd + np.float32(1e-16)), -100.0, 100.0).astype(np.float32)
            xpad = np.zeros((R, G * fpg), dtype=np.float32)
            ipad = np.zeros((R, G * fpg), dtype=np.float32)
            xpad[:, : st.n_features] = xn
            ipad[:, : st.n_features] = ind
            xpad = xpad.reshape(R, G, fpg) * es.gscale[None, :, None]
            ipad = ipad.reshape(R, G, fpg)
            feats = np.concatenate([xpad, ipad], axis=-1)  # [R, G, 4] = [x_a, x_b, ind_a, ind_b]
            out[e, :, :G, :] = (feats @ W.T) + pe[None, :G, :]
            if train_y is not None:
                ty = train_y[e] if train_y.ndim == 2 else train_y   # [E, n]: per-estimator labels
                yin = np.stack([ty, np.zeros_like(ty)], -1)
            else:
                yb = st.ybar_e[e] if st.ybar_e is not None else st.ybar_z
                yin = np.tile(np.array([[yb, NAN_INDICATOR]], dtype=np.float32), (R, 1))
            out[e, :, G, :] = yin @ Wy.T
        return out

    # ------------------------------------------------------------------ layer
    def _layer(self, x: np.ndarray, l: int, st: FitState, train: bool) -> np.ndarray:
        E, R, C, d = x.shape
        H, hd = self.H, self.hd
        p = f"l{l}."
        # feature attention (per row over its C tokens)
        qkv = self._bf(self._mm(x, p + "feat_qkv")).reshape(E * R, C, 3, H, hd)
        o = np.empty((E * R, C, H, hd), dtype=np.float32)

        def feat_chunk(rg):
            a, b = rg
            q, k, v = qkv[a:b, :, 0], qkv[a:b, :, 1], qkv[a:b, :, 2]
            sc = np.einsum("rchd,rkhd->rhck", q, k, optimize=True) / np.float32(math.sqrt(hd))
            o[a:b] = np.einsum("rhck,rkhd->rchd", softmax(sc, -1), v, optimize=True)

        _pmap(feat_chunk, _row_chunks(E * R, 4 * n_threads()))
        o = self._bf(o.reshape(E, R, C, d))
        x = self._ln(x + self._mm(o, p + "feat_out"), p + "ln1")
        # item attention (rows attend to the train rows of the same column)
        if train:
            qkv = self._bf(self._mm(x, p + "item_qkv")).reshape(E, R, C, 3, d)
            q = qkv[..., 0, :]
            kv = qkv[..., 1:, :]                     # [E, n, C, 2, d]
            st.kv.append(kv)
        else:
            wq = self.w[p + "item_qkv"][:d]
            q = self._bf((self._bf(x) @ wq.T).astype(np.float32))
            kv = st.kv[l]
        o = np.zeros((E, R, C, d), dtype=np.float32)
        scale = np.float32(1.0 / math.sqrt(hd))
        qblk = max(1, min(R, 2048))

        def item_task(t):
            e, c, h, r0 = t
            r1 = min(R, r0 + qblk)
            qh = q[e, r0:r1, c, h * hd:(h + 1) * hd]                          # [r, hd]
            kh = kv[e, :, c, 0, h * hd:(h + 1) * hd]                           # [n, hd]
            vh = kv[e, :, c, 1, h * hd:(h + 1) * hd]
            sc = (qh @ kh.T) * scale
            o[e, r0:r1, c, h * hd:(h + 1) * hd] = softmax(sc, -1) @ vh

        _pmap(item_task, [(e, c, h, r0) for e in range(E) for c in range(C) for h in range(H)
                          for r0 in range(0, R, qblk)])
        o = self._bf(o)
        x = self._ln(x + self._mm(o, p + "item_out"), p + "ln2")
        if train and l == self.L - 1:
            return x  # nothing reads train rows after the last item attention
        h = self._bf(self._gelu(self._mm(x, p + "mlp_w1")))
        x = self._ln(x + self._mm(h, p + "mlp_w2"), p + "ln3")
        return x

    def _ln(self, x, pre):
        x = np.ascontiguousarray(x, dtype=np.float32)
        flat = x.reshape(-1, x.shape[-1])
        out = np.empty_like(flat)
        g, b = self.w[pre + "_g"], self.w[pre + "_b"]

        def f(rg):
            out[rg[0]:rg[1]] = layer_norm(flat[rg[0]:rg[1]], g, b)

        _pmap(f, _row_chunks(flat.shape[0], 4 * n_threads()))
        return out.reshape(x.shape)

    def _gelu(self, x):
        x = np.ascontiguousarray(x, dtype=np.float32)
        flat = x.reshape(-1, x.shape[-1])
        out = np.empty_like(flat)

        def f(rg):
            out[rg[0]:rg[1]] = gelu(flat[rg[0]:rg[1]])

        _pmap(f, _row_chunks(flat.shape[0], 4 * n_threads()))
        return out.reshape(x.shape)

    # ---------------------------------------------------------------- predict
    def predict_probs(self, Xq: np.ndarray, return_estimator_logits: bool = False):
        st = self.state
        assert st is not None, "fit() first"
        Xq = np.asarray(Xq, dtype=np.float32)
        assert Xq.shape[1] == st.n_features
        x = self._encode(Xq, st, train_y=None)
        for l in range(self.L):
            x = self._layer(x, l, st, train=False)
        z = x[:, :, st.n_groups, :]                              # target token [E, R, d]
        h = self._bf(self._gelu(self._mm(z, "dec_w1") + self.w["dec_b1"]))
        logits = (self._mm(h, "dec_w2") + self.w["dec_b2"]).astype(np.float32)  # [E, R, nb]
        probs = np.empty((logits.shape[1], logits.shape[2]), dtype=np.float32)
        invT = np.float32(1.0 / self.T)

        def mix(rg):
            a, b = rg
            pe = softmax(logits[:, a:b] * invT, -1).astype(np.float64)
            probs[a:b] = pe.mean(0).astype(np.float32)

        _pmap(mix, _row_chunks(logits.shape[1], 4 * n_threads()))
        if return_estimator_logits:
            return probs, logits
        return probs

    def predict_proba(self, Xq: np.ndarray) -> np.ndarray:
        """Classifier probabilities [R, K] (TabPFNClassifier.predict_proba, npe_pfn.py:697).

        Per estimator: decoder logits of the permuted classes, softmax(logits / T)
        over the K classes present, mapped back to the original labels; the
        estimators' probabilities are averaged [ext: tabpfn 2.2.1 classifier].
        """
        st = self.state
        assert st is not None and st.n_classes > 0, "fit_classes() first"
        Xq = np.asarray(Xq, dtype=np.float32)
        assert Xq.shape[1] == st.n_features
        x = self._encode(Xq, st, train_y=None)
        for l in range(self.L):
            x = self._layer(x, l, st, train=False)
        z = x[:, :, st.n_groups, :]
        h = self._bf(self._gelu(self._mm(z, "dec_w1") + self.w["dec_b1"]))
        logits = (self._mm(h, "dec_w2") + self.w["dec_b2"]).astype(np.float32)  # [E, R, n_out]
        invT = np.float32(1.0 / self.T)
        acc = np.zeros((logits.shape[1], st.n_classes), dtype=np.float64)
        for e in range(self.E):
            acc += softmax(logits[e][:, st.cperm[e]] * invT, -1).astype(np.float64)
        return (acc / self.E).astype(np.float32)

    def borders(self) -> np.ndarray:
        st = self.state
        return (self.w["borders"] * np.float32(st.y_std) + np.float32(st.y_mean)).astype(np.float32)


# ------------------------------------------------------------ bar distribution
def bar_sample(logits: np.ndarray, borders: np.ndarray, u: np.ndarray) -> np.ndarray:
    """Inverse-CDF sample with linear interpolation in the bucket.

    [ext: tabpfn 2.2.1 BarDistribution.sample/icdf]; called at npe_pfn.py:146,220.
    """
    p = softmax(np.asarray(logits, dtype=np.float32), -1).astype(np.float64)
    nb = p.shape[1]
    cdf = np.cumsum(p, axis=1)
    u64 = np.asarray(u, dtype=np.float64)
    idx = np.array([np.searchsorted(cdf[i], u64[i], side="left") for i in range(p.shape[0])])
    idx = np.clip(idx, 0, nb - 1)
    cdf0 = np.concatenate([np.zeros((p.shape[0], 1)), cdf], axis=1)
    rows = np.arange(p.shape[0])
    rest = u64 - cdf0[rows, idx]
    b = np.asarray(borders, dtype=np.float64)
    left, right = b[idx], b[idx + 1]
    return (left + (right - left) * rest / p[rows, idx]).astype(np.float32)


def bar_bucket(borders: np.ndarray, y: np.ndarray) -> np.ndarray:
    """searchsorted(borders, y) - 1 with the end-border fix-ups, clamped [ext: map_to_bucket_idx]."""
    b = np.asarray(borders, dtype=np.float32)
    y = np.asarray(y, dtype=np.float32)
    nb = b.shape[0] - 1
    idx = np.searchsorted(b, y, side="left") - 1
    idx = np.where(y == b[0], 0, idx)
    idx = np.where(y == b[-1], nb - 1, idx)
    return np.clip(idx, 0, nb - 1)


def bar_nll(logits: np.ndarray, borders: np.ndarray, y: np.ndarray) -> np.ndarray:
    """FullSupportBarDistribution NLL [ext: tabpfn 2.2.1 FullSupportBarDistribution.forward].

    Called as ``criterion(logits, y)`` at npe_pfn.py:149,226,510.
    """
    logits = np.asarray(logits, dtype=np.float32).astype(np.float64)
    b = np.asarray(borders, dtype=np.float32).astype(np.float64)
    y64 = np.asarray(y, dtype=np.float32).astype(np.float64)
    nb = b.shape[0] - 1
    w = np.diff(b)
    m = logits.max(1, keepdims=True)
    lsm = logits - m - np.log(np.exp(logits - m).sum(1, keepdims=True))
    idx = bar_bucket(borders, y)
    rows = np.arange(logits.shape[0])
    lp = lsm[rows, idx] - np.log(w[idx])
    s0 = w[0] / HALFNORMAL_MEDIAN
    s1 = w[-1] / HALFNORMAL_MEDIAN

    def hn_logpdf(v, s):
        return np.log(np.sqrt(2.0 / np.pi) / s) - v * v / (2.0 * s * s)

    left = idx == 0
    right = idx == nb - 1
    lp = np.where(left, lp + hn_logpdf(np.maximum(b[1] - y64, 1e-8), s0) + np.log(w[0]), lp)
    lp = np.where(right, lp + hn_logpdf(np.maximum(y64 - b[-2], 1e-8), s1) + np.log(w[-1]), lp)
    return (-lp).astype(np.float32)


class OracleRegressor:
    """tabpfn.TabPFNRegressor-compatible wrapper around OracleTabPFN.

    Implements exactly the surface the reference uses:
    ``fit(X, y)``, ``predict(X, output_type="full", quantiles=[])`` returning
    ``{"logits", "criterion"}``, ``criterion.sample(logits)`` (one Philox
    counter per call) and ``criterion(logits, y)``.
    """

    default_weights: Optional[Dict[str, np.ndarray]] = None

    def __init__(self, n_estimators: int = 8, softmax_temperature: float = 0.9,
                 random_state: int = 0, weights=None, emulate_bf16: bool = False, **_ignored):
        w = weights if weights is not None else OracleRegressor.default_weights
        if w is None:
            raise RuntimeError("OracleRegressor needs weights (set OracleRegressor.default_weights)")
        self.model = OracleTabPFN(w, n_estimators, softmax_temperature, random_state, emulate_bf16)
        self.random_state = int(random_state)
        self.sample_counter = 0
        self.calls: List[tuple] = []

    def fit(self, X, y):
        X = _np(X)
        y = _np(y)
        self.calls.append(("fit", tuple(X.shape), tuple(y.shape)))
        self.model.fit(X, y)
        return self

    def predict(self, X, output_type="full", quantiles=None):
        import torch

        X = _np(X)
        self.calls.append(("predict", tuple(X.shape), output_type))
        probs = self.model.predict_probs(X)
        logits = np.log(np.maximum(probs, np.float32(1e-38))).astype(np.float32)
        return {"logits": torch.from_numpy(logits), "criterion": OracleCriterion(self, self.model.borders())}


class OracleCriterion:
    def __init__(self, reg: OracleRegressor, borders: np.ndarray):
        self.reg = reg
        self.borders = borders

    def sample(self, logits, t: float = 1.0):
        import torch

        lg = _np(logits) / np.float32(t)
        u = uniforms(self.reg.random_state, self.reg.sample_counter, lg.shape[0])
        self.reg.sample_counter += 1
        return torch.from_numpy(bar_sample(lg, self.borders, u))

    def __call__(self, logits, y):
        import torch

        return torch.from_numpy(bar_nll(_np(logits), self.borders, _np(y)))


class OracleClassifier:
    """tabpfn.TabPFNClassifier-compatible wrapper around OracleTabPFN.fit_classes.

    The surface the reference uses: ``fit(X, y)`` (npe_pfn.py:661)
    and ``predict_proba(X)`` returning a numpy ``[N, n_classes]`` array in the
    order of ``classes_`` (npe_pfn.py:697-701).  Labels are encoded like
    sklearn's LabelEncoder (sorted unique values).
    """

    default_weights: Optional[Dict[str, np.ndarray]] = None

    def __init__(self, n_estimators: int = 8, softmax_temperature: float = 0.9,
                 random_state: int = 0, weights=None, emulate_bf16: bool = False, **_ignored):
        w = weights if weights is not None else OracleClassifier.default_weights
        if w is None:
            raise RuntimeError("OracleClassifier needs weights (set OracleClassifier.default_weights)")
        self.model = OracleTabPFN(w, n_estimators, softmax_temperature, random_state, emulate_bf16)
        self.classes_ = None
        self.calls: List[tuple] = []

    def fit(self, X, y):
        X = _np(X)
        yv = np.asarray(y.detach().cpu().numpy() if hasattr(y, "detach") else y).reshape(-1)
        self.classes_, yi = np.unique(yv, return_inverse=True)
        if self.classes_.shape[0] < 2:
            raise ValueError("classifier fit needs at least two classes")
        self.calls.append(("fit", tuple(X.shape), tuple(yv.shape)))
        self.model.fit_classes(X, yi, self.classes_.shape[0])
        return self

    def predict_proba(self, X) -> np.ndarray:
        X = _np(X)
        self.calls.append(("predict_proba", tuple(X.shape)))
        return self.model.predict_proba(X)


def _np(t) -> np.ndarray:
    if hasattr(t, "detach"):
        t = t.detach().cpu().numpy()
    return np.asarray(t, dtype=np.float32)
