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
  (population std); per-estimator preprocessing (``preprocessing`` mode, see
  oracle/preprocess_oracle.py): 0 = feature shuffle only, 1 / 2 = quantile / Yeo-Johnson
  views on alternating estimators, 3 = the default regressor ensemble of tabpfn
  (quantile + original + SVD | Yeo-Johnson features, fingerprint feature, Yeo-Johnson
  target transform with border translation), each followed by the feature shuffle
  (``oracle.philox.estimator_permutation``).  Mode 3 is the OracleRegressor default,
  as ``preprocessing="ensemble"`` is the engine regressor's.
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
from oracle.preprocess_oracle import (MODE_ENSEMBLE, QUANTILE_DIV, QUANTILE_DIV_COARSE, T_PFP, T_POWER, T_QSVD, T_QUANT, T_RAW, T_RFP, cancel_broken_borders,
                                      estimator_configs, fingerprint, fingerprint_salt, n_features_of,
                                      power_transform_vec, quantile_fit, quantile_subsample, quantile_transform_vec,
                                      svd_components,
                                      svd_fit, svd_transform, translate_probs, translation_table, yeo_johnson_inverse,
                                      yj_fit)

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
    ftype: int             # feature pipeline (preprocess_oracle.T_*)
    target_tf: bool        # Yeo-Johnson target transform (ensemble mode)
    n_feat: int            # features after the pipeline (F_e)
    n_groups: int          # G_e = ceil(F_e / 2); tokens C_e = G_e + 1
    perm: np.ndarray       # [F_e] column order for this estimator
    mu: np.ndarray         # [F_e] train mean of permuted columns
    sd: np.ndarray         # [F_e] train std (ddof=1) of permuted columns
    gscale: np.ndarray     # [G_e] sqrt(fpg / used features in group)
    salt: int = 0          # fingerprint salt (T_QSVD / T_PFP)
    ystats: tuple = (0.0, 1.0, 0.0)   # (mean, std, mean of standardized) of its train target


@dataclass
class FitState:
    n_features: int
    n_groups: int          # of the plain pipeline (modes 0-2: every estimator)
    y_mean: float
    y_std: float
    ybar_z: float
    estimators: List[EstimatorState]
    kv: List[List[np.ndarray]]   # per estimator group (_groups), per layer: [E_g, n, C, 2, d] train K/V
    n_classes: int = 0                     # > 0: classifier fit (fit_classes)
    cperm: Optional[np.ndarray] = None     # [E, K] per-estimator class permutation
    ybar_e: Optional[np.ndarray] = None    # [E] test-row target value per estimator
    qtab: Optional[list] = None            # per column quantile table
    plam: Optional[list] = None            # per column Yeo-Johnson lambda
    svd: Optional[tuple] = None            # (scale, components) of the Q+SVD pipeline
    ylam: Optional[float] = None           # target Yeo-Johnson lambda (ensemble mode)
    trans: Optional[tuple] = None          # (idx, share, flag, cancel) target-border translation


class OracleTabPFN:
    """numpy restatement of the v2 regressor forward (see module docstring)."""

    def __init__(self, weights: Dict[str, np.ndarray], n_estimators: int = 8,
                 softmax_temperature: float = 0.9, seed: int = 0,
                 emulate_bf16: bool = False, n_heads: int = 6, features_per_group: int = 2,
                 preprocessing: int = 0, average_before_softmax: bool = False):
        self.w = {k: np.asarray(v, dtype=np.float32) for k, v in weights.items()}
        # tabpfn's average_before_softmax [ext]: mix the ensemble as softmax(mean_e log q_e)
        self.avg_before_softmax = bool(average_before_softmax)
        self.pre = int(preprocessing)   # preprocess_oracle MODE_*: 0 none, 1 quantile, 2 +power, 3 ensemble
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
        # multiplies every item-attention score (the engine's npfn_debug_item_attn_scale; stress tests)
        self.item_attn_scale = 1.0
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

    @staticmethod
    def _ystats(y: np.ndarray):
        """(mean, population std + 1e-20, mean of the standardized values), float32 like the engine."""
        y64 = np.asarray(y, dtype=np.float32).astype(np.float64)
        m = float(np.float32(y64.mean()))
        s = float(np.float32(y64.std() + 1e-20))
        z = ((np.asarray(y, dtype=np.float32) - np.float32(m)) / np.float32(s)).astype(np.float32)
        return m, s, float(np.float32(z.astype(np.float64).mean())), z

    # -------------------------------------------------------------------- fit
    def fit(self, X: np.ndarray, y: np.ndarray) -> FitState:
        """Regressor fit (npe_pfn.py:140, 215, 502): standardized target token."""
        X = np.asarray(X, dtype=np.float32)
        y = np.asarray(y, dtype=np.float32).reshape(-1)
        assert y.shape[0] == X.shape[0]
        y_mean, y_std, ybar_z, y_z = self._ystats(y)
        st = self._fit_features(X, y_mean, y_std, ybar_z)
        ty = np.stack([y_z] * self.E)
        if any(es.target_tf for es in st.estimators):
            st.ylam = yj_fit(y)
            yt = power_transform_vec(y, st.ylam)
            tm, ts, tz, yt_z = self._ystats(yt)
            bz = self.w["borders"].astype(np.float64)
            frm = yeo_johnson_inverse(bz * np.float32(ts) + np.float32(tm), st.ylam)
            frm, cancel = cancel_broken_borders(frm)
            idx, share, flag = translation_table(frm.astype(np.float32), self.borders_of(st))
            st.trans = (idx, share, flag, cancel)
            for e, es in enumerate(st.estimators):
                if es.target_tf:
                    es.ystats = (tm, ts, tz)
                    ty[e] = yt_z
        return self._fit_forward(X, st, ty)

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
        st = self._fit_features(X, 0.0, 1.0, 0.0, classifier=True)
        st.n_classes, st.cperm, st.ybar_e = K, cperm, ybar_e
        return self._fit_forward(X, st, ty)

    def _fit_features(self, X: np.ndarray, y_mean: float, y_std: float, ybar_z: float,
                      classifier: bool = False) -> FitState:
        n, F = X.shape
        fpg = self.fpg
        cfgs = estimator_configs(self.pre, self.E, classifier)
        types = {t for t, _ in cfgs}
        st = FitState(F, (F + fpg - 1) // fpg, y_mean, y_std, ybar_z, [], [])
        if types & {T_QUANT, T_QSVD}:
            # the classifier's ensemble uses tabpfn's "quantile_uni_coarse" (n // 10 quantiles)
            div = QUANTILE_DIV_COARSE if classifier and self.pre == MODE_ENSEMBLE else QUANTILE_DIV
            sub = quantile_subsample(n, self.seed)  # sklearn's subsample=10_000 (engine k_qt_subsample)
            st.qtab = [quantile_fit(X[:, j], n, div, sub) for j in range(F)]
        if types & {T_POWER, T_PFP}:
            st.plam = [yj_fit(X[:, j]) for j in range(F)]
        if T_QSVD in types:
            k = svd_components(n, F)
            if k:
                Z = np.concatenate([X, self._quant(X, st)], 1).astype(np.float64)
                st.svd = svd_fit(Z, k)
        for e, (ftype, ttf) in enumerate(cfgs):
            salt = fingerprint_salt(self.seed, e) if ftype in (T_QSVD, T_PFP, T_RFP) else 0
            es = EstimatorState(ftype, ttf, n_features_of(ftype, F, n), 0, None, None, None, None, salt,
                                (y_mean, y_std, ybar_z))
            es.n_groups = (es.n_feat + fpg - 1) // fpg
            es.perm = estimator_permutation(self.seed, e, es.n_feat)
            Xp = self._features(X, st, es, train=True)[:, es.perm].astype(np.float64)
            finite = np.isfinite(Xp)
            cnt = finite.sum(0)
            s1 = np.where(finite, Xp, 0.0).sum(0)
            mu = s1 / np.maximum(cnt, 1)
            dev = np.where(finite, Xp - mu, 0.0)
            sd = np.sqrt((dev**2).sum(0) / np.maximum(cnt - 1, 1))
            mx = np.where(finite, Xp, -np.inf).max(0)
            mn = np.where(finite, Xp, np.inf).min(0)
            used = (mx > mn).astype(np.int64)
            used_pad = np.zeros(es.n_groups * fpg, dtype=np.int64)
            used_pad[: es.n_feat] = used
            ug = used_pad.reshape(es.n_groups, fpg).sum(1)
            es.mu, es.sd = mu.astype(np.float32), sd.astype(np.float32)
            es.gscale = np.sqrt(fpg / np.maximum(ug, 1)).astype(np.float32)
            st.estimators.append(es)
        return st

    # ------------------------------------------------------ feature pipelines
    @staticmethod
    def _quant(X, st):
        return np.stack([quantile_transform_vec(X[:, j], st.qtab[j]) for j in range(X.shape[1])], 1)

    @staticmethod
    def _power(X, st):
        return np.stack([power_transform_vec(X[:, j], st.plam[j]) for j in range(X.shape[1])], 1)

    def _features(self, X: np.ndarray, st: FitState, es: EstimatorState, train: bool) -> np.ndarray:
        """The table [R, F_e] as estimator es sees it, before its shuffle (float32)."""
        X = np.asarray(X, dtype=np.float32)
        if es.ftype == T_RAW:
            return X
        if es.ftype == T_QUANT:
            return self._quant(X, st)
        if es.ftype == T_POWER:
            return self._power(X, st)
        fp = fingerprint(X, es.salt, train)[:, None]
        if es.ftype == T_PFP:
            return np.concatenate([self._power(X, st), fp], 1)
        if es.ftype == T_RFP:
            return np.concatenate([X, fp], 1)
        q = self._quant(X, st)
        parts = [X, q]
        if st.svd is not None:
            parts.append(svd_transform(np.concatenate([X, q], 1).astype(np.float64), *st.svd))
        return np.concatenate(parts + [fp], 1).astype(np.float32)

    @staticmethod
    def _groups(st: FitState):
        """Runs of consecutive estimators with the same token count, forwarded together."""
        out, a = [], 0
        ests = st.estimators
        for e in range(1, len(ests) + 1):
            if e == len(ests) or ests[e].n_groups != ests[a].n_groups:
                out.append((a, e))
                a = e
        return out

    def _fit_forward(self, X: np.ndarray, st: FitState, train_y: np.ndarray) -> FitState:
        self.state = st
        st.kv = []
        for a, b in self._groups(st):
            x = np.stack([self._encode_one(X, st, e, train_y=train_y[e], train=True) for e in range(a, b)])
            kv = []
            for l in range(self.L):
                x = self._layer(x, l, None, kv_out=kv)
            st.kv.append(kv)
        return st

    # ----------------------------------------------------------------- encode
    def _encode_one(self, Xrows: np.ndarray, st: FitState, e: int, train_y: Optional[np.ndarray],
                    train: bool) -> np.ndarray:
        """Token embeddings [R, C_e, d] of estimator e (C_e = groups + target token)."""
        es = st.estimators[e]
        R = Xrows.shape[0]
        G, fpg, d = es.n_groups, self.fpg, self.d
        C = G + 1
        W = self.w["enc_w"]          # [d, 4]
        Wy = self.w["y_enc_w"]       # [d, 2]
        pe = self.w["pos_emb"]       # [Gmax, d]
        out = np.zeros((R, C, d), dtype=np.float32)
        xp = self._features(Xrows, st, es, train)[:, es.perm]
        isnan = np.isnan(xp)
        ispinf = np.isposinf(xp)
        isninf = np.isneginf(xp)
        ind = (isnan * NAN_INDICATOR + ispinf * INF_INDICATOR + isninf * NEG_INF_INDICATOR).astype(np.float32)
        v = np.where(isnan | ispinf | isninf, es.mu[None, :], xp).astype(np.float32)
        xn = np.clip((v - es.mu) / (es.sd + np.float32(1e-16)), -100.0, 100.0).astype(np.float32)
        xpad = np.zeros((R, G * fpg), dtype=np.float32)
        ipad = np.zeros((R, G * fpg), dtype=np.float32)
        xpad[:, : es.n_feat] = xn
        ipad[:, : es.n_feat] = ind
        xpad = xpad.reshape(R, G, fpg) * es.gscale[None, :, None]
        ipad = ipad.reshape(R, G, fpg)
        feats = np.concatenate([xpad, ipad], axis=-1)  # [R, G, 4] = [x_a, x_b, ind_a, ind_b]
        out[:, :G, :] = (feats @ W.T) + pe[None, :G, :]
        if train_y is not None:
            yin = np.stack([train_y, np.zeros_like(train_y)], -1)
        else:
            yb = st.ybar_e[e] if st.ybar_e is not None else es.ystats[2]
            yin = np.tile(np.array([[yb, NAN_INDICATOR]], dtype=np.float32), (R, 1))
        out[:, G, :] = yin @ Wy.T
        return out

    # ------------------------------------------------------------------ layer
    def _layer(self, x: np.ndarray, l: int, kv_in: Optional[list], kv_out: Optional[list] = None) -> np.ndarray:
        """One post-norm layer on a group of estimators' tokens x [E, R, C, d].  Train side
        (kv_out is a list): the item attention runs over x itself and its K/V [E, n, C, 2, d]
        is appended to kv_out; test side: over the cached kv_in[l]."""
        E, R, C, d = x.shape
        H, hd = self.H, self.hd
        p = f"l{l}."
        train = kv_out is not None
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
            kv_out.append(kv)
        else:
            wq = self.w[p + "item_qkv"][:d]
            q = self._bf((self._bf(x) @ wq.T).astype(np.float32))
            kv = kv_in[l]
        o = np.zeros((E, R, C, d), dtype=np.float32)
        scale = np.float32(self.item_attn_scale / math.sqrt(hd))
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
    def _estimator_logits(self, Xq: np.ndarray) -> np.ndarray:
        """Decoder logits [E, R, n_out] of every estimator for the query rows."""
        st = self.state
        assert st is not None, "fit() first"
        Xq = np.asarray(Xq, dtype=np.float32)
        assert Xq.shape[1] == st.n_features
        out = []
        for g, (a, b) in enumerate(self._groups(st)):
            x = np.stack([self._encode_one(Xq, st, e, train_y=None, train=False) for e in range(a, b)])
            for l in range(self.L):
                x = self._layer(x, l, st.kv[g])
            z = x[:, :, st.estimators[a].n_groups, :]              # target token [Eg, R, d]
            h = self._bf(self._gelu(self._mm(z, "dec_w1") + self.w["dec_b1"]))
            lg = (self._mm(h, "dec_w2") + self.w["dec_b2"]).astype(np.float32)
            if self.emulate:  # the engine stores the decoder logits as fp16 (npfn_kernels.h logit_t)
                lg = lg.astype(np.float16).astype(np.float32)
            out.append(lg)
        return np.concatenate(out, 0)

    def predict_probs(self, Xq: np.ndarray, return_estimator_logits: bool = False):
        """Ensemble-mean bar probabilities [R, n_bars] over the common borders: per estimator
        softmax(logits / T); a target-transformed estimator's bars cancelled where its
        translated borders broke, its probabilities translated to the common borders."""
        st = self.state
        logits = self._estimator_logits(Xq)   # [E, R, nb]
        probs = np.zeros((logits.shape[1], logits.shape[2]), dtype=np.float64)
        invT = np.float32(1.0 / self.T)
        for e, es in enumerate(st.estimators):
            lg = logits[e] * invT
            if es.target_tf:
                idx, share, flag, cancel = st.trans
                lg = np.where(cancel[None, :], np.float32(-np.inf), lg)
                pe = translate_probs(softmax(lg, -1), idx, share, flag)
            else:
                pe = softmax(lg, -1)
            if self.avg_before_softmax:  # log of the float32 probabilities (0 -> -inf), as tabpfn's .log()
                with np.errstate(divide="ignore"):
                    probs += np.log(np.maximum(pe.astype(np.float64), 0.0))
            else:
                probs += pe.astype(np.float64)
        probs = probs / self.E
        if self.avg_before_softmax:
            probs = np.exp(probs - probs.max(1, keepdims=True))
            probs = probs / probs.sum(1, keepdims=True)
        probs = probs.astype(np.float32)
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
        logits = self._estimator_logits(Xq)   # [E, R, n_out]
        invT = np.float32(1.0 / self.T)
        acc = np.zeros((logits.shape[1], st.n_classes), dtype=np.float64)
        for e in range(self.E):
            lg = (logits[e][:, st.cperm[e]] * invT).astype(np.float64)
            if self.avg_before_softmax:  # tabpfn [ext]: the estimators' logits averaged, then softmax
                acc += lg
            else:
                acc += softmax(lg.astype(np.float32), -1).astype(np.float64)
        if self.avg_before_softmax:
            z = acc / self.E
            z = np.exp(z - z.max(1, keepdims=True))
            return (z / z.sum(1, keepdims=True)).astype(np.float32)
        return (acc / self.E).astype(np.float32)

    def borders_of(self, st: FitState) -> np.ndarray:
        return (self.w["borders"] * np.float32(st.y_std) + np.float32(st.y_mean)).astype(np.float32)

    def borders(self) -> np.ndarray:
        return self.borders_of(self.state)


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
                 random_state: int = 0, weights=None, emulate_bf16: bool = False,
                 preprocessing=MODE_ENSEMBLE, average_before_softmax: bool = False, **_ignored):
        w = weights if weights is not None else OracleRegressor.default_weights
        if w is None:
            raise RuntimeError("OracleRegressor needs weights (set OracleRegressor.default_weights)")
        modes = {"none": 0, "quantile": 1, "quantile+power": 2, "ensemble": MODE_ENSEMBLE}
        pre = modes[preprocessing] if isinstance(preprocessing, str) else int(preprocessing)
        self.model = OracleTabPFN(w, n_estimators, softmax_temperature, random_state, emulate_bf16,
                                  preprocessing=pre, average_before_softmax=average_before_softmax)
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
                 random_state: int = 0, weights=None, emulate_bf16: bool = False, preprocessing=0,
                 average_before_softmax: bool = False, **_ignored):
        """``preprocessing`` defaults to 0 ("none"): the mode the reference-generated golden
        fixtures (tests/golden/ratio.npz) were made with; MODE_ENSEMBLE / "ensemble" is the
        classifier's ensemble (TabPFNClassifier's default)."""
        w = weights if weights is not None else OracleClassifier.default_weights
        if w is None:
            raise RuntimeError("OracleClassifier needs weights (set OracleClassifier.default_weights)")
        modes = {"none": 0, "quantile": 1, "quantile+power": 2, "ensemble": MODE_ENSEMBLE}
        pre = modes[preprocessing] if isinstance(preprocessing, str) else int(preprocessing)
        self.model = OracleTabPFN(w, n_estimators, softmax_temperature, random_state, emulate_bf16,
                                  preprocessing=pre, average_before_softmax=average_before_softmax)
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
