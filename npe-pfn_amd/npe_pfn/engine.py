"""ctypes binding of the C-ABI engine (include/npfn.h, libnpfn.so).

The library is built in-tree for gfx950 (``make -C npe-pfn_amd`` or
``__graft_entry__.build()``).  There is no CPU fallback: constructing an
:class:`Engine` without the library or without a ROCm device raises.

torch is imported first so that libnpfn.so binds to the HIP runtime torch
already loaded (same SONAME), which makes torch's device pointers and streams
valid inside the engine.
"""

from __future__ import annotations

import ctypes
import os
from typing import Dict, Optional, Tuple

import numpy as np
import torch

from .limits import check_engine_table
from .weights import ModelConfig, pack_weights, synthetic_weights

LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_lib", "libnpfn.so")

# packed weight blobs of the last few weight sets (pack_weights costs ~30 ms per engine, paid
# again by every engine of a run_tsnpe_pfn round); keyed by the weight dict's identity, which
# the entry keeps alive, so a key is never reused by another dict
_PACK_CACHE: "Dict[Tuple[int, ModelConfig], Tuple[Dict[str, np.ndarray], np.ndarray]]" = {}
_PACK_CACHE_MAX = 3  # the regressor and classifier weight sets of a run_tsnpe_pfn round, and one more


def _packed(weights: Dict[str, np.ndarray], cfg: ModelConfig) -> np.ndarray:
    key = (id(weights), cfg)
    hit = _PACK_CACHE.get(key)
    if hit is not None and hit[0] is weights:
        return hit[1]
    blob = pack_weights(weights, cfg)
    if len(_PACK_CACHE) >= _PACK_CACHE_MAX:
        _PACK_CACHE.pop(next(iter(_PACK_CACHE)))
    _PACK_CACHE[key] = (weights, blob)
    return blob

# (name, restype, argtypes) of every entry point in include/npfn.h
_vp, _i64, _i32, _u64, _f = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32, ctypes.c_uint64, ctypes.c_float


class NpfnConfig(ctypes.Structure):
    _fields_ = [
        ("d_model", ctypes.c_int32),
        ("n_heads", ctypes.c_int32),
        ("n_layers", ctypes.c_int32),
        ("d_ff", ctypes.c_int32),
        ("n_bars", ctypes.c_int32),
        ("features_per_group", ctypes.c_int32),
        ("max_groups", ctypes.c_int32),
        ("n_estimators", ctypes.c_int32),
        ("softmax_temperature", ctypes.c_float),
        ("device", ctypes.c_int32),
        ("random_state", ctypes.c_uint64),
    ]


class NpfnProfEntry(ctypes.Structure):
    _fields_ = [
        ("name", ctypes.c_char * 48),
        ("launches", ctypes.c_int64),
        ("ms", ctypes.c_double),
        ("flops", ctypes.c_double),
        ("bytes", ctypes.c_double),
    ]


SIGNATURES = {
    "npfn_version": (ctypes.c_int, []),
    "npfn_last_error": (ctypes.c_char_p, []),
    "npfn_weights_size": (ctypes.c_size_t, [ctypes.POINTER(NpfnConfig)]),
    "npfn_engine_create": (ctypes.c_int, [ctypes.POINTER(NpfnConfig), _vp, ctypes.c_size_t, ctypes.POINTER(_vp)]),
    "npfn_engine_destroy": (ctypes.c_int, [_vp]),
    "npfn_fit": (ctypes.c_int, [_vp, _vp, _i64, _vp, _i64, _i64, _i32, _vp]),
    "npfn_predict": (ctypes.c_int, [_vp, _vp, _i64, _i64, _vp, _vp]),
    "npfn_set_preprocessing": (ctypes.c_int, [_vp, _i32]),
    "npfn_set_average_before_softmax": (ctypes.c_int, [_vp, _i32]),
    "npfn_fit_classes": (ctypes.c_int, [_vp, _vp, _i64, _vp, _i64, _i64, _i32, _i32, _vp]),
    "npfn_predict_proba": (ctypes.c_int, [_vp, _vp, _i64, _i64, _vp, _vp]),
    "npfn_get_borders": (ctypes.c_int, [_vp, _vp, _vp]),
    "npfn_bar_sample": (ctypes.c_int, [_vp, _vp, _i64, _i32, _u64, _u64, _vp, _vp]),
    "npfn_bar_nll": (ctypes.c_int, [_vp, _vp, _vp, _i64, _i32, _vp, _vp]),
    "npfn_ar_sample": (ctypes.c_int, [_vp, _vp, _vp, _i64, _i32, _i32, _vp, _i64, _u64, _i64, _vp, _vp, _f, _vp]),
    "npfn_ar_sample_repeated": (ctypes.c_int, [_vp, _vp, _vp, _i64, _i32, _i32, _vp, _i64, _i64, _u64, _i64, _vp, _vp,
                                               _f, _vp]),
    "npfn_ar_log_prob": (ctypes.c_int, [_vp, _vp, _vp, _i64, _i32, _i32, _vp, _vp, _i64, _vp, _f, _vp]),
    "npfn_ar_log_prob_repeated": (ctypes.c_int, [_vp, _vp, _vp, _i64, _i32, _i32, _vp, _i64, _vp, _i64, _vp, _f, _vp]),
    "npfn_box_support": (ctypes.c_int, [_vp, _i64, _i32, _vp, _vp, _vp, _vp]),
    "npfn_compact_rows": (ctypes.c_int, [_vp, _vp, _i64, _i32, _vp, _vp, _vp]),
    "npfn_filter_stdeuclid": (ctypes.c_int, [_vp, _i64, _i32, _vp, _i64, _vp, _vp]),
    "npfn_sir_select": (ctypes.c_int, [_vp, _vp, _vp, _i64, _i32, _u64, _u64, _i64, _vp, _i32, _vp, _vp, _vp, _vp]),
    "npfn_set_estimator_range": (ctypes.c_int, [_vp, _i32, _i32]),
    "npfn_set_estimator_set": (ctypes.c_int, [_vp, _i32, _i32, _i32]),
    "npfn_forward_targets": (ctypes.c_int, [_vp, _vp, _i64, _i64, _vp, _vp]),
    "npfn_head_sample": (ctypes.c_int, [_vp, _vp, _i32, _i64, _u64, _i64, _vp, _vp, _f, _vp]),
    "npfn_ar_fit_begin": (ctypes.c_int, [_vp, _vp, _vp, _i64, _i32, _i32, _vp]),
    "npfn_ar_fit_step": (ctypes.c_int, [_vp, _i32, _vp]),
    "npfn_set_fit_token": (ctypes.c_int, [_vp, _u64]),
    "npfn_set_chunk_rows": (ctypes.c_int, [_vp, _i64]),
    "npfn_prof_enable": (ctypes.c_int, [_vp, ctypes.c_int]),
    "npfn_prof_read": (ctypes.c_int, [_vp, ctypes.POINTER(NpfnProfEntry), _i32, ctypes.POINTER(_i32)]),
    "npfn_debug_views": (ctypes.c_int, [_vp, _vp, _i64, _i32, ctypes.POINTER(_i32)]),
    "npfn_debug_item_attn_online": (ctypes.c_int, [ctypes.c_int]),
    "npfn_debug_item_attn_scale": (ctypes.c_int, [_f]),
    "npfn_debug_fail_row_launch": (ctypes.c_int, [_vp, _i32]),
    "npfn_item_attn_fallback": (ctypes.c_int, [_vp, ctypes.POINTER(_u64), ctypes.c_int]),
    "npfn_item_attn_fallback_causes": (ctypes.c_int, [_vp, ctypes.POINTER(_u64)]),
}

_LIB = None
# A/B switch (tools/ab_bench.py): NPFN_NO_REPEATED=1 runs repeated query rows through the
# plain npfn_ar_sample / npfn_ar_log_prob (step 0 over every row)
_NO_REPEATED = os.environ.get("NPFN_NO_REPEATED") == "1"


class EngineError(RuntimeError):
    pass


def load_library(path: Optional[str] = None) -> ctypes.CDLL:
    """Load libnpfn.so and declare every entry point (raises if missing).

    NPFN_LIB overrides the path (diagnostic builds, e.g. a ``-DNPFN_DIAG_*`` timing build, or an older build in an
    A/B run, which may lack entry points added since: those are left unbound)."""
    global _LIB
    override = path is None and bool(os.environ.get("NPFN_LIB"))
    path = path or os.environ.get("NPFN_LIB") or LIB_PATH
    if _LIB is not None and _LIB._name == path:
        return _LIB
    if not os.path.exists(path):
        raise ImportError(
            f"NPE-PFN engine library not found at {path}; build it with `make -C npe-pfn_amd` "
            "(or __graft_entry__.build()). There is no CPU fallback."
        )
    lib = ctypes.CDLL(path)
    for name, (res, args) in SIGNATURES.items():
        if override and not hasattr(lib, name):
            continue
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _LIB = lib
    return lib


def _ptr(t: Optional[torch.Tensor]):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def _check(lib, rc: int, what: str):
    if rc != 0:
        msg = lib.npfn_last_error()
        raise EngineError(f"{what} failed ({rc}): {msg.decode() if msg else ''}")


def _dev_f32(t, device) -> torch.Tensor:
    t = torch.as_tensor(t)
    return t.to(device=device, dtype=torch.float32).contiguous()


class Engine:
    """One engine handle on one device: weights resident in HBM, fit state, workspaces."""

    def __init__(self, cfg: ModelConfig = ModelConfig(), weights: Optional[Dict[str, np.ndarray]] = None,
                 device: Optional[torch.device] = None, random_state: int = 0, preprocessing: str = "ensemble"):
        """``preprocessing``: the engine's per-estimator preprocessing (:meth:`set_preprocessing`);
        the default "ensemble" is tabpfn's default and the C engine's initial mode, as for
        ``TabPFNRegressor`` (npe_pfn/tabpfn.py)."""
        if not torch.cuda.is_available():
            raise EngineError("the NPE-PFN engine needs a ROCm GPU (torch.cuda.is_available() is False)")
        self.lib = load_library()
        self.cfg = cfg
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        if self.device.type != "cuda":
            raise EngineError(f"engine device must be a GPU, got {self.device}")
        if weights is None:
            weights = synthetic_weights(cfg, seed=0)
        blob = _packed(weights, cfg)
        self.c_cfg = NpfnConfig(cfg.d_model, cfg.n_heads, cfg.n_layers, cfg.d_ff, cfg.n_bars,
                                cfg.features_per_group, cfg.max_groups, cfg.n_estimators,
                                float(cfg.softmax_temperature), self.device.index or 0,
                                int(random_state) & 0xFFFFFFFFFFFFFFFF)
        want = self.lib.npfn_weights_size(ctypes.byref(self.c_cfg))
        if want != blob.size:
            raise EngineError(f"weight blob has {blob.size} floats, engine expects {want}")
        h = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            _check(self.lib, self.lib.npfn_engine_create(ctypes.byref(self.c_cfg), blob.ctypes.data_as(ctypes.c_void_p),
                                                         blob.size, ctypes.byref(h)), "npfn_engine_create")
        self.h = h
        self.random_state = int(random_state)
        self.n_features: Optional[int] = None
        self.n_classes = 0
        self.preprocessing = self.DEFAULT_PREPROCESSING  # npfn_engine_create starts in mode 3
        self.e0, self.ne = 0, cfg.n_estimators
        self.ep_set = None  # (rank, count, stride) of npe_pfn.distributed's estimator-parallel split
        if preprocessing != self.preprocessing:
            self.set_preprocessing(preprocessing)

    def full_range(self) -> None:
        """Back to all estimators after an estimator-parallel split (the single-engine entry
        points need the whole ensemble)."""
        if self.e0 != 0 or self.ne != self.cfg.n_estimators:
            self.set_estimator_range(0, self.cfg.n_estimators)

    PREPROCESSING_MODES = {"none": 0, "quantile": 1, "quantile+power": 2, "ensemble": 3}
    DEFAULT_PREPROCESSING = "ensemble"

    def set_preprocessing(self, mode: str) -> None:
        """Per-estimator preprocessing from the next fit on (include/npfn.h
        ``npfn_set_preprocessing``): "none"; "quantile" = sklearn QuantileTransformer
        (uniform, n_quantiles=max(n//5, 2)) on even estimators [ext: tabpfn "quantile_uni"];
        "quantile+power" = that plus the Yeo-Johnson power transform on odd estimators
        [ext: tabpfn "safepower"]; "ensemble" = tabpfn's default regressor ensemble
        (quantile + original + SVD | Yeo-Johnson features, fingerprint feature, Yeo-Johnson
        target transform on half the estimators; oracle/preprocess_oracle.py MODE_ENSEMBLE)."""
        if mode not in self.PREPROCESSING_MODES:
            raise ValueError(f"preprocessing must be one of {sorted(self.PREPROCESSING_MODES)}, got {mode!r}")
        _check(self.lib, self.lib.npfn_set_preprocessing(self.h, self.PREPROCESSING_MODES[mode]),
               "npfn_set_preprocessing")
        self.preprocessing = mode
        self.n_features = None

    def set_average_before_softmax(self, enable: bool) -> None:
        """tabpfn's ``average_before_softmax`` (npfn_set_average_before_softmax): the ensemble is
        mixed as softmax(mean of the estimators' log probabilities) instead of the mean of their
        probabilities, from the next predict / AR call on."""
        _check(self.lib, self.lib.npfn_set_average_before_softmax(self.h, 1 if enable else 0),
               "npfn_set_average_before_softmax")
        self.average_before_softmax = bool(enable)

    def check_table(self, n_rows: int, n_features: int, classifier: bool = False) -> None:
        """ValueError naming the limit when a fit on [n_rows, n_features] exceeds the engine's
        capacity under its preprocessing (npe_pfn.limits; raised before any C call)."""
        check_engine_table(int(n_rows), int(n_features), self.PREPROCESSING_MODES[self.preprocessing], classifier,
                           self.cfg.max_groups)

    def __del__(self):
        h = getattr(self, "h", None)
        if h is not None and h.value:
            try:
                self.lib.npfn_engine_destroy(h)
            except Exception:
                pass
            self.h = None

    @property
    def stream(self):
        return ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    # ------------------------------------------------------------ TabPFN surface
    def fit(self, X, y) -> None:
        """npfn_fit of this engine's estimator set (a partial set is a building block of the
        estimator-parallel split: fit + forward_targets; the mixing calls need the full set)."""
        X = _dev_f32(X, self.device)
        y = _dev_f32(y, self.device).reshape(-1)
        if X.ndim != 2 or X.shape[0] != y.shape[0]:
            raise ValueError(f"fit: X {tuple(X.shape)} and y {tuple(y.shape)} do not match")
        self.check_table(X.shape[0], X.shape[1])
        _check(self.lib, self.lib.npfn_fit(self.h, _ptr(X), X.shape[1], _ptr(y), 1, X.shape[0], X.shape[1],
                                           self.stream), "npfn_fit")
        self.n_features = X.shape[1]
        self._keep = (X, y)  # inputs stay alive until the stream consumed them

    def predict_logits(self, Xq) -> torch.Tensor:
        if self.n_features is None:
            raise EngineError("predict before fit")
        Xq = _dev_f32(Xq, self.device)
        if Xq.ndim != 2 or Xq.shape[1] != self.n_features:
            raise ValueError(f"predict: X has shape {tuple(Xq.shape)}, fit had {self.n_features} features")
        out = torch.empty((Xq.shape[0], self.cfg.n_bars), dtype=torch.float32, device=self.device)
        _check(self.lib, self.lib.npfn_predict(self.h, _ptr(Xq), Xq.shape[1], Xq.shape[0], _ptr(out), self.stream),
               "npfn_predict")
        return out

    # -------------------------------------------------------- classifier surface
    def fit_classes(self, X, y_idx, n_classes: int) -> None:
        """Classifier fit on label indices 0..n_classes-1 (npfn_fit_classes)."""
        self.full_range()
        X = _dev_f32(X, self.device)
        y = _dev_f32(y_idx, self.device).reshape(-1)
        if X.ndim != 2 or X.shape[0] != y.shape[0]:
            raise ValueError(f"fit: X {tuple(X.shape)} and y {tuple(y.shape)} do not match")
        self.check_table(X.shape[0], X.shape[1], classifier=True)
        _check(self.lib, self.lib.npfn_fit_classes(self.h, _ptr(X), X.shape[1], _ptr(y), 1, X.shape[0], X.shape[1],
                                                   int(n_classes), self.stream), "npfn_fit_classes")
        self.n_features = X.shape[1]
        self.n_classes = int(n_classes)
        self._keep = (X, y)

    def predict_proba(self, Xq) -> torch.Tensor:
        """[N, n_classes] estimator-mean class probabilities on the device (npfn_predict_proba)."""
        if self.n_features is None or not getattr(self, "n_classes", 0):
            raise EngineError("predict_proba before fit_classes")
        Xq = _dev_f32(Xq, self.device)
        if Xq.ndim != 2 or Xq.shape[1] != self.n_features:
            raise ValueError(f"predict_proba: X has shape {tuple(Xq.shape)}, fit had {self.n_features} features")
        out = torch.empty((Xq.shape[0], self.n_classes), dtype=torch.float32, device=self.device)
        _check(self.lib, self.lib.npfn_predict_proba(self.h, _ptr(Xq), Xq.shape[1], Xq.shape[0], _ptr(out),
                                                     self.stream), "npfn_predict_proba")
        return out

    def borders(self) -> torch.Tensor:
        out = torch.empty(self.cfg.n_bars + 1, dtype=torch.float32, device=self.device)
        _check(self.lib, self.lib.npfn_get_borders(self.h, _ptr(out), self.stream), "npfn_get_borders")
        return out

    def bar_sample(self, logits: torch.Tensor, borders: torch.Tensor, counter: int) -> torch.Tensor:
        logits = _dev_f32(logits, self.device)
        borders = _dev_f32(borders, self.device)
        out = torch.empty(logits.shape[0], dtype=torch.float32, device=self.device)
        _check(self.lib, self.lib.npfn_bar_sample(_ptr(logits), _ptr(borders), logits.shape[0], logits.shape[1],
                                                  self.random_state, int(counter), _ptr(out), self.stream),
               "npfn_bar_sample")
        return out

    def bar_nll(self, logits: torch.Tensor, borders: torch.Tensor, y) -> torch.Tensor:
        logits = _dev_f32(logits, self.device)
        borders = _dev_f32(borders, self.device)
        y = _dev_f32(y, self.device).reshape(-1)
        out = torch.empty(logits.shape[0], dtype=torch.float32, device=self.device)
        _check(self.lib, self.lib.npfn_bar_nll(_ptr(logits), _ptr(borders), _ptr(y), logits.shape[0],
                                               logits.shape[1], _ptr(out), self.stream), "npfn_bar_nll")
        return out

    # -------------------------------------------------------------- fused paths
    def ar_sample(self, x_ctx, theta_ctx, x_query, counter: int, with_log_prob: bool = False,
                  eps: float = 1e-15, row_base: int = 0,
                  x_unique: Optional[torch.Tensor] = None) -> Tuple[torch.Tensor, Optional[torch.Tensor]]:
        """``x_unique``: the distinct rows of ``x_query`` when ``x_query`` is
        ``x_unique.repeat_interleave(N // U, 0)`` (one observation repeated, or sample_batched's
        obs-major batch): npfn_ar_sample_repeated runs AR step 0 once per distinct row."""
        self.full_range()
        x_ctx = _dev_f32(x_ctx, self.device)
        theta_ctx = _dev_f32(theta_ctx, self.device)
        n, dx = x_ctx.shape
        dth = theta_ctx.shape[1]
        N = x_query.shape[0]
        if theta_ctx.shape[0] != n or x_query.shape[1] != dx:
            raise ValueError("ar_sample: inconsistent shapes")
        self.check_table(n, dx + dth - 1)
        theta = torch.empty((N, dth), dtype=torch.float32, device=self.device)
        lp = torch.empty(N, dtype=torch.float32, device=self.device) if with_log_prob else None
        if x_unique is not None and not _NO_REPEATED:
            x_unique = _dev_f32(x_unique, self.device)
            U = x_unique.shape[0]
            if x_unique.ndim != 2 or x_unique.shape[1] != dx or U < 1 or N % U:
                raise ValueError(f"ar_sample: x_unique {tuple(x_unique.shape)} does not repeat into {N} rows of {dx}")
            _check(self.lib, self.lib.npfn_ar_sample_repeated(
                self.h, _ptr(x_ctx), _ptr(theta_ctx), n, dx, dth, _ptr(x_unique), U, N, int(counter), int(row_base),
                _ptr(theta), _ptr(lp), float(eps), self.stream), "npfn_ar_sample_repeated")
        else:
            x_query = _dev_f32(x_query, self.device)
            _check(self.lib, self.lib.npfn_ar_sample(self.h, _ptr(x_ctx), _ptr(theta_ctx), n, dx, dth, _ptr(x_query),
                                                     N, int(counter), int(row_base), _ptr(theta), _ptr(lp),
                                                     float(eps), self.stream),
                   "npfn_ar_sample")
        self.n_features = dx + dth - 1
        return theta, lp

    def ar_log_prob(self, x_ctx, theta_ctx, x_query, theta, eps: float = 1e-15,
                    x_unique: Optional[torch.Tensor] = None) -> torch.Tensor:
        """``x_unique``: the distinct rows ``x_query`` repeats (as in :meth:`ar_sample`)."""
        self.full_range()
        x_ctx = _dev_f32(x_ctx, self.device)
        theta_ctx = _dev_f32(theta_ctx, self.device)
        theta = _dev_f32(theta, self.device)
        n, dx = x_ctx.shape
        dth = theta_ctx.shape[1]
        N = x_query.shape[0]
        if theta.shape != (N, dth):
            raise ValueError("ar_log_prob: theta shape mismatch")
        self.check_table(n, dx + dth - 1)
        out = torch.empty(N, dtype=torch.float32, device=self.device)
        if x_unique is not None and not _NO_REPEATED:
            x_unique = _dev_f32(x_unique, self.device)
            U = x_unique.shape[0]
            if x_unique.ndim != 2 or x_unique.shape[1] != dx or U < 1 or N % U:
                raise ValueError(f"ar_log_prob: x_unique {tuple(x_unique.shape)} does not repeat into {N} rows")
            _check(self.lib, self.lib.npfn_ar_log_prob_repeated(
                self.h, _ptr(x_ctx), _ptr(theta_ctx), n, dx, dth, _ptr(x_unique), U, _ptr(theta), N, _ptr(out),
                float(eps), self.stream), "npfn_ar_log_prob_repeated")
        else:
            x_query = _dev_f32(x_query, self.device)
            _check(self.lib, self.lib.npfn_ar_log_prob(self.h, _ptr(x_ctx), _ptr(theta_ctx), n, dx, dth,
                                                       _ptr(x_query), _ptr(theta), N, _ptr(out), float(eps),
                                                       self.stream),
                   "npfn_ar_log_prob")
        self.n_features = dx + dth - 1
        return out

    # ------------------------------------------------------- support kernels
    def box_support(self, theta: torch.Tensor, low: torch.Tensor, high: torch.Tensor) -> torch.Tensor:
        """K9 mask of a box prior; scalar or broadcastable bounds are expanded to theta's
        width first (the kernel reads low[j] / high[j] for every column j)."""
        theta = _dev_f32(theta, self.device)
        if theta.ndim != 2:
            raise ValueError(f"box_support: theta must be [N, dim], got {tuple(theta.shape)}")
        dim = theta.shape[1]
        low = torch.broadcast_to(_dev_f32(low, self.device).reshape(-1), (dim,)).contiguous()
        high = torch.broadcast_to(_dev_f32(high, self.device).reshape(-1), (dim,)).contiguous()
        mask = torch.empty(theta.shape[0], dtype=torch.uint8, device=self.device)
        _check(self.lib, self.lib.npfn_box_support(_ptr(theta), theta.shape[0], theta.shape[1], _ptr(low), _ptr(high),
                                                   _ptr(mask), self.stream), "npfn_box_support")
        return mask.bool()

    def compact_rows(self, src: torch.Tensor, mask: torch.Tensor) -> torch.Tensor:
        src = _dev_f32(src, self.device)
        m = mask.to(device=self.device, dtype=torch.uint8).contiguous()
        dst = torch.empty_like(src)
        cnt = torch.zeros(1, dtype=torch.int64, device=self.device)
        _check(self.lib, self.lib.npfn_compact_rows(_ptr(src), _ptr(m), src.shape[0], src.shape[1], _ptr(dst),
                                                    _ptr(cnt), self.stream), "npfn_compact_rows")
        return dst[: int(cnt.item())]

    def filter_stdeuclid(self, x: torch.Tensor, obs: torch.Tensor, k: int) -> torch.Tensor:
        x = _dev_f32(x, self.device)
        obs = _dev_f32(obs, self.device).reshape(-1)
        idx = torch.empty(int(k), dtype=torch.int64, device=self.device)
        _check(self.lib, self.lib.npfn_filter_stdeuclid(_ptr(x), x.shape[0], x.shape[1], _ptr(obs), int(k), _ptr(idx),
                                                        self.stream), "npfn_filter_stdeuclid")
        return idx

    # ------------------------------------------------- estimator-parallel split
    def set_estimator_range(self, e0: int, count: int) -> None:
        """Fits / forwards compute estimators [e0, e0 + count) only (npfn_set_estimator_range)."""
        _check(self.lib, self.lib.npfn_set_estimator_range(self.h, int(e0), int(count)), "npfn_set_estimator_range")
        self.e0, self.ne = int(e0), int(count)
        self.n_features = None
        self.ep_set = None  # npe_pfn.distributed's cached strided set is gone

    def set_estimator_set(self, e0: int, count: int, stride: int) -> None:
        """Fits / forwards compute estimators e0 + stride * i, i < count (npfn_set_estimator_set);
        forward_targets returns their tokens in that order."""
        _check(self.lib, self.lib.npfn_set_estimator_set(self.h, int(e0), int(count), int(stride)),
               "npfn_set_estimator_set")
        self.e0, self.ne = int(e0), int(count)
        self.n_features = None
        self.ep_set = None

    def forward_targets(self, Xq) -> torch.Tensor:
        """[count, N, 192] bf16 decoder-input tokens of this engine's estimators (npfn_forward_targets)."""
        if self.n_features is None:
            raise EngineError("forward_targets before fit")
        Xq = _dev_f32(Xq, self.device)
        if Xq.ndim != 2 or Xq.shape[1] != self.n_features:
            raise ValueError(f"forward_targets: X has shape {tuple(Xq.shape)}, fit had {self.n_features} features")
        out = torch.empty((getattr(self, "ne", self.cfg.n_estimators), Xq.shape[0], self.cfg.d_model),
                          dtype=torch.bfloat16, device=self.device)
        _check(self.lib, self.lib.npfn_forward_targets(self.h, _ptr(Xq), Xq.shape[1], Xq.shape[0], _ptr(out),
                                                       self.stream), "npfn_forward_targets")
        return out

    def head_sample(self, tokens: torch.Tensor, counter: int, row_base: int = 0,
                    log_prob_acc: Optional[torch.Tensor] = None, eps: float = 1e-15) -> torch.Tensor:
        """Decoder + ensemble mix + bar sample of one AR step from [E, N, 192] bf16 tokens of all
        estimators (npfn_head_sample); adds the step's log density into ``log_prob_acc``."""
        if tokens.dtype != torch.bfloat16 or tokens.ndim != 3 or tokens.shape[2] != self.cfg.d_model:
            raise ValueError(f"head_sample: tokens must be bf16 [E, N, {self.cfg.d_model}], got "
                             f"{tokens.dtype} {tuple(tokens.shape)}")
        tokens = tokens.to(self.device).contiguous()
        n = tokens.shape[1]
        out = torch.empty(n, dtype=torch.float32, device=self.device)
        if log_prob_acc is not None and (log_prob_acc.shape != (n,) or log_prob_acc.dtype != torch.float32
                                         or not log_prob_acc.is_contiguous() or log_prob_acc.device != self.device):
            raise ValueError("head_sample: log_prob_acc must be a contiguous float32 [N] tensor on the engine device")
        _check(self.lib, self.lib.npfn_head_sample(self.h, _ptr(tokens), tokens.shape[0], n, int(counter),
                                                   int(row_base), _ptr(out), _ptr(log_prob_acc), float(eps),
                                                   self.stream), "npfn_head_sample")
        return out

    def ar_fit_begin(self, x_ctx, theta_ctx) -> None:
        """npfn_ar_fit_begin: the per-step fits of an AR call on (x_ctx, theta_ctx), driven by
        :meth:`ar_fit_step` (under a fit token every step's preprocessing fit is queued at once)."""
        x_ctx = _dev_f32(x_ctx, self.device).contiguous()
        theta_ctx = _dev_f32(theta_ctx, self.device).contiguous()
        if x_ctx.ndim != 2 or theta_ctx.ndim != 2 or x_ctx.shape[0] != theta_ctx.shape[0]:
            raise ValueError(f"ar_fit_begin: x_ctx {tuple(x_ctx.shape)} and theta_ctx {tuple(theta_ctx.shape)} "
                             "do not match")
        self.check_table(x_ctx.shape[0], x_ctx.shape[1] + theta_ctx.shape[1] - 1)
        _check(self.lib, self.lib.npfn_ar_fit_begin(self.h, _ptr(x_ctx), _ptr(theta_ctx), x_ctx.shape[0],
                                                    x_ctx.shape[1], theta_ctx.shape[1], self.stream),
               "npfn_ar_fit_begin")
        self._ar_dims = (x_ctx.shape[1], theta_ctx.shape[1])
        self._keep = (x_ctx, theta_ctx)

    def ar_fit_step(self, k: int) -> None:
        """npfn_ar_fit_step: step k's fit (on x_ctx | theta_ctx[:, :k] -> theta_ctx[:, k]) becomes
        the current fit of forward_targets / head_sample."""
        _check(self.lib, self.lib.npfn_ar_fit_step(self.h, int(k), self.stream), "npfn_ar_fit_step")
        self.n_features = self._ar_dims[0] + int(k)

    def set_fit_token(self, token: int) -> None:
        """npfn_set_fit_token: ar_sample / ar_log_prob calls under one non-zero token reuse the
        per-step fits of the first (the context must be the same for all of them)."""
        _check(self.lib, self.lib.npfn_set_fit_token(self.h, int(token) & 0xFFFFFFFFFFFFFFFF), "npfn_set_fit_token")

    def set_chunk_rows(self, rows: int) -> None:
        """Query rows per forward chunk (npfn_set_chunk_rows; default 16384)."""
        _check(self.lib, self.lib.npfn_set_chunk_rows(self.h, int(rows)), "npfn_set_chunk_rows")

    # -------------------------------------------------------------- profiling
    def prof_enable(self, on: bool = True) -> None:
        _check(self.lib, self.lib.npfn_prof_enable(self.h, 1 if on else 0), "npfn_prof_enable")

    def prof_read(self) -> list:
        """Per-kernel totals since the last read: [{name, launches, ms, flops, bytes}] (synchronizes)."""
        buf = (NpfnProfEntry * 32)()
        n = ctypes.c_int32(0)
        _check(self.lib, self.lib.npfn_prof_read(self.h, buf, 32, ctypes.byref(n)), "npfn_prof_read")
        return [dict(name=buf[i].name.decode(), launches=int(buf[i].launches), ms=float(buf[i].ms),
                     flops=float(buf[i].flops), bytes=float(buf[i].bytes)) for i in range(n.value)]

    def debug_views(self, rows: int, max_cols: int = 1024) -> np.ndarray:
        """[rows, Vw] preprocessed table of the last fit / forward (npfn_debug_views; synchronous)."""
        buf = np.empty((int(rows), int(max_cols)), dtype=np.float32)
        vw = ctypes.c_int32(0)
        _check(self.lib, self.lib.npfn_debug_views(self.h, buf.ctypes.data_as(ctypes.c_void_p), int(rows),
                                                   int(max_cols), ctypes.byref(vw)), "npfn_debug_views")
        return buf.reshape(-1)[: int(rows) * vw.value].reshape(int(rows), vw.value).copy()

    def debug_item_attn_online(self, on: bool = True) -> None:
        """Process-wide: every item-attention block also runs its online-softmax fallback pass
        (npfn_debug_item_attn_online) -- lets the tests pin both passes against the oracle."""
        _check(self.lib, self.lib.npfn_debug_item_attn_online(1 if on else 0), "npfn_debug_item_attn_online")

    def debug_item_attn_scale(self, scale: float = 1.0) -> None:
        """Process-wide: multiply every item-attention score by ``scale`` (stress runs of the
        first pass's fallback; npfn_debug_item_attn_scale).  1.0 restores the model."""
        _check(self.lib, self.lib.npfn_debug_item_attn_scale(float(scale)), "npfn_debug_item_attn_scale")

    def debug_fail_row_launch(self, n: int = 1) -> None:
        """The ``n``-th next row-kernel launch is refused by the runtime (0 = off;
        npfn_debug_fail_row_launch): the error path's test."""
        _check(self.lib, self.lib.npfn_debug_fail_row_launch(self.h, int(n)), "npfn_debug_fail_row_launch")

    def item_attn_fallback(self, reset: bool = True) -> dict:
        """Item-attention launches since the last reset: blocks / query rows that ran or took the
        online-softmax fallback pass, and their totals (npfn_item_attn_fallback; synchronizes); the
        fallback rows split by cause -- sum overflow, underflow, padding-dominated / forced
        (npfn_item_attn_fallback_causes)."""
        cause = (ctypes.c_uint64 * 2)()
        if hasattr(self.lib, "npfn_item_attn_fallback_causes"):  # an older library in an A/B run has none
            _check(self.lib, self.lib.npfn_item_attn_fallback_causes(self.h, cause), "npfn_item_attn_fallback_causes")
        buf = (ctypes.c_uint64 * 4)()
        _check(self.lib, self.lib.npfn_item_attn_fallback(self.h, buf, 1 if reset else 0), "npfn_item_attn_fallback")
        b_fb, b_all, r_fb, r_all = (int(v) for v in buf)
        r_over, r_under = int(cause[0]), int(cause[1])
        return {"blocks_fallback": b_fb, "blocks": b_all, "rows_fallback": r_fb, "rows": r_all,
                "rows_overflow": r_over, "rows_underflow": r_under,
                "rows_padding": max(r_fb - r_over - r_under, 0),
                "fallback_frac": (r_fb / r_all) if r_all else 0.0,
                "block_fallback_frac": (b_fb / b_all) if b_all else 0.0}
