"""``tabpfn``-compatible estimator objects backed by the HIP engine (the drop-in boundary).

The reference holds ``TabPFNRegressor(**regressor_init_kwargs)`` in
``NPE_PFN_Core._model`` (npe_pfn/npe_pfn.py:48, rebuilt on unpickle :69) and
uses exactly this surface of it:

* ``fit(X, y)`` -- npe_pfn.py:140, 215, 502;
* ``predict(X, output_type="full", quantiles=[])`` returning ``{"logits",
  "criterion"}`` -- npe_pfn.py:143, 217, 505;
* ``criterion.sample(logits)`` -- npe_pfn.py:146, 220;
* ``criterion(logits, y)`` (NLL) -- npe_pfn.py:149, 226, 510.

:class:`TabPFNRegressor` provides that surface over ``libnpfn.so`` and, in
addition, the fused autoregressive entry points (``ar_sample``,
``ar_log_prob``) that :class:`npe_pfn.npe_pfn.NPE_PFN_Core` uses when its
estimator offers them.

Sampling randomness: tabpfn draws ``criterion.sample`` uniforms from torch's
global RNG [ext]; here they come from Philox4x32-10 keyed by
``random_state`` with one counter per ``criterion.sample`` call (the fused
sampler consumes one counter per autoregressive step), so results are
reproducible and identical between the engine and the CPU oracle.
"""

from __future__ import annotations

import contextlib
import itertools
import warnings
from typing import Optional

import torch

from .limits import MAX_NUMBER_OF_SAMPLES, check_pretraining_limits  # noqa: F401 (re-exported)
from .weights import (ModelConfig, classifier_config, config_for, load_weights, synthetic_classifier_weights,
                      synthetic_weights)

# tabpfn 2.2.1's remaining TabPFNRegressor / TabPFNClassifier keyword arguments [ext] (the
# reference forwards regressor_init_kwargs / classifier_init_kwargs unchanged, npe_pfn.py:45-48,
# 610) and how this engine takes each (INTEGRATION.md "tabpfn keyword arguments"):
# * no effect on results -- accepted and ignored:
_NOOP_KWARGS = {"fit_mode", "memory_saving_mode", "n_jobs", "n_preprocessing_jobs"}
# * honoured: average_before_softmax (npfn_set_average_before_softmax), inference_precision
#   ("auto" / "autocast" only: the engine computes with bf16 MFMA operands and fp32 accumulation,
#   as tabpfn's GPU autocast does; any other precision raises), balance_probabilities
#   (classifier only: the class probabilities divided by the training class frequencies and
#   renormalized, as tabpfn does);
# * would change results in a way the engine does not compute -- accepted only at tabpfn's
#   default, anything else raises ValueError:
_DEFAULT_ONLY_KWARGS = {"categorical_features_indices": None, "differentiable_input": False,
                        "inference_config": None}
_PRECISIONS = ("auto", "autocast")


def _take_kwargs(cls_name: str, kwargs: dict, classifier: bool) -> dict:
    """Split tabpfn's extra keyword arguments (see above): returns the honoured ones with their
    defaults filled in; raises TypeError for names tabpfn does not have and ValueError for
    values the engine cannot honour."""
    kw = dict(kwargs)
    honoured = {"average_before_softmax": bool(kw.pop("average_before_softmax", False)),
                "inference_precision": kw.pop("inference_precision", "auto")}
    if classifier:
        honoured["balance_probabilities"] = bool(kw.pop("balance_probabilities", False))
    prec = honoured["inference_precision"]
    if not (isinstance(prec, str) and prec in _PRECISIONS):
        raise ValueError(f"{cls_name}: inference_precision={prec!r} is not supported -- the HIP engine computes "
                         "with bf16 MFMA operands and fp32 accumulation (tabpfn's 'auto' / 'autocast' on a GPU); "
                         "pass 'auto' or 'autocast'")
    for name, default in _DEFAULT_ONLY_KWARGS.items():
        if name in kw:
            val = kw.pop(name)
            if val != default:
                raise ValueError(f"{cls_name}: {name}={val!r} is not supported by the HIP engine (only tabpfn's "
                                 f"default {default!r})")
    ignored = {k: kw.pop(k) for k in list(kw) if k in _NOOP_KWARGS}
    if kw:
        raise TypeError(f"{cls_name} got unsupported keyword arguments: {sorted(kw)}")
    if ignored:
        warnings.warn(f"{cls_name}: ignoring {sorted(ignored)} (no effect on the results of the HIP engine)",
                      stacklevel=3)
    return honoured


_WEIGHTS_CACHE = {}


def _check_table(n: int, n_features: int, ignore_pretraining_limits: bool) -> None:
    """tabpfn refuses more than 10 000 context rows or 500 features unless
    ``ignore_pretraining_limits=True`` [ext]; the same errors here, raised before any engine
    call (the engine's own capacity is checked by ``Engine.check_table``, npe_pfn.limits)."""
    check_pretraining_limits(int(n), int(n_features), ignore_pretraining_limits)


def _n_features(X) -> int:
    shape = getattr(X, "shape", None)
    return int(shape[1]) if shape is not None and len(shape) == 2 else 0


_FIT_TOKENS = itertools.count(1)   # process-unique fit tokens (npfn_set_fit_token)


_CKPT_SUFFIXES = (".ckpt", ".pt", ".pth")


def _load_file(model_path: str, cfg: ModelConfig, classifier: bool):
    """A converted ``.npz`` (weights.load_weights) or a TabPFN-v2 ``.ckpt`` converted on
    load (checkpoint.load_tabpfn_checkpoint); the file's architecture must be ``cfg``'s."""
    if not model_path.endswith(_CKPT_SUFFIXES):
        return load_weights(model_path, cfg)
    from .checkpoint import load_tabpfn_checkpoint

    ck_cfg, w = load_tabpfn_checkpoint(model_path, classifier=classifier, n_estimators=cfg.n_estimators,
                                       softmax_temperature=cfg.softmax_temperature, max_groups=cfg.max_groups)
    if ck_cfg != cfg:
        raise ValueError(f"{model_path}: checkpoint architecture {ck_cfg} differs from the engine's {cfg}")
    return w


def _resolve_weights(model_path, weights, weight_seed: int, cfg: ModelConfig, classifier: bool = False):
    if weights is not None:
        return weights
    if model_path in (None, "auto"):
        key = ("synthetic", weight_seed, cfg)
        if key not in _WEIGHTS_CACHE:
            _WEIGHTS_CACHE[key] = synthetic_weights(cfg, seed=weight_seed)
        return _WEIGHTS_CACHE[key]
    key = ("file", str(model_path), cfg, classifier)
    if key not in _WEIGHTS_CACHE:
        _WEIGHTS_CACHE[key] = _load_file(str(model_path), cfg, classifier)
    return _WEIGHTS_CACHE[key]


def _resolve_device(device) -> torch.device:
    if device in (None, "auto"):
        if not torch.cuda.is_available():
            raise RuntimeError("TabPFNRegressor (NPE-PFN engine) needs a ROCm GPU; none is visible")
        return torch.device("cuda", torch.cuda.current_device())
    dev = torch.device(device)
    if dev.type != "cuda":
        raise ValueError(f"the NPE-PFN engine runs on the GPU only, got device={device!r}")
    return dev


class TabPFNRegressor:
    """Engine-backed stand-in for ``tabpfn.TabPFNRegressor`` (v2.2.1 surface used by npe_pfn)."""

    def __init__(self, n_estimators: int = 8, softmax_temperature: float = 0.9, random_state: Optional[int] = 0,
                 device="auto", model_path="auto", weights=None, weight_seed: int = 0,
                 preprocessing: str = "ensemble", ignore_pretraining_limits: bool = False, **kwargs):
        kw = _take_kwargs("TabPFNRegressor", kwargs, classifier=False)
        self.average_before_softmax = kw["average_before_softmax"]
        self.inference_precision = kw["inference_precision"]
        self.n_estimators = int(n_estimators)
        self.softmax_temperature = float(softmax_temperature)
        self.random_state = 0 if random_state is None else int(random_state)
        self.device = device
        self.model_path = model_path
        self._weights = weights
        self.weight_seed = int(weight_seed)
        self.ignore_pretraining_limits = bool(ignore_pretraining_limits)
        # "ensemble" (tabpfn's default regressor preprocessing) | "none" | "quantile" |
        # "quantile+power" (Engine.set_preprocessing)
        self.preprocessing = preprocessing
        self.sample_counter = 0
        self._engine = None

    # -------------------------------------------------------------- engine
    @property
    def config(self) -> ModelConfig:
        return ModelConfig(n_estimators=self.n_estimators, softmax_temperature=self.softmax_temperature)

    @property
    def engine(self):
        if self._engine is None:
            from .engine import Engine

            cfg = self.config
            w = _resolve_weights(self.model_path, self._weights, self.weight_seed, cfg)
            cfg = config_for(w, cfg)  # the table the weights bring
            self._engine = Engine(cfg, w, device=_resolve_device(self.device), random_state=self.random_state,
                                  preprocessing=self.preprocessing)
            if self.average_before_softmax:
                self._engine.set_average_before_softmax(True)
        return self._engine

    def __getstate__(self):
        st = self.__dict__.copy()
        st["_engine"] = None
        return st

    # ------------------------------------------------------- tabpfn surface
    def fit(self, X, y):
        _check_table(len(X), _n_features(X), self.ignore_pretraining_limits)
        self.engine.fit(X, y)
        return self

    def predict(self, X, output_type: str = "full", quantiles=None):
        if output_type != "full":
            raise NotImplementedError(f"output_type={output_type!r}: only 'full' is used by NPE-PFN")
        eng = self.engine
        logits = eng.predict_logits(X)
        return {"logits": logits, "criterion": BarCriterion(self, eng.borders())}

    # ------------------------------------------------------------ fused path
    def ar_sample(self, x_ctx, theta_ctx, x_query, with_log_prob: bool = False, eps: float = 1e-15,
                  row_base: int = 0, x_unique=None):
        """Fused AR sampler; query row i draws at Philox row ``row_base + i`` (sharded batches);
        ``x_unique``: the distinct rows x_query repeats (Engine.ar_sample)."""
        _check_table(len(x_ctx), x_ctx.shape[1] + theta_ctx.shape[1] - 1, self.ignore_pretraining_limits)
        counter = self.sample_counter
        self.sample_counter += int(theta_ctx.shape[1])
        return self.engine.ar_sample(x_ctx, theta_ctx, x_query, counter, with_log_prob, eps, row_base=row_base,
                                     x_unique=x_unique)

    def ar_log_prob(self, x_ctx, theta_ctx, x_query, theta, eps: float = 1e-15, x_unique=None):
        _check_table(len(x_ctx), x_ctx.shape[1] + theta_ctx.shape[1] - 1, self.ignore_pretraining_limits)
        return self.engine.ar_log_prob(x_ctx, theta_ctx, x_query, theta, eps, x_unique=x_unique)

    @contextlib.contextmanager
    def reuse_fits(self):
        """Within the block, ar_sample / ar_log_prob calls share their per-step fits (one fresh
        token; the caller guarantees one context for the whole block -- one sample() call)."""
        eng = self.engine
        eng.set_fit_token(next(_FIT_TOKENS))
        try:
            yield
        finally:
            eng.set_fit_token(0)


class BarCriterion:
    """``FullSupportBarDistribution`` returned by ``predict(...)["criterion"]``."""

    def __init__(self, reg: TabPFNRegressor, borders: torch.Tensor):
        self._reg = reg
        self.borders = borders

    @property
    def num_bars(self) -> int:
        return int(self.borders.numel()) - 1

    def sample(self, logits: torch.Tensor, t: float = 1.0) -> torch.Tensor:
        """One inverse-CDF draw per row; returned on the CPU like tabpfn's [ext]."""
        if t != 1.0:
            logits = logits / t
        out = self._reg.engine.bar_sample(logits, self.borders, self._reg.sample_counter)
        self._reg.sample_counter += 1
        return out.cpu()

    def __call__(self, logits: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
        """NLL per row, returned on the device of ``y``."""
        y = torch.as_tensor(y)
        out = self._reg.engine.bar_nll(logits, self.borders, y)
        return out.to(y.device)


class TabPFNClassifier:
    """Engine-backed stand-in for ``tabpfn.TabPFNClassifier`` (the surface npe_pfn uses).

    ``DensityRatioWrapper`` (npe_pfn.py:603-704) creates it with
    ``classifier_init_kwargs`` (:610), calls ``fit(X[2n, dθ], y in {0, 1})`` (:661)
    and ``predict_proba(theta)`` (:697), expecting a numpy ``[N, n_classes]`` array
    in the order of ``classes_`` (labels sorted, as sklearn's LabelEncoder).
    The forward is the same per-feature transformer as the regressor with a
    class head (``weights.classifier_config``); ``weight_seed`` selects the
    synthetic classifier weights when no ``model_path`` / ``weights`` is given.
    """

    def __init__(self, n_estimators: int = 8, softmax_temperature: float = 0.9, random_state: Optional[int] = 0,
                 device="auto", model_path="auto", weights=None, weight_seed: int = 1,
                 preprocessing: str = "ensemble", ignore_pretraining_limits: bool = False, **kwargs):
        kw = _take_kwargs("TabPFNClassifier", kwargs, classifier=True)
        self.average_before_softmax = kw["average_before_softmax"]
        self.inference_precision = kw["inference_precision"]
        self.balance_probabilities = kw["balance_probabilities"]
        self.class_counts_ = None
        self.n_estimators = int(n_estimators)
        self.softmax_temperature = float(softmax_temperature)
        self.random_state = 0 if random_state is None else int(random_state)
        self.device = device
        self.model_path = model_path
        self._weights = weights
        self.weight_seed = int(weight_seed)
        self.ignore_pretraining_limits = bool(ignore_pretraining_limits)
        # "ensemble" (tabpfn's default classifier preprocessing: coarse-quantile + original + SVD |
        # original, fingerprint; oracle/preprocess_oracle.py) | "none" | "quantile" | "quantile+power"
        self.preprocessing = preprocessing
        self.classes_ = None
        self._engine = None

    @property
    def config(self) -> ModelConfig:
        return classifier_config(self.n_estimators, self.softmax_temperature)

    @property
    def engine(self):
        if self._engine is None:
            from .engine import Engine

            cfg = self.config
            if self._weights is not None:
                w = self._weights
            elif self.model_path in (None, "auto"):
                key = ("synthetic-classifier", self.weight_seed, cfg)
                if key not in _WEIGHTS_CACHE:
                    _WEIGHTS_CACHE[key] = synthetic_classifier_weights(cfg, seed=self.weight_seed)
                w = _WEIGHTS_CACHE[key]
            else:
                w = _resolve_weights(self.model_path, None, self.weight_seed, cfg, classifier=True)
            cfg = config_for(w, cfg)  # the table the weights bring
            self._engine = Engine(cfg, w, device=_resolve_device(self.device), random_state=self.random_state,
                                  preprocessing=self.preprocessing)
            if self.average_before_softmax:
                self._engine.set_average_before_softmax(True)
        return self._engine

    def __getstate__(self):
        st = self.__dict__.copy()
        st["_engine"] = None
        return st

    def fit(self, X, y):
        _check_table(len(X), _n_features(X), self.ignore_pretraining_limits)
        y = torch.as_tensor(y).reshape(-1)
        classes, y_idx, counts = torch.unique(y, sorted=True, return_inverse=True, return_counts=True)
        if classes.numel() < 2:
            raise ValueError("TabPFNClassifier.fit needs at least two classes")
        self.classes_ = classes.cpu().numpy()
        self.class_counts_ = counts.cpu().numpy()
        self.engine.fit_classes(X, y_idx.to(torch.float32), int(classes.numel()))
        return self

    def predict_proba_tensor(self, X) -> torch.Tensor:
        """Device tensor variant of predict_proba (no host copy)."""
        if self.classes_ is None:
            raise RuntimeError("TabPFNClassifier: predict_proba before fit")
        p = self.engine.predict_proba(X)
        if self.balance_probabilities:  # tabpfn [ext]: divide by the train class frequencies, renormalize
            freq = torch.as_tensor(self.class_counts_ / self.class_counts_.sum(), dtype=torch.float32,
                                   device=p.device)
            p = p / freq
            p = p / p.sum(-1, keepdim=True)
        return p

    def predict_proba(self, X):
        """numpy [N, n_classes], as tabpfn returns it (npe_pfn.py:697-701)."""
        return self.predict_proba_tensor(X).cpu().numpy()
