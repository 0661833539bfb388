"""Model configuration and weight sets for the NPE-PFN engine.

The reference obtains its TabPFN-v2 regressor from ``tabpfn.TabPFNRegressor``
(``npe_pfn/npe_pfn.py:8,48``), which downloads a checkpoint on first use
(``model_path="auto"``; tabpfn 2.2.1, poetry.lock:4455-4464).  Neither the
package nor a checkpoint exists in this environment, so the engine runs on a
weight set with the architecture of the v2 regressor:

* d_model 192, 6 heads x 32, 12 layers, MLP width 768 (nhid_factor 4),
  2 features per group, 5000 Riemann bars [ext: tabpfn v2 regressor config];
* ``n_estimators`` 8, softmax temperature 0.9 [ext: tabpfn 2.2.1 defaults].

``synthetic_weights(seed)`` draws that weight set deterministically from
``numpy.random.default_rng(seed)`` (PCG64, stable across platforms), so the
engine and the CPU oracle in ``oracle/`` see identical numbers.  A locally
provisioned checkpoint converted to the same named-tensor layout can be passed
instead (``load_weights``); see INTEGRATION.md.

Weight tensors are stored ``[out_features, in_features]`` (nn.Linear layout),
which is also the layout the engine's GEMMs consume (the B operand of
``Y = X @ W^T`` is read along K for each output column).
"""

from __future__ import annotations

import hashlib
from dataclasses import dataclass, asdict
from typing import Dict, Optional

import numpy as np

__all__ = [
    "ModelConfig",
    "synthetic_weights",
    "synthetic_borders",
    "CLASSIFIER_N_OUT",
    "classifier_config",
    "synthetic_classifier_weights",
    "pack_weights",
    "weight_names",
    "config_for",
    "weights_digest",
    "load_weights",
    "save_weights",
]


@dataclass(frozen=True)
class ModelConfig:
    """Architecture of the per-feature transformer (tabpfn v2 regressor shape)."""

    d_model: int = 192
    n_heads: int = 6
    n_layers: int = 12
    d_ff: int = 768
    n_bars: int = 5000
    features_per_group: int = 2
    # rows of the positional table: tabpfn's 500-feature limit under the default ensemble
    # (2F + k + 1 <= 1251 features, 626 groups) fits
    max_groups: int = 640
    n_estimators: int = 8
    softmax_temperature: float = 0.9

    @property
    def head_dim(self) -> int:
        return self.d_model // self.n_heads

    def to_dict(self) -> dict:
        return asdict(self)


def synthetic_borders(n_bars: int, scale: float = 40.0, a: float = 4.0) -> np.ndarray:
    """Bar borders in the standardized target space.

    sinh-spaced, symmetric, dense near 0 (spacing ~2.3e-3) and reaching +-scale,
    mimicking the shape of TabPFN's full-support bar distribution borders
    [ext: FullSupportBarDistribution borders are data-derived in the checkpoint].
    """
    t = np.linspace(-1.0, 1.0, n_bars + 1, dtype=np.float64)
    b = scale * np.sinh(a * t) / np.sinh(a)
    b[n_bars // 2] = 0.0 if n_bars % 2 == 0 else b[n_bars // 2]
    return b.astype(np.float32)


def weight_names(cfg: ModelConfig):
    """Canonical order of named tensors (also the C-ABI blob order, include/npfn.h)."""
    d, dff, nb, G = cfg.d_model, cfg.d_ff, cfg.n_bars, cfg.max_groups
    names = [
        ("enc_w", (d, 4)),
        ("y_enc_w", (d, 2)),
        ("pos_emb", (G, d)),
    ]
    for l in range(cfg.n_layers):
        names += [
            (f"l{l}.feat_qkv", (3 * d, d)),
            (f"l{l}.feat_out", (d, d)),
            (f"l{l}.item_qkv", (3 * d, d)),
            (f"l{l}.item_out", (d, d)),
            (f"l{l}.mlp_w1", (dff, d)),
            (f"l{l}.mlp_w2", (d, dff)),
            (f"l{l}.ln1_g", (d,)),
            (f"l{l}.ln1_b", (d,)),
            (f"l{l}.ln2_g", (d,)),
            (f"l{l}.ln2_b", (d,)),
            (f"l{l}.ln3_g", (d,)),
            (f"l{l}.ln3_b", (d,)),
        ]
    names += [
        ("dec_w1", (dff, d)),
        ("dec_b1", (dff,)),
        ("dec_w2", (nb, dff)),
        ("dec_b2", (nb,)),
        ("borders", (nb + 1,)),
    ]
    return names


def synthetic_weights(cfg: ModelConfig = ModelConfig(), seed: int = 0) -> Dict[str, np.ndarray]:
    """Deterministic weight set with the v2-regressor architecture.

    Initialisation: linear maps ~ N(0, 1/fan_in); LayerNorm gains 1 + 0.1 N,
    biases 0.05 N.  The decoder's output bias is the log of a unit Gaussian
    bump over the bar centres (plus log bar width), so the untrained head
    already predicts a sensible standardized density that the inputs modulate.
    """
    rng = np.random.default_rng(seed)
    d, dff, nb = cfg.d_model, cfg.d_ff, cfg.n_bars
    w: Dict[str, np.ndarray] = {}

    def lin(out_f, in_f, gain=1.0):
        return (rng.standard_normal((out_f, in_f)) * (gain / np.sqrt(in_f))).astype(np.float32)

    w["enc_w"] = lin(d, 4, gain=np.sqrt(2.0))
    w["y_enc_w"] = lin(d, 2, gain=np.sqrt(2.0))
    w["pos_emb"] = (rng.standard_normal((min(cfg.max_groups, 256), d)) * 0.5).astype(np.float32)
    for l in range(cfg.n_layers):
        w[f"l{l}.feat_qkv"] = lin(3 * d, d)
        w[f"l{l}.feat_out"] = lin(d, d)
        w[f"l{l}.item_qkv"] = lin(3 * d, d)
        w[f"l{l}.item_out"] = lin(d, d)
        w[f"l{l}.mlp_w1"] = lin(dff, d)
        w[f"l{l}.mlp_w2"] = lin(d, dff)
        for k in (1, 2, 3):
            w[f"l{l}.ln{k}_g"] = (1.0 + 0.1 * rng.standard_normal(d)).astype(np.float32)
            w[f"l{l}.ln{k}_b"] = (0.05 * rng.standard_normal(d)).astype(np.float32)
    w["dec_w1"] = lin(dff, d)
    w["dec_b1"] = (0.1 * rng.standard_normal(dff)).astype(np.float32)
    w["dec_w2"] = lin(nb, dff, gain=1.5)
    borders = synthetic_borders(nb)
    centers = 0.5 * (borders[1:].astype(np.float64) + borders[:-1])
    widths = np.diff(borders.astype(np.float64))
    w["dec_b2"] = (-0.5 * centers**2 + np.log(widths)).astype(np.float32)
    w["borders"] = borders
    if cfg.max_groups > 256:  # rows past 256 from their own stream: the first 256 rows (and every
        # other tensor) are those of a 256-row table, so the golden fixtures made with it still hold
        extra = np.random.default_rng([seed, 0x9E5]).standard_normal((cfg.max_groups - 256, d)) * 0.5
        w["pos_emb"] = np.concatenate([w["pos_emb"], extra.astype(np.float32)])
    for name, shape in weight_names(cfg):
        assert w[name].shape == shape, (name, w[name].shape, shape)
    return w


CLASSIFIER_N_OUT = 10  # decoder width of the v2 classifier = max classes [ext: tabpfn 2.2.1]


def classifier_config(n_estimators: int = 8, softmax_temperature: float = 0.9) -> ModelConfig:
    """Architecture of the TabPFN-v2 classifier (npe_pfn.py:610, ``TabPFNClassifier``).

    Same per-feature transformer as the regressor; the decoder ends in
    ``CLASSIFIER_N_OUT`` class logits instead of the Riemann bars (the
    ``n_bars`` field carries the decoder width; the ``borders`` tensor of the
    blob is present for layout uniformity and unused).
    """
    return ModelConfig(n_bars=CLASSIFIER_N_OUT, n_estimators=n_estimators, softmax_temperature=softmax_temperature)


def synthetic_classifier_weights(cfg: Optional[ModelConfig] = None, seed: int = 1) -> Dict[str, np.ndarray]:
    """Deterministic classifier weight set: the trunk of ``synthetic_weights`` plus a
    class head with zero bias and moderate gain, so the untrained head is not
    saturated and its probabilities follow the inputs."""
    cfg = cfg or classifier_config()
    w = synthetic_weights(cfg, seed=seed)
    rng = np.random.default_rng(seed + 0x5EED)
    nb, dff = cfg.n_bars, cfg.d_ff
    w["dec_w2"] = (rng.standard_normal((nb, dff)) * (2.0 / np.sqrt(dff))).astype(np.float32)
    w["dec_b2"] = np.zeros(nb, dtype=np.float32)
    w["borders"] = np.arange(nb + 1, dtype=np.float32)
    return w


def pack_weights(w: Dict[str, np.ndarray], cfg: ModelConfig) -> np.ndarray:
    """Flatten a named weight set into the contiguous float32 blob of include/npfn.h."""
    parts = []
    for name, shape in weight_names(cfg):
        t = np.asarray(w[name], dtype=np.float32)
        if t.shape != shape:
            raise ValueError(f"weight {name}: shape {t.shape} != expected {shape}")
        parts.append(t.reshape(-1))
    return np.ascontiguousarray(np.concatenate(parts), dtype=np.float32)


def weights_digest(w: Dict[str, np.ndarray], cfg: ModelConfig) -> str:
    return hashlib.sha256(pack_weights(w, cfg).tobytes()).hexdigest()[:16]


def save_weights(path: str, w: Dict[str, np.ndarray], cfg: ModelConfig) -> None:
    np.savez(path, __config__=np.frombuffer(repr(cfg.to_dict()).encode(), dtype=np.uint8), **w)


def load_weights(path: str, cfg: ModelConfig) -> Dict[str, np.ndarray]:
    """Load a named-tensor ``.npz`` (no pickle) and check it against ``cfg`` (the positional
    table may have any number of rows: ``config_for`` takes its capacity from it)."""
    with np.load(path, allow_pickle=False) as z:
        w = {k: z[k] for k in z.files if k != "__config__"}
    for name, shape in weight_names(cfg):
        if name not in w:
            raise KeyError(f"weights file {path} lacks tensor {name}")
        got = tuple(w[name].shape)
        if got != shape and not (name == "pos_emb" and len(got) == 2 and got[1] == shape[1]):
            raise ValueError(f"weights file {path}: {name} has shape {w[name].shape}, want {shape}")
    return w


def config_for(w: Dict[str, np.ndarray], cfg: ModelConfig) -> ModelConfig:
    """``cfg`` with ``max_groups`` = the rows of ``w``'s positional table: weights converted or
    saved with another table size (e.g. round 4's 256 rows) keep their own capacity."""
    from dataclasses import replace

    g = int(np.asarray(w["pos_emb"]).shape[0])
    return cfg if g == cfg.max_groups else replace(cfg, max_groups=g)
