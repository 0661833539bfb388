"""TabPFN-v2 checkpoint -> engine weight layout.

The reference gets its regressor and classifier weights from
``TabPFNRegressor(model_path="auto")`` / ``TabPFNClassifier`` (npe_pfn.py:48,
:69, :610), which resolve a ``.ckpt`` through the tabpfn package [ext:
tabpfn==2.2.1, poetry.lock:4455-4464; ``model/loading.py``].  Neither the
package nor a checkpoint exists offline, so this module restates the
checkpoint's published layout and maps it onto the named tensors of
``weights.weight_names`` (the C-ABI blob of include/npfn.h):

==========================================================  ======================
checkpoint ``state_dict`` key [ext]                          engine tensor
==========================================================  ======================
``encoder.<i>.layer.weight``            [d, 2*fpg]           ``enc_w``
``y_encoder.<i>.layer.weight``          [d, 2]               ``y_enc_w``
``feature_positional_embedding_embeddings.{weight,bias}``    ``pos_emb`` (see below)
``transformer_encoder.layers.<l>.self_attn_between_features._w_qkv`` [3,H,hd,d]
                                                             ``l<l>.feat_qkv`` [3d, d]
``..._w_out``                           [H, hd, d]           ``l<l>.feat_out`` [d, d]
``...self_attn_between_items._w_qkv / _w_out``               ``l<l>.item_qkv / item_out``
``...mlp.linear1.weight / linear2.weight``                   ``l<l>.mlp_w1 / mlp_w2``
``...layer_norms.<0|1|2>.{weight,bias}``                     ``l<l>.ln<1|2|3>_{g,b}``
``decoder_dict.standard.0.{weight,bias}``                    ``dec_w1``, ``dec_b1``
``decoder_dict.standard.2.{weight,bias}``                    ``dec_w2``, ``dec_b2``
``criterion.borders``                   [n_bars+1]           ``borders``
==========================================================  ======================

Layout notes.  ``_w_qkv`` is einsum-shaped ``[3, H, hd, d]``: flattening its
first three axes gives the ``[q | k | v] x (head, dim)`` row order that the
engine's fused QKV GEMM produces (``oracle/tabpfn_oracle.py`` reshapes the
output as ``(3, H, hd)``).  ``_w_out`` ``[H, hd, d]`` contracts over
``(H, hd)``, so as an ``nn.Linear`` matrix it is ``reshape(H*hd, d).T``.
Checkpoints that split the projection (``_w_q`` ``[1,H,hd,d]`` plus
``_w_kv`` ``[2,H,hd,d]``) are concatenated.  LayerNorms without elementwise
affine parameters map to gain 1 / bias 0.

Feature positional embedding.  TabPFN v2 adds, per feature group ``g``,
``Linear(d/4 -> d)(r_g)`` with ``r`` drawn by ``torch.randn`` from a generator
seeded with ``random_embedding_seed`` (42) [ext].  The engine stores the
resulting ``[max_groups, d]`` table (``pos_emb``); it is generated here on the
CPU generator.  Whether the package draws ``r`` on the CPU or on the model's
device, and whether a prefix of the draw is independent of the group count,
are not verifiable offline: **parity with the package is unpinned** for this
term (and for the whole checkpoint path), see DESIGN.md §3.

Anything the engine cannot represent (an encoder or MLP bias that is not zero,
attention biases, a different width / head count, a decoder hidden width other
than ``d_ff``) raises ``ValueError`` rather than being silently dropped.

Loading executes nothing from the file: ``torch.load(..., weights_only=True)``.
A checkpoint whose config the safe loader refuses cannot be used; convert it
once where it was produced (``state_dict`` + a plain-dict config).

Command line: ``python -m npe_pfn.checkpoint IN.ckpt OUT.npz [--classifier]``
writes the named-tensor ``.npz`` that ``model_path=`` accepts.
"""

from __future__ import annotations

import argparse
import re
from typing import Dict, Mapping, Optional, Tuple

import numpy as np

from .weights import CLASSIFIER_N_OUT, ModelConfig, save_weights, weight_names

__all__ = [
    "RANDOM_EMBEDDING_SEED",
    "config_from_checkpoint",
    "tabpfn_state_to_weights",
    "weights_to_tabpfn_state",
    "load_tabpfn_checkpoint",
    "positional_table",
]

RANDOM_EMBEDDING_SEED = 42  # [ext: tabpfn v2 PerFeatureTransformer default]
_LAYER = "transformer_encoder.layers.{l}."


def _np(t) -> np.ndarray:
    if hasattr(t, "detach"):
        t = t.detach().to("cpu").float().numpy()
    return np.asarray(t, dtype=np.float32)


def _find(sd: Mapping[str, object], pattern: str, what: str) -> str:
    rx = re.compile(pattern)
    hits = sorted(k for k in sd if rx.fullmatch(k))
    if len(hits) != 1:
        raise ValueError(f"checkpoint: expected one key for {what} (/{pattern}/), found {hits}")
    return hits[0]


def _zero_or_absent(sd, key: str) -> None:
    if key in sd and np.any(_np(sd[key]) != 0):
        raise ValueError(f"checkpoint: {key} is non-zero; the engine has no slot for this bias")


def config_from_checkpoint(state: Mapping[str, object], cfg_dict: Optional[Mapping] = None,
                           classifier: bool = False, n_estimators: int = 8,
                           softmax_temperature: float = 0.9,
                           max_groups: int = ModelConfig.max_groups) -> ModelConfig:
    """Architecture from the checkpoint config (``emsize``, ``nhead``, ``nlayers``,
    ``nhid_factor``, ``features_per_group`` [ext]), cross-checked with tensor shapes."""
    cfg_dict = dict(cfg_dict or {})
    qkv0 = _np(state[_LAYER.format(l=0) + "self_attn_between_features._w_qkv"]) \
        if _LAYER.format(l=0) + "self_attn_between_features._w_qkv" in state else None
    lin1 = _np(state[_LAYER.format(l=0) + "mlp.linear1.weight"])
    d = int(cfg_dict.get("emsize", lin1.shape[1]))
    H = int(cfg_dict.get("nhead", qkv0.shape[1] if qkv0 is not None else 6))
    n_layers = int(cfg_dict.get("nlayers", 1 + max(int(m.group(1)) for k in state
                                                     for m in [re.match(r"transformer_encoder\.layers\.(\d+)\.", k)] if m)))
    d_ff = int(d * cfg_dict["nhid_factor"]) if "nhid_factor" in cfg_dict else int(lin1.shape[0])
    fpg = int(cfg_dict.get("features_per_group", _np(state[_find(state, r"encoder\.\d+\.layer\.weight", "encoder")]).shape[1] // 2))
    if lin1.shape != (d_ff, d):
        raise ValueError(f"checkpoint: mlp.linear1 has shape {lin1.shape}, config says ({d_ff}, {d})")
    if classifier:
        n_out = _np(state["decoder_dict.standard.2.weight"]).shape[0]
        if n_out != CLASSIFIER_N_OUT:
            raise ValueError(f"checkpoint: classifier decoder width {n_out} != {CLASSIFIER_N_OUT}")
        n_bars = n_out
    else:
        n_bars = _np(state["criterion.borders"]).shape[0] - 1
    return ModelConfig(d_model=d, n_heads=H, n_layers=n_layers, d_ff=d_ff, n_bars=n_bars,
                       features_per_group=fpg, max_groups=max_groups, n_estimators=n_estimators,
                       softmax_temperature=softmax_temperature)


def positional_table(W: np.ndarray, b: Optional[np.ndarray], n_groups: int,
                     seed: int = RANDOM_EMBEDDING_SEED) -> np.ndarray:
    """``Linear(d/4 -> d)`` applied to ``randn(n_groups, d/4)`` from a CPU generator
    seeded with ``seed`` [ext; device/prefix behaviour unpinned, module docstring]."""
    import torch

    g = torch.Generator(device="cpu").manual_seed(seed)
    r = torch.randn((n_groups, W.shape[1]), generator=g, dtype=torch.float32).numpy()
    out = r.astype(np.float64) @ W.astype(np.float64).T
    if b is not None:
        out = out + b
    return out.astype(np.float32)


def _qkv(sd, prefix: str, H: int, hd: int, d: int) -> np.ndarray:
    if prefix + "_w_qkv" in sd:
        w = _np(sd[prefix + "_w_qkv"])
    elif prefix + "_w_q" in sd and prefix + "_w_kv" in sd:
        w = np.concatenate([_np(sd[prefix + "_w_q"]), _np(sd[prefix + "_w_kv"])], 0)
    else:
        raise ValueError(f"checkpoint: no QKV projection under {prefix}")
    if w.shape != (3, H, hd, d):
        raise ValueError(f"checkpoint: {prefix} QKV has shape {w.shape}, want (3, {H}, {hd}, {d})")
    return w.reshape(3 * H * hd, d)


def _out(sd, prefix: str, H: int, hd: int, d: int) -> np.ndarray:
    w = _np(sd[prefix + "_w_out"])
    if w.shape != (H, hd, d):
        raise ValueError(f"checkpoint: {prefix}_w_out has shape {w.shape}, want ({H}, {hd}, {d})")
    return np.ascontiguousarray(w.reshape(H * hd, d).T)


def tabpfn_state_to_weights(state: Mapping[str, object], cfg: ModelConfig,
                            classifier: bool = False) -> Dict[str, np.ndarray]:
    """Map a TabPFN-v2 ``state_dict`` onto the engine's named tensors (module docstring)."""
    d, H, hd = cfg.d_model, cfg.n_heads, cfg.head_dim
    w: Dict[str, np.ndarray] = {}
    ek = _find(state, r"encoder\.\d+\.layer\.weight", "the input encoder")
    _zero_or_absent(state, ek[: -len("weight")] + "bias")
    w["enc_w"] = _np(state[ek])
    yk = _find(state, r"y_encoder\.\d+\.layer\.weight", "the target encoder")
    _zero_or_absent(state, yk[: -len("weight")] + "bias")
    w["y_enc_w"] = _np(state[yk])
    pk = "feature_positional_embedding_embeddings."
    if pk + "weight" in state:
        b = _np(state[pk + "bias"]) if pk + "bias" in state else None
        w["pos_emb"] = positional_table(_np(state[pk + "weight"]), b, cfg.max_groups)
    else:
        w["pos_emb"] = np.zeros((cfg.max_groups, d), np.float32)
    for l in range(cfg.n_layers):
        p = _LAYER.format(l=l)
        for kind, name in (("feat", "self_attn_between_features."), ("item", "self_attn_between_items.")):
            for bias in ("_b_qkv", "_b_q", "_b_kv", "_b_out"):
                _zero_or_absent(state, p + name + bias)
            w[f"l{l}.{kind}_qkv"] = _qkv(state, p + name, H, hd, d)
            w[f"l{l}.{kind}_out"] = _out(state, p + name, H, hd, d)
        for lin in ("linear1", "linear2"):
            _zero_or_absent(state, p + f"mlp.{lin}.bias")
        w[f"l{l}.mlp_w1"] = _np(state[p + "mlp.linear1.weight"])
        w[f"l{l}.mlp_w2"] = _np(state[p + "mlp.linear2.weight"])
        for i in range(3):
            g, b = p + f"layer_norms.{i}.weight", p + f"layer_norms.{i}.bias"
            w[f"l{l}.ln{i + 1}_g"] = _np(state[g]) if g in state else np.ones(d, np.float32)
            w[f"l{l}.ln{i + 1}_b"] = _np(state[b]) if b in state else np.zeros(d, np.float32)
    dp = "decoder_dict.standard."
    w["dec_w1"] = _np(state[dp + "0.weight"])
    w["dec_b1"] = _np(state[dp + "0.bias"]) if dp + "0.bias" in state else np.zeros(cfg.d_ff, np.float32)
    w["dec_w2"] = _np(state[dp + "2.weight"])
    w["dec_b2"] = _np(state[dp + "2.bias"]) if dp + "2.bias" in state else np.zeros(cfg.n_bars, np.float32)
    if classifier:
        w["borders"] = np.arange(cfg.n_bars + 1, dtype=np.float32)
    else:
        w["borders"] = _np(state["criterion.borders"])
    for name, shape in weight_names(cfg):
        if tuple(w[name].shape) != shape:
            raise ValueError(f"checkpoint: converted {name} has shape {w[name].shape}, the engine needs {shape}")
    return w


def weights_to_tabpfn_state(w: Mapping[str, np.ndarray], cfg: ModelConfig, pos_base: Optional[np.ndarray] = None,
                            encoder_index: int = 5, y_encoder_index: int = 2) -> Dict[str, np.ndarray]:
    """Inverse map into a TabPFN-v2-keyed state dict (test fixture builder).

    ``pos_base`` = ``(W [d, d/4], b [d])`` of the positional ``Linear``; when given, the
    positional keys are emitted (and ``w["pos_emb"]`` is ignored)."""
    d, H, hd = cfg.d_model, cfg.n_heads, cfg.head_dim
    sd: Dict[str, np.ndarray] = {
        f"encoder.{encoder_index}.layer.weight": np.asarray(w["enc_w"]),
        f"y_encoder.{y_encoder_index}.layer.weight": np.asarray(w["y_enc_w"]),
    }
    if pos_base is not None:
        sd["feature_positional_embedding_embeddings.weight"] = pos_base[0]
        sd["feature_positional_embedding_embeddings.bias"] = pos_base[1]
    for l in range(cfg.n_layers):
        p = _LAYER.format(l=l)
        for kind, name in (("feat", "self_attn_between_features."), ("item", "self_attn_between_items.")):
            sd[p + name + "_w_qkv"] = np.asarray(w[f"l{l}.{kind}_qkv"]).reshape(3, H, hd, d)
            sd[p + name + "_w_out"] = np.ascontiguousarray(np.asarray(w[f"l{l}.{kind}_out"]).T).reshape(H, hd, d)
        sd[p + "mlp.linear1.weight"] = np.asarray(w[f"l{l}.mlp_w1"])
        sd[p + "mlp.linear2.weight"] = np.asarray(w[f"l{l}.mlp_w2"])
        for i in range(3):
            sd[p + f"layer_norms.{i}.weight"] = np.asarray(w[f"l{l}.ln{i + 1}_g"])
            sd[p + f"layer_norms.{i}.bias"] = np.asarray(w[f"l{l}.ln{i + 1}_b"])
    sd["decoder_dict.standard.0.weight"] = np.asarray(w["dec_w1"])
    sd["decoder_dict.standard.0.bias"] = np.asarray(w["dec_b1"])
    sd["decoder_dict.standard.2.weight"] = np.asarray(w["dec_w2"])
    sd["decoder_dict.standard.2.bias"] = np.asarray(w["dec_b2"])
    sd["criterion.borders"] = np.asarray(w["borders"])
    return sd


def load_tabpfn_checkpoint(path: str, classifier: bool = False, n_estimators: int = 8,
                           softmax_temperature: float = 0.9,
                           max_groups: int = ModelConfig.max_groups) -> Tuple[ModelConfig, Dict[str, np.ndarray]]:
    """Read a TabPFN-v2 ``.ckpt`` with the safe loader and convert it.

    Accepts ``{"state_dict": ..., "config": {...}}`` (the package's format [ext]) or a
    bare state dict.  ``torch.load(weights_only=True)`` executes nothing from the file;
    if it refuses the file, that error propagates."""
    import torch

    obj = torch.load(path, map_location="cpu", weights_only=True)
    if isinstance(obj, Mapping) and "state_dict" in obj:
        state, cfg_dict = obj["state_dict"], obj.get("config")
    else:
        state, cfg_dict = obj, None
    if not isinstance(state, Mapping):
        raise ValueError(f"{path}: no state_dict mapping in the checkpoint")
    if cfg_dict is not None and not isinstance(cfg_dict, Mapping):
        cfg_dict = None
    cfg = config_from_checkpoint(state, cfg_dict, classifier, n_estimators, softmax_temperature, max_groups)
    return cfg, tabpfn_state_to_weights(state, cfg, classifier)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description="convert a TabPFN-v2 .ckpt to the engine's named-tensor .npz")
    ap.add_argument("src")
    ap.add_argument("dst")
    ap.add_argument("--classifier", action="store_true")
    a = ap.parse_args(argv)
    cfg, w = load_tabpfn_checkpoint(a.src, classifier=a.classifier)
    save_weights(a.dst, w, cfg)
    print(f"wrote {a.dst}: {cfg}")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
