"""TabPFN-v2 checkpoint converter (npe_pfn/checkpoint.py).

No TabPFN checkpoint exists offline, so the checkpoints here are built from the
synthetic weight set through the inverse key map, written with ``torch.save`` in
the package's ``{"state_dict", "config"}`` format [ext], and read back through the
safe loader.  The einsum test pins the layout conversion independently: it
applies the checkpoint-shaped ``_w_qkv [3,H,hd,d]`` / ``_w_out [H,hd,d]`` the way
the v2 attention module does [ext] and compares with the engine's ``nn.Linear``
form.  Parity with the package itself is unpinned (module docstring).
"""
import numpy as np
import pytest
import torch

from npe_pfn.checkpoint import (config_from_checkpoint, load_tabpfn_checkpoint, positional_table,
                                tabpfn_state_to_weights, weights_to_tabpfn_state)
from npe_pfn.weights import (ModelConfig, classifier_config, synthetic_classifier_weights, synthetic_weights,
                             weight_names)

CFG = ModelConfig(n_layers=2, n_bars=64, max_groups=16)


def _save_ckpt(path, sd, cfg, with_config=True):
    state = {k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in sd.items()}
    obj = {"state_dict": state}
    if with_config:
        obj["config"] = {"emsize": cfg.d_model, "nhead": cfg.n_heads, "nlayers": cfg.n_layers,
                         "nhid_factor": cfg.d_ff // cfg.d_model, "features_per_group": cfg.features_per_group}
    torch.save(obj, path)


@pytest.mark.parametrize("with_config", [True, False])
def test_round_trip_through_torch_save(tmp_path, with_config):
    w = synthetic_weights(CFG, seed=5)
    path = str(tmp_path / "m.ckpt")
    _save_ckpt(path, weights_to_tabpfn_state(w, CFG), CFG, with_config)
    cfg2, w2 = load_tabpfn_checkpoint(path, max_groups=CFG.max_groups)
    assert cfg2 == CFG
    for name, shape in weight_names(CFG):
        if name == "pos_emb":
            continue  # no positional keys emitted: zero table
        np.testing.assert_array_equal(w2[name], w[name], err_msg=name)
    assert not w2["pos_emb"].any()


def test_attention_layout_matches_einsum_form():
    """q/k/v = einsum('rs,jhds->rjhd', x, _w_qkv); out = einsum('rhd,hds->rs', a, _w_out) [ext]."""
    w = synthetic_weights(CFG, seed=2)
    sd = weights_to_tabpfn_state(w, CFG)
    conv = tabpfn_state_to_weights(sd, CFG)
    H, hd, d = CFG.n_heads, CFG.head_dim, CFG.d_model
    rng = np.random.default_rng(0)
    x = rng.standard_normal((7, d)).astype(np.float64)
    for kind, mod in (("feat", "self_attn_between_features"), ("item", "self_attn_between_items")):
        wqkv = sd[f"transformer_encoder.layers.1.{mod}._w_qkv"].astype(np.float64)
        wout = sd[f"transformer_encoder.layers.1.{mod}._w_out"].astype(np.float64)
        ref = np.einsum("rs,jhds->rjhd", x, wqkv)
        got = (x @ conv[f"l1.{kind}_qkv"].astype(np.float64).T).reshape(7, 3, H, hd)  # oracle's (3, H, hd) split
        np.testing.assert_allclose(got, ref, rtol=1e-12, atol=1e-12)
        a = rng.standard_normal((7, H, hd))
        ref_o = np.einsum("rhd,hds->rs", a, wout)
        got_o = a.reshape(7, H * hd) @ conv[f"l1.{kind}_out"].astype(np.float64).T
        np.testing.assert_allclose(got_o, ref_o, rtol=1e-12, atol=1e-12)


def test_split_q_kv_projection_is_concatenated():
    w = synthetic_weights(CFG, seed=1)
    sd = weights_to_tabpfn_state(w, CFG)
    k = "transformer_encoder.layers.0.self_attn_between_items."
    qkv = sd.pop(k + "_w_qkv")
    sd[k + "_w_q"], sd[k + "_w_kv"] = qkv[:1], qkv[1:]
    conv = tabpfn_state_to_weights(sd, CFG)
    np.testing.assert_array_equal(conv["l0.item_qkv"], w["l0.item_qkv"])


def test_positional_table_is_linear_of_seeded_randn():
    rng = np.random.default_rng(3)
    d = CFG.d_model
    W = rng.standard_normal((d, d // 4)).astype(np.float32)
    b = rng.standard_normal(d).astype(np.float32)
    w = synthetic_weights(CFG, seed=0)
    conv = tabpfn_state_to_weights(weights_to_tabpfn_state(w, CFG, pos_base=(W, b)), CFG)
    g = torch.Generator().manual_seed(42)
    r = torch.randn((CFG.max_groups, d // 4), generator=g)
    ref = torch.nn.functional.linear(r.double(), torch.from_numpy(W).double(), torch.from_numpy(b).double())
    np.testing.assert_allclose(conv["pos_emb"], ref.numpy(), rtol=1e-5, atol=1e-5)
    assert positional_table(W, b, 4).shape == (4, d)


def test_unrepresentable_parameters_raise():
    w = synthetic_weights(CFG, seed=0)
    sd = weights_to_tabpfn_state(w, CFG)
    sd["transformer_encoder.layers.0.mlp.linear1.bias"] = np.ones(CFG.d_ff, np.float32)
    with pytest.raises(ValueError, match="non-zero"):
        tabpfn_state_to_weights(sd, CFG)
    sd = weights_to_tabpfn_state(w, CFG)
    sd["encoder.5.layer.bias"] = np.zeros(CFG.d_model, np.float32)  # zero bias: accepted
    tabpfn_state_to_weights(sd, CFG)
    sd["encoder.1.layer.weight"] = sd["encoder.5.layer.weight"]      # ambiguous encoder
    with pytest.raises(ValueError, match="expected one key"):
        tabpfn_state_to_weights(sd, CFG)


def test_missing_layer_norm_affine_maps_to_identity():
    w = synthetic_weights(CFG, seed=0)
    sd = weights_to_tabpfn_state(w, CFG)
    for k in [k for k in sd if ".layer_norms." in k]:
        del sd[k]
    conv = tabpfn_state_to_weights(sd, CFG)
    assert (conv["l1.ln2_g"] == 1).all() and (conv["l1.ln2_b"] == 0).all()


def test_classifier_checkpoint(tmp_path):
    cfg = classifier_config()
    cfg = ModelConfig(**{**cfg.to_dict(), "n_layers": 1, "max_groups": 8})
    w = synthetic_classifier_weights(cfg, seed=4)
    sd = weights_to_tabpfn_state(w, cfg)
    del sd["criterion.borders"]
    path = str(tmp_path / "c.ckpt")
    _save_ckpt(path, sd, cfg)
    cfg2, w2 = load_tabpfn_checkpoint(path, classifier=True, max_groups=8)
    assert cfg2.n_bars == cfg.n_bars and cfg2.n_layers == 1
    np.testing.assert_array_equal(w2["dec_w2"], w["dec_w2"])


def test_config_mismatch_raises():
    w = synthetic_weights(CFG, seed=0)
    sd = weights_to_tabpfn_state(w, CFG)
    with pytest.raises(ValueError, match="linear1"):
        config_from_checkpoint(sd, {"emsize": 192, "nhead": 6, "nlayers": 2, "nhid_factor": 2})


def test_regressor_shim_loads_ckpt_path(tmp_path):
    """TabPFNRegressor(model_path=*.ckpt) resolves through the converter (no GPU needed to resolve)."""
    from npe_pfn.tabpfn import _resolve_weights

    cfg = ModelConfig()
    w = synthetic_weights(cfg, seed=9)
    path = str(tmp_path / "full.ckpt")
    _save_ckpt(path, weights_to_tabpfn_state(w, cfg), cfg)
    got = _resolve_weights(path, None, 0, cfg)
    np.testing.assert_array_equal(got["l11.mlp_w2"], w["l11.mlp_w2"])
    with pytest.raises(ValueError, match="differs"):
        _resolve_weights(path, None, 0, ModelConfig(n_estimators=4, n_layers=6))
