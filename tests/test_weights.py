"""Synthetic weight set: shapes, determinism, packing order, checkpoint round trip."""
import numpy as np

from npe_pfn.weights import (ModelConfig, load_weights, pack_weights, save_weights, synthetic_borders,
                             synthetic_weights, weight_names, weights_digest)


def test_deterministic_and_named():
    cfg = ModelConfig(n_layers=2)
    a = synthetic_weights(cfg, seed=3)
    b = synthetic_weights(cfg, seed=3)
    assert weights_digest(a, cfg) == weights_digest(b, cfg)
    assert weights_digest(a, cfg) != weights_digest(synthetic_weights(cfg, seed=4), cfg)
    assert [n for n, _ in weight_names(cfg)] == list(a.keys())


def test_borders_monotone_symmetric():
    b = synthetic_borders(5000)
    assert b.shape == (5001,) and np.all(np.diff(b) > 0)
    np.testing.assert_allclose(b, -b[::-1], atol=1e-5)


def test_decoder_bias_is_a_density_prior():
    cfg = ModelConfig()
    w = synthetic_weights(cfg, seed=0)
    b = w["borders"].astype(np.float64)
    p = np.exp(w["dec_b2"] - w["dec_b2"].max())
    p /= p.sum()
    centers = 0.5 * (b[1:] + b[:-1])
    mean = (p * centers).sum()
    sd = np.sqrt((p * (centers - mean) ** 2).sum())
    assert abs(mean) < 1e-3 and abs(sd - 1.0) < 1e-2


def test_npz_round_trip(tmp_path):
    cfg = ModelConfig(n_layers=1, n_bars=16, max_groups=8)
    w = synthetic_weights(cfg, seed=0)
    path = str(tmp_path / "w.npz")
    save_weights(path, w, cfg)
    w2 = load_weights(path, cfg)
    np.testing.assert_array_equal(pack_weights(w, cfg), pack_weights(w2, cfg))


def test_positional_table_extension_keeps_every_other_tensor():
    """ModelConfig() has 640 positional rows (tabpfn's 500 features under the ensemble); rows past
    256 come from their own stream, so a 256-row table's weights -- the golden fixtures' -- are the
    first rows, and every other tensor is unchanged."""
    small, big = ModelConfig(max_groups=256), ModelConfig()
    a, b = synthetic_weights(small, seed=0), synthetic_weights(big, seed=0)
    assert big.max_groups == 640 and b["pos_emb"].shape == (640, 192)
    np.testing.assert_array_equal(a["pos_emb"], b["pos_emb"][:256])
    for name in a:
        if name != "pos_emb":
            np.testing.assert_array_equal(a[name], b[name])


def test_weights_bring_their_table_size(tmp_path):
    """Weights saved (or converted) with another positional-table size load into the default
    config, and config_for takes the capacity from the table (the engine's max_groups)."""
    from npe_pfn.weights import config_for

    small = ModelConfig(n_layers=1, n_bars=16, max_groups=8)
    w = synthetic_weights(small, seed=0)
    path = str(tmp_path / "w.npz")
    save_weights(path, w, small)
    cfg = ModelConfig(n_layers=1, n_bars=16)  # 640 rows by default
    w2 = load_weights(path, cfg)
    cfg2 = config_for(w2, cfg)
    assert cfg2.max_groups == 8 and cfg2.n_layers == 1
    np.testing.assert_array_equal(pack_weights(w, small), pack_weights(w2, cfg2))
    assert config_for(synthetic_weights(cfg, seed=0), cfg) is cfg
