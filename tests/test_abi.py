"""The C-ABI library loads on a CPU-only host and exports every entry point of include/npfn.h.

No compute calls are made here (no GPU); the GPU tests call through the same
symbols (tests/test_gpu_*.py).
"""
import ctypes
import os
import re

import pytest

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "npfn.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(npfn_[a-z_0-9]+)\s*\(", src)))


def test_header_declares_the_boundary():
    names = declared_functions()
    for must in ("npfn_engine_create", "npfn_fit", "npfn_predict", "npfn_bar_sample", "npfn_bar_nll",
                 "npfn_ar_sample", "npfn_ar_log_prob", "npfn_box_support", "npfn_compact_rows",
                 "npfn_filter_stdeuclid", "npfn_sir_select", "npfn_last_error"):
        assert must in names


def test_library_exports_every_declared_symbol():
    from npe_pfn.engine import LIB_PATH, SIGNATURES, load_library

    if not os.path.exists(LIB_PATH):
        pytest.fail("libnpfn.so is not built; run `make -C npe-pfn_amd` (__graft_entry__.build())")
    lib = load_library()
    for name in declared_functions():
        assert hasattr(lib, name), name
        assert name in SIGNATURES, f"{name} has no ctypes signature in npe_pfn/engine.py"
    assert lib.npfn_version() >= 1


def test_weights_size_matches_python_packing():
    import numpy as np

    from npe_pfn.engine import NpfnConfig, load_library
    from npe_pfn.weights import ModelConfig, pack_weights, synthetic_weights

    lib = load_library()
    for cfg in (ModelConfig(), ModelConfig(n_layers=2, n_bars=64, max_groups=16)):
        c = NpfnConfig(cfg.d_model, cfg.n_heads, cfg.n_layers, cfg.d_ff, cfg.n_bars, cfg.features_per_group,
                       cfg.max_groups, cfg.n_estimators, cfg.softmax_temperature, 0, 0)
        blob = pack_weights(synthetic_weights(cfg, seed=1), cfg)
        assert lib.npfn_weights_size(ctypes.byref(c)) == blob.size
        assert blob.dtype == np.float32


def test_config_struct_layout():
    from npe_pfn.engine import NpfnConfig, NpfnProfEntry

    assert ctypes.sizeof(NpfnConfig) == 48
    assert NpfnConfig.random_state.offset == 40
    assert ctypes.sizeof(NpfnProfEntry) == 48 + 8 + 8 + 8 + 8


def test_engine_fails_loudly_without_gpu():
    import torch

    from npe_pfn.engine import Engine, EngineError

    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(EngineError):
        Engine()


def test_regressor_rejects_unknown_kwargs_and_cpu_device():
    from npe_pfn.tabpfn import TabPFNRegressor

    with pytest.raises(TypeError):
        TabPFNRegressor(not_a_tabpfn_kwarg=1)
    reg = TabPFNRegressor(device="cpu")
    with pytest.raises((ValueError, RuntimeError)):
        reg.engine
