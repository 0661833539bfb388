"""Host-side logic that needs no GPU: when fits may be reused across accept/reject batches,
the tabpfn context-row limit, the boundary's default preprocessing mode, and EP argument
validation."""
import contextlib
import os
import re

import pytest
import torch

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")


class _RecordingModel:
    """Stands in for TabPFNRegressor: records whether reuse_fits was entered."""

    def __init__(self):
        self.entered = 0

    @contextlib.contextmanager
    def reuse_fits(self):
        self.entered += 1
        yield


@pytest.mark.parametrize("filter_type,expect", [("standardized_euclidean_filtering", True), ("no_filtering", True),
                                                ("latest_filtering", True), ("random_filtering", False),
                                                (lambda obs, th, x, k: (th, x), False)])
def test_fit_reuse_only_for_deterministic_contexts(filter_type, expect):
    """random_filtering draws a new context per accept/reject batch and the reference refits on
    each (npe_pfn.py:128 via support_posterior.py:351); a user callable is not known to be
    deterministic -- neither may share one fit token across batches."""
    from npe_pfn import TabPFN_Based_NPE_PFN

    post = TabPFN_Based_NPE_PFN(filter_type=filter_type)
    post._model = _RecordingModel()
    with post._reuse_fits():
        pass
    assert post._model.entered == (1 if expect else 0)


def test_core_context_reuses_fits():
    from npe_pfn import NPE_PFN_Core

    core = NPE_PFN_Core()
    core._model = _RecordingModel()
    with core._reuse_fits():
        pass
    assert core._model.entered == 1


def test_context_row_limit_is_tabpfns():
    """More than 10 000 context rows: tabpfn's ValueError before any engine call, unless
    ignore_pretraining_limits=True (then the engine is asked, and needs a GPU here)."""
    from npe_pfn.tabpfn import TabPFNClassifier, TabPFNRegressor

    X = torch.zeros(10_001, 2)
    y = torch.zeros(10_001)
    with pytest.raises(ValueError, match="ignore_pretraining_limits"):
        TabPFNRegressor().fit(X, y)
    with pytest.raises(ValueError, match="ignore_pretraining_limits"):
        TabPFNRegressor().ar_sample(X, y[:, None], X[:4])
    with pytest.raises(ValueError, match="ignore_pretraining_limits"):
        TabPFNClassifier().fit(X, torch.arange(10_001) % 2)
    reg = TabPFNRegressor(ignore_pretraining_limits=True)
    assert reg.ignore_pretraining_limits
    if not torch.cuda.is_available():
        with pytest.raises(RuntimeError):  # past the limit check: the engine needs a GPU
            reg.fit(X, y)


def test_default_preprocessing_agrees_across_the_boundary():
    """TabPFNRegressor, Engine, the C engine (npfn_engine_create) and the INTEGRATION stub all
    start in tabpfn's ensemble (mode 3)."""
    import inspect

    from npe_pfn.engine import Engine
    from npe_pfn.tabpfn import TabPFNRegressor

    assert TabPFNRegressor().preprocessing == "ensemble"
    assert inspect.signature(Engine.__init__).parameters["preprocessing"].default == "ensemble"
    assert Engine.DEFAULT_PREPROCESSING == "ensemble" and Engine.PREPROCESSING_MODES["ensemble"] == 3
    src = open(os.path.join(ROOT, "npe-pfn_amd", "csrc", "npfn_engine.hip")).read()
    create = src[src.index("int npfn_engine_create("):]
    assert re.search(r"apply_preprocessing\(h, 3\)", create[:2000])
    hdr = open(os.path.join(ROOT, "include", "npfn.h")).read()
    assert "mode 3 (the DEFAULT of a new engine)" in hdr
    integ = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    assert "npfn_set_preprocessing(h, 3)" in integ


def test_ep_size_must_divide_world_and_estimators():
    from npe_pfn.distributed import sample_estimator_parallel

    class _Eng:
        class cfg:
            n_estimators = 8

    class _Reg:
        engine = _Eng()

    class _Post:
        _model = _Reg()

    with pytest.raises(ValueError, match="ep_size"):
        sample_estimator_parallel(_Post(), torch.zeros(1, 2), (10,), ep_size=3)


def test_packed_weight_blobs_cached_per_weight_set():
    """engine._packed: one pack_weights per weight dict (the blob is reused by every engine built
    from that dict, e.g. the regressor and classifier engines of each run_tsnpe_pfn round), a new
    blob for another dict, and at most _PACK_CACHE_MAX entries."""
    import numpy as np

    from npe_pfn import engine as E
    from npe_pfn.weights import ModelConfig, synthetic_weights

    cfg = ModelConfig(n_layers=1)
    w0 = synthetic_weights(cfg, seed=0)
    w1 = synthetic_weights(cfg, seed=1)
    E._PACK_CACHE.clear()
    b0 = E._packed(w0, cfg)
    assert E._packed(w0, cfg) is b0
    b1 = E._packed(w1, cfg)
    assert b1 is not b0 and not np.array_equal(b0, b1)
    np.testing.assert_array_equal(b0, E.pack_weights(w0, cfg))
    extra = [synthetic_weights(cfg, seed=s) for s in range(2, 2 + E._PACK_CACHE_MAX)]
    for w in extra:
        E._packed(w, cfg)
    assert len(E._PACK_CACHE) <= E._PACK_CACHE_MAX
    E._PACK_CACHE.clear()


def test_c2_logprob_fixture_is_the_c2_task():
    """tests/golden/c2_logprob.npz (the c2-size AR log-prob golden, make_golden_c2_logprob.py)
    holds exactly the c2 context npe_pfn.tasks generates, and finite per-step densities with
    the far-tail query in the half-normal end bars."""
    import numpy as np

    from npe_pfn.tasks import gaussian_linear_task

    g = np.load(os.path.join(os.path.dirname(__file__), "golden", "c2_logprob.npz"))
    theta, x, x_o = (t.numpy() for t in gaussian_linear_task(10, 1000, seed=0))
    assert np.array_equal(g["theta"], theta) and np.array_equal(g["x"], x)
    assert np.array_equal(g["xq"], np.repeat(x_o, g["tq"].shape[0], 0))
    assert g["steps"].shape == (10, g["tq"].shape[0]) and np.isfinite(g["steps"]).all()
    assert g["steps"][:, -1].sum() < -100 < g["steps"][:, :-1].sum(0).min()
