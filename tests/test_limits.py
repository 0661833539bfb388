"""Where each remaining cap on the tables the engine takes sits, and its message (CPU).

npe_pfn.limits mirrors csrc/npfn_engine.hip ``fit_prep``: the constants are parsed from
csrc/npfn_kernels.h so the two cannot drift; every cap raises a ValueError naming it before
any C call (tabpfn's own 10 000-row / 500-feature errors first, then the engine's).
Reference: the reference's published workload of notebooks/sampling_comparison.ipynb:85-106
(theta 2-D, x 50-D, 100 simulations) fits 50 and 51 features (npe_pfn.py:140-143).
"""
import os
import re

import pytest
import torch

from npe_pfn import limits

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = open(os.path.join(ROOT, "npe-pfn_amd", "csrc", "npfn_kernels.h")).read()


def _const(name):
    m = re.search(rf"constexpr int {name} = ([^;]+);", HDR)
    assert m, name
    return int(eval(m.group(1)))


def test_constants_match_the_engine_header():
    from npe_pfn.weights import ModelConfig

    assert _const("kRowMaxC") == limits.ROW_MAX_TOKENS
    assert _const("kFeatAttnMaxC") == limits.UNFUSED_MAX_TOKENS
    assert _const("kWideMaxC") == limits.WIDE_MAX_TOKENS
    assert _const("kSvdMaxM") == limits.SVD_MAX_M == 2 * limits.SVD_MAX_FEATURES
    assert _const("kSvdLargeMaxM") == limits.SVD_LARGE_MAX_M
    assert _const("kQtSubsample") == limits.QT_SUBSAMPLE
    assert _const("kQtSubsampleMaxRows") == limits.QT_SUBSAMPLE_MAX_ROWS
    assert _const("kFpBlock") == limits.FP_BLOCK
    assert ModelConfig().max_groups == limits.DEFAULT_MAX_GROUPS


def test_reference_sampling_comparison_shape_is_accepted():
    """theta 2-D / x 50-D, 100 simulations: 50 and 51 features under every preprocessing mode."""
    for mode in range(4):
        for F in (50, 51):
            limits.check_engine_table(100, F, mode)
            limits.check_engine_table(100, F, mode, classifier=True)
    # its widest estimator: 2 * 51 + 11 SVD components + fingerprint = 114 features, 58 tokens
    assert limits.pipeline_features(limits.T_QSVD, 100, 51) == 114


def test_wide_tables_under_the_ensemble():
    """The ensemble's quantile + original + SVD pipeline has 2F + k + 1 features.  Up to 256 tokens
    per row (510 features) an estimator runs the fused row kernel; wider ones the per-sublayer
    path with the long-row feature attention.  tabpfn's own maximum, 500 features, fits under the
    ensemble at any context size the SVD takes: 2 * 500 + 250 + 1 = 1251 features, 626 groups of
    the 640-row positional table."""
    assert limits.pipeline_features(limits.T_QSVD, 1000, 204) == 510   # the r04 cap, now the fused one
    assert limits.pipeline_features(limits.T_QSVD, 100, 500) == 1012
    for n in (100, 512, 1000, 10_000):
        limits.check_engine_table(n, 500, 3)
        limits.check_engine_table(n, 500, 3, classifier=True)
    # the model's positional table, not the engine, is the cap: 2F + k + 1 features in 640 groups
    assert limits.max_ensemble_features(100) == 634
    assert limits.max_ensemble_features(1000) == 589
    assert limits.max_ensemble_features(10_000) == 511
    # "none": one feature per token slot pair; past the positional table the message names it
    limits.check_engine_table(1000, 1280, 0)
    with pytest.raises(ValueError, match=r"positional table holds 640 groups"):
        limits.check_engine_table(1000, 1281, 0)
    with pytest.raises(ValueError, match=r"positional table holds 16 groups"):
        limits.check_engine_table(100, 40, 3, max_groups=16)
    # a larger table: the engine's own cap, 1024 tokens per row
    with pytest.raises(ValueError, match=r"\(1024 tokens\)"):
        limits.check_engine_table(1000, 2047, 0, max_groups=4096)


def test_quantile_caps():
    """sklearn's own check: n_quantiles = n // 5 may not exceed subsample = 10 000 (n // 10 for
    the classifier's coarse transform); the row subsample's index array holds 65 536 rows."""
    limits.check_engine_table(50_004, 10, 1)
    with pytest.raises(ValueError, match="10001 quantiles and 10000 samples"):
        limits.check_engine_table(50_005, 10, 1)
    with pytest.raises(ValueError, match="10001 quantiles"):
        limits.check_engine_table(50_005, 10, 3)
    limits.check_engine_table(65_536, 10, 3, classifier=True)
    with pytest.raises(ValueError, match="at most 65536 context rows"):
        limits.check_engine_table(65_537, 10, 3, classifier=True)
    limits.check_engine_table(1_000_000, 10, 0)  # no quantile pipeline: no row cap
    limits.check_engine_table(1_000_000, 10, 2 - 2)


def test_svd_cap():
    """The Gram matrix [2F, 2F] by the one-block Jacobi up to 256 features, its n x n dual up to 512
    context rows, else the dense Gram matrix by dsyevd up to 1024 features."""
    limits.check_engine_table(10_000, 256, 3, max_groups=4096)
    limits.check_engine_table(512, 900, 3, max_groups=4096)
    limits.check_engine_table(513, 960, 3, max_groups=4096)
    with pytest.raises(ValueError, match="SVD takes at most 1024 features past 512 context rows"):
        limits.check_engine_table(513, 1025, 3, max_groups=4096)


def test_tabpfn_pretraining_limits():
    limits.check_pretraining_limits(10_000, 500, False)
    with pytest.raises(ValueError, match="Number of samples 10001"):
        limits.check_pretraining_limits(10_001, 5, False)
    with pytest.raises(ValueError, match="Number of features 501"):
        limits.check_pretraining_limits(100, 501, False)
    limits.check_pretraining_limits(20_000, 600, True)


def test_estimator_shims_check_features_before_the_engine():
    from npe_pfn.tabpfn import TabPFNRegressor

    X = torch.zeros(100, 501)
    with pytest.raises(ValueError, match="Number of features 501"):
        TabPFNRegressor().fit(X, torch.zeros(100))
    with pytest.raises(ValueError, match="Number of features 501"):
        TabPFNRegressor().ar_sample(torch.zeros(100, 500), torch.zeros(100, 2), torch.zeros(4, 500))
