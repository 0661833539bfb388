"""Which tables the engine takes, checked before any C call (no GPU needed).

tabpfn's own input checks [ext: tabpfn 2.2.1 ``validate_Xy_fit``] refuse more than 10 000
context rows or 500 features unless ``ignore_pretraining_limits=True``; the estimator shims
(``npe_pfn/tabpfn.py``) raise the same ``ValueError`` here.  Past those, the engine's own
capacity (include/npfn.h, ``fit_prep`` in csrc/npfn_engine.hip) is raised as a ``ValueError``
naming the limit, before the C call would return ``NPFN_EINVAL``:

* feature groups of 2 per estimator <= the model's positional table (``ModelConfig.max_groups``,
  640 by default: tabpfn's 500 features under the default ensemble need at most 626) and tokens
  per row (groups + the target token) <= 1024 (``kWideMaxC``).  Rows of up to 256 tokens run the
  fused ``k_row_layer`` (whole rows in a 256-slot tile); wider estimator groups run the
  per-sublayer kernels with the long-row feature attention (``k_feat_attn_wide``);
* the ensemble's TruncatedSVD: the Gram matrix [2F, 2F] by the one-block Jacobi up to 256 features,
  the dual [n, n] up to 512 context rows, else the dense Gram matrix by rocSOLVER's dsyevd up to
  1024 features (``kSvdLargeMaxM`` = 2048; the 1024-token rows hold ~1000 input features anyway);
* quantile pipelines: sklearn's own ``ValueError`` when n_quantiles = n // 5 (n // 10 for the
  classifier's coarse transform) exceeds ``subsample`` = 10 000, and the engine's row
  subsample takes at most 65 536 context rows.
"""

from __future__ import annotations

MAX_NUMBER_OF_SAMPLES = 10_000   # tabpfn's pretraining limits [ext: tabpfn 2.2.1]
MAX_NUMBER_OF_FEATURES = 500
ROW_MAX_TOKENS = 256             # npfn_kernels.h kRowMaxC: the fused row kernel's tile
UNFUSED_MAX_TOKENS = 160 * 1024 // (576 * 2)  # kFeatAttnMaxC: k_feat_attn (longer rows: k_feat_attn_wide)
WIDE_MAX_TOKENS = 1024           # kWideMaxC
SVD_MAX_M = 512                  # kSvdMaxM: the Jacobi forms (Gram matrix or its n x n dual)
SVD_MAX_FEATURES = SVD_MAX_M // 2
SVD_LARGE_MAX_M = 2048           # kSvdLargeMaxM: the dsyevd form (2F > 512 and n > 512)
DEFAULT_MAX_GROUPS = 640         # weights.ModelConfig.max_groups
QT_SUBSAMPLE = 10_000            # kQtSubsample (sklearn's default subsample)
QT_SUBSAMPLE_MAX_ROWS = 65_536   # kQtSubsampleMaxRows
FP_BLOCK = 10_000                # kFpBlock: train rows per block of distinct fingerprint hashes

# feature pipelines (oracle/preprocess_oracle.py T_*, csrc/npfn_kernels.h)
T_RAW, T_QUANT, T_POWER, T_QSVD, T_PFP, T_RFP = 0, 1, 2, 3, 4, 5
MODES = {"none": 0, "quantile": 1, "quantile+power": 2, "ensemble": 3}


def check_pretraining_limits(n_rows: int, n_features: int, ignore_pretraining_limits: bool) -> None:
    """tabpfn's ``ValueError`` for more than 10 000 rows / 500 features [ext]."""
    if ignore_pretraining_limits:
        return
    if n_rows > MAX_NUMBER_OF_SAMPLES:
        raise ValueError(f"Number of samples {n_rows} in the input data is greater than the maximum number of samples "
                         f"{MAX_NUMBER_OF_SAMPLES} officially supported by TabPFN. Set "
                         "`ignore_pretraining_limits=True` to override this error!")
    if n_features > MAX_NUMBER_OF_FEATURES:
        raise ValueError(f"Number of features {n_features} in the input data is greater than the maximum number of "
                         f"features {MAX_NUMBER_OF_FEATURES} officially supported by the TabPFN model. Set "
                         "`ignore_pretraining_limits=True` to override this error!")


def pipeline_types(mode: int, classifier: bool):
    """The feature pipelines a preprocessing mode uses (any estimator count >= 2 uses all)."""
    if mode == 3:
        return (T_QSVD, T_RFP) if classifier else (T_QSVD, T_PFP)
    if mode == 2:
        return (T_QUANT, T_POWER)
    if mode == 1:
        return (T_QUANT, T_RAW)
    return (T_RAW,)


def svd_components(n_rows: int, n_features: int) -> int:
    return 0 if n_features < 2 else max(1, min(n_rows // 10 + 1, n_features // 2))


def pipeline_features(t: int, n_rows: int, n_features: int) -> int:
    if t == T_QSVD:
        return 2 * n_features + svd_components(n_rows, n_features) + 1
    if t in (T_PFP, T_RFP):
        return n_features + 1
    return n_features


def check_engine_table(n_rows: int, n_features: int, mode: int, classifier: bool = False,
                       max_groups: int = DEFAULT_MAX_GROUPS) -> None:
    """The engine's capacity for a fit on [n_rows, n_features] under preprocessing ``mode``
    (the checks of csrc/npfn_engine.hip ``fit_prep``, same order and limits)."""
    types = pipeline_types(mode, classifier)
    if T_QUANT in types or T_QSVD in types:
        div = 10 if (classifier and mode == 3) else 5
        nq = max(n_rows // div, 2)
        if nq > QT_SUBSAMPLE:
            raise ValueError(f"The number of quantiles cannot be greater than the number of samples used. Got {nq} "
                             f"quantiles and {QT_SUBSAMPLE} samples.")
        if n_rows > QT_SUBSAMPLE_MAX_ROWS:
            raise ValueError(f"the quantile preprocessing's row subsample takes at most {QT_SUBSAMPLE_MAX_ROWS} context "
                             f"rows ({n_rows} given)")
    if T_QSVD in types and n_features >= 2 and 2 * n_features > SVD_LARGE_MAX_M and n_rows > SVD_MAX_M:
        raise ValueError(f"the ensemble's SVD takes at most {SVD_LARGE_MAX_M // 2} features past {SVD_MAX_M} "
                         f"context rows ({n_features} features, {n_rows} rows given)")
    for t in types:
        fe = pipeline_features(t, n_rows, n_features)
        g = (fe + 1) // 2
        if g > max_groups:
            raise ValueError(f"an estimator's pipeline has {fe} features ({g} feature groups); the model's positional "
                             f"table holds {max_groups} groups ({2 * max_groups} features) per estimator")
        if g + 1 > WIDE_MAX_TOKENS:
            raise ValueError(f"an estimator's pipeline has {fe} features ({g + 1} tokens per row); the engine holds at "
                             f"most {2 * (WIDE_MAX_TOKENS - 1)} features ({WIDE_MAX_TOKENS} tokens) per estimator")


def max_ensemble_features(n_rows: int) -> int:
    """Largest feature count the default (ensemble) preprocessing takes at n_rows context rows."""
    f = 1
    while True:
        try:
            check_engine_table(n_rows, f + 1, 3)
        except ValueError:
            return f
        f += 1
