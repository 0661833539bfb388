"""Which tables the engine takes, checked before any C call (no GPU needed).

tabpfn's own input checks [ext: tabpfn 2.2.1 ``validate_Xy_fit``] refuse more than 10 000
context rows or 500 features unless ``ignore_pretraining_limits=True``; the estimator shims
(``npe_pfn/tabpfn.py``) raise the same ``ValueError`` here.  Past those, the engine's own
capacity (include/npfn.h, ``fit_prep`` in csrc/npfn_engine.hip) is raised as a ``ValueError``
naming the limit, before the C call would return ``NPFN_EINVAL``:

* tokens per row (feature groups of 2 + the target token) <= 256: ``k_row_layer`` holds whole
  rows in a 256-slot tile (142 on the unfused ``NPFN_UNFUSED=1`` path);
* the ensemble's TruncatedSVD takes at most 256 features (its Gram matrix is [2F, 2F]);
* quantile pipelines: sklearn's own ``ValueError`` when n_quantiles = n // 5 (n // 10 for the
  classifier's coarse transform) exceeds ``subsample`` = 10 000, and the engine's row
  subsample takes at most 65 536 context rows.
"""

from __future__ import annotations

MAX_NUMBER_OF_SAMPLES = 10_000   # tabpfn's pretraining limits [ext: tabpfn 2.2.1]
MAX_NUMBER_OF_FEATURES = 500
ROW_MAX_TOKENS = 256             # npfn_kernels.h kRowMaxC
UNFUSED_MAX_TOKENS = 160 * 1024 // (576 * 2)  # kFeatAttnMaxC
SVD_MAX_FEATURES = 256           # 2F <= kSvdMaxM = 512
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


def check_engine_table(n_rows: int, n_features: int, mode: int, classifier: bool = False, fused: bool = True) -> None:
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
    if T_QSVD in types and n_features >= 2 and n_features > SVD_MAX_FEATURES:
        raise ValueError(f"the ensemble's SVD takes at most {SVD_MAX_FEATURES} features ({n_features} given)")
    cmax = ROW_MAX_TOKENS if fused else UNFUSED_MAX_TOKENS
    for t in types:
        fe = pipeline_features(t, n_rows, n_features)
        c = (fe + 1) // 2 + 1
        if c > cmax:
            raise ValueError(f"an estimator's pipeline has {fe} features ({c} tokens per row); the engine holds at most "
                             f"{2 * (cmax - 1)} features ({cmax} tokens) per estimator")


def max_ensemble_features(n_rows: int) -> int:
    """Largest feature count the default (ensemble) preprocessing takes at n_rows context rows."""
    f = 1
    while True:
        try:
            check_engine_table(n_rows, f + 1, 3)
        except ValueError:
            return f
        f += 1
