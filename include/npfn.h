/*
 * npfn.h -- C-ABI of the MI355X NPE-PFN engine (libnpfn.so).
 *
 * Drop-in boundary: the reference reaches this arithmetic through the
 * tabpfn estimator object held by NPE_PFN_Core (npe_pfn/npe_pfn.py:48,69;
 * tabpfn==2.2.1, poetry.lock:4455-4464).  Each entry point below replaces one
 * call the reference makes on it; the Python host package
 * (npe-pfn_amd/npe_pfn/tabpfn.py) binds them with ctypes, and INTEGRATION.md
 * shows the binding a maintainer would add to the reference.
 *
 * Conventions
 *  - every function returns 0 on success, a negative NPFN_E* code on failure;
 *    npfn_last_error() returns the thread-local message of the last failure;
 *  - all float/int buffers are DEVICE pointers owned by the caller (e.g.
 *    torch tensors' data_ptr()), row-major, float32 unless stated;
 *  - `stream` is a hipStream_t (NULL = legacy default stream); work is
 *    stream-ordered and asynchronous unless stated;
 *  - one engine handle per (device, thread); concurrent use of a handle is
 *    undefined (the reference is single-threaded).
 */
#ifndef NPFN_H
#define NPFN_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define NPFN_OK 0
#define NPFN_EINVAL (-1)   /* bad argument or shape */
#define NPFN_EHIP (-2)     /* HIP runtime error */
#define NPFN_ESTATE (-3)   /* call out of order (e.g. predict before fit) */
#define NPFN_ENOMEM (-4)   /* device allocation failed */

typedef struct npfn_engine npfn_engine; /* opaque */

typedef struct npfn_config {
  int32_t d_model;            /* 192  [ext: tabpfn v2 regressor emsize] */
  int32_t n_heads;            /* 6    (head_dim must be 32) */
  int32_t n_layers;           /* 12 */
  int32_t d_ff;               /* 768 */
  int32_t n_bars;             /* 5000 Riemann bars */
  int32_t features_per_group; /* 2 */
  int32_t max_groups;         /* rows of the positional-embedding table */
  int32_t n_estimators;       /* 8  (TabPFNRegressor(n_estimators=...)) */
  float softmax_temperature;  /* 0.9 (TabPFNRegressor(softmax_temperature=...)) */
  int32_t device;             /* HIP device ordinal */
  uint64_t random_state;      /* TabPFNRegressor(random_state=...): feature
                                 permutations and the Philox key of sampling */
} npfn_config;

/* Library identity. */
int npfn_version(void);
const char* npfn_last_error(void);

/* Number of float32 values in the weight blob for `cfg` (layout: named tensors
 * in the order of npe_pfn/weights.py::weight_names, each [out, in] row-major). */
size_t npfn_weights_size(const npfn_config* cfg);

/* Create / destroy an engine.  `weights` is a HOST pointer to the blob; it is
 * converted (bf16 for GEMM weights) and uploaded once.  Replaces
 * `TabPFNRegressor(**regressor_init_kwargs)` (npe_pfn.py:48, :69). */
int npfn_engine_create(const npfn_config* cfg, const float* weights, size_t n_weights,
                       npfn_engine** out);
int npfn_engine_destroy(npfn_engine* h);

/* Per-estimator preprocessing of the feature columns, applied from the next fit on.
 * mode 3 (the DEFAULT of a new engine): tabpfn's default preprocessing ensemble [ext:
 * tabpfn 2.2.1, reached from TabPFNRegressor(**regressor_init_kwargs), npe_pfn.py:48;
 * restated in oracle/preprocess_oracle.py, parity pinned to that restatement and to
 * sklearn / hashlib only]: estimators 0-3 quantile-uniform features appended to the
 * original ones plus a TruncatedSVD of both, estimators 4-7 Yeo-Johnson features, every
 * estimator a SHA-256 fingerprint feature, every second estimator of each pipeline a
 * Yeo-Johnson transform of the target.  Table caps (npfn_fit returns NPFN_EINVAL past
 * them, npfn_last_error() naming the cap; npe_pfn/limits.py checks the same in Python):
 * at most max_groups feature groups per estimator row (2 features each; the default table has
 * 640 rows: tabpfn's 500 features under the ensemble need 626) and 1024 tokens; rows of up to
 * 256 tokens run the fused row kernel, wider estimator groups the per-sublayer kernels with the
 * long-row feature attention (memory: a wide group's train forward holds ~4.2 KB of per-sublayer
 * workspace per token -- E * n * C * 4.2 KB, ~26 GB per estimator group at 10 000 rows x 627
 * tokens -- plus its K/V cache; tested on the GPU up to 1 000 context rows x 298 features and
 * 100 rows x 500 features; past the device's memory npfn_fit returns NPFN_ENOMEM naming the
 * failed allocation); the SVD on at most 1024 features (a one-block Jacobi up to 256,
 * the n x n dual up to 512 context rows, else rocSOLVER dsyevd); for the quantile pipelines
 * sklearn's n_quantiles (n/5, the classifier's n/10) <= its 10000-row subsample, the
 * subsample itself from at most 65536 rows.  Above
 * 10000 context rows the quantile fit uses sklearn's 10000-row subsample and the train
 * fingerprints are made distinct among the 10000 hash buckets within blocks of 10000 rows
 * (tabpfn itself refuses more than 10000 rows unless ignore_pretraining_limits=True).
 * For npfn_fit_classes mode 3 is the
 * classifier's ensemble (quantile-uniform + original + SVD on every estimator, with the
 * fingerprint; the class shuffle is always on).
 * mode 0: standardization only -- NOT tabpfn's default; kept for the reference-anchored
 * golden fixtures.  mode 1: sklearn QuantileTransformer (uniform, n_quantiles =
 * max(n/5, 2)) on even estimators (`PreprocessorConfig("quantile_uni")`).  mode 2: mode 1
 * plus the Yeo-Johnson power transform (sklearn PowerTransformer, lambda by maximum
 * likelihood) on odd estimators ("safepower"); the quantile caps as for mode 3.
 * Invalidates the fit. */
int npfn_set_preprocessing(npfn_engine* h, int32_t mode);

/* TabPFNRegressor / TabPFNClassifier(average_before_softmax=...) [ext: tabpfn 2.2.1, reached
 * through regressor_init_kwargs / classifier_init_kwargs, npe_pfn.py:45-48, 610]: 0 (default)
 * mixes the ensemble as the mean of the estimators' probabilities; 1 as softmax(mean_e log q_e)
 * -- the estimators' (border-translated) log probabilities averaged, then renormalized; for the
 * classifier the estimators' class logits averaged, then softmax.  Applies from the next
 * predict / predict_proba / AR call on; the fit is kept. */
int npfn_set_average_before_softmax(npfn_engine* h, int32_t enable);

/* Fit: X [n_ctx, n_features] (row stride ldx), y [n_ctx] (element stride ldy).
 * Computes target standardization, per-estimator preprocessing and the
 * train-side forward (item-attention K/V cache of every layer).
 * Errors: NPFN_EINVAL past a table cap (npfn_set_preprocessing); NPFN_ENOMEM when a workspace
 * does not fit; NPFN_EHIP for a HIP error, or when the wide-table SVD's rocSOLVER dsyevd reports
 * no convergence (its info flag is checked before its vectors are used; that path alone waits on
 * the stream).
 * Replaces `self._model.fit(joint[:, :F], joint[:, F])` (npe_pfn.py:140,215,502). */
int npfn_fit(npfn_engine* h, const float* X, int64_t ldx, const float* y, int64_t ldy,
             int64_t n_ctx, int32_t n_features, void* stream);

/* Predict: Xq [n_rows, n_features of the last fit] (row stride ldq) ->
 * logits [n_rows, n_bars] = log of the ensemble-mean bar probabilities.
 * Replaces `predict(X, output_type="full", quantiles=[])["logits"]`
 * (npe_pfn.py:143-145, 217-219, 505-507). */
int npfn_predict(npfn_engine* h, const float* Xq, int64_t ldq, int64_t n_rows, float* logits,
                 void* stream);

/* Classifier fit (TabPFNClassifier.fit, npe_pfn.py:661): X [n_ctx, n_features],
 * y [n_ctx] = label INDICES 0..n_classes-1 as float (the host label-encodes, as
 * sklearn's LabelEncoder does in tabpfn).  The engine must have been created
 * with a classifier weight blob (decoder width cfg.n_bars >= n_classes; the
 * v2 classifier has 10).  Per estimator the labels are permuted; the train-side
 * forward fills the item-attention K/V cache exactly as npfn_fit does. */
int npfn_fit_classes(npfn_engine* h, const float* X, int64_t ldx, const float* y, int64_t ldy,
                     int64_t n_ctx, int32_t n_features, int32_t n_classes, void* stream);

/* Classifier probabilities: probs [n_rows, n_classes] = estimator mean of
 * softmax(class logits / T), in label-index order.  Replaces
 * `self._classifier.predict_proba(theta[mask])` (npe_pfn.py:697). */
int npfn_predict_proba(npfn_engine* h, const float* Xq, int64_t ldq, int64_t n_rows, float* probs,
                       void* stream);

/* Borders [n_bars + 1] of the last fit's criterion (standardized borders *
 * y_std + y_mean): the `criterion` half of predict(...)["criterion"]. */
int npfn_get_borders(npfn_engine* h, float* borders, void* stream);

/* criterion.sample(logits) (npe_pfn.py:146, 220): inverse-CDF sample of each
 * row with u = Philox4x32-10(counter=(row, counter), key=seed). */
int npfn_bar_sample(const float* logits, const float* borders, int64_t n_rows, int32_t n_bars,
                    uint64_t seed, uint64_t counter, float* out, void* stream);

/* criterion(logits, y) (npe_pfn.py:149, 226, 510): full-support bar NLL. */
int npfn_bar_nll(const float* logits, const float* borders, const float* y, int64_t n_rows,
                 int32_t n_bars, float* out, void* stream);

/* Fused autoregressive sampler: the whole `for param_idx in range(dim_theta)`
 * loop of NPE_PFN_Core._sample / _sample_batched (npe_pfn.py:135-169,
 * 211-241) on the device.  x_ctx [n_ctx, dim_x], theta_ctx [n_ctx, dim_theta]
 * (context), x_query [n_rows, dim_x] (already repeated / interleaved).
 * Step k uses Philox counter `counter + k`; query row i draws its uniform at
 * Philox row `row_base + i`, so a batch split into shards (rows [a, b) with
 * row_base = a, e.g. one observation shard per GPU) draws exactly the numbers
 * of the unsplit batch.  Writes theta_out [n_rows,
 * dim_theta] and, if log_prob_out != NULL, the summed per-step log densities
 * with -inf replaced by log(eps) (npe_pfn.py:148-159). */
int npfn_ar_sample(npfn_engine* h, const float* x_ctx, const float* theta_ctx, int64_t n_ctx,
                   int32_t dim_x, int32_t dim_theta, const float* x_query, int64_t n_rows,
                   uint64_t counter, int64_t row_base, float* theta_out, float* log_prob_out,
                   float eps, void* stream);

/* npfn_ar_sample over repeated query rows: x_unique [n_unique, dim_x] holds the distinct rows
 * and query row i is x_unique[i / (n_rows / n_unique)] (n_unique divides n_rows) -- the
 * `x.repeat(batch, 1)` of one observation (npe_pfn.py:122, n_unique = 1) and the obs-major
 * `x.repeat_interleave(n, 0)` of sample_batched (npe_pfn.py:199).  AR step 0, whose features
 * are the query rows alone, runs the forward, decoder and ensemble mix once per distinct row;
 * every row then draws from its row's mixture with its own uniform.  Same results as
 * npfn_ar_sample on the repeated rows, bit for bit: the forward is batch-invariant (a row's
 * result does not depend on its slot in the row kernel's token tile). */
int npfn_ar_sample_repeated(npfn_engine* h, const float* x_ctx, const float* theta_ctx, int64_t n_ctx,
                            int32_t dim_x, int32_t dim_theta, const float* x_unique, int64_t n_unique,
                            int64_t n_rows, uint64_t counter, int64_t row_base, float* theta_out,
                            float* log_prob_out, float eps, void* stream);

/* Teacher-forced autoregressive log density (npe_pfn.py:462-524):
 * log_prob_out [n_rows] = sum_k -NLL_k(theta[:, k] | x, theta[:, :k]). */
int npfn_ar_log_prob(npfn_engine* h, const float* x_ctx, const float* theta_ctx, int64_t n_ctx,
                     int32_t dim_x, int32_t dim_theta, const float* x_query, const float* theta,
                     int64_t n_rows, float* log_prob_out, float eps, void* stream);

/* npfn_ar_log_prob over repeated query rows (the `x.repeat(num_samples, 1)` of npe_pfn.py:480):
 * x_unique [n_unique, dim_x], query row i = x_unique[i / (n_rows / n_unique)]; step 0 runs once
 * per distinct row and every row's theta is scored under its row's mixture, which is the
 * repeated rows' own (the forward is batch-invariant). */
int npfn_ar_log_prob_repeated(npfn_engine* h, const float* x_ctx, const float* theta_ctx, int64_t n_ctx,
                              int32_t dim_x, int32_t dim_theta, const float* x_unique, int64_t n_unique,
                              const float* theta, int64_t n_rows, float* log_prob_out, float eps,
                              void* stream);

/* K9: prior-support check of a box prior (npe_pfn.py:581-600 with
 * BoxUniform): mask[i] = all_j(low_j <= theta[i,j] <= high_j). */
int npfn_box_support(const float* theta, int64_t n_rows, int32_t dim, const float* low,
                     const float* high, uint8_t* mask, void* stream);

/* K9/K10 stream compaction: rows of src [n_rows, dim] with mask != 0 are
 * written in order to dst; *count_out (device int64) receives the count. */
int npfn_compact_rows(const float* src, const uint8_t* mask, int64_t n_rows, int32_t dim,
                      float* dst, int64_t* count_out, void* stream);

/* K12 standardized-Euclidean context filter (support_posterior.py:357-369):
 * idx_out[0:k] = indices of the k rows of x [n_rows, dim] closest to obs in
 * z-scored Euclidean distance, ascending (ties by lower index). */
int npfn_filter_stdeuclid(const float* x, int64_t n_rows, int32_t dim, const float* obs, int64_t k,
                          int64_t* idx_out, void* stream);

/* K11 SIR resampling step of PosteriorSupport.sample_sir (support_posterior.py:
 * 216-241).  lpr, lq [n_groups * k]: prior / posterior log densities of the
 * proposals, group g = rows g*k .. g*k+k-1; thr: DEVICE float (the lq quantile).
 * Per group: log_ratio = nan_to_num(lpr - lq, nan=-inf) with lpr := -inf where
 * lq < *thr; ess_out[g] = 1 / sum softmax(log_ratio)^2; pick_out[g] = inverse-CDF
 * index of softmax(log_ratio) at u = Philox4x32-10(counter=(group_offset + g,
 * counter), key=seed).  If theta_out != NULL, theta_out[g, :] = theta[g*k + pick, :]
 * (theta [n_groups * k, dim]). */
int npfn_sir_select(const float* lpr, const float* lq, const float* thr, int64_t n_groups, int32_t k,
                    uint64_t seed, uint64_t counter, int64_t group_offset, const float* theta,
                    int32_t dim, int64_t* pick_out, float* ess_out, float* theta_out, void* stream);

/* Estimator-parallel split (npe_pfn/distributed.py): from the next fit on,
 * fits and forwards compute only estimators [e0, e0 + count) of cfg.n_estimators (the
 * feature permutation and preprocessing of estimator e are the same as in the full
 * ensemble).  Calls that mix the ensemble (predict, predict_proba, ar_sample, ar_log_prob,
 * fit_classes) need the full range (0, n_estimators).  Invalidates the fit. */
int npfn_set_estimator_range(npfn_engine* h, int32_t e0, int32_t count);
/* The strided generalisation: fits and forwards compute estimators e0 + stride * i,
 * i < count (npfn_set_estimator_range = stride 1).  npfn_forward_targets writes their target
 * tokens in that order.  Estimator-parallel sampling gives rank r of an EP group of g ranks
 * the set (r, E / g, g), so that every rank holds the same mix of the ensemble's
 * preprocessing pipelines (the ensemble mode's estimators 0-3 and 4-7 differ in token
 * count by about 2x, which a contiguous split would put on different ranks). */
int npfn_set_estimator_set(npfn_engine* h, int32_t e0, int32_t count, int32_t stride);

/* The test-side forward of the estimator range over Xq [n_rows, n_features of the last
 * fit]: tokens_out (bf16, [count][n_rows][192]) = the last layer's target token of every
 * (estimator, row) -- the decoder input of predict (npe_pfn.py:143 up to the head). */
int npfn_forward_targets(npfn_engine* h, const float* Xq, int64_t ldq, int64_t n_rows, void* tokens_out,
                         void* stream);

/* Decoder head + ensemble mix + criterion.sample (+ NLL) of one autoregressive step
 * (npe_pfn.py:143-159) from the target tokens of ALL estimators: tokens (bf16,
 * [n_est][n_rows][192], n_est = cfg.n_estimators).  theta_out [n_rows]; row i draws
 * Philox row row_base + i at `counter`; if log_prob_acc != NULL its row i gets the step's
 * log density added (-inf -> log(eps)).  npfn_forward_targets + this = one step of
 * npfn_ar_sample, bit for bit. */
int npfn_head_sample(npfn_engine* h, const void* tokens, int32_t n_est, int64_t n_rows, uint64_t counter,
                     int64_t row_base, float* theta_out, float* log_prob_acc, float eps, void* stream);

/* The per-step fits of an autoregressive call driven step by step (the fit of
 * npe_pfn.py:135-140 for AR dimension k = fit on (x_ctx, theta_ctx[:, :k]) -> theta_ctx[:, k]),
 * for callers that run the steps themselves (estimator-parallel sampling: npfn_forward_targets
 * + an exchange + npfn_head_sample per step).  npfn_ar_fit_begin copies the context and, under
 * a fit token (npfn_set_fit_token), queues every step's preprocessing fit on the engine's side
 * stream at once (they read only the context); npfn_ar_fit_step(k) then makes step k's fit the
 * current one (its train forward after its preprocessing, or nothing when an earlier call under
 * the same token fitted it).  Without a token, step k is fitted in order on `stream`.  The
 * results equal npfn_fit(x_ctx | theta_ctx[:, :k], theta_ctx[:, k]) bit for bit. */
int npfn_ar_fit_begin(npfn_engine* h, const float* x_ctx, const float* theta_ctx, int64_t n_ctx, int32_t dim_x,
                      int32_t dim_theta, void* stream);
int npfn_ar_fit_step(npfn_engine* h, int32_t k, void* stream);

/* Fit reuse across calls (the reference refits inside every accept/reject batch,
 * npe_pfn.py:135-140 reached from accept_reject_sampler.py:51; the fit is deterministic):
 * while token != 0, npfn_ar_sample / npfn_ar_log_prob keep the fit of every AR step and
 * the next call with the same token, context shape, mode and estimator range uses them
 * instead of refitting.  The caller promises that the context (x_ctx, theta_ctx) is the
 * same for all calls under one token -- e.g. one token per sample() call.  0 (default)
 * refits every call.  npfn_fit / npfn_fit_classes never touch the cached fits. */
int npfn_set_fit_token(npfn_engine* h, uint64_t token);

/* Query rows per forward chunk of npfn_predict / npfn_predict_proba / npfn_ar_sample /
 * npfn_ar_log_prob (default 16384).  The reference runs one `predict` over every query
 * row (960 000 at config c5, npe_pfn.py:199, 211-241); the engine splits it into chunks
 * of this many rows to bound its workspaces.  Results do not depend on it beyond
 * floating-point summation order (tests cross the chunk boundaries this way). */
int npfn_set_chunk_rows(npfn_engine* h, int64_t rows);

/* Live per-kernel timing for bench.py: while enabled, every launch the engine
 * makes is bracketed by a HIP event pair on its stream; npfn_prof_read
 * synchronizes, returns per-kernel-function totals (launch count, summed
 * duration, algorithmic FLOPs and bytes) and resets the record.  While enabled, the AR
 * calls' fits run in order on the caller's stream instead of on the side streams, so that
 * every event pair times its launch alone (same results, less overlap). */
typedef struct npfn_prof_entry {
  char name[48];
  int64_t launches;
  double ms;
  double flops;
  double bytes;
} npfn_prof_entry;

int npfn_prof_enable(npfn_engine* h, int enable);
int npfn_prof_read(npfn_engine* h, npfn_prof_entry* out, int32_t max_entries, int32_t* n_entries);

/* Diagnostics: copies the first `rows` rows of the preprocessed table of the last fit or
 * forward ([rows][*vw_out] float32: raw | quantile | SVD | power | fingerprints, see
 * npfn_kernels.h ViewLayout) to the HOST buffer out (capacity rows * max_cols floats).
 * Synchronous.  Used by the tests to pin the device SVD and SHA-256 fingerprints. */
int npfn_debug_views(npfn_engine* h, float* out, int64_t rows, int32_t max_cols, int32_t* vw_out);

/* Diagnostics (process-wide): enable != 0 makes every item-attention block run its
 * online-softmax pass as well (the fallback of the reference-free first pass), so the
 * tests can compare both.  Off by default. */
int npfn_debug_item_attn_online(int enable);

/* Diagnostics (process-wide): every item-attention score is multiplied by scale (> 0; 1 by
 * default) -- stress runs that push queries out of the reference-free first pass's range
 * (bench.py --ia-stress).  Changes results; never set on a sampling path. */
int npfn_debug_item_attn_scale(float scale);

/* Diagnostics: the engine's n-th next row-kernel launch (n >= 1; 0 = off) is refused by the
 * HIP runtime (an oversized block; nothing runs on the device).  The call that hits one returns
 * NPFN_EHIP and leaves the engine usable: the stream's tile counter is not advanced for a
 * launch that did not go in, so later calls compute every tile (tests/test_gpu_engine.py). */
int npfn_debug_fail_row_launch(npfn_engine* h, int32_t n);

/* Item-attention fallback accounting of this engine since the last reset: out4[0] blocks that
 * ran the online-softmax pass, out4[1] blocks launched, out4[2] query rows that took the online
 * pass's result, out4[3] query rows ((token, head) queries / 32 lanes: ny * R per launch).
 * HOST output, synchronous; reset != 0 clears the counters.  Reference call of the path:
 * npe_pfn.py:143 (predict) -- the first pass is exact while every query's row sum stays in
 * [2^-100, 2^100]. */
int npfn_item_attn_fallback(npfn_engine* h, uint64_t* out4, int reset);

/* The fallback rows of npfn_item_attn_fallback split by cause (HOST output, synchronous, since
 * that call's last reset): out2[0] query rows whose first-pass sum overflowed (> 2^100, inf or
 * NaN), out2[1] rows whose sum underflowed (< 2^-100); the rest of out4[2] were forced
 * (npfn_debug_item_attn_online).  The padding keys of the last step are masked to P = 0 in both
 * passes, so padding never causes a fallback.  A query whose max over its FIRST 32 keys lies
 * outside [-64, 16] (log2 units) runs the first pass relative to that max + 60 (its own lane-local
 * reference), so a uniformly large or small score level no longer fails; only a spread of more
 * than ~160 log2 units between those first 32 keys and the rest does (csrc/npfn_kernels.hip,
 * kIaShiftHi / kIaShiftLo / kIaShiftMargin and the comment above them). */
int npfn_item_attn_fallback_causes(npfn_engine* h, uint64_t* out2);

#ifdef __cplusplus
}
#endif
#endif /* NPFN_H */
