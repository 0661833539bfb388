// npfn_kernels.h -- launcher interface between the engine and the kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace npfn {

typedef uint16_t bf16_t;

// Sets the thread-local message npfn_last_error() returns and passes `code` through
// (defined in npfn_engine.hip, used by every translation unit's entry points).
int set_error(int code, const char* msg);

enum { EPI_BF16 = 0, EPI_BF16_GELU = 1, EPI_LOGIT = 2, EPI_LN = 3 };
// Storage type of the decoder logits (h->logits, [E][rows][n_bars], EPI_LOGIT): f32
// accumulation in the GEMM, stored as fp16 -- the type tabpfn's decoder Linear returns under
// its default autocast forward on a GPU [ext] -- and widened to f32 by every mix kernel on load.
// r05 A/B against f32 storage: the decoder GEMM -20 % (8.53 -> 6.85 ms per c2 call), the mix
// -4 %, c2 +0.5 %, the c2 posterior tests unchanged (profiles/r05/ab_logit_f16_r05t.txt)
typedef _Float16 logit_t;

struct EpiParams {
  const float* bias = nullptr;  // [N]
  bf16_t* out_bf = nullptr;     // EPI_BF16*, row stride ldo
  logit_t* out_l = nullptr;     // EPI_LOGIT, row stride ldo
  int64_t ldo = 0;
  float* resid = nullptr;       // EPI_LN: fp32 residual stream [M][192], updated in place
  bf16_t* resid_bf = nullptr;   // EPI_LN: bf16 copy of the result
  const float* ln_g = nullptr;
  const float* ln_b = nullptr;
};

// Feature pipelines of an estimator (oracle/preprocess_oracle.py T_*): which columns of the
// preprocessed table ("views", [rows][Vw]) it reads, before its feature shuffle.
// T_RFP: original features + fingerprint (the classifier ensemble's "none" pipeline)
enum { T_RAW = 0, T_QUANT = 1, T_POWER = 2, T_QSVD = 3, T_PFP = 4, T_RFP = 5 };

// Column layout of the views table of one forward: raw F | quantile F | SVD k | power F |
// fingerprint of estimator e (E columns).  Columns a mode does not use are not written.
struct ViewLayout {
  int F, k, E, Vw;
  int q_off, s_off, p_off, fp_off;
  int has_q, has_p, has_fp;
};
__host__ __device__ inline ViewLayout view_layout(int F, int k, int E, int has_q, int has_p, int has_fp) {
  ViewLayout v;
  v.F = F; v.k = k; v.E = E;
  v.q_off = F; v.s_off = 2 * F; v.p_off = 2 * F + k; v.fp_off = 3 * F + k;
  v.Vw = 3 * F + k + E;
  v.has_q = has_q; v.has_p = has_p; v.has_fp = has_fp;
  return v;
}

// Fit state as seen by the encoder (one launch = one group of estimators with equal C).
struct DevFit {
  const int* vcol;      // [Etot][Fmax] views column of feature position j (after the shuffle)
  const float* mu;      // [Etot][Fmax]
  const float* sd;      // [Etot][Fmax]
  const float* gscale;  // [Etot][Gmax]
  const int* eF;        // [Etot] features of the estimator's pipeline
  const int* ett;       // [Etot] 1: target transform (ensemble mode)
  const float* ystats;  // [2][3]: (mean, std, mean of standardized) of y | of Yeo-Johnson(y)
  const double* ylam;   // target Yeo-Johnson lambda (ensemble mode)
  const int* cperm;     // classifier: [Etot][KMAX_CLS] class permutation (ncls > 0)
  const float* ybar_e;  // classifier: [Etot] target value of test rows
  const float* views;   // [R][Vw] preprocessed table of the current forward rows
  int Vw;
  int E, G, C, Fmax, Gmax;
  int e0;               // global index of the group's first estimator: every per-estimator
                        // table is indexed globally (npfn_set_estimator_set, groups)
  int es;               // global index stride of the group's estimators (e0 + es * local)
  int ncls;             // 0: regressor fit; K > 0: classifier fit with K classes
};

// What the view kernels compute from the raw rows (fit state of the preprocessing).
struct ViewParams {
  ViewLayout L;
  const double* qtab;   // [F][nqmax] quantiles
  const int* qn;        // [F] table length (0: column passes through)
  int nqmax;
  const double* plam;   // [F] Yeo-Johnson lambdas
  const double* svd;    // [m] scale then [k][m] components (m = 2F), f64
  const int* fp_salt;   // [E] fingerprint salt, -1: the estimator has no fingerprint column
};
constexpr int QT_SORT_MAX = 16384;  // values a quantile fit sorts in LDS (>= kQtSubsample)
// sklearn QuantileTransformer's default subsample: contexts of more rows fit the quantiles on
// kQtSubsample rows drawn by numpy's RandomState (k_qt_subsample; oracle quantile_subsample)
constexpr int kQtSubsample = 10000;
constexpr int kQtSubsampleMaxRows = 65536;  // the shuffle's uint16 index array in LDS
// item attention: one 64-key step per K/V barrier (r03: two per barrier changed nothing); the key
// tiles (32 keys) of a context are rounded up to a multiple of 2 (padding keys are packed as zeros)
constexpr int kIaTileQuantum = 2;
constexpr int KMAX_CLS = 16;

// Fused row-tile layer kernel (npfn_rowk2.hip).  One launch runs a layer for up to kRowSegs
// SEGMENTS (estimator groups of one forward: same layer weights, each its own token count C
// and token tensor); its tiles are the segments' tiles one after the other, so the persistent
// grid has one tail per layer instead of one per group.
constexpr int kRowSegs = 4;
// tokens per row the fused path (k_row_layer: whole rows in a 256-slot tile) and the unfused
// per-sublayer path (k_feat_attn: a row's q|k|v in LDS, 1152 B per token) accept; wider rows
// (wide tables: an estimator group with C > kRowMaxC) run the per-sublayer path with
// k_feat_attn_wide (one head's K|V of the row in LDS, 128 B per token) up to kWideMaxC
constexpr int kRowMaxC = 256;
constexpr int kFeatAttnMaxC = 160 * 1024 / (576 * 2);
constexpr int kWideMaxC = 1024;
struct RowSeg {
  int64_t tile0;           // the segment's first tile in the launch
  int64_t rows;            // rows (E_g * R) of the segment's token tensor [rows][C][192]
  int C, rpt;              // tokens per row (as tiled), rows per tile
  const bf16_t* o_item;    // [tok][192] item-attention output of layer l (do_post)
  float* resid;            // [tok][192] fp32 residual stream (in / out)
  bf16_t* out;             // q [tok][192] | qkv [tok][576] | last layer: x bf16 [rows][192] (packed)
  // memory token of slot t of a tile starting at row r0: r0 * tmem + tofs + t * tstride.
  // Tiles of whole rows: tmem = C, tofs = 0, tstride = 1.  The last layer's post-only launch
  // runs the rows' target tokens alone (C = 1; tmem = tstride = the rows' token count,
  // tofs = that count - 1): the decoder reads nothing else of the last layer.
  int tmem, tofs, tstride;
};
// NPFN_GELU_F16: the row kernel's MLP hidden slabs go to W2 as fp16 B fragments from a packed-f16
// GELU (v_pk_*_f16), and the W2 chunk images of the weight stream are fp16 (v_mfma_f32_16x16x32_f16);
// 0: GELU in f32, bf16 fragments and W2 images (npfn_rowk2.hip run_w2_gelu)
#ifndef NPFN_GELU_F16
#define NPFN_GELU_F16 0
#endif
struct RowLayerParams {
  int64_t R;               // rows per estimator: a tile never spans two estimators, so a
                           // row's tile position (and its result, bit for bit) does not
                           // depend on how many estimators or segments the launch holds
  int64_t ntiles;          // tiles of all segments
  int nseg;
  RowSeg seg[kRowSegs];
  int dff;                 // MLP width
  int do_post, do_pre, out_qkv;
  // the pre part is the LAST layer's: only each row's target token (its last slot, C - 1) has its
  // residual and item projections read afterwards (the last layer runs the target column only),
  // so the other tokens' stores are skipped
  int tgt_only;
  // weight stream of one tile, in consumption order: [192][64] chunk images (npfn_engine.hip
  // build_rowk_streams), 3 per GEMM; the kernel replays it for every tile
  const bf16_t* stream;
  int stream_chunks;
  const float *ln2g, *ln2b, *ln3g, *ln3b;
  const float *ln1g, *ln1b;
  // dynamic tile schedule (npfn_rowk2.hip): a workgroup takes its next tile from a per-stream
  // device counter, tile = atomicAdd(tile_ctr, 1) - tile_base; the counter only grows (every
  // launch advances it by ntiles + grid: each workgroup's last fetch overshoots once).
  // nullptr: the static schedule (workgroup w takes tiles w, w + grid, ...)
  unsigned* tile_ctr;
  unsigned tile_base;
};
void rowk_setup();
// grid of a row-kernel launch over `ntiles` tiles (the counter advance is ntiles + grid)
int64_t rowk_grid(int64_t ntiles);
int rowk_rows_per_tile(int C);
hipError_t launch_row_layer(const RowLayerParams& p, hipStream_t s, bool inject_fail = false);  // the launch's error (hipGetLastError)

void gemm_setup();
void launch_col_stats(const float* X, int64_t ldx, const float* y, int64_t ldy, int64_t n, int F,
                      float* colstat, float* ystats, hipStream_t s);
void launch_build_params(const float* colstat, int F, int k, int E, int Fmax, int Gmax, uint64_t seed,
                         const int* ftype, ViewLayout L, int* vcol, float* mu, float* sd, float* gscale, int* eF,
                         hipStream_t s);
// Yeo-Johnson lambdas of the F columns of X and, when y != null, of the target column y in the
// same launch (its lambda into ylam, its statistics into ypstat)
void launch_power_fit(const float* X, int64_t ldx, int64_t n, int F, double* plam, float* pstat, hipStream_t s,
                      const float* y = nullptr, int64_t ldy = 0, double* ylam = nullptr, float* ypstat = nullptr);
// div: n_quantiles = max(n / div, 2) -- 5 (tabpfn "quantile_uni"), 10 ("quantile_uni_coarse")
// sub: kQtSubsample row indices (launch_qt_subsample) when n > kQtSubsample, else null
void launch_quantile_fit(const float* X, int64_t ldx, int64_t n, int F, int div, int nqmax, const int* sub,
                         double* qtab, int* qn, float* qstat, hipStream_t s);
// idx [kQtSubsample]: the rows sklearn's QuantileTransformer(random_state=seed) fits on
// (kQtSubsample < n <= kQtSubsampleMaxRows)
void launch_qt_subsample(int64_t n, uint32_t seed, int* idx, hipStream_t s);
__host__ __device__ int quantile_count(int64_t n, int div);
// views [R][Vw] of rows X: raw / quantile / power columns, then the SVD columns (they read the
// raw and quantile ones), then the fingerprints of TEST rows (train rows: launch_fp_train)
void launch_views_base(const float* X, int64_t ldx, int64_t R, const ViewParams& vp, float* views, hipStream_t s);
void launch_views_svd(int64_t R, const ViewParams& vp, float* views, hipStream_t s);
void launch_views_fp_test(const float* X, int64_t ldx, int64_t R, const ViewParams& vp, float* views, hipStream_t s);
// fingerprints of TRAIN rows: collision-free per estimator within each kFpBlock rows (tabpfn's
// re-hash with +1, +2, ...); htab: workspace [E][fp_total(n)] int
void launch_fp_train(const float* X, int64_t ldx, int64_t n, const ViewParams& vp, int* htab, float* views,
                     hipStream_t s);
constexpr int kFpBuckets = 10000;  // hash values: sha256 % 10000 / 10000
// candidate hashes precomputed for the train row at position k of its block: enough that a
// row needs more with probability ~1e-3 once k hashes are taken (7 / p - 3 for a free fraction
// p = (kFpBuckets - k) / kFpBuckets; -ln(1e-3) ~ 6.9), within [4, 256]
constexpr int kFpMin = 4, kFpCap = 256;
__host__ __device__ constexpr int fp_count(int k) {
  const int q = (7 * kFpBuckets + (kFpBuckets - k) - 1) / (kFpBuckets - k) - 3;
  return q < kFpMin ? kFpMin : (q > kFpCap ? kFpCap : q);
}
int fp_stride(int64_t n);  // the largest fp_count of an n-row fit's rows, rounded up to 4
// candidates of all rows of an n-row fit per estimator: row r's fp_count(r % kFpBlock), rounded up
// to 4 (16-byte pieces), at prefix offsets -- not every row at the largest count (r04: ~20x the
// bytes at 10 000 rows)
int64_t fp_total(int64_t n);
constexpr int kFpBlock = 10000;    // train rows per block of distinct hashes
// StandardScaler(with_mean=False) + truncated SVD of the train views' [raw | quantile] block:
// out = [m] scale then [k][m] components (f64); m = 2F <= kSvdMaxM (the m x m Gram matrix by the
// one-block Jacobi), any m with n <= kSvdMaxM rows (the n x n dual), else m <= kSvdLargeMaxM (the
// dense Gram matrix by rocSOLVER dsyevd); work: svd_work_bytes(n, m) bytes.
// Returns 0, or -1 for a shape it does not take.
constexpr int kSvdMaxM = 512;
constexpr int kSvdLargeMaxM = 2048;
size_t svd_work_bytes(int64_t n, int m);
void svd_setup();
// 0 ok; -1 shape out of range or a launch / the eigensolver's start failed; -2 the large form's
// dsyevd reported no convergence (info != 0; checked synchronously on that path only)
int launch_svd_fit(const float* views, int64_t n, ViewLayout L, void* work, double* out, hipStream_t s);
struct TransEntry;
// target transform of the ensemble mode: Yeo-Johnson fit of y (lambda), stats of YJ(y) into
// ystats[3..5], and the translation of the transformed estimators' bars back to the common borders:
// tab [nb + 1], tcancel [nb]; pscratch: 3 floats
void launch_target_tf(const float* y, int64_t ldy, int64_t n, const float* bz, int nb, double* ylam, float* ystats,
                      TransEntry* tab, uint8_t* tcancel, float* pscratch, hipStream_t s, bool fit_lambda = true);
void launch_encode(const float* ytr, int64_t ldy, int64_t R, const DevFit& fp, const float* encw,
                   const float* yencw, const float* pos, float* resid, bf16_t* resid_bf, hipStream_t s);
void launch_gemm(int epi, const bf16_t* A, int64_t lda, const bf16_t* W, int64_t M, int N, int K,
                 const EpiParams& p, hipStream_t s);
void launch_feat_attn(const bf16_t* qkv, bf16_t* out, int64_t rows, int C, hipStream_t s);
// c_lo: pack columns [c_lo, C) only (the last layer's cache: the target column)
void launch_kv_pack(const bf16_t* qkv, int64_t n, int C, int E, int ntile, bf16_t* kvc, hipStream_t s, int c_lo = 0);
void set_item_attn_online(int on);
// Item attention of up to kIaSegs estimator groups in one launch (grid.y = the segments'
// (estimator, column, head) triples one after the other).
constexpr int kIaSegs = 4;
struct IaSeg {
  int y0;               // first grid.y of the segment
  int C;                // tokens per row
  int c_lo;             // first column attended (the last layer: C - 1, the target column)
  const bf16_t* q;      // [E_g * R][C][ldq] (queries at column 0)
  const bf16_t* kvc;    // the segment's packed K/V cache of this layer
  bf16_t* out;          // [E_g * R][C][192]
};
struct IaParams {
  int nseg;
  IaSeg seg[kIaSegs];
  int ny;               // grid.y: (estimator, column >= c_lo, head) triples of all segments
  int64_t ldq, R, n;
  int ntile;
  // fallback counters (nullable): [0] += blocks that ran the online-softmax pass, [1] += query
  // rows that took its result
  unsigned long long* fb;
};
void launch_item_attn(const IaParams& p, hipStream_t s);
int64_t item_attn_blocks(const IaParams& p);  // blocks of a launch (queries: ny * R)
void set_item_attn_scale(float s);
void launch_class_params(const float* y, int64_t ldy, int64_t n, int K, int E, uint64_t seed, int* cperm,
                         float* ybar_e, hipStream_t s);
void launch_cls_mix(const logit_t* logits, int64_t R, int E, int nout, int K, float invT, const int* cperm, int geo,
                    float* probs, int64_t ldo, hipStream_t s);
// Target-border translation of the ensemble's target-transformed estimators (null: none).
// Per common border b: (source bucket, share of it left of the border) with the flag folded
// into the share: -1 = at / below the source range (cdf 0), 2 = at / above it (cdf 1).
struct TransEntry {
  int idx;
  float share;
};
struct MixTrans {
  const int* ett = nullptr;           // [E] 1: estimator e's probabilities are translated
  const TransEntry* tab = nullptr;    // [nb + 1]
  const uint8_t* tcancel = nullptr;   // [nb] bars with no mass after the border repair
  int geo = 0;                        // 1: tabpfn's average_before_softmax -- the mixture is
                                      // softmax(mean_e log q_e) instead of mean_e q_e
};
void launch_mix_log(const logit_t* logits, int64_t R, int E, int nb, float invT, const MixTrans& tr, float* out,
                    int64_t ldo, hipStream_t s);
void launch_mix_sample(const logit_t* logits, int64_t R, int E, int nb, float invT, const MixTrans& tr,
                       const float* bz, const float* ystats, uint64_t seed, uint64_t counter, int64_t row_offset,
                       uint64_t philox_row0, float* feat, int64_t ldf, int col, float* logp_acc, float log_eps,
                       hipStream_t s);
// Draws that share their query row (npfn_ar_sample_repeated, AR step 0): k_mix_prob writes the
// mixture of each distinct row once, k_group_sample draws row r of [row_offset, row_offset + R)
// from the mixture of row (row_offset + r) / per -- the same p, uniform and arithmetic as
// k_mix_sample on the repeated rows
void launch_mix_prob(const logit_t* logits, int64_t R, int E, int nb, float invT, const MixTrans& tr, float* p_out,
                     hipStream_t s);
void launch_group_sample(const float* p_rows, int64_t per, int64_t R, int nb, const float* bz, const float* ystats,
                         uint64_t seed, uint64_t counter, int64_t row_offset, uint64_t philox_row0, float* feat,
                         int64_t ldf, int col, float* logp_acc, float log_eps, hipStream_t s);
void launch_group_nll(const float* p_rows, int64_t per, int64_t R, int nb, const float* bz, const float* ystats,
                      int64_t row_offset, const float* feat, int64_t ldf, int col, float* logp_acc, float log_eps,
                      hipStream_t s);
void launch_mix_nll(const logit_t* logits, int64_t R, int E, int nb, float invT, const MixTrans& tr, const float* bz,
                    const float* ystats, int64_t row_offset, const float* feat, int64_t ldf, int col,
                    float* logp_acc, float log_eps, hipStream_t s);
void launch_bar_sample(const float* logits, const float* borders, int64_t R, int nb, uint64_t seed,
                       uint64_t counter, float* out, hipStream_t s);
void launch_bar_nll(const float* logits, const float* borders, const float* y, int64_t R, int nb, float* out,
                    hipStream_t s);
void launch_borders(const float* bz, const float* ystats, int nb, float* out, hipStream_t s);
// dst[r][dst_col0 + c] = src[r / per][c] (per = 1: a plain column copy; per > 1: rows repeated
// obs-major, as x.repeat_interleave(per, 0))
void launch_copy_cols(const float* src, int64_t lds, float* dst, int64_t ldd, int64_t rows, int cols,
                      int dst_col0, hipStream_t s, int64_t per = 1);
void launch_fill(float* dst, int64_t n, float v, hipStream_t s);
void launch_box_support(const float* th, int64_t n, int dim, const float* lo, const float* hi, uint8_t* mask,
                        hipStream_t s);

}  // namespace npfn
