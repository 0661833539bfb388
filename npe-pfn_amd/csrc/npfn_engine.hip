// npfn_engine.hip -- engine state and the C-ABI of include/npfn.h.
//
// Data layout in HBM:
//   tokens   [E][rows][C][192]  fp32 residual stream + bf16 copy (GEMM A operand)
//   qkv      [E*rows*C][576]    bf16 (feature attention; item attention on train rows)
//   q        [E*rows*C][192]    bf16 (item attention queries of test rows)
//   kv cache [L][E][C][6][ntile][2048] bf16, MFMA-fragment packed (k_kv_pack)
//   hidden   [E*rows*C][768]    bf16 (MLP)
//   logits   [E][rows][5000]    logit_t (fp16; decoder), mixed + sampled by k_mix_*
// All estimators share the weights, so every GEMM runs over all E at once.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "npfn.h"
#include "npfn_kernels.h"

using namespace npfn;

static constexpr bool kFusedDefault = true;

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

}  // namespace

// shared with npfn_support.hip: every entry point reports through npfn_last_error()
int npfn::set_error(int code, const char* msg) { return fail(code, msg ? msg : ""); }

namespace {

#define HIPCHK(x)                                                                          \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) return fail(NPFN_EHIP, std::string(#x) + ": " + hipGetErrorString(e_)); \
  } while (0)

struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
};

uint16_t host_f2bf(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  if ((u & 0x7fffffffu) > 0x7f800000u) return 0x7fc0;
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}

struct LayerW {
  bf16_t *feat_qkv, *feat_out, *item_qkv, *item_out, *w1, *w2;
  float* ln[6];
};

// Live per-kernel timing (npfn_prof_*): a HIP event pair around every launch,
// accumulated per kernel function with its algorithmic FLOPs and bytes.
enum ProfCat {
  P_ENCODE, P_GEMM_BF16, P_GEMM_GELU, P_GEMM_F32, P_GEMM_LN, P_FEAT_ATTN, P_KV_PACK, P_ITEM_ATTN,
  P_MIX_SAMPLE, P_MIX_NLL, P_MIX_LOG, P_STATS, P_ROW_LAYER, P_CLS_MIX, P_VIEWS, P_QUANT_FIT, P_POWER_FIT,
  P_SVD_FIT, P_FP_TRAIN, P_TARGET_TF, P_OTHER, P_NCAT
};
const char* kProfNames[P_NCAT] = {
  "k_encode", "k_gemm<EPI_BF16>", "k_gemm<EPI_BF16_GELU>", "k_gemm<EPI_LOGIT>", "k_gemm<EPI_LN>", "k_feat_attn",
  "k_kv_pack", "k_item_attn", "k_mix_sample", "k_mix_nll", "k_mix_log", "k_col_stats+k_build_params", "k_row_layer",
  "k_cls_mix", "k_views", "k_quantile_fit", "k_power_fit", "k_svd_fit", "k_fp_train", "k_target_tf", "other"};

struct ProfRec {
  int cat;  // + P_NCAT: launched on a side stream (the AR fits' preprocessing / train forwards)
  hipEvent_t a, b;
  double flops, bytes;
};

struct Profiler {
  bool on = false;
  std::vector<hipEvent_t> pool;
  size_t used = 0;
  std::vector<ProfRec> recs;
  hipEvent_t get() {
    if (used == pool.size()) {
      hipEvent_t e;
      (void)hipEventCreate(&e);
      pool.push_back(e);
    }
    return pool[used++];
  }
};

}  // namespace

// The state one fit leaves for predicts: preprocessing fits, per-estimator tables, the
// estimator groups and their train-side K/V caches.
struct Fit {
  bool fitted = false;
  int F = 0, ntile = 0;
  int64_t n = 0;
  DevBuf colstat, ystats, vcol, mu, sd, gscale, eF, kvc;
  int ncls = 0;          // > 0 after a classifier fit (npfn_fit_classes)
  DevBuf cperm, ybar_e;  // classifier: [E][KMAX_CLS] label permutation, [E] test target value
  size_t kv_elems = 0;   // K/V cache size of the groups (fit_prep)
  int nqmax = 0;
  DevBuf qtab, qn, qstat;  // [F][nqmax] f64 quantiles, [F] lengths, [F][3] scratch
  DevBuf qsub;             // [kQtSubsample] rows of the quantile fit's subsample (n > kQtSubsample)
  DevBuf plam, pstat;      // [F] f64 Yeo-Johnson lambdas, [F][3] scratch
  DevBuf svd;              // [m] scale + [k][m] components (f64), m = 2F
  DevBuf svdw;             // SVD workspace (svd_work_bytes)
  DevBuf htab;             // [E][fp_total(n)] train fingerprint candidates
  DevBuf ylam, ttab, tcancel, tscratch;  // ensemble target transform
  DevBuf tviews;           // [n][Vw] preprocessed table of the train rows (read by the train forward)
  ViewLayout vl{};
  // estimator groups of the fit: consecutive estimators of the range with equal C
  struct Group {
    int e0, ne, C;
    size_t kv_off;  // elements into kvc
  };
  std::vector<Group> groups;
  void release();
};

// Forward workspaces of one stream (token tensors of the rows in flight).
struct Work {
  DevBuf resid, resid_bf, qkv, attn, hid;
  void release();
};

struct npfn_engine {
  npfn_config cfg{};
  std::vector<void*> weight_allocs;
  float *encw = nullptr, *yencw = nullptr, *pos = nullptr, *bz = nullptr;
  float *dec_b1 = nullptr, *dec_b2 = nullptr;
  bf16_t *dec_w1 = nullptr, *dec_w2 = nullptr;
  std::vector<LayerW> layers;
  // k_row_layer weight streams (build_rowk_streams): stream j = [post of layer j-1 | pre of
  // layer j] as consecutive [192][64] chunk images; rowk_post[j] = chunks of the post part
  std::vector<bf16_t*> rowk_stream;
  std::vector<int> rowk_post;
  // preprocessing (npfn_set_preprocessing): per-estimator pipeline and target transform,
  // uploaded once per mode (oracle preprocess_oracle.estimator_configs)
  int pre_mode = 0;
  bool pre_cls = false;  // mode 3's pipelines are the classifier's (npfn_fit_classes)
  int qdiv = 5;          // n_quantiles = max(n / qdiv, 2)
  std::vector<int> h_ftype, h_tt, h_salt;
  DevBuf ftype, ett, fp_salt;
  bool any_tt = false;
  DevBuf views;            // [rows][Vw] preprocessed table of the current test forward (k_views*)
  const DevBuf* last_views = nullptr;  // views of the last fit (its tviews) or test forward (npfn_debug_views)
  // side stream of the AR calls' preprocessing fits (ar_prefit): every step's fit statistics
  // are computed there up front, while the main stream runs the earlier steps
  hipStream_t side = nullptr;
  hipStream_t side_t = nullptr;  // train forwards of the AR fits (steps >= 1)
  std::vector<hipEvent_t> prep_done;  // per AR step: its fit (preprocessing + train forward) is complete
  std::vector<hipEvent_t> stat_done;  // per AR step: its preprocessing fit is complete
  hipEvent_t setup_done = nullptr;
  // npfn_ar_fit_begin / npfn_ar_fit_step: the AR fits of a call driven step by step
  bool ar_active = false, ar_piped = false, ar_reuse = false;
  int64_t ar_n = 0;
  int ar_dx = 0, ar_dth = 0;
  // fit state: `f` is the fit predict / forward read; fit0 unless npfn_ar_sample reuses the
  // per-step fits of an earlier call with the same fit token (npfn_set_fit_token)
  Fit fit0;
  Fit* f = &fit0;
  std::vector<Fit> slots;      // per AR step k: the fit of step k
  uint64_t fit_token = 0;      // npfn_set_fit_token
  uint64_t slot_key[6] = {0, 0, 0, 0, 0, 0};  // token, n, dim_x, dim_theta, mode, range of the cached slots
  // workspaces: the forwards' token tensors per stream (w = the one in use: wmain on the
  // caller's stream, wside for the AR train forwards on side_t)
  Work wmain, wside;
  Work* w = &wmain;
  DevBuf dh, logits, tgt;
  DevBuf joint, feat, logp;
  DevBuf pu;  // [n_unique][nb] step-0 mixtures of npfn_ar_sample_repeated
  int64_t chunk_rows = 16384;
  // estimator set of fits and forwards (npfn_set_estimator_set): estimators e0 + es * i,
  // i < ne, of cfg.n_estimators; a partial set is the estimator-parallel multi-GPU split
  int e0 = 0, ne = 0, es = 1;
  bool fused = true;  // k_row_layer path (NPFN_UNFUSED=1 selects the per-sublayer kernels)
  // dynamic row-kernel tile schedule (RowLayerParams::tile_ctr): one device counter per stream
  // the row kernel runs on (the caller's, side_t), the host keeps each counter's running base
  static constexpr int kTileCtrs = 8;
  unsigned* tile_ctrs = nullptr;  // [kTileCtrs], zeroed at creation
  // item-attention fallback counters (IaParams::fb): device [blocks, rows] that took the online
  // pass; host totals of the launches since the last read (npfn_item_attn_fallback)
  unsigned long long* ia_fb = nullptr;
  uint64_t ia_blocks = 0, ia_rows = 0;
  hipStream_t tile_ctr_stream[kTileCtrs] = {};
  unsigned tile_ctr_base[kTileCtrs] = {};
  int n_tile_ctr = 0;
  bool dyn_tiles = true;  // NPFN_ROWK_STATIC=1: the static schedule
  int avg_before_softmax = 0;  // npfn_set_average_before_softmax (tabpfn's kwarg)
  int debug_fail_row = 0;  // npfn_debug_fail_row_launch: the n-th next row-kernel launch is refused
  Profiler prof;

  int Fmax() const { return 2 * cfg.max_groups; }
  DevFit devfit(const Fit::Group& g, bool train) const {
    DevFit d;
    d.vcol = (const int*)f->vcol.p;
    d.mu = (const float*)f->mu.p;
    d.sd = (const float*)f->sd.p;
    d.gscale = (const float*)f->gscale.p;
    d.eF = (const int*)f->eF.p;
    d.ett = (const int*)ett.p;
    d.ystats = (const float*)f->ystats.p;
    d.ylam = (const double*)f->ylam.p;
    d.cperm = (const int*)f->cperm.p;
    d.ybar_e = (const float*)f->ybar_e.p;
    d.views = (const float*)(train ? f->tviews.p : views.p);
    d.Vw = f->vl.Vw;
    d.E = g.ne;
    d.e0 = g.e0;
    d.es = es;
    d.C = g.C;
    d.G = g.C - 1;
    d.Fmax = Fmax();
    d.Gmax = cfg.max_groups;
    d.ncls = f->ncls;
    return d;
  }
  ViewParams viewparams() const {
    ViewParams v;
    v.L = f->vl;
    v.qtab = (const double*)f->qtab.p;
    v.qn = (const int*)f->qn.p;
    v.nqmax = f->nqmax;
    v.plam = (const double*)f->plam.p;
    v.svd = (const double*)f->svd.p;
    v.fp_salt = (const int*)fp_salt.p;
    return v;
  }
  MixTrans mixtrans() const {
    MixTrans t;
    t.geo = avg_before_softmax;
    if (!any_tt) return t;
    t.ett = (const int*)ett.p;
    t.tab = (const TransEntry*)f->ttab.p;
    t.tcancel = (const uint8_t*)f->tcancel.p;
    return t;
  }
};

namespace {

int ensure(DevBuf& b, size_t bytes, hipStream_t s) {
  if (bytes == 0) bytes = 16;
  if (b.bytes >= bytes) return NPFN_OK;
  if (b.p) {
    HIPCHK(hipStreamSynchronize(s));
    HIPCHK(hipFree(b.p));
    b.p = nullptr;
    b.bytes = 0;
  }
  const size_t want = bytes + bytes / 8;
  if (hipMalloc(&b.p, want) != hipSuccess) {
    b.p = nullptr;
    (void)hipGetLastError();
    return fail(NPFN_ENOMEM, "hipMalloc of " + std::to_string(want) + " bytes failed");
  }
  b.bytes = want;
  return NPFN_OK;
}

void free_buf(DevBuf& b) {
  if (b.p) (void)hipFree(b.p);
  b.p = nullptr;
  b.bytes = 0;
}

}  // namespace

void Work::release() {
  DevBuf* bufs[] = {&resid, &resid_bf, &qkv, &attn, &hid};
  for (DevBuf* b : bufs) free_buf(*b);
}

void Fit::release() {
  DevBuf* bufs[] = {&colstat, &ystats, &vcol, &mu,   &sd,   &gscale, &eF,  &kvc,  &cperm,   &ybar_e,  &qtab,
                    &qn,      &qstat, &qsub,  &plam, &pstat, &svd, &svdw, &htab,   &ylam, &ttab, &tcancel, &tscratch,
                    &tviews};
  for (DevBuf* b : bufs) free_buf(*b);
  fitted = false;
}

namespace {

struct ProfGuard {
  npfn_engine* h;
  int cat;
  double flops, bytes;
  hipStream_t s;
  hipEvent_t a = nullptr;
  ProfGuard(npfn_engine* h_, int c, double f, double b, hipStream_t s_) : h(h_), cat(c), flops(f), bytes(b), s(s_) {
    if (h->prof.on) {
      a = h->prof.get();
      (void)hipEventRecord(a, s);
    }
  }
  ~ProfGuard() {
    if (a) {
      hipEvent_t b = h->prof.get();
      (void)hipEventRecord(b, s);
      const bool side = s != nullptr && (s == h->side || s == h->side_t);
      h->prof.recs.push_back({cat + (side ? P_NCAT : 0), a, b, flops, bytes});
    }
  }
};

double gemm_bytes(int64_t M, int N, int K, int epi) {
  double b = 2.0 * M * K + 2.0 * N * K;
  if (epi == EPI_LOGIT) b += (double)sizeof(logit_t) * M * N;
  else if (epi == EPI_LN) b += M * 192.0 * (4 + 4 + 2);
  else b += 2.0 * M * N;
  return b;
}

void gemm_p(npfn_engine* h, int epi, const bf16_t* A, int64_t lda, const bf16_t* W, int64_t M, int N, int K,
            const EpiParams& p, hipStream_t s) {
  static const int cat_of[4] = {P_GEMM_BF16, P_GEMM_GELU, P_GEMM_F32, P_GEMM_LN};
  ProfGuard g(h, cat_of[epi], 2.0 * M * N * K, gemm_bytes(M, N, K, epi), s);
  launch_gemm(epi, A, lda, W, M, N, K, p, s);
}

int check_cfg(const npfn_config* c) {
  if (!c) return fail(NPFN_EINVAL, "null config");
  if (c->d_model != 192 || c->n_heads != 6)
    return fail(NPFN_EINVAL, "engine kernels are built for d_model=192, 6 heads of 32");
  if (c->features_per_group != 2) return fail(NPFN_EINVAL, "features_per_group must be 2");
  if (c->d_ff % 192 != 0 || c->d_ff <= 0) return fail(NPFN_EINVAL, "d_ff must be a positive multiple of 192");
  if (c->n_layers <= 0 || c->n_bars <= 1 || c->n_estimators <= 0 || c->n_estimators > 64)
    return fail(NPFN_EINVAL, "bad n_layers / n_bars / n_estimators");
  if (c->max_groups <= 0 || c->max_groups > 4096) return fail(NPFN_EINVAL, "bad max_groups");
  if (!(c->softmax_temperature > 0.f)) return fail(NPFN_EINVAL, "softmax_temperature must be > 0");
  return NPFN_OK;
}

size_t blob_size(const npfn_config* c) {
  const size_t d = c->d_model, dff = c->d_ff, nb = c->n_bars, G = c->max_groups;
  size_t per_layer = 3 * d * d + d * d + 3 * d * d + d * d + dff * d + d * dff + 6 * d;
  return d * 4 + d * 2 + G * d + c->n_layers * per_layer + dff * d + dff + nb * dff + nb + (nb + 1);
}

int upload_f32(npfn_engine* h, const float* src, size_t n, float** dst) {
  void* p = nullptr;
  HIPCHK(hipMalloc(&p, n * sizeof(float)));
  h->weight_allocs.push_back(p);
  HIPCHK(hipMemcpy(p, src, n * sizeof(float), hipMemcpyHostToDevice));
  *dst = (float*)p;
  return NPFN_OK;
}

// a row-kernel weight stream: chunk c (192 x 64 values) as fp16 where f16[c] (NPFN_GELU_F16: the
// W2 chunks), else bf16
int upload_stream(npfn_engine* h, const std::vector<float>& img, const std::vector<uint8_t>& f16, bf16_t** dst) {
  const size_t n = img.size(), ce = 192 * 64;
  std::vector<uint16_t> tmp(n);
  for (size_t i = 0; i < n; ++i)
    tmp[i] = f16[i / ce] ? __builtin_bit_cast(uint16_t, (_Float16)img[i]) : host_f2bf(img[i]);
  void* p = nullptr;
  HIPCHK(hipMalloc(&p, n * sizeof(uint16_t)));
  h->weight_allocs.push_back(p);
  HIPCHK(hipMemcpy(p, tmp.data(), n * sizeof(uint16_t), hipMemcpyHostToDevice));
  *dst = (bf16_t*)p;
  return NPFN_OK;
}

int upload_bf16(npfn_engine* h, const float* src, size_t n, bf16_t** dst) {
  std::vector<uint16_t> tmp(n);
  for (size_t i = 0; i < n; ++i) tmp[i] = host_f2bf(src[i]);
  void* p = nullptr;
  HIPCHK(hipMalloc(&p, n * sizeof(uint16_t)));
  h->weight_allocs.push_back(p);
  HIPCHK(hipMemcpy(p, tmp.data(), n * sizeof(uint16_t), hipMemcpyHostToDevice));
  *dst = (bf16_t*)p;
  return NPFN_OK;
}

// Row-kernel chunk images (npfn_rowk2.hip): 192 image rows x 64 bf16 columns (24 KB), each
// stored exactly as its LDS image -- 16-byte unit u of image row r at unit u ^ (r & 7) -- so
// a chunk is one contiguous LDS-DMA copy; within each 32 columns, column s holds source
// column pi(s), pi(8g + j) = j < 4 ? 4g + j : 16 + 4g + j - 4 (the order in which a product's
// D tiles pack into the next B fragment).
//   S chunk: source rows [r0, r0 + 192) x columns [k0, k0 + 64)
//   O chunk: source rows [r0, r0 + 64) x all 192 columns, image row 64 kb + r = source row
//            r0 + r, columns [64 kb, 64 kb + 64)
void chunk_image(std::vector<float>& img, const float* src, size_t K, bool o_chunk, size_t r0, size_t k0,
                 float scale = 1.0f) {
  const size_t base = img.size();
  img.resize(base + 192 * 64);
  for (size_t vr = 0; vr < 192; ++vr)
    for (size_t tc = 0; tc < 64; ++tc) {
      const size_t sc = tc & 31, g = sc >> 3, j = sc & 7;
      const size_t pk = (tc & ~(size_t)31) + (j < 4 ? 4 * g + j : 16 + 4 * g + j - 4);
      const size_t row = o_chunk ? r0 + (vr & 63) : r0 + vr;
      const size_t kcol = o_chunk ? 64 * (vr >> 6) + pk : k0 + pk;
      const size_t unit = (tc >> 3) ^ (vr & 7);
      img[base + vr * 64 + unit * 8 + (tc & 7)] = src[row * K + kcol] * scale;
    }
}

#define RCHK_(x)                  \
  do {                            \
    int r_ = (x);                 \
    if (r_ != NPFN_OK) return r_; \
  } while (0)

// Per-layer host copies of the row-kernel matrices (float, [rows][K] as in the weights file)
struct RowkHost {
  std::vector<float> feat_qkv, feat_out, item_qkv, item_out, w1, w2;
};

// feature-attention q rows of the row-kernel stream carry the softmax scale 1/sqrt(32) and
// log2(e) (the kernel's S is then in log2 units); folded here instead of one multiply per
// q value per token in k_row_layer
constexpr float kFeatQScale = 0.17677669529663687f * 1.4426950408889634f;

// The weight streams k_row_layer replays per tile, one per launch position j = 0..L, in its
// consumption order (npfn_rowk2.hip):
//   post(l) = Wo_i S x3 | W1_0 O | W1_1 O, W2_0 S | ... | W1_11 O, W2_10 S | W2_11 S   layer l = j-1
//   pre(l)  = per head pair hp: Wv_hp O, Wk_hp O, Wq_hp O, Wo_f[:, hp] S | Wq_i S x3
//             (train: + Wk_i S x3, Wv_i S x3)                                          layer l = j
int build_rowk_streams(npfn_engine* h, const std::vector<RowkHost>& hw) {
  const int L = (int)hw.size(), d = h->cfg.d_model, dff = h->cfg.d_ff, ns = dff / 64;
  for (int j = 0; j <= L; ++j) {
    std::vector<float> img;
    std::vector<uint8_t> f16;  // per chunk: stored as fp16 (the W2 chunks under NPFN_GELU_F16)
    auto mark = [&](bool h16) { f16.resize(img.size() / (192 * 64), 0); f16.back() = h16 ? 1 : 0; };
    if (j >= 1) {
      const RowkHost& w = hw[j - 1];
      for (int kc = 0; kc < 3; ++kc) chunk_image(img, w.item_out.data(), d, false, 0, 64 * kc);
      chunk_image(img, w.w1.data(), d, true, 0, 0);
      for (int s = 1; s < ns; ++s) {
        chunk_image(img, w.w1.data(), d, true, 64 * s, 0);
        chunk_image(img, w.w2.data(), dff, false, 0, 64 * (s - 1));
        mark(NPFN_GELU_F16 != 0);
      }
      chunk_image(img, w.w2.data(), dff, false, 0, 64 * (ns - 1));
      mark(NPFN_GELU_F16 != 0);
    }
    const int post = (int)(img.size() / (192 * 64));
    if (j < L) {
      const RowkHost& w = hw[j];
      for (int hp = 0; hp < 3; ++hp) {
        chunk_image(img, w.feat_qkv.data(), d, true, 2 * d + 64 * hp, 0);               // v of the pair
        chunk_image(img, w.feat_qkv.data(), d, true, d + 64 * hp, 0);                   // k of the pair
        chunk_image(img, w.feat_qkv.data(), d, true, 64 * hp, 0, kFeatQScale);          // q of the pair
        chunk_image(img, w.feat_out.data(), d, false, 0, 64 * hp);                      // Wo_f slice
      }
      for (int m = 0; m < 3; ++m)  // item q | k | v (the test side stops after q)
        for (int kc = 0; kc < 3; ++kc) chunk_image(img, w.item_qkv.data(), d, false, (size_t)m * d, 64 * kc);
    }
    f16.resize(img.size() / (192 * 64), 0);
    bf16_t* dptr = nullptr;
    RCHK_(upload_stream(h, img, f16, &dptr));
    h->rowk_stream.push_back(dptr);
    h->rowk_post.push_back(post);
  }
  return NPFN_OK;
}

#define RCHK(x)                 \
  do {                          \
    int r_ = (x);               \
    if (r_ != NPFN_OK) return r_; \
  } while (0)

// ---------------------------------------------------------------- forward
// A row-kernel launch with the stream's tile counter (dynamic schedule): every launch advances
// it by ntiles + grid (each workgroup's last fetch overshoots once), so the next launch on the
// same stream starts from the host's running base; launches on one stream run in order.  A
// stream beyond the kTileCtrs counters takes the static schedule.
// Errors: a HIP error still pending from an earlier (unchecked) launch is returned before
// anything is launched, so it is never blamed on this launch; the launch's own error is
// returned too.  In both cases the host base stays where the device counter is (no launch
// went in), so the stream's later launches keep their tiles.
int row_launch(npfn_engine* h, RowLayerParams& rp, hipStream_t s) {
  const hipError_t pend = hipGetLastError();
  if (pend != hipSuccess)
    return fail(NPFN_EHIP, std::string("HIP error pending before a row-kernel launch: ") + hipGetErrorString(pend));
  rp.tile_ctr = nullptr;
  rp.tile_base = 0;
  int k = -1;
  if (h->dyn_tiles && h->tile_ctrs) {
    for (int i = 0; i < h->n_tile_ctr; ++i)
      if (h->tile_ctr_stream[i] == s) k = i;
    if (k < 0 && h->n_tile_ctr < npfn_engine::kTileCtrs) {
      k = h->n_tile_ctr++;
      h->tile_ctr_stream[k] = s;
    }
  }
  if (k >= 0) {
    rp.tile_ctr = h->tile_ctrs + k;
    rp.tile_base = h->tile_ctr_base[k];
  }
  // the counter advances only when the launch went in (a failed launch leaves it untouched)
  const bool inject = h->debug_fail_row > 0 && --h->debug_fail_row == 0;
  const hipError_t e = launch_row_layer(rp, s, inject);
  if (e != hipSuccess) return fail(NPFN_EHIP, std::string("row-kernel launch: ") + hipGetErrorString(e));
  if (k >= 0) h->tile_ctr_base[k] += (unsigned)(rp.ntiles + rowk_grid(rp.ntiles));
  return NPFN_OK;
}

// An item-attention launch with the engine's fallback counters.
void ia_launch(npfn_engine* h, IaParams& ip, hipStream_t s) {
  ip.fb = h->ia_fb;
  h->ia_blocks += (uint64_t)item_attn_blocks(ip);
  h->ia_rows += (uint64_t)ip.ny * (uint64_t)ip.R;
  launch_item_attn(ip, s);
}

// Item attention of one estimator group (the unfused path's form of launch_item_attn).
void item_attn_one(npfn_engine* h, const bf16_t* q, int64_t ldq, const bf16_t* kvc, bf16_t* out, int64_t R, int C,
                   int E, int64_t n, int ntile, hipStream_t s) {
  IaParams ip{};
  ip.nseg = 1;
  ip.seg[0] = IaSeg{0, C, 0, q, kvc, out};
  ip.ny = E * C * 6;
  ip.ldq = ldq;
  ip.R = R;
  ip.n = n;
  ip.ntile = ntile;
  ia_launch(h, ip, s);
}

// Runs the encoder + L layers of one estimator group over `rows` rows (views of those rows
// already in h->views).  train: ytr != nullptr, item attention against itself, K/V packed into
// the group's cache.
// test-side tokens per forward_rows call of a wide group (~4.2 KB of per-sublayer tensors each)
constexpr int64_t kWideTokens = int64_t(1) << 22;

// Test side: rows [r_off, r_off + rows) of the views (a wide group runs its test rows in chunks).
int forward_rows(npfn_engine* h, const Fit::Group& grp, const float* ytr, int64_t ldy, int64_t rows,
                 bool train, hipStream_t s, int64_t r_off = 0) {
  const int E = grp.ne, C = grp.C, L = h->cfg.n_layers, dff = h->cfg.d_ff;
  const int64_t tokens = (int64_t)E * rows * C;
  Work& wk = *h->w;
  RCHK(ensure(wk.resid, tokens * 192 * sizeof(float), s));
  RCHK(ensure(wk.resid_bf, tokens * 192 * sizeof(bf16_t), s));
  RCHK(ensure(wk.qkv, tokens * 576 * sizeof(bf16_t), s));
  RCHK(ensure(wk.attn, tokens * 192 * sizeof(bf16_t), s));
  RCHK(ensure(wk.hid, tokens * (size_t)dff * sizeof(bf16_t), s));
  float* resid = (float*)wk.resid.p;
  bf16_t* rbf = (bf16_t*)wk.resid_bf.p;
  bf16_t* qkv = (bf16_t*)wk.qkv.p;
  bf16_t* attn = (bf16_t*)wk.attn.p;
  bf16_t* hid = (bf16_t*)wk.hid.p;
  DevFit fp = h->devfit(grp, train);
  fp.views += r_off * fp.Vw;
  {
    ProfGuard g(h, P_ENCODE, 0.0, (double)tokens * 192 * 6, s);
    launch_encode(ytr, ldy, rows, fp, h->encw, h->yencw, h->pos, resid, rbf, s);
  }
  const double n_keys = (double)h->f->n;
  const double q_tok = (double)tokens * 6;  // (token, head) queries of the item attention
  const double kv_bytes_l = (double)E * C * 6 * h->f->ntile * 2048 * 2;
  const size_t kv_layer = (size_t)E * C * 6 * h->f->ntile * 2048;
  for (int l = 0; l < L; ++l) {
    const LayerW& w = h->layers[l];
    bf16_t* kvc = (bf16_t*)h->f->kvc.p + grp.kv_off + (size_t)l * kv_layer;
    EpiParams pq;
    pq.out_bf = qkv;
    pq.ldo = 576;
    gemm_p(h, EPI_BF16, rbf, 192, w.feat_qkv, tokens, 576, 192, pq, s);
    {
      ProfGuard g(h, P_FEAT_ATTN, (double)tokens * C * 6 * 128, (double)tokens * (576 + 192) * 2, s);
      launch_feat_attn(qkv, attn, (int64_t)E * rows, C, s);
    }
    EpiParams pln;
    pln.resid = resid;
    pln.resid_bf = rbf;
    pln.ln_g = w.ln[0];
    pln.ln_b = w.ln[1];
    gemm_p(h, EPI_LN, attn, 192, w.feat_out, tokens, 192, 192, pln, s);
    if (train) {
      gemm_p(h, EPI_BF16, rbf, 192, w.item_qkv, tokens, 576, 192, pq, s);
      {
        ProfGuard g(h, P_KV_PACK, 0.0, (double)tokens * 384 * 2 + kv_bytes_l, s);
        launch_kv_pack(qkv, rows, C, E, h->f->ntile, kvc, s);
      }
      {
        ProfGuard g(h, P_ITEM_ATTN, q_tok * 128 * n_keys, (double)tokens * 192 * 4 + kv_bytes_l, s);
        item_attn_one(h, qkv, 576, kvc, attn, rows, C, E, h->f->n, h->f->ntile, s);
      }
    } else {
      EpiParams pq2;
      pq2.out_bf = qkv;
      pq2.ldo = 192;
      gemm_p(h, EPI_BF16, rbf, 192, w.item_qkv, tokens, 192, 192, pq2, s);
      {
        ProfGuard g(h, P_ITEM_ATTN, q_tok * 128 * n_keys, (double)tokens * 192 * 4 + kv_bytes_l, s);
        item_attn_one(h, qkv, 192, kvc, attn, rows, C, E, h->f->n, h->f->ntile, s);
      }
    }
    pln.ln_g = w.ln[2];
    pln.ln_b = w.ln[3];
    gemm_p(h, EPI_LN, attn, 192, w.item_out, tokens, 192, 192, pln, s);
    if (train && l == L - 1) break;  // train rows are not read after the last item attention
    EpiParams ph;
    ph.out_bf = hid;
    ph.ldo = dff;
    gemm_p(h, EPI_BF16_GELU, rbf, 192, w.w1, tokens, dff, 192, ph, s);
    pln.ln_g = w.ln[4];
    pln.ln_b = w.ln[5];
    gemm_p(h, EPI_LN, hid, dff, w.w2, tokens, 192, dff, pln, s);
  }
  HIPCHK(hipGetLastError());
  return NPFN_OK;
}

// Fused variant over up to kRowSegs estimator groups at once: the encoder per group, then per
// layer ONE item-attention launch and ONE k_row_layer launch for all of them (each group a
// segment with its own token count and token tensor, all tensors of the batch live in the
// workspace at token offsets tok0[g]), so each layer's persistent row-kernel grid has one
// tail instead of one per group -- at 8 GPUs a rank's group launches are a few tile rounds
// each, where a tail is a large share.  Per-tile arithmetic is unchanged: results are bit for
// bit those of one launch per group.
// Test side (tgt != null): the last layer runs the rows' target tokens only -- the item
// attention of the target column and a post-only row-kernel launch over the target tokens,
// which writes them packed to tgt + tgt_off[g] ([ne][rows][192], the decoder input); nothing
// else of the last layer is read.  Train side: the last layer's item attention is skipped
// (only its K/V cache is read).  Both bit for bit the target tokens of the full layer.
int forward_groups_fused(npfn_engine* h, const Fit::Group* gs, int ng, const float* ytr, int64_t ldy, int64_t rows,
                         bool train, hipStream_t s, int64_t* tok0, bf16_t* tgt = nullptr,
                         const int64_t* tgt_off = nullptr) {
  if (ng < 1 || ng > kRowSegs) return fail(NPFN_EINVAL, "forward: bad group batch");
  const int L = h->cfg.n_layers, dff = h->cfg.d_ff;
  int64_t tokens = 0;
  for (int g = 0; g < ng; ++g) {
    tok0[g] = tokens;
    tokens += (int64_t)gs[g].ne * rows * gs[g].C;
  }
  const int qw = train ? 576 : 192;
  Work& wk = *h->w;
  RCHK(ensure(wk.resid, tokens * 192 * sizeof(float), s));
  RCHK(ensure(wk.qkv, tokens * qw * sizeof(bf16_t), s));
  RCHK(ensure(wk.attn, tokens * 192 * sizeof(bf16_t), s));
  float* resid = (float*)wk.resid.p;
  bf16_t* qkv = (bf16_t*)wk.qkv.p;
  bf16_t* attn = (bf16_t*)wk.attn.p;
  if (!train && !tgt) return fail(NPFN_EINVAL, "forward: the test side needs the target-token buffer");
  for (int g = 0; g < ng; ++g) {
    const int64_t tg = (int64_t)gs[g].ne * rows * gs[g].C;
    const DevFit fp = h->devfit(gs[g], train);
    ProfGuard pg(h, P_ENCODE, 0.0, (double)tg * 192 * 4, s);
    launch_encode(ytr, ldy, rows, fp, h->encw, h->yencw, h->pos, resid + tok0[g] * 192, nullptr, s);
  }
  const double n_keys = (double)h->f->n;
  const int nproj = train ? 3 : 1;
  const double post_flops = 2.0 * (192.0 * 192 + 2.0 * 192 * dff);
  double pre_flops_sum = 0.0, kv_bytes_l = 0.0;  // over the batch's tokens / caches
  for (int g = 0; g < ng; ++g) {
    const double tg = (double)gs[g].ne * rows * gs[g].C;
    pre_flops_sum += tg * (2.0 * (576.0 * 192 + 192.0 * 192 + nproj * 192.0 * 192) + 128.0 * 6 * gs[g].C);
    kv_bytes_l += (double)gs[g].ne * gs[g].C * 6 * h->f->ntile * 2048 * 2;
  }
  RowLayerParams rp{};
  rp.R = rows;
  rp.nseg = ng;
  rp.ntiles = 0;
  for (int g = 0; g < ng; ++g) {
    RowSeg& sg = rp.seg[g];
    sg.tile0 = rp.ntiles;
    sg.rows = (int64_t)gs[g].ne * rows;
    sg.C = gs[g].C;
    sg.rpt = rowk_rows_per_tile(gs[g].C);
    sg.resid = resid + tok0[g] * 192;
    sg.o_item = attn + tok0[g] * 192;
    sg.tmem = gs[g].C;
    sg.tofs = 0;
    sg.tstride = 1;
    rp.ntiles += (rows + sg.rpt - 1) / sg.rpt * gs[g].ne;
  }
  rp.dff = dff;
  rp.out_qkv = train ? 1 : 0;
  auto set_out = [&](bf16_t* base, int width) {
    for (int g = 0; g < ng; ++g) rp.seg[g].out = base + tok0[g] * width;
  };
  // launch position j = l + 1 streams [post(l) | pre(l + 1)] (build_rowk_streams)
  auto set_stream = [&](int j) {
    rp.stream = h->rowk_stream[j];
    rp.stream_chunks = (rp.do_post ? h->rowk_post[j] : 0) + (rp.do_pre ? 3 * (rp.out_qkv ? 7 : 5) : 0);
  };
  auto set_pre = [&](int l) {
    const LayerW& w = h->layers[l];
    rp.ln1g = w.ln[0];
    rp.ln1b = w.ln[1];
  };
  auto set_post = [&](int l) {
    const LayerW& w = h->layers[l];
    rp.ln2g = w.ln[2];
    rp.ln2b = w.ln[3];
    rp.ln3g = w.ln[4];
    rp.ln3b = w.ln[5];
  };
  IaParams ip{};
  ip.nseg = ng;
  ip.ldq = qw;
  ip.R = rows;
  ip.n = h->f->n;
  ip.ntile = h->f->ntile;
  ip.ny = 0;
  auto set_cols = [&](bool target_only) {  // the columns the item attention runs
    ip.ny = 0;
    for (int g = 0; g < ng; ++g) {
      ip.seg[g].y0 = ip.ny;
      ip.seg[g].C = gs[g].C;
      ip.seg[g].c_lo = target_only ? gs[g].C - 1 : 0;
      ip.seg[g].q = qkv + tok0[g] * qw;
      ip.seg[g].out = attn + tok0[g] * 192;
      ip.ny += gs[g].ne * (gs[g].C - ip.seg[g].c_lo) * 6;
    }
  };
  set_cols(false);
  // layer 0 entry: feature attention of layer 0 + item projections
  rp.do_post = 0;
  rp.do_pre = 1;
  rp.tgt_only = L == 1;  // the last layer's pre part: only the target tokens' rows are read later
  set_out(qkv, qw);
  set_pre(0);
  set_stream(0);
  {
    ProfGuard pg(h, P_ROW_LAYER, pre_flops_sum, (double)tokens * (192 * 8 + nproj * 384), s);
    RCHK(row_launch(h, rp, s));
  }
  for (int l = 0; l < L; ++l) {
    for (int g = 0; g < ng; ++g) {
      const size_t kv_layer = (size_t)gs[g].ne * gs[g].C * 6 * h->f->ntile * 2048;
      bf16_t* kvc = (bf16_t*)h->f->kvc.p + gs[g].kv_off + (size_t)l * kv_layer;
      ip.seg[g].kvc = kvc;
      if (train) {
        // the last layer's item attention reads the target column's cache only (set_cols(true)),
        // and only the target tokens' q | k | v were stored (RowLayerParams::tgt_only)
        const int c_lo = l == L - 1 ? gs[g].C - 1 : 0;
        const double frac = (double)(gs[g].C - c_lo) / gs[g].C;
        const int64_t tg = (int64_t)gs[g].ne * rows * gs[g].C;
        ProfGuard pg(h, P_KV_PACK, 0.0, ((double)tg * 384 * 2 + (double)kv_layer * 2) * frac, s);
        launch_kv_pack(qkv + tok0[g] * 576, rows, gs[g].C, gs[g].ne, h->f->ntile, kvc, s, c_lo);
      }
    }
    if (train && l == L - 1) break;  // train rows' last-layer outputs are never read: K/V only
    const bool last = l == L - 1;
    int64_t ltok = tokens;  // tokens the item attention and the post part run
    if (last) {
      ltok = 0;
      for (int g = 0; g < ng; ++g) ltok += (int64_t)gs[g].ne * rows;
      set_cols(true);
    }
    {
      ProfGuard pg(h, P_ITEM_ATTN, (double)ltok * 6 * 128 * n_keys, (double)ltok * 192 * 4 + kv_bytes_l, s);
      ia_launch(h, ip, s);
    }
    set_post(l);
    rp.do_post = 1;
    rp.do_pre = last ? 0 : 1;
    rp.tgt_only = l + 1 == L - 1;
    if (rp.do_pre) {
      set_pre(l + 1);
      set_out(qkv, qw);
    } else {  // last layer: the rows' target tokens, packed into tgt for the decoder
      rp.ntiles = 0;
      for (int g = 0; g < ng; ++g) {
        RowSeg& sg = rp.seg[g];
        sg.tile0 = rp.ntiles;
        sg.C = 1;
        sg.rpt = rowk_rows_per_tile(1);
        sg.tmem = sg.tstride = gs[g].C;
        sg.tofs = gs[g].C - 1;
        sg.out = tgt + tgt_off[g];
        rp.ntiles += (rows + sg.rpt - 1) / sg.rpt * gs[g].ne;
      }
    }
    set_stream(l + 1);
    ProfGuard pg(h, P_ROW_LAYER, ltok * post_flops + (rp.do_pre ? pre_flops_sum : 0.0),
                 (double)ltok * (192 * 2 + 192 * 8 + 384) + (rp.do_pre ? (double)tokens * 384 * nproj : 0.0), s);
    RCHK(row_launch(h, rp, s));
  }
  HIPCHK(hipGetLastError());
  return NPFN_OK;
}

// The forward of every estimator group of the range over `rows` rows of X.  Test side: the
// views of X are computed first and every group's last-layer target tokens are packed into
// h->tgt [ne][rows][192] (the decoder input).  Train side: the fit has already written the
// train views (with collision-resolved fingerprints); the groups fill the K/V cache.
int forward_any(npfn_engine* h, const float* X, int64_t ldx, const float* ytr, int64_t ldy, int64_t rows, bool train,
                hipStream_t s) {
  if (!train) {
    RCHK(ensure(h->views, (size_t)std::max<int64_t>(rows, 1) * h->f->vl.Vw * sizeof(float), s));
    const ViewParams vp = h->viewparams();
    ProfGuard g(h, P_VIEWS, 0.0, (double)rows * (h->f->F + h->f->vl.Vw) * 4, s);
    launch_views_base(X, ldx, rows, vp, (float*)h->views.p, s);
    launch_views_svd(rows, vp, (float*)h->views.p, s);
    launch_views_fp_test(X, ldx, rows, vp, (float*)h->views.p, s);
    h->last_views = &h->views;
    RCHK(ensure(h->tgt, (size_t)h->ne * std::max<int64_t>(rows, 1) * 192 * sizeof(bf16_t), s));
  }
  const std::vector<Fit::Group>& groups = h->f->groups;
  for (size_t g0 = 0; g0 < groups.size();) {
    // the fused path batches up to kRowSegs consecutive groups that fit its 256-slot tile; a wide
    // group (C > kRowMaxC) or the NPFN_UNFUSED=1 path runs alone through the per-sublayer kernels
    if (h->fused && groups[g0].C <= kRowMaxC) {
      int ng = 1;
      while (ng < kRowSegs && g0 + ng < groups.size() && groups[g0 + ng].C <= kRowMaxC) ++ng;
      int64_t tok0[kRowSegs] = {0, 0, 0, 0};
      // the target tokens land packed in h->tgt [ne][rows][192] straight from the last layer
      int64_t toff[kRowSegs] = {0, 0, 0, 0};
      for (int g = 0; g < ng; ++g) toff[g] = (int64_t)((groups[g0 + g].e0 - h->e0) / h->es) * rows * 192;
      RCHK(forward_groups_fused(h, &groups[g0], ng, ytr, ldy, rows, train, s, tok0,
                                train ? nullptr : (bf16_t*)h->tgt.p, toff));
      g0 += ng;
      continue;
    }
    const Fit::Group& grp = groups[g0++];
    if (train) {
      RCHK(forward_rows(h, grp, ytr, ldy, rows, true, s));
      continue;
    }
    // test rows in chunks of about kWideTokens tokens (a wide group's per-sublayer tensors hold
    // ~4.2 KB per token), each chunk's target tokens (index C - 1) copied into h->tgt
    const int64_t step = std::max<int64_t>(1, kWideTokens / ((int64_t)grp.ne * grp.C));
    for (int64_t r0 = 0; r0 < rows; r0 += step) {
      const int64_t rr = std::min(step, rows - r0);
      RCHK(forward_rows(h, grp, nullptr, 0, rr, false, s, r0));
      const bf16_t* src = (const bf16_t*)h->w->resid_bf.p + (size_t)(grp.C - 1) * 192;
      for (int e = 0; e < grp.ne; ++e) {
        bf16_t* dst = (bf16_t*)h->tgt.p + ((size_t)((grp.e0 - h->e0) / h->es + e) * rows + r0) * 192;
        HIPCHK(hipMemcpy2DAsync(dst, 192 * sizeof(bf16_t), src + (size_t)e * rr * grp.C * 192,
                                (size_t)grp.C * 192 * sizeof(bf16_t), 192 * sizeof(bf16_t), (size_t)rr,
                                hipMemcpyDeviceToDevice, s));
      }
    }
  }
  return NPFN_OK;
}

// host copy of preprocess_oracle.svd_components / n_features_of
int svd_components(int64_t n, int F) { return F < 2 ? 0 : (int)std::max<int64_t>(1, std::min<int64_t>(n / 10 + 1, F / 2)); }
int pipeline_features_host(int t, int F, int k) {
  return t == T_QSVD ? 2 * F + k + 1 : ((t == T_PFP || t == T_RFP) ? F + 1 : F);
}

// Preprocessing part of a fit into h->f (everything the train forward reads: estimator groups,
// view layout and fit statistics, per-estimator tables, the train rows' views).  It reads only
// the context, so the AR calls run every step's on a side stream ahead of time (ar_prefit).
int fit_prep(npfn_engine* h, const float* X, int64_t ldx, const float* y, int64_t ldy, int64_t n, int F,
             hipStream_t s, int ncls = 0) {
  if (!X || !y) return fail(NPFN_EINVAL, "fit: null X or y");
  if (n < 1) return fail(NPFN_EINVAL, "fit: need at least one context row");
  if (F < 1) return fail(NPFN_EINVAL, "fit: need at least one feature");
  if (ldx < F) return fail(NPFN_EINVAL, "fit: ldx < n_features");
  const int E = h->cfg.n_estimators;
  bool need_q = false, need_p = false, need_svd = false, need_fp = false;
  for (int e = 0; e < E; ++e) {
    const int t = h->h_ftype[e];
    need_q |= t == T_QUANT || t == T_QSVD;
    need_p |= t == T_POWER || t == T_PFP;
    need_svd |= t == T_QSVD;
    need_fp |= t == T_QSVD || t == T_PFP || t == T_RFP;
  }
  if (need_q && quantile_count(n, h->qdiv) > kQtSubsample)  // sklearn QuantileTransformer.fit's ValueError
    return fail(NPFN_EINVAL, "fit: The number of quantiles cannot be greater than the number of samples used. Got " +
                                 std::to_string(quantile_count(n, h->qdiv)) + " quantiles and " +
                                 std::to_string(kQtSubsample) + " samples.");
  if (need_q && n > kQtSubsampleMaxRows)
    return fail(NPFN_EINVAL, "fit: the quantile preprocessing's row subsample takes at most " +
                                 std::to_string(kQtSubsampleMaxRows) + " context rows (" + std::to_string(n) +
                                 " given)");
  const int k = need_svd ? svd_components(n, F) : 0;
  if (need_svd && F >= 2 && 2 * F > kSvdLargeMaxM && n > kSvdMaxM)
    return fail(NPFN_EINVAL, "fit: the ensemble's SVD takes at most " + std::to_string(kSvdLargeMaxM / 2) +
                                 " features past " + std::to_string(kSvdMaxM) + " context rows (" + std::to_string(F) +
                                 " features, " + std::to_string(n) + " rows given)");
  // estimator groups of the range: consecutive estimators with equal token count
  h->f->groups.clear();
  size_t kv_off = 0;
  // 32-key tiles, rounded up to whole 64-key steps of k_item_attn: the padding keys are packed
  // as zeros (K = V = 0), which the item attention's first pass counts instead of masking
  h->f->ntile = (int)((n + 32 * kIaTileQuantum - 1) / (32 * kIaTileQuantum)) * kIaTileQuantum;
  for (int i = 0; i < h->ne; ++i) {
    const int e = h->e0 + h->es * i;
    const int Fe = pipeline_features_host(h->h_ftype[e], F, k);
    const int Ge = (Fe + 1) / 2, Ce = Ge + 1;
    if (Ge > h->cfg.max_groups) return fail(NPFN_EINVAL, "fit: too many features for max_groups");
    const int cmax = kWideMaxC;  // C > kRowMaxC (or NPFN_UNFUSED=1): the per-sublayer path
    if (Ce > cmax)
      return fail(NPFN_EINVAL, "fit: an estimator's pipeline has " + std::to_string(Fe) + " features (" +
                                   std::to_string(Ce) + " tokens per row); the engine holds at most " +
                                   std::to_string(2 * (cmax - 1)) + " features (" + std::to_string(cmax) +
                                   " tokens) per estimator");
    if (!h->f->groups.empty() && h->f->groups.back().C == Ce) {
      h->f->groups.back().ne += 1;
    } else {
      h->f->groups.push_back({e, 1, Ce, 0});
    }
  }
  for (auto& g : h->f->groups) {
    g.kv_off = kv_off;
    kv_off += (size_t)h->cfg.n_layers * g.ne * g.C * 6 * h->f->ntile * 2048;
  }
  h->f->fitted = false;
  h->f->vl = view_layout(F, k, E, need_q ? 1 : 0, need_p ? 1 : 0, need_fp ? 1 : 0);
  const int Vw = h->f->vl.Vw;
  RCHK(ensure(h->f->colstat, (size_t)Vw * 3 * sizeof(float), s));
  RCHK(ensure(h->f->ystats, 6 * sizeof(float), s));
  RCHK(ensure(h->f->vcol, (size_t)E * h->Fmax() * sizeof(int), s));
  RCHK(ensure(h->f->mu, (size_t)E * h->Fmax() * sizeof(float), s));
  RCHK(ensure(h->f->sd, (size_t)E * h->Fmax() * sizeof(float), s));
  RCHK(ensure(h->f->gscale, (size_t)E * h->cfg.max_groups * sizeof(float), s));
  RCHK(ensure(h->f->eF, (size_t)E * sizeof(int), s));
  RCHK(ensure(h->f->tviews, (size_t)n * Vw * sizeof(float), s));
  RCHK(ensure(h->f->ylam, sizeof(double), s));
  h->f->F = F;
  h->f->n = n;
  float* views = (float*)h->f->tviews.p;
  h->last_views = &h->f->tviews;
  // one profiler entry per preprocessing kernel (each a separate launch on s)
  if (need_q) {
    h->f->nqmax = quantile_count(n, h->qdiv);
    RCHK(ensure(h->f->qtab, (size_t)F * h->f->nqmax * sizeof(double), s));
    RCHK(ensure(h->f->qn, (size_t)F * sizeof(int), s));
    RCHK(ensure(h->f->qstat, (size_t)F * 3 * sizeof(float), s));
    const int* sub = nullptr;
    if (n > kQtSubsample) {
      RCHK(ensure(h->f->qsub, (size_t)kQtSubsample * sizeof(int), s));
      launch_qt_subsample(n, (uint32_t)h->cfg.random_state, (int*)h->f->qsub.p, s);
      sub = (const int*)h->f->qsub.p;
    }
    ProfGuard g(h, P_QUANT_FIT, 0.0, (double)n * F * 4, s);
    launch_quantile_fit(X, ldx, n, F, h->qdiv, h->f->nqmax, sub, (double*)h->f->qtab.p, (int*)h->f->qn.p,
                        (float*)h->f->qstat.p, s);
  }
  // the target's Yeo-Johnson lambda (ensemble regressor) rides in the features' power-fit launch
  const bool tt = h->any_tt && ncls == 0;
  if (tt) RCHK(ensure(h->f->tscratch, 4 * sizeof(float), s));
  if (need_p) {
    RCHK(ensure(h->f->plam, (size_t)F * sizeof(double), s));
    RCHK(ensure(h->f->pstat, (size_t)F * 3 * sizeof(float), s));
    ProfGuard g(h, P_POWER_FIT, 0.0, (double)n * (F + (tt ? 1 : 0)) * 4, s);
    launch_power_fit(X, ldx, n, F, (double*)h->f->plam.p, (float*)h->f->pstat.p, s, tt ? y : nullptr, ldy,
                     (double*)h->f->ylam.p, (float*)h->f->tscratch.p);
  }
  if (k > 0) {
    RCHK(ensure(h->f->svd, (size_t)(2 * F) * (k + 1) * sizeof(double), s));
    RCHK(ensure(h->f->svdw, svd_work_bytes(n, 2 * F), s));
  }
  if (need_fp) RCHK(ensure(h->f->htab, (size_t)E * fp_total(n) * sizeof(int), s));
  const ViewParams vp = h->viewparams();
  {
    ProfGuard g(h, P_VIEWS, 0.0, (double)n * (F + Vw) * 4, s);
    launch_views_base(X, ldx, n, vp, views, s);
  }
  if (k > 0) {
    {
      ProfGuard g(h, P_SVD_FIT, 0.0, (double)n * 2 * F * 4, s);
      const int src = launch_svd_fit(views, n, h->f->vl, h->f->svdw.p, (double*)h->f->svd.p, s);
      if (src == -2)
        return fail(NPFN_EHIP, "fit: the SVD's eigensolver (rocSOLVER dsyevd) did not converge (info != 0)");
      if (src != 0)
        return fail(NPFN_EINVAL, "fit: the SVD's shape is out of range or its eigensolver (rocSOLVER) failed to start");
    }
    ProfGuard g(h, P_VIEWS, 0.0, (double)n * (2 * F + k) * 4, s);
    launch_views_svd(n, vp, views, s);
  }
  if (need_fp) {
    ProfGuard g(h, P_FP_TRAIN, 0.0, (double)n * F * 4, s);
    launch_fp_train(X, ldx, n, vp, (int*)h->f->htab.p, views, s);
  }
  {
    ProfGuard gst(h, P_STATS, 0.0, (double)n * (Vw + 1) * 4 * 2, s);
    launch_col_stats(views, Vw, y, ldy, n, Vw, (float*)h->f->colstat.p, (float*)h->f->ystats.p, s);
    launch_build_params((const float*)h->f->colstat.p, F, k, E, h->Fmax(), h->cfg.max_groups, h->cfg.random_state,
                        (const int*)h->ftype.p, h->f->vl, (int*)h->f->vcol.p, (float*)h->f->mu.p, (float*)h->f->sd.p,
                        (float*)h->f->gscale.p, (int*)h->f->eF.p, s);
  }
  if (tt) {
    const int nb = h->cfg.n_bars;
    RCHK(ensure(h->f->ttab, (size_t)(nb + 1) * sizeof(TransEntry), s));
    RCHK(ensure(h->f->tcancel, (size_t)nb + 4, s));
    ProfGuard g(h, P_TARGET_TF, 0.0, (double)n * 4, s);
    launch_target_tf(y, ldy, n, h->bz, nb, (double*)h->f->ylam.p, (float*)h->f->ystats.p, (TransEntry*)h->f->ttab.p,
                     (uint8_t*)h->f->tcancel.p, (float*)h->f->tscratch.p, s, /*fit_lambda=*/!need_p);
  }
  h->f->ncls = ncls;
  if (ncls > 0) {
    RCHK(ensure(h->f->cperm, (size_t)E * KMAX_CLS * sizeof(int), s));
    RCHK(ensure(h->f->ybar_e, (size_t)E * sizeof(float), s));
    ProfGuard gst(h, P_STATS, 0.0, (double)n * 4, s);
    launch_class_params(y, ldy, n, ncls, E, h->cfg.random_state, (int*)h->f->cperm.p, (float*)h->f->ybar_e.p, s);
  }
  h->f->kv_elems = kv_off;
  return NPFN_OK;
}

// Train-side forward of a prepared fit: fills the K/V cache.
int fit_train(npfn_engine* h, const float* X, int64_t ldx, const float* y, int64_t ldy, int64_t n, hipStream_t s) {
  RCHK(ensure(h->f->kvc, h->f->kv_elems * sizeof(bf16_t), s));
  RCHK(forward_any(h, X, ldx, y, ldy, n, true, s));
  h->f->fitted = true;
  return NPFN_OK;
}

int fit_impl(npfn_engine* h, const float* X, int64_t ldx, const float* y, int64_t ldy, int64_t n, int F,
             hipStream_t s, int ncls = 0) {
  RCHK(fit_prep(h, X, ldx, y, ldy, n, F, s, ncls));
  return fit_train(h, X, ldx, y, ldy, n, s);
}

// Decoder head over E x rows target tokens -> h->logits [E][rows][nb]: token (e, r) is the
// bf16 row A + (e * rows + r) * lda (the last layer's target token in the forward's token
// tensor, lda = C * 192, or a packed [E][rows][192] buffer from npfn_forward_targets).
// Every output element's K order is fixed, so a row's logits do not depend on lda or rows.
int decode_chunk(npfn_engine* h, const bf16_t* A, int64_t lda, int E, int64_t rows, hipStream_t s) {
  const int dff = h->cfg.d_ff, nb = h->cfg.n_bars;
  RCHK(ensure(h->dh, (size_t)E * rows * dff * sizeof(bf16_t), s));
  RCHK(ensure(h->logits, (size_t)E * rows * nb * sizeof(logit_t), s));
  EpiParams p1;
  p1.out_bf = (bf16_t*)h->dh.p;
  p1.ldo = dff;
  p1.bias = h->dec_b1;
  gemm_p(h, EPI_BF16_GELU, A, lda, h->dec_w1, (int64_t)E * rows, dff, 192, p1, s);
  EpiParams p2;
  p2.out_l = (logit_t*)h->logits.p;
  p2.ldo = nb;
  p2.bias = h->dec_b2;
  gemm_p(h, EPI_LOGIT, (const bf16_t*)h->dh.p, dff, h->dec_w2, (int64_t)E * rows, nb, dff, p2, s);
  HIPCHK(hipGetLastError());
  return NPFN_OK;
}

// Test-side forward + decoder for rows [0, rows) of Xq -> h->logits [E][rows][nb]
int predict_logits_chunk(npfn_engine* h, const float* Xq, int64_t ldq, int64_t rows, hipStream_t s) {
  RCHK(forward_any(h, Xq, ldq, nullptr, 0, rows, false, s));
  return decode_chunk(h, (const bf16_t*)h->tgt.p, 192, h->ne, rows, s);
}

int need_full_range(npfn_engine* h, const char* what) {
  if (h->e0 != 0 || h->ne != h->cfg.n_estimators)
    return fail(NPFN_ESTATE, std::string(what) + " mixes all estimators: call npfn_set_estimator_range(h, 0, "
                                                 "n_estimators) first (this engine holds a partial range)");
  return NPFN_OK;
}

// Per-estimator pipeline / target transform / fingerprint salt of a preprocessing mode
// (oracle preprocess_oracle.estimator_configs, fingerprint_salt), uploaded synchronously:
// not on the sampling path.
int apply_preprocessing(npfn_engine* h, int mode, bool classifier = false) {
  const int E = h->cfg.n_estimators;
  h->h_ftype.assign(E, T_RAW);
  h->h_tt.assign(E, 0);
  h->h_salt.assign(E, -1);
  h->qdiv = 5;
  if (mode == 3) {
    // regressor: 2 feature pipelines x 2 target transforms; classifier (oracle
    // preprocess_oracle estimator_configs(classifier=True)): coarse-quantile + SVD | original,
    // both with the fingerprint, no target transform
    const int ncombo = classifier ? 2 : 4;
    const int combo_t[4] = {T_QSVD, T_QSVD, T_PFP, T_PFP}, combo_tt[4] = {0, 1, 0, 1};
    const int ccombo_t[2] = {T_QSVD, T_RFP};
    const int bc = E / ncombo;
    for (int e = 0; e < E; ++e) {
      const int c = e < ncombo * bc ? e / bc : e - ncombo * bc;  // balanced in product order, leftovers in order
      h->h_ftype[e] = classifier ? ccombo_t[c] : combo_t[c];
      h->h_tt[e] = classifier ? 0 : combo_tt[c];
      uint64_t st = ((h->cfg.random_state & 0xFFFFFFFFull) | ((uint64_t)(e & 0xFFFF) << 32)) ^ 0xF1A6E4A7F1A6E4A7ull;
      st += 0x9E3779B97F4A7C15ull;  // splitmix64_next
      uint64_t z = st;
      z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
      z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
      z ^= z >> 31;
      h->h_salt[e] = (int)(z % 65536ull);
    }
    if (classifier) h->qdiv = 10;  // tabpfn "quantile_uni_coarse"
  } else if (mode == 1 || mode == 2) {
    for (int e = 0; e < E; ++e) h->h_ftype[e] = (e % 2 == 0) ? T_QUANT : (mode == 2 ? T_POWER : T_RAW);
  }
  h->any_tt = false;
  for (int e = 0; e < E; ++e) h->any_tt |= h->h_tt[e] != 0;
  RCHK(ensure(h->ftype, E * sizeof(int), nullptr));
  RCHK(ensure(h->ett, E * sizeof(int), nullptr));
  RCHK(ensure(h->fp_salt, E * sizeof(int), nullptr));
  HIPCHK(hipMemcpy(h->ftype.p, h->h_ftype.data(), E * sizeof(int), hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(h->ett.p, h->h_tt.data(), E * sizeof(int), hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(h->fp_salt.p, h->h_salt.data(), E * sizeof(int), hipMemcpyHostToDevice));
  h->pre_mode = mode;
  h->pre_cls = classifier;
  return NPFN_OK;
}
// the pipeline assignment of the engine's mode for a regressor (classifier = false) or a
// classifier fit; mode 3 differs between the two (re-uploaded only on a switch)
int ensure_pipelines(npfn_engine* h, bool classifier) {
  if (h->pre_mode != 3 || h->pre_cls == classifier) return NPFN_OK;
  RCHK(apply_preprocessing(h, 3, classifier));
  h->ar_active = false;  // an AR fit sequence begun under the other pipelines is void (as in the other setters)
  h->ar_reuse = false;
  for (Fit& sl : h->slots) sl.fitted = false;
  std::memset(h->slot_key, 0, sizeof(h->slot_key));
  h->fit0.fitted = false;
  return NPFN_OK;
}

int check_engine(npfn_engine* h) {
  if (!h) return fail(NPFN_EINVAL, "null engine");
  HIPCHK(hipSetDevice(h->cfg.device));
  return NPFN_OK;
}

// per > 1: xq holds N / per distinct rows, query row i = xq[i / per] (npfn_ar_sample_repeated)
int ar_common_setup(npfn_engine* h, const float* x_ctx, const float* theta_ctx, int64_t n, int dx, int dth,
                    const float* xq, int64_t N, hipStream_t s, int64_t per = 1) {
  if (!x_ctx || !theta_ctx || !xq) return fail(NPFN_EINVAL, "ar: null input");
  if (dx < 1 || dth < 1 || n < 1 || N < 0) return fail(NPFN_EINVAL, "ar: bad dimensions");
  const int Ft = dx + dth;
  RCHK(ensure(h->joint, (size_t)n * Ft * sizeof(float), s));
  RCHK(ensure(h->feat, (size_t)std::max<int64_t>(N, 1) * Ft * sizeof(float), s));
  RCHK(ensure(h->logp, (size_t)std::max<int64_t>(N, 1) * sizeof(float), s));
  launch_copy_cols(x_ctx, dx, (float*)h->joint.p, Ft, n, dx, 0, s);
  launch_copy_cols(theta_ctx, dth, (float*)h->joint.p, Ft, n, dth, dx, s);
  launch_copy_cols(xq, dx, (float*)h->feat.p, Ft, N, dx, 0, s, per);
  launch_fill((float*)h->logp.p, N, 0.f, s);
  return NPFN_OK;
}

// Selects the fit of AR step k (npfn_ar_sample / npfn_ar_log_prob).  Without a fit token:
// fit0, refitted every call.  With one (npfn_set_fit_token): the per-step slot k, refitted
// only when the token or the call's shape changed since the slots were filled -- the
// accept/reject batches of one sample() call share their context (npe_pfn.py:284-292).
// Returns in `refit` whether step k must be fitted.
void begin_ar_fits(npfn_engine* h, int64_t n, int dx, int dth, bool& reuse) {
  const uint64_t key[6] = {h->fit_token, (uint64_t)n, (uint64_t)dx, (uint64_t)dth, (uint64_t)h->pre_mode,
                           ((uint64_t)h->es << 48) | ((uint64_t)h->e0 << 24) | (uint64_t)h->ne};
  reuse = h->fit_token != 0 && (int)h->slots.size() >= dth && std::memcmp(key, h->slot_key, sizeof(key)) == 0;
  if (h->fit_token != 0 && !reuse) {
    if ((int)h->slots.size() < dth) h->slots.resize(dth);
    std::memset(h->slot_key, 0, sizeof(h->slot_key));
    // a slot filled under another token, context or estimator set is not a fit of this call
    for (Fit& sl : h->slots) sl.fitted = false;
  }
}
void end_ar_fits(npfn_engine* h, int64_t n, int dx, int dth) {
  if (h->fit_token == 0) return;
  const uint64_t key[6] = {h->fit_token, (uint64_t)n, (uint64_t)dx, (uint64_t)dth, (uint64_t)h->pre_mode,
                           ((uint64_t)h->es << 48) | ((uint64_t)h->e0 << 24) | (uint64_t)h->ne};
  std::memcpy(h->slot_key, key, sizeof(key));
}
Fit* step_fit(npfn_engine* h, int k) { return h->fit_token != 0 ? &h->slots[k] : &h->fit0; }

// The fits of the AR steps (slot k: fit on x | theta[:, :k] -> theta[:, k]) depend on the
// context only, not on the samples of the earlier steps, so with per-step slots they run
// ahead of the main stream.  Every step's preprocessing fit goes on the engine's
// (lowest-priority) side stream, in order, right after the call's setup (one-block,
// latency-bound kernels: Yeo-Johnson searches, SVD sweeps, fingerprint hashing).  Step 0's
// train forward is on the critical path (nothing else can run before it), so it runs on the
// main stream as soon as its preprocessing is done; step k >= 1's train forward runs on
// side_t (own workspaces wside), queued kTrainAhead steps ahead -- steps 1 and
// 2 with the preprocessing, step k + 2 when the main stream starts step k -- not all at once:
// a forward is ~37 launches, and a deep backlog fills the side queues' packet rings, so that
// the host blocks inside a launch and issues the main stream's work late (measured: all ten
// queued up front held step 0 back 40 ms).  The train forwards fill the tails of the main
// stream's test-side launches.  prep_done[k] = step
// k's fit is complete.  `piped` = whether that happened (no fit token: fit0 is refitted in
// order on the main stream).
// A/B switch: NPFN_TRAIN_AHEAD=<steps> (default 2)
static const int kTrainAhead = [] {
  const char* e = getenv("NPFN_TRAIN_AHEAD");
  const int v = e ? atoi(e) : 2;
  return v < 0 ? 0 : v;  // 0: every train forward in order on the main stream
}();
int ar_side_train(npfn_engine* h, const float* joint, int Ft, int64_t n, int F, int k) {
  hipStream_t t = h->side_t;
  Fit* keep_f = h->f;
  Work* keep_w = h->w;
  h->f = &h->slots[k];
  h->w = &h->wside;
  int rc = hipStreamWaitEvent(t, h->stat_done[k], 0) == hipSuccess ? NPFN_OK : fail(NPFN_EHIP, "stream wait");
  if (rc == NPFN_OK) rc = fit_train(h, joint, Ft, joint + F, Ft, n, t);
  h->f = keep_f;
  h->w = keep_w;
  RCHK(rc);
  HIPCHK(hipEventRecord(h->prep_done[k], t));
  return NPFN_OK;
}
int ar_prefit(npfn_engine* h, const float* joint, int Ft, int64_t n, int dx, int dth, hipStream_t s, bool& piped) {
  piped = false;
  // while the live profiler is on, the fits run in order on the main stream: an event pair
  // then times its launch alone, not the launch plus whatever shared the CUs with it
  static const bool serial = [] { const char* e = getenv("NPFN_SERIAL_FITS"); return e && e[0] == '1'; }();  // A/B
  if (h->fit_token == 0 || dth < 2 || h->prof.on || serial) return NPFN_OK;
  if (!h->side) {
    int least = 0, greatest = 0;
    HIPCHK(hipDeviceGetStreamPriorityRange(&least, &greatest));
    HIPCHK(hipStreamCreateWithPriority(&h->side, hipStreamNonBlocking, least));
    HIPCHK(hipStreamCreateWithPriority(&h->side_t, hipStreamNonBlocking, least));
    HIPCHK(hipEventCreateWithFlags(&h->setup_done, hipEventDisableTiming));
  }
  while ((int)h->prep_done.size() < dth) {
    hipEvent_t e, e2;
    HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    HIPCHK(hipEventCreateWithFlags(&e2, hipEventDisableTiming));
    h->prep_done.push_back(e);
    h->stat_done.push_back(e2);
  }
  // the context table was written on s, and the slots' buffers may still be read by s's work
  // of the previous call
  HIPCHK(hipEventRecord(h->setup_done, s));
  HIPCHK(hipStreamWaitEvent(h->side, h->setup_done, 0));
  HIPCHK(hipStreamWaitEvent(h->side_t, h->setup_done, 0));
  // issue order: the preprocessing of steps 0 .. kTrainAhead, each early step's train forward
  // right behind its preprocessing, then the remaining steps' preprocessing
  Fit* keep_f = h->f;
  for (int k = 0; k < dth; ++k) {
    const int F = dx + k;
    h->f = &h->slots[k];
    int rc = fit_prep(h, joint, Ft, joint + F, Ft, n, F, h->side);
    if (rc == NPFN_OK && hipEventRecord(h->stat_done[k], h->side) != hipSuccess) rc = fail(NPFN_EHIP, "event");
    if (rc == NPFN_OK && k == 0) {  // step 0 on the main stream, in its own workspaces
      if (hipStreamWaitEvent(s, h->stat_done[0], 0) != hipSuccess) rc = fail(NPFN_EHIP, "stream wait");
      if (rc == NPFN_OK) rc = fit_train(h, joint, Ft, joint + F, Ft, n, s);
    }
    h->f = keep_f;
    RCHK(rc);
    if (k >= 1 && k <= kTrainAhead) RCHK(ar_side_train(h, joint, Ft, n, F, k));
  }
  piped = true;
  return NPFN_OK;
}
// Fit of AR step k (h->f = its slot) unless reused: when piped, wait for it on s and queue
// step k + kTrainAhead's train forward (step 0: already on s); otherwise the whole fit in
// order on s.
int ar_step_fit(npfn_engine* h, const float* joint, int Ft, int64_t n, int dx, int dth, int k, bool piped,
                hipStream_t s) {
  if (!piped) return fit_impl(h, joint, Ft, joint + dx + k, Ft, n, dx + k, s);
  if (k == 0) return NPFN_OK;  // fitted on s by ar_prefit
  if (kTrainAhead == 0) {
    HIPCHK(hipStreamWaitEvent(s, h->stat_done[k], 0));
    return fit_train(h, joint, Ft, joint + dx + k, Ft, n, s);
  }
  HIPCHK(hipStreamWaitEvent(s, h->prep_done[k], 0));
  if (k + kTrainAhead < dth) RCHK(ar_side_train(h, joint, Ft, n, dx + k + kTrainAhead, k + kTrainAhead));
  return NPFN_OK;
}

// npfn_ar_sample (n_unique = 0: x_query [n_rows][dim_x]) and npfn_ar_sample_repeated
// (x_query [n_unique][dim_x], query row i = x_query[i / (n_rows / n_unique)]).  With repeated
// rows, step 0 -- whose features are the query rows alone -- runs the forward, decoder and
// ensemble mix once per distinct row and every draw samples from its row's mixture
// (k_group_sample); steps >= 1 see distinct sampled columns and run over every row.
int ar_sample_impl(npfn_engine* h, const float* x_ctx, const float* theta_ctx, int64_t n_ctx, int dim_x,
                   int dim_theta, const float* x_query, int64_t n_unique, int64_t n_rows, uint64_t counter,
                   int64_t row_base, float* theta_out, float* log_prob_out, float eps, hipStream_t s) {
  if (!theta_out) return fail(NPFN_EINVAL, "ar_sample: null theta_out");
  if (row_base < 0) return fail(NPFN_EINVAL, "ar_sample: negative row_base");
  RCHK(need_full_range(h, "ar_sample"));
  RCHK(ensure_pipelines(h, false));
  const int64_t per = n_unique > 0 ? n_rows / n_unique : 1;
  RCHK(ar_common_setup(h, x_ctx, theta_ctx, n_ctx, dim_x, dim_theta, x_query, n_rows, s, per));
  const int Ft = dim_x + dim_theta, E = h->cfg.n_estimators, nb = h->cfg.n_bars;
  const float invT = 1.0f / h->cfg.softmax_temperature;
  const float log_eps = logf(eps);
  float* joint = (float*)h->joint.p;
  float* feat = (float*)h->feat.p;
  float* logp = log_prob_out ? (float*)h->logp.p : nullptr;
  bool reuse = false, piped = false;
  begin_ar_fits(h, n_ctx, dim_x, dim_theta, reuse);
  if (!reuse) RCHK(ar_prefit(h, joint, Ft, n_ctx, dim_x, dim_theta, s, piped));
  for (int k = 0; k < dim_theta; ++k) {
    const int F = dim_x + k;
    h->f = step_fit(h, k);
    if (!reuse) RCHK(ar_step_fit(h, joint, Ft, n_ctx, dim_x, dim_theta, k, piped, s));
    if (k == 0 && n_unique > 0 && n_rows > 0) {
      RCHK(ensure(h->pu, (size_t)n_unique * nb * sizeof(float), s));
      float* pu = (float*)h->pu.p;
      for (int64_t u0 = 0; u0 < n_unique; u0 += h->chunk_rows) {
        const int64_t rows = std::min(h->chunk_rows, n_unique - u0);
        RCHK(predict_logits_chunk(h, x_query + u0 * dim_x, dim_x, rows, s));
        ProfGuard g(h, P_MIX_SAMPLE, 0.0, (double)E * rows * nb * sizeof(logit_t), s);
        launch_mix_prob((const logit_t*)h->logits.p, rows, E, nb, invT, h->mixtrans(), pu + u0 * nb, s);
      }
      ProfGuard g(h, P_MIX_SAMPLE, 0.0, (double)n_rows * nb * 4, s);
      launch_group_sample(pu, per, n_rows, nb, h->bz, (const float*)h->f->ystats.p, h->cfg.random_state,
                          counter + (uint64_t)k, 0, (uint64_t)row_base, feat, Ft, F, logp, log_eps, s);
      continue;
    }
    for (int64_t r0 = 0; r0 < n_rows; r0 += h->chunk_rows) {
      const int64_t rows = std::min(h->chunk_rows, n_rows - r0);
      RCHK(predict_logits_chunk(h, feat + r0 * Ft, Ft, rows, s));
      ProfGuard g(h, P_MIX_SAMPLE, 0.0, (double)E * rows * nb * sizeof(logit_t), s);
      launch_mix_sample((const logit_t*)h->logits.p, rows, E, nb, invT, h->mixtrans(), h->bz, (const float*)h->f->ystats.p,
                        h->cfg.random_state, counter + (uint64_t)k, r0, (uint64_t)row_base, feat, Ft, F, logp,
                        log_eps, s);
    }
  }
  end_ar_fits(h, n_ctx, dim_x, dim_theta);
  launch_copy_cols(feat + dim_x, Ft, theta_out, dim_theta, n_rows, dim_theta, 0, s);
  if (log_prob_out && n_rows > 0)
    HIPCHK(hipMemcpyAsync(log_prob_out, h->logp.p, n_rows * sizeof(float), hipMemcpyDeviceToDevice, s));
  HIPCHK(hipGetLastError());
  return NPFN_OK;
}

// npfn_ar_log_prob (n_unique = 0) and npfn_ar_log_prob_repeated: step 0 once per distinct query
// row (k_mix_prob), every row's log density of its own theta from its row's mixture (k_group_nll).
int ar_log_prob_impl(npfn_engine* h, const float* x_ctx, const float* theta_ctx, int64_t n_ctx, int dim_x,
                     int dim_theta, const float* x_query, int64_t n_unique, const float* theta, int64_t n_rows,
                     float* log_prob_out, float eps, hipStream_t s) {
  if (!theta || !log_prob_out) return fail(NPFN_EINVAL, "ar_log_prob: null pointer");
  RCHK(need_full_range(h, "ar_log_prob"));
  RCHK(ensure_pipelines(h, false));
  const int64_t per = n_unique > 0 ? n_rows / n_unique : 1;
  RCHK(ar_common_setup(h, x_ctx, theta_ctx, n_ctx, dim_x, dim_theta, x_query, n_rows, s, per));
  const int Ft = dim_x + dim_theta, E = h->cfg.n_estimators, nb = h->cfg.n_bars;
  const float invT = 1.0f / h->cfg.softmax_temperature;
  const float log_eps = logf(eps);
  float* joint = (float*)h->joint.p;
  float* feat = (float*)h->feat.p;
  launch_copy_cols(theta, dim_theta, feat, Ft, n_rows, dim_theta, dim_x, s);
  bool reuse = false, piped = false;
  begin_ar_fits(h, n_ctx, dim_x, dim_theta, reuse);
  if (!reuse) RCHK(ar_prefit(h, joint, Ft, n_ctx, dim_x, dim_theta, s, piped));
  for (int k = 0; k < dim_theta; ++k) {
    const int F = dim_x + k;
    h->f = step_fit(h, k);
    if (!reuse) RCHK(ar_step_fit(h, joint, Ft, n_ctx, dim_x, dim_theta, k, piped, s));
    if (k == 0 && n_unique > 0 && n_rows > 0) {
      RCHK(ensure(h->pu, (size_t)n_unique * nb * sizeof(float), s));
      float* pu = (float*)h->pu.p;
      for (int64_t u0 = 0; u0 < n_unique; u0 += h->chunk_rows) {
        const int64_t rows = std::min(h->chunk_rows, n_unique - u0);
        RCHK(predict_logits_chunk(h, x_query + u0 * dim_x, dim_x, rows, s));
        ProfGuard g(h, P_MIX_NLL, 0.0, (double)E * rows * nb * sizeof(logit_t), s);
        launch_mix_prob((const logit_t*)h->logits.p, rows, E, nb, invT, h->mixtrans(), pu + u0 * nb, s);
      }
      ProfGuard g(h, P_MIX_NLL, 0.0, (double)n_rows * nb * 4, s);
      launch_group_nll(pu, per, n_rows, nb, h->bz, (const float*)h->f->ystats.p, 0, feat, Ft, F, (float*)h->logp.p,
                       log_eps, s);
      continue;
    }
    for (int64_t r0 = 0; r0 < n_rows; r0 += h->chunk_rows) {
      const int64_t rows = std::min(h->chunk_rows, n_rows - r0);
      RCHK(predict_logits_chunk(h, feat + r0 * Ft, Ft, rows, s));
      ProfGuard g(h, P_MIX_NLL, 0.0, (double)E * rows * nb * sizeof(logit_t), s);
      launch_mix_nll((const logit_t*)h->logits.p, rows, E, nb, invT, h->mixtrans(), h->bz, (const float*)h->f->ystats.p, r0, feat,
                     Ft, F, (float*)h->logp.p, log_eps, s);
    }
  }
  end_ar_fits(h, n_ctx, dim_x, dim_theta);
  if (n_rows > 0)
    HIPCHK(hipMemcpyAsync(log_prob_out, h->logp.p, n_rows * sizeof(float), hipMemcpyDeviceToDevice, s));
  HIPCHK(hipGetLastError());
  return NPFN_OK;
}

}  // namespace

// =================================================================== C-ABI
extern "C" {

int npfn_version(void) { return 1; }

const char* npfn_last_error(void) { return g_err.c_str(); }

size_t npfn_weights_size(const npfn_config* cfg) {
  if (!cfg) return 0;
  return blob_size(cfg);
}

int npfn_engine_create(const npfn_config* cfg, const float* weights, size_t n_weights, npfn_engine** out) {
  RCHK(check_cfg(cfg));
  if (!weights || !out) return fail(NPFN_EINVAL, "null weights or out pointer");
  if (n_weights != blob_size(cfg))
    return fail(NPFN_EINVAL, "weight blob has " + std::to_string(n_weights) + " floats, expected " +
                                 std::to_string(blob_size(cfg)));
  int ndev = 0;
  HIPCHK(hipGetDeviceCount(&ndev));
  if (cfg->device < 0 || cfg->device >= ndev) return fail(NPFN_EINVAL, "bad device ordinal");
  HIPCHK(hipSetDevice(cfg->device));
  npfn_engine* h = new npfn_engine();
  h->cfg = *cfg;
  h->ne = cfg->n_estimators;
  if (apply_preprocessing(h, 3) != NPFN_OK) {
    const int rc2 = NPFN_ENOMEM;
    npfn_engine_destroy(h);
    return rc2;
  }
  const size_t d = cfg->d_model, dff = cfg->d_ff, nb = cfg->n_bars, G = cfg->max_groups;
  const float* p = weights;
  int rc = NPFN_OK;
  auto f32 = [&](size_t n, float** dst) {
    if (rc == NPFN_OK) rc = upload_f32(h, p, n, dst);
    p += n;
  };
  auto b16 = [&](size_t n, bf16_t** dst) {
    if (rc == NPFN_OK) rc = upload_bf16(h, p, n, dst);
    p += n;
  };
  // row-kernel matrix: plain copy (per-sublayer kernels) + host copy (row-kernel streams)
  std::vector<RowkHost> rowk_host(cfg->n_layers);
  auto b16p = [&](size_t rows, size_t K, bf16_t** dst, std::vector<float>* img) {
    if (rc == NPFN_OK) rc = upload_bf16(h, p, rows * K, dst);
    img->assign(p, p + rows * K);
    p += rows * K;
  };
  f32(d * 4, &h->encw);
  f32(d * 2, &h->yencw);
  f32(G * d, &h->pos);
  h->layers.resize(cfg->n_layers);
  for (int l = 0; l < cfg->n_layers; ++l) {
    LayerW& w = h->layers[l];
    RowkHost& hw = rowk_host[l];
    b16p(3 * d, d, &w.feat_qkv, &hw.feat_qkv);
    b16p(d, d, &w.feat_out, &hw.feat_out);
    b16p(3 * d, d, &w.item_qkv, &hw.item_qkv);
    b16p(d, d, &w.item_out, &hw.item_out);
    b16p(dff, d, &w.w1, &hw.w1);
    b16p(d, dff, &w.w2, &hw.w2);
    for (int k = 0; k < 6; ++k) f32(d, &w.ln[k]);
  }
  b16(dff * d, &h->dec_w1);
  f32(dff, &h->dec_b1);
  b16(nb * dff, &h->dec_w2);
  f32(nb, &h->dec_b2);
  f32(nb + 1, &h->bz);
  if (rc == NPFN_OK) rc = build_rowk_streams(h, rowk_host);
  if (rc != NPFN_OK) {
    npfn_engine_destroy(h);
    return rc;
  }
  gemm_setup();
  rowk_setup();
  svd_setup();
  {
    // NPFN_UNFUSED=1 / =0 forces the per-sublayer / fused path; unset = default
    const char* env = getenv("NPFN_UNFUSED");
    h->fused = env ? (env[0] != '1') : kFusedDefault;
    const char* dt = getenv("NPFN_ROWK_STATIC");
    h->dyn_tiles = !(dt && dt[0] == '1');
    const char* cr = getenv("NPFN_CHUNK_ROWS");  // A/B: query rows per forward chunk (npfn_set_chunk_rows)
    if (cr && atoll(cr) > 0) h->chunk_rows = atoll(cr);
    if (hipMalloc((void**)&h->tile_ctrs, npfn_engine::kTileCtrs * sizeof(unsigned)) == hipSuccess)
      (void)hipMemset(h->tile_ctrs, 0, npfn_engine::kTileCtrs * sizeof(unsigned));
    else
      h->tile_ctrs = nullptr;
    if (hipMalloc((void**)&h->ia_fb, 4 * sizeof(unsigned long long)) == hipSuccess)
      (void)hipMemset(h->ia_fb, 0, 4 * sizeof(unsigned long long));
    else
      h->ia_fb = nullptr;
  }
  *out = h;
  return NPFN_OK;
}

int npfn_engine_destroy(npfn_engine* h) {
  if (!h) return NPFN_OK;
  (void)hipSetDevice(h->cfg.device);
  (void)hipDeviceSynchronize();
  for (void* p : h->weight_allocs) (void)hipFree(p);
  for (hipEvent_t e : h->prof.pool) (void)hipEventDestroy(e);
  if (h->tile_ctrs) (void)hipFree(h->tile_ctrs);
  if (h->ia_fb) (void)hipFree(h->ia_fb);
  for (hipEvent_t e : h->prep_done) (void)hipEventDestroy(e);
  for (hipEvent_t e : h->stat_done) (void)hipEventDestroy(e);
  if (h->side_t) (void)hipStreamDestroy(h->side_t);
  if (h->setup_done) (void)hipEventDestroy(h->setup_done);
  if (h->side) (void)hipStreamDestroy(h->side);
  h->fit0.release();
  for (Fit& f : h->slots) f.release();
  h->wmain.release();
  h->wside.release();
  DevBuf* bufs[] = {&h->dh,      &h->logits, &h->tgt,
                    &h->joint, &h->feat,     &h->logp, &h->pu, &h->views, &h->ftype, &h->ett,     &h->fp_salt};
  for (DevBuf* b : bufs) free_buf(*b);
  delete h;
  return NPFN_OK;
}

int npfn_fit(npfn_engine* h, const float* X, int64_t ldx, const float* y, int64_t ldy, int64_t n_ctx,
             int32_t n_features, void* stream) {
  RCHK(check_engine(h));
  h->f = &h->fit0;  // never overwrite a cached per-step fit of npfn_ar_sample
  RCHK(ensure_pipelines(h, false));
  return fit_impl(h, X, ldx, y, ldy, n_ctx, n_features, (hipStream_t)stream);
}

int npfn_set_preprocessing(npfn_engine* h, int32_t mode) {
  RCHK(check_engine(h));
  if (mode < 0 || mode > 3)
    return fail(NPFN_EINVAL,
                "set_preprocessing: mode must be 0 (none), 1 (quantile), 2 (quantile+power) or 3 (ensemble)");
  RCHK(apply_preprocessing(h, mode));
  h->f = &h->fit0;
  h->f->fitted = false;
  for (Fit& sl : h->slots) sl.fitted = false;
  std::memset(h->slot_key, 0, sizeof(h->slot_key));
  h->ar_active = false;
  return NPFN_OK;
}

int npfn_fit_classes(npfn_engine* h, const float* X, int64_t ldx, const float* y, int64_t ldy, int64_t n_ctx,
                     int32_t n_features, int32_t n_classes, void* stream) {
  RCHK(check_engine(h));
  h->f = &h->fit0;
  RCHK(need_full_range(h, "fit_classes"));
  RCHK(ensure_pipelines(h, true));  // mode 3: the classifier's ensemble
  if (n_classes < 2 || n_classes > KMAX_CLS || n_classes > h->cfg.n_bars)
    return fail(NPFN_EINVAL, "fit_classes: n_classes must be in [2, min(16, decoder width)]");
  return fit_impl(h, X, ldx, y, ldy, n_ctx, n_features, (hipStream_t)stream, n_classes);
}

int npfn_predict_proba(npfn_engine* h, const float* Xq, int64_t ldq, int64_t n_rows, float* probs, void* stream) {
  RCHK(check_engine(h));
  if (!h->f->fitted || h->f->ncls == 0) return fail(NPFN_ESTATE, "predict_proba before fit_classes");
  RCHK(need_full_range(h, "predict_proba"));
  if (!Xq || !probs) return fail(NPFN_EINVAL, "predict_proba: null pointer");
  if (ldq < h->f->F) return fail(NPFN_EINVAL, "predict_proba: ldq < n_features");
  hipStream_t s = (hipStream_t)stream;
  const int E = h->cfg.n_estimators, nb = h->cfg.n_bars;
  const float invT = 1.0f / h->cfg.softmax_temperature;
  for (int64_t r0 = 0; r0 < n_rows; r0 += h->chunk_rows) {
    const int64_t rows = std::min(h->chunk_rows, n_rows - r0);
    RCHK(predict_logits_chunk(h, Xq + r0 * ldq, ldq, rows, s));
    ProfGuard g(h, P_CLS_MIX, 0.0, (double)E * rows * nb * sizeof(logit_t) + (double)rows * h->f->ncls * 4, s);
    launch_cls_mix((const logit_t*)h->logits.p, rows, E, nb, h->f->ncls, invT, (const int*)h->f->cperm.p,
                   h->avg_before_softmax, probs + r0 * h->f->ncls, h->f->ncls, s);
  }
  HIPCHK(hipGetLastError());
  return NPFN_OK;
}

int npfn_predict(npfn_engine* h, const float* Xq, int64_t ldq, int64_t n_rows, float* logits, void* stream) {
  RCHK(check_engine(h));
  if (!h->f->fitted) return fail(NPFN_ESTATE, "predict before fit");
  if (h->f->ncls > 0) return fail(NPFN_ESTATE, "predict (bar logits) after a classifier fit; use predict_proba");
  RCHK(need_full_range(h, "predict"));
  if (!Xq || !logits) return fail(NPFN_EINVAL, "predict: null pointer");
  if (ldq < h->f->F) return fail(NPFN_EINVAL, "predict: ldq < n_features");
  hipStream_t s = (hipStream_t)stream;
  const int E = h->cfg.n_estimators, nb = h->cfg.n_bars;
  const float invT = 1.0f / h->cfg.softmax_temperature;
  for (int64_t r0 = 0; r0 < n_rows; r0 += h->chunk_rows) {
    const int64_t rows = std::min(h->chunk_rows, n_rows - r0);
    RCHK(predict_logits_chunk(h, Xq + r0 * ldq, ldq, rows, s));
    ProfGuard g(h, P_MIX_LOG, 0.0, (double)E * rows * nb * sizeof(logit_t) + (double)rows * nb * 4, s);
    launch_mix_log((const logit_t*)h->logits.p, rows, E, nb, invT, h->mixtrans(), logits + r0 * nb, nb, s);
  }
  HIPCHK(hipGetLastError());
  return NPFN_OK;
}

int npfn_get_borders(npfn_engine* h, float* borders, void* stream) {
  RCHK(check_engine(h));
  if (!h->f->fitted) return fail(NPFN_ESTATE, "get_borders before fit");
  launch_borders(h->bz, (const float*)h->f->ystats.p, h->cfg.n_bars, borders, (hipStream_t)stream);
  HIPCHK(hipGetLastError());
  return NPFN_OK;
}

int npfn_bar_sample(const float* logits, const float* borders, int64_t n_rows, int32_t n_bars, uint64_t seed,
                    uint64_t counter, float* out, void* stream) {
  if (!logits || !borders || !out || n_bars < 2) return fail(NPFN_EINVAL, "bar_sample: bad arguments");
  if (n_rows == 0) return NPFN_OK;
  launch_bar_sample(logits, borders, n_rows, n_bars, seed, counter, out, (hipStream_t)stream);
  HIPCHK(hipGetLastError());
  return NPFN_OK;
}

int npfn_bar_nll(const float* logits, const float* borders, const float* y, int64_t n_rows, int32_t n_bars,
                 float* out, void* stream) {
  if (!logits || !borders || !y || !out || n_bars < 2) return fail(NPFN_EINVAL, "bar_nll: bad arguments");
  if (n_rows == 0) return NPFN_OK;
  launch_bar_nll(logits, borders, y, n_rows, n_bars, out, (hipStream_t)stream);
  HIPCHK(hipGetLastError());
  return NPFN_OK;
}

int npfn_ar_sample(npfn_engine* h, const float* x_ctx, const float* theta_ctx, int64_t n_ctx, int32_t dim_x,
                   int32_t dim_theta, const float* x_query, int64_t n_rows, uint64_t counter, int64_t row_base,
                   float* theta_out, float* log_prob_out, float eps, void* stream) {
  RCHK(check_engine(h));
  return ar_sample_impl(h, x_ctx, theta_ctx, n_ctx, dim_x, dim_theta, x_query, 0, n_rows, counter, row_base,
                        theta_out, log_prob_out, eps, (hipStream_t)stream);
}

int npfn_ar_sample_repeated(npfn_engine* h, const float* x_ctx, const float* theta_ctx, int64_t n_ctx, int32_t dim_x,
                            int32_t dim_theta, const float* x_unique, int64_t n_unique, int64_t n_rows,
                            uint64_t counter, int64_t row_base, float* theta_out, float* log_prob_out, float eps,
                            void* stream) {
  RCHK(check_engine(h));
  if (n_unique < 1 || n_rows < 0 || n_rows % n_unique != 0)
    return fail(NPFN_EINVAL, "ar_sample_repeated: need n_unique >= 1 dividing n_rows");
  return ar_sample_impl(h, x_ctx, theta_ctx, n_ctx, dim_x, dim_theta, x_unique, n_unique, n_rows, counter, row_base,
                        theta_out, log_prob_out, eps, (hipStream_t)stream);
}

int npfn_ar_log_prob(npfn_engine* h, const float* x_ctx, const float* theta_ctx, int64_t n_ctx, int32_t dim_x,
                     int32_t dim_theta, const float* x_query, const float* theta, int64_t n_rows,
                     float* log_prob_out, float eps, void* stream) {
  RCHK(check_engine(h));
  return ar_log_prob_impl(h, x_ctx, theta_ctx, n_ctx, dim_x, dim_theta, x_query, 0, theta, n_rows, log_prob_out, eps,
                          (hipStream_t)stream);
}

int npfn_ar_log_prob_repeated(npfn_engine* h, const float* x_ctx, const float* theta_ctx, int64_t n_ctx,
                              int32_t dim_x, int32_t dim_theta, const float* x_unique, int64_t n_unique,
                              const float* theta, int64_t n_rows, float* log_prob_out, float eps, void* stream) {
  RCHK(check_engine(h));
  if (n_unique < 1 || n_rows < 0 || n_rows % n_unique != 0)
    return fail(NPFN_EINVAL, "ar_log_prob_repeated: need n_unique >= 1 dividing n_rows");
  return ar_log_prob_impl(h, x_ctx, theta_ctx, n_ctx, dim_x, dim_theta, x_unique, n_unique, theta, n_rows,
                          log_prob_out, eps, (hipStream_t)stream);
}

int npfn_ar_fit_begin(npfn_engine* h, const float* x_ctx, const float* theta_ctx, int64_t n_ctx, int32_t dim_x,
                      int32_t dim_theta, void* stream) {
  RCHK(check_engine(h));
  if (!x_ctx || !theta_ctx) return fail(NPFN_EINVAL, "ar_fit_begin: null input");
  if (dim_x < 1 || dim_theta < 1 || n_ctx < 1) return fail(NPFN_EINVAL, "ar_fit_begin: bad dimensions");
  hipStream_t s = (hipStream_t)stream;
  const int Ft = dim_x + dim_theta;
  h->ar_active = false;
  RCHK(ensure_pipelines(h, false));
  RCHK(ensure(h->joint, (size_t)n_ctx * Ft * sizeof(float), s));
  float* joint = (float*)h->joint.p;
  launch_copy_cols(x_ctx, dim_x, joint, Ft, n_ctx, dim_x, 0, s);
  launch_copy_cols(theta_ctx, dim_theta, joint, Ft, n_ctx, dim_theta, dim_x, s);
  bool reuse = false, piped = false;
  begin_ar_fits(h, n_ctx, dim_x, dim_theta, reuse);
  if (!reuse) RCHK(ar_prefit(h, joint, Ft, n_ctx, dim_x, dim_theta, s, piped));
  // the slots are keyed now; a slot's `fitted` says whether its train forward ran
  end_ar_fits(h, n_ctx, dim_x, dim_theta);
  h->ar_n = n_ctx;
  h->ar_dx = dim_x;
  h->ar_dth = dim_theta;
  h->ar_piped = piped;
  h->ar_reuse = reuse;
  h->ar_active = true;
  HIPCHK(hipGetLastError());
  return NPFN_OK;
}

int npfn_ar_fit_step(npfn_engine* h, int32_t k, void* stream) {
  RCHK(check_engine(h));
  if (!h->ar_active) return fail(NPFN_ESTATE, "ar_fit_step before ar_fit_begin");
  if (k < 0 || k >= h->ar_dth) return fail(NPFN_EINVAL, "ar_fit_step: step out of range");
  const int Ft = h->ar_dx + h->ar_dth;
  h->f = step_fit(h, k);
  // reuse: an earlier call under the same token, context shape and estimator set fitted every
  // slot (nothing queued); a slot's `fitted` alone may be left over from another context
  if (h->ar_reuse && h->f->fitted) return NPFN_OK;
  RCHK(ar_step_fit(h, (const float*)h->joint.p, Ft, h->ar_n, h->ar_dx, h->ar_dth, k, h->ar_piped,
                   (hipStream_t)stream));
  HIPCHK(hipGetLastError());
  return NPFN_OK;
}

int npfn_set_fit_token(npfn_engine* h, uint64_t token) {
  RCHK(check_engine(h));
  h->fit_token = token;
  if (token == 0) h->f = &h->fit0;
  return NPFN_OK;
}

int npfn_set_estimator_range(npfn_engine* h, int32_t e0, int32_t count) {
  return npfn_set_estimator_set(h, e0, count, 1);
}

int npfn_set_estimator_set(npfn_engine* h, int32_t e0, int32_t count, int32_t stride) {
  RCHK(check_engine(h));
  if (e0 < 0 || count < 1 || stride < 1 || e0 + (int64_t)stride * (count - 1) >= h->cfg.n_estimators)
    return fail(NPFN_EINVAL, "set_estimator_set: need 0 <= e0, 1 <= count, 1 <= stride and "
                             "e0 + stride * (count - 1) < n_estimators");
  h->e0 = e0;
  h->ne = count;
  h->es = count == 1 ? 1 : stride;
  h->f = &h->fit0;
  h->f->fitted = false;
  for (Fit& sl : h->slots) sl.fitted = false;  // per-estimator layouts of the old set
  std::memset(h->slot_key, 0, sizeof(h->slot_key));
  h->ar_active = false;
  return NPFN_OK;
}

int npfn_forward_targets(npfn_engine* h, const float* Xq, int64_t ldq, int64_t n_rows, void* tokens_out,
                         void* stream) {
  RCHK(check_engine(h));
  if (!h->f->fitted || h->f->ncls > 0) return fail(NPFN_ESTATE, "forward_targets before a regressor fit");
  if (!Xq || !tokens_out) return fail(NPFN_EINVAL, "forward_targets: null pointer");
  if (ldq < h->f->F) return fail(NPFN_EINVAL, "forward_targets: ldq < n_features");
  if (n_rows < 0) return fail(NPFN_EINVAL, "forward_targets: negative n_rows");
  hipStream_t s = (hipStream_t)stream;
  bf16_t* out = (bf16_t*)tokens_out;
  for (int64_t r0 = 0; r0 < n_rows; r0 += h->chunk_rows) {
    const int64_t rows = std::min(h->chunk_rows, n_rows - r0);
    RCHK(forward_any(h, Xq + r0 * ldq, ldq, nullptr, 0, rows, false, s));
    for (int e = 0; e < h->ne; ++e)
      HIPCHK(hipMemcpyAsync(out + ((size_t)e * n_rows + r0) * 192, (const bf16_t*)h->tgt.p + (size_t)e * rows * 192,
                            (size_t)rows * 192 * sizeof(bf16_t), hipMemcpyDeviceToDevice, s));
  }
  HIPCHK(hipGetLastError());
  return NPFN_OK;
}

int npfn_head_sample(npfn_engine* h, const void* tokens, int32_t n_est, int64_t n_rows, uint64_t counter,
                     int64_t row_base, float* theta_out, float* log_prob_acc, float eps, void* stream) {
  RCHK(check_engine(h));
  if (!h->f->fitted || h->f->ncls > 0) return fail(NPFN_ESTATE, "head_sample before a regressor fit");
  if (!tokens || !theta_out) return fail(NPFN_EINVAL, "head_sample: null pointer");
  if (n_est != h->cfg.n_estimators)
    return fail(NPFN_EINVAL, "head_sample: the ensemble mean needs the target tokens of all n_estimators");
  if (n_rows < 0 || row_base < 0) return fail(NPFN_EINVAL, "head_sample: negative n_rows or row_base");
  hipStream_t s = (hipStream_t)stream;
  const int nb = h->cfg.n_bars;
  const float invT = 1.0f / h->cfg.softmax_temperature;
  const bf16_t* tok = (const bf16_t*)tokens;
  for (int64_t r0 = 0; r0 < n_rows; r0 += h->chunk_rows) {
    const int64_t rows = std::min(h->chunk_rows, n_rows - r0);
    const bf16_t* blk = tok;
    if (rows != n_rows) {  // gather the chunk's rows of every estimator into one [E][rows][192] block
      RCHK(ensure(h->wmain.attn, (size_t)n_est * rows * 192 * sizeof(bf16_t), s));
      bf16_t* b = (bf16_t*)h->wmain.attn.p;
      for (int e = 0; e < n_est; ++e)
        HIPCHK(hipMemcpyAsync(b + (size_t)e * rows * 192, tok + ((size_t)e * n_rows + r0) * 192,
                              (size_t)rows * 192 * sizeof(bf16_t), hipMemcpyDeviceToDevice, s));
      blk = b;
    }
    RCHK(decode_chunk(h, blk, 192, n_est, rows, s));
    ProfGuard g(h, P_MIX_SAMPLE, 0.0, (double)n_est * rows * nb * sizeof(logit_t), s);
    launch_mix_sample((const logit_t*)h->logits.p, rows, n_est, nb, invT, h->mixtrans(), h->bz, (const float*)h->f->ystats.p,
                      h->cfg.random_state, counter, r0, (uint64_t)row_base, theta_out, 1, 0, log_prob_acc,
                      logf(eps), s);
  }
  HIPCHK(hipGetLastError());
  return NPFN_OK;
}

int npfn_set_chunk_rows(npfn_engine* h, int64_t rows) {
  RCHK(check_engine(h));
  if (rows < 1) return fail(NPFN_EINVAL, "set_chunk_rows: rows must be >= 1");
  h->chunk_rows = rows;
  return NPFN_OK;
}

int npfn_prof_enable(npfn_engine* h, int enable) {
  RCHK(check_engine(h));
  h->prof.on = enable != 0;
  return NPFN_OK;
}

int npfn_prof_read(npfn_engine* h, npfn_prof_entry* out, int32_t max_entries, int32_t* n_entries) {
  RCHK(check_engine(h));
  if (!out || !n_entries) return fail(NPFN_EINVAL, "prof_read: null pointer");
  HIPCHK(hipDeviceSynchronize());
  // a side-stream launch's event pair also spans the time its low-priority stream waited for
  // CUs, so side-stream launches are reported apart ("<kernel> (side stream)")
  double ms[2 * P_NCAT] = {0}, fl[2 * P_NCAT] = {0}, by[2 * P_NCAT] = {0};
  int64_t cnt[2 * P_NCAT] = {0};
  for (const ProfRec& r : h->prof.recs) {
    float t = 0.f;
    HIPCHK(hipEventElapsedTime(&t, r.a, r.b));
    ms[r.cat] += t;
    fl[r.cat] += r.flops;
    by[r.cat] += r.bytes;
    cnt[r.cat] += 1;
  }
  h->prof.recs.clear();
  h->prof.used = 0;
  int k = 0;
  for (int c = 0; c < 2 * P_NCAT && k < max_entries; ++c) {
    if (cnt[c] == 0) continue;
    std::memset(&out[k], 0, sizeof(npfn_prof_entry));
    const std::string nm = std::string(kProfNames[c % P_NCAT]) + (c >= P_NCAT ? " (side stream)" : "");
    std::strncpy(out[k].name, nm.c_str(), sizeof(out[k].name) - 1);
    out[k].launches = cnt[c];
    out[k].ms = ms[c];
    out[k].flops = fl[c];
    out[k].bytes = by[c];
    ++k;
  }
  *n_entries = k;
  return NPFN_OK;
}

int npfn_debug_views(npfn_engine* h, float* out, int64_t rows, int32_t max_cols, int32_t* vw_out) {
  RCHK(check_engine(h));
  if (!out || !vw_out) return fail(NPFN_EINVAL, "debug_views: null pointer");
  const DevBuf* v = h->last_views;
  if (!v || !v->p || h->f->vl.Vw == 0) return fail(NPFN_ESTATE, "debug_views before a fit");
  *vw_out = h->f->vl.Vw;
  if (h->f->vl.Vw > max_cols) return fail(NPFN_EINVAL, "debug_views: max_cols < views width");
  if ((size_t)rows * h->f->vl.Vw * sizeof(float) > v->bytes) return fail(NPFN_EINVAL, "debug_views: too many rows");
  HIPCHK(hipDeviceSynchronize());
  HIPCHK(hipMemcpy(out, v->p, (size_t)rows * h->f->vl.Vw * sizeof(float), hipMemcpyDeviceToHost));
  return NPFN_OK;
}

int npfn_debug_item_attn_online(int enable) {
  set_item_attn_online(enable);
  return NPFN_OK;
}

int npfn_debug_item_attn_scale(float scale) {
  if (!(scale > 0.f)) return fail(NPFN_EINVAL, "item-attention score scale must be > 0");
  set_item_attn_scale(scale);
  return NPFN_OK;
}

int npfn_set_average_before_softmax(npfn_engine* h, int32_t enable) {
  RCHK(check_engine(h));
  h->avg_before_softmax = enable ? 1 : 0;
  return NPFN_OK;
}

int npfn_debug_fail_row_launch(npfn_engine* h, int32_t n) {
  RCHK(check_engine(h));
  if (n < 0) return fail(NPFN_EINVAL, "npfn_debug_fail_row_launch: n must be >= 0 (0 = off)");
  h->debug_fail_row = n;
  return NPFN_OK;
}

int npfn_item_attn_fallback(npfn_engine* h, uint64_t* out4, int reset) {
  RCHK(check_engine(h));
  if (!out4) return fail(NPFN_EINVAL, "npfn_item_attn_fallback: null output");
  unsigned long long dev[4] = {0ull, 0ull, 0ull, 0ull};
  HIPCHK(hipDeviceSynchronize());
  if (h->ia_fb) HIPCHK(hipMemcpy(dev, h->ia_fb, sizeof(dev), hipMemcpyDeviceToHost));
  out4[0] = dev[0];
  out4[1] = h->ia_blocks;
  out4[2] = dev[1];
  out4[3] = h->ia_rows;
  if (reset) {
    if (h->ia_fb) HIPCHK(hipMemset(h->ia_fb, 0, sizeof(dev)));
    h->ia_blocks = h->ia_rows = 0;
  }
  return NPFN_OK;
}

int npfn_item_attn_fallback_causes(npfn_engine* h, uint64_t* out2) {
  RCHK(check_engine(h));
  if (!out2) return fail(NPFN_EINVAL, "npfn_item_attn_fallback_causes: null output");
  unsigned long long dev[4] = {0ull, 0ull, 0ull, 0ull};
  HIPCHK(hipDeviceSynchronize());
  if (h->ia_fb) HIPCHK(hipMemcpy(dev, h->ia_fb, sizeof(dev), hipMemcpyDeviceToHost));
  out2[0] = dev[2];
  out2[1] = dev[3];
  return NPFN_OK;
}

int npfn_box_support(const float* theta, int64_t n_rows, int32_t dim, const float* low, const float* high,
                     uint8_t* mask, void* stream) {
  if (n_rows == 0 && dim >= 1) return NPFN_OK;
  if (!theta || !low || !high || !mask || dim < 1 || n_rows < 0) return fail(NPFN_EINVAL, "box_support: bad arguments");
  launch_box_support(theta, n_rows, dim, low, high, mask, (hipStream_t)stream);
  HIPCHK(hipGetLastError());
  return NPFN_OK;
}

}  // extern "C"
