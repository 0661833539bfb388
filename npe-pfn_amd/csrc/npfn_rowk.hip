// npfn_rowk.hip -- fused row-tile layer kernel (everything of a PerFeatureEncoderLayer
// except the item attention, which needs other rows), register-resident.
//
// One workgroup (8 waves) owns a tile of whole rows (rpt = floor(128 / C) rows x C tokens
// <= 128 token slots); wave w owns slots 16w .. 16w+15, one token per lane column
// (lane & 15).  The chain of the layer runs on those 16 tokens in the wave's registers:
//
//   [post of layer l]  x = LN2(x + o_item Wo_i^T); per 64-wide hidden slab s < 12:
//                      h_s = GELU(x W1_s^T), x += h_s W2[:, s]^T; x = LN3(x)
//   [pre of layer l+1] v = x Wv_f^T (-> v^T image in LDS); per head pair hp < 3:
//                      k_hp, q_hp = x Wk_hp^T, x Wq_hp^T; feature attention of the pair over
//                      the row's C tokens; x += o_hp Wo_f[:, hp]^T; then x = LN1(x);
//                      out = x Wq_i^T (test) or x Wqkv_i^T (train)
//
// Every matrix product is cut into CHUNKS of 24 KB of weights = 24 v_mfma_f32_16x16x32_bf16
// per wave, of two kinds (A = weights from LDS, B = the wave's activations):
//   S chunk  [192 outputs][64 of K]: acc[12 tiles] (+)= W X^T over 2 K-steps -- the 192-wide
//            products (Wo_i, W2 slabs, Wv_f, Wo_f pair slices, item projections) accumulate
//            into the residual x (MFMA C operand) or a 192-wide accumulator;
//   O chunk  [64 outputs][192 = all of K]: acc[4 tiles] = W_s X^T over 6 K-steps -- the
//            64-wide slabs (W1 hidden slabs, per-head-pair k and q).
// A slab's output is consumed right away (GELU, keys, queries), so the live register set
// stays small (x 48 + LN(x) 24 + slab 16 + ...) and every chunk can hold all 24 of its A
// fragments in flight: one burst of 24 ds_read_b128 after the chunk's barrier, then 24
// MFMAs as the fragments land (the 192-wide formulation sat at 256 VGPRs with one or two
// LDS reads in flight per MFMA).  The GELU of slab s runs inside the W2 chunk of slab s-1
// (software pipeline: W1_0, W1_1, W2_0, W1_2, W2_1, ..., W1_11, W2_10, W2_11), so its VALU
// work shares the SIMD with matrix work instead of idling the matrix pipe.
//
// A product's D tile of features 16f.. leaves lane (g = lane >> 4) features 16f + 4g + {0..3};
// packing D tiles 2m and 2m+1 gives the B fragment of K-step m in the order
//     slot 8g + j  <->  feature 32m + pi(8g + j),  pi = j < 4 ? 4g + j : 16 + 4g + j - 4,
// so a product's output is the next product's input without leaving the registers,
// provided the weights' K axis is stored in the same order (npfn_engine.hip builds
// pi-permuted chunk images).  LayerNorm over a token's 192 features is an in-lane sum + two
// lane shuffles.
//
// Weights stream through a 3-slot LDS ring filled by LDS-DMA (global_load_lds_dwordx4, the
// bank swizzle applied in the image): every wave copies 3 KB of each chunk.  At the open of
// chunk i each wave waits for its own pieces of chunk i with a counted vmcnt(3) (chunk i+1
// stays in flight), passes the barrier (everyone's pieces landed, everyone finished chunk
// i-1), and refills chunk i-1's slot with chunk i+2.  Barriers are raw s_barrier after
// lgkmcnt(0): a __syncthreads() fence would drain the DMA queue.
#include "npfn_common.h"
#include "npfn_kernels.h"

namespace npfn {
namespace {

constexpr int RT = 128;                              // token slots per tile (8 waves x 16)
#ifndef NPFN_ROWK_SLOTS
#define NPFN_ROWK_SLOTS 3
#endif
constexpr int NSLOT = NPFN_ROWK_SLOTS;               // weight ring depth (3, or 4 for the stagger)
static_assert(NSLOT == 3 || NSLOT == 4, "3 or 4 ring slots");
#ifndef NPFN_ROWK_STAGGER
#define NPFN_ROWK_STAGGER 0
#endif
static_assert(!NPFN_ROWK_STAGGER || NSLOT == 4, "the stagger needs the 4-slot ring");
constexpr int WS_ELEMS = 192 * 64;                   // one chunk image (bf16)
constexpr int WS_BYTES = WS_ELEMS * 2;
constexpr int WS_OFF = 0;
// Feature-attention images of one head pair (rows = token slots; RTP = RT + 32 zeroed pad rows
// for the values, whose 32-key steps may run 31 rows past a row's end, RTQ = RT + 16 for the
// keys and queries, whose 16-row blocks run at most 15 past it)
// that the last row's key blocks / value steps may cover):
constexpr int RTP = RT + 32;
constexpr int RTQ = RT + 16;
constexpr int KH_ELEMS = RTQ * 32;                   // one head: bf16 [RTQ][32], dims in pi order
constexpr int KH_OFF = WS_OFF + NSLOT * WS_BYTES;    // keys: 2 heads
constexpr int QH_OFF = KH_OFF + 2 * KH_ELEMS * 2;    // queries: 2 heads; overwritten by the outputs
constexpr int VV_OFF = QH_OFF + 2 * KH_ELEMS * 2;    // values: bf16 [RTP][64] (the pair's dims), token-major
constexpr int FA_END = VV_OFF + RTP * 64 * 2;
constexpr int LNP_OFF = FA_END;                      // float [6][192]: ln2 g,b | ln3 g,b | ln1 g,b
constexpr int SMEM_BYTES = LNP_OFF + 6 * 192 * 4;
#ifndef NPFN_ROWK_DMA_WAVES
#define NPFN_ROWK_DMA_WAVES 8
#endif
constexpr int DMA_WAVES = NPFN_ROWK_DMA_WAVES;        // waves that copy the weight chunks
constexpr int GLDS_PER_WAVE = 24 / DMA_WAVES;        // 1 KB LDS-DMA pieces per copying wave per chunk
static_assert(24 % DMA_WAVES == 0, "a chunk is 24 pieces");

typedef f32x4 Acc[12];   // D of a 192-feature product for the wave's 16 tokens
typedef f32x4 Acc4[4];   // D of a 64-feature slab
typedef bf16x8 Frag[6];  // B operand of a K = 192 product (pi order per 32-feature step)

__device__ __forceinline__ void bar() { lds_barrier(); }
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// head-key image [RT][32] (4 units per token row)
__device__ __forceinline__ int kh_idx(int t, int u) { return t * 32 + ((u ^ ((t >> 2) & 3)) << 3); }
// value image [RTP][64]: 8-byte granule gi (dims 4gi .. 4gi+3) of row t at granule gi ^ (((t >> 1) & 3) << 2):
// the 8 consecutive rows x 4 granules of one ds_read_b64_tr_b16 half-wave hit 32 distinct bank pairs
// for ANY first row (the rows of a key step start wherever the token's row starts)
__device__ __forceinline__ int vv_idx(int t, int gi) { return t * 64 + ((gi ^ (((t >> 1) & 3) << 2)) << 2); }

__device__ __forceinline__ bf16x8 pack8(const f32x4& lo, const f32x4& hi) {
  uint4 u;
  u.x = pack_bf2(lo[0], lo[1]);
  u.y = pack_bf2(lo[2], lo[3]);
  u.z = pack_bf2(hi[0], hi[1]);
  u.w = pack_bf2(hi[2], hi[3]);
  return __builtin_bit_cast(bf16x8, u);
}
__device__ __forceinline__ void to_frag(const Acc& a, Frag& f) {
#pragma unroll
  for (int m = 0; m < 6; ++m) f[m] = pack8(a[2 * m], a[2 * m + 1]);
}

// The weight stream of one tile: P.stream_chunks chunk images in consumption order
// (npfn_engine.hip build_rowk_streams), replayed from the start for every tile.
struct Ring {
  const char* istart;  // stream of this launch
  const char* iend;
  const char* isrc;    // next chunk to issue
  uint32_t ws_lds;     // LDS byte address of slot 0
  int slot;            // slot of the chunk being read (chunk i)

  // next chunk of the stream -> slot `dslot`: wave w copies bytes [3 KB w, 3 KB (w + 1)),
  // 1 KB per wave instruction (scalar source base + per-lane offset).  The stream wraps to
  // the next tile's first chunk (after the last tile it lands in a slot never read, and the
  // kernel drains it before exiting).
  __device__ __forceinline__ void issue(int dslot) {
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
#ifdef NPFN_ROWK_DMA_HIGH
    const int dw = wave - (8 - DMA_WAVES);  // the last DMA_WAVES waves copy
#else
    const int dw = wave;                    // the first DMA_WAVES waves copy
#endif
    if (DMA_WAVES == 8 || (dw >= 0 && dw < DMA_WAVES)) {
      const uint32_t voff = (threadIdx.x & 63) * 16u;
      const uint32_t dst = ws_lds + (uint32_t)(dslot * WS_BYTES) + (uint32_t)dw * (GLDS_PER_WAVE * 1024u);
      const char* src = isrc + dw * (GLDS_PER_WAVE * 1024);
#pragma unroll
      for (int p = 0; p < GLDS_PER_WAVE; ++p) glds16_s(src + p * 1024, voff, dst + (uint32_t)p * 1024u);
    }
    isrc += WS_BYTES;
    if (isrc == iend) isrc = istart;
  }
  // the same copy one piece at a time (NPFN_ROWK_DMA_SPREAD: the pieces are spread over the
  // second half of the chunk instead of issued back to back right after the barrier)
  const char* psrc;
  uint32_t pdst;
  __device__ __forceinline__ void begin_issue(int dslot) {
    const int dw = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    pdst = ws_lds + (uint32_t)(dslot * WS_BYTES) + (uint32_t)dw * (GLDS_PER_WAVE * 1024u);
    psrc = isrc + dw * (GLDS_PER_WAVE * 1024);
    isrc += WS_BYTES;
    if (isrc == iend) isrc = istart;
  }
  __device__ __forceinline__ void issue_piece(int p) {
    glds16_s(psrc + p * 1024, (threadIdx.x & 63) * 16u, pdst + (uint32_t)p * 1024u);
  }
#ifdef NPFN_ROWK_STAMPS
  unsigned long long* ph;  // diagnostics: [1] chunk bodies, [3] vmcnt waits, [8] barrier waits, [7] DMA issue
  unsigned long long* tprev;
  __device__ __forceinline__ void stamp(int k) {
    const unsigned long long now = __builtin_amdgcn_s_memtime();
    ph[k] += now - *tprev;
    *tprev = now;
  }
#else
  __device__ __forceinline__ void stamp(int) {}
#endif
  __device__ __forceinline__ const bf16_t* cur(const char* smem) const {
    return reinterpret_cast<const bf16_t*>(smem + WS_OFF) + slot * WS_ELEMS;
  }
  // Barrier beta_i, in the middle of chunk i (after its last reads were issued): this wave's
  // reads of chunk i have landed in its registers (lds_barrier's lgkmcnt(0)) and its DMA
  // pieces of chunk i+1 in LDS (counted vmcnt(3): chunk i+2's stay in flight); after the
  // barrier both hold for every wave, so chunk i's slot is free -- refilled with chunk i+3 --
  // and chunk i+1 may be read.  Returns chunk i+1's weights.
  __device__ __forceinline__ const bf16_t* advance(const char* smem) {
    stamp(1);
    wait_vmcnt<GLDS_PER_WAVE>();
    stamp(3);
    if constexpr (NSLOT == 4) {
      // 4 slots: the refill goes to chunk i-1's slot, whose reads every wave consumed in its
      // MFMAs before this barrier -- chunk i's reads may stay in flight across it
      asm volatile("s_barrier" ::: "memory");
    } else {
      bar();
    }
    stamp(8);
#ifdef NPFN_ROWK_DMA_SPREAD
    begin_issue(slot);
#else
    issue(NSLOT == 3 ? slot : (slot + NSLOT - 1) % NSLOT);
#endif
    slot = slot == NSLOT - 1 ? 0 : slot + 1;
    stamp(7);
    return reinterpret_cast<const bf16_t*>(smem + WS_OFF) + slot * WS_ELEMS;
  }
};

// Chunk pipeline.  A chunk's 24 A fragments (in MFMA order) flow through a window of 12
// registers: run_*() enters with fragments 0-11 of chunk i already loaded, issues MFMA k
// and then the read of fragment k+12 into the register MFMA k consumed (k < 12), passes
// beta_i (Ring::advance: this wave's reads of chunk i landed, its DMA pieces of chunk i+1
// too, then the barrier), and issues MFMA 12+k followed by the read of fragment k of chunk
// i+1 (k < 12).  So every wave keeps about 12 reads in flight, LDS latency hides behind its
// MFMAs, and the barrier comes while the first half's MFMAs are still in the pipe.
// NT = the kind of chunk i+1 (its fragment addresses differ).
enum { CK_S = 0, CK_O = 1 };
typedef bf16x8 AWin[12];

// lane offsets (elements) of the two 32-K halves of a 64-K block row (unit u of image row r
// at u ^ (r & 7), 8 units per row); image row f*16 + (lane & 15) adds f * 1024
__device__ __forceinline__ int frag_off(int half) {
  const int lane = threadIdx.x & 63;
  return (lane & 15) * 64 + (((4 * half + (lane >> 4)) ^ (lane & 7)) << 3);
}
// fragment k of a chunk, in MFMA order: S k = 12 k2 + f (K-half k2, output tile f < 12);
// O k = 4 ks + f (K-step ks < 6, output tile f < 4; image rows 64 (ks / 2) + 16 f + r)
template <int T>
__device__ __forceinline__ bf16x8 read_frag(const bf16_t* w, int k, int o0, int o1) {
  const int e = T == CK_S ? (k % 12) * 1024 + (k >= 12 ? o1 : o0)
                          : ((k >> 2) >> 1) * 4096 + (k & 3) * 1024 + (((k >> 2) & 1) ? o1 : o0);
  return *reinterpret_cast<const bf16x8*>(w + e);
}
template <int T>
__device__ __forceinline__ void read_first_half(const bf16_t* w, AWin& a) {
  const int o0 = frag_off(0), o1 = frag_off(1);
#pragma unroll
  for (int k = 0; k < 12; ++k) a[k] = read_frag<T>(w, k, o0, o1);
}

// Scheduling: nothing crosses a chunk half, and inside a half each MFMA is followed by the
// read that refills its fragment register (+ VALU filler of a fused epilogue).
__device__ __forceinline__ void sched_fence() { __builtin_amdgcn_sched_barrier(0); }
template <int VALU_PER_MFMA>
__device__ __forceinline__ void sched_half() {
#pragma unroll
  for (int i = 0; i < 12; ++i) {
    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
    __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // DS read into its fragment register
    if (VALU_PER_MFMA > 0) __builtin_amdgcn_sched_group_barrier(0x002, VALU_PER_MFMA, 0);
  }
}

// generic chunk: MFMA(k) for k < 24 through the window; `mma(k, frag)` issues MFMA k
template <bool LAG, int T, int NT, int VALU, class MMA, class EPI>
__device__ __forceinline__ void run_chunk(Ring& ring, const char* smem, AWin& a, MMA&& mma, EPI&& epi_half) {
  const int o0 = frag_off(0), o1 = frag_off(1);
  const bf16_t* w = ring.cur(smem);
  // Stagger (NPFN_ROWK_STAGGER, LAG = waves 4-7, which run their own instance of the layer
  // body): they pass each chunk's barrier at the chunk's start instead of its middle, so they run half a chunk behind waves 0-3 and a SIMD's two waves
  // (w, w + 4) reach their VALU phases (LayerNorm, stores, GELU) at different times.  Legal
  // with the 4-slot ring: at barrier i the lagging half has read chunk i-1 completely (not
  // chunk i), so the refill goes to chunk i-1's slot.
  const bf16_t* wn = w;
  if constexpr (LAG) wn = ring.advance(smem);
  sched_fence();
#pragma unroll
  for (int k = 0; k < 12; ++k) {
    mma(k, a[k]);
    a[k] = read_frag<T>(w, k + 12, o0, o1);
  }
  epi_half(0);
  sched_half<VALU>();
  sched_fence();
  if constexpr (!LAG) wn = ring.advance(smem);
#pragma unroll
  for (int k = 0; k < 12; ++k) {
    mma(k + 12, a[k]);
    a[k] = read_frag<NT>(wn, k, o0, o1);
#ifdef NPFN_ROWK_DMA_SPREAD
    static_assert(GLDS_PER_WAVE == 3 && NSLOT == 3 && !NPFN_ROWK_STAGGER, "spread: 3 pieces per wave, 3 slots");
    if (k % 4 == 1) ring.issue_piece(k / 4);
#endif
  }
  epi_half(1);
  sched_half<VALU>();
  sched_fence();
}

// S chunk: acc (+)= W X^T for 192 outputs over the 64-K slice whose B fragments are b0, b1.
// SWAP: D = X W^T (rows = the wave's tokens 4g+i, cols = features) -- the v^T image layout.
template <bool LAG, bool INIT, bool SWAP, int NT>
__device__ __forceinline__ void run_s(Ring& ring, const char* smem, AWin& a, const bf16x8& b0, const bf16x8& b1,
                                      Acc& acc) {
  run_chunk<LAG, CK_S, NT, 0>(
      ring, smem, a,
      [&](int k, const bf16x8& fr) {
        const int f = k % 12;
        const bool first = k < 12;
        const f32x4 c = (INIT && first) ? f32x4{0.f, 0.f, 0.f, 0.f} : acc[f];
        acc[f] = SWAP ? __builtin_amdgcn_mfma_f32_16x16x32_bf16(first ? b0 : b1, fr, c, 0, 0, 0)
                      : __builtin_amdgcn_mfma_f32_16x16x32_bf16(fr, first ? b0 : b1, c, 0, 0, 0);
      },
      [](int) {});
}

// O chunk: acc = W_s X^T for a 64-output slab over all of K = 192 (B = the 6 fragments of b)
template <bool LAG, int NT>
__device__ __forceinline__ void run_o(Ring& ring, const char* smem, AWin& a, const Frag& b, Acc4& acc) {
  run_chunk<LAG, CK_O, NT, 0>(
      ring, smem, a,
      [&](int k, const bf16x8& fr) {
        const int ks = k >> 2, f = k & 3;
        acc[f] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fr, b[ks], ks == 0 ? f32x4{0.f, 0.f, 0.f, 0.f} : acc[f], 0,
                                                         0, 0);
      },
      [](int) {});
}

// GELU of hidden values -> bf16 pairs
__device__ __forceinline__ void gelu4(f32x4& h) {
#ifndef NPFN_DIAG_NOGELU
#pragma unroll
  for (int r = 0; r < 4; ++r) h[r] = gelu_tanh(h[r]);
#endif
}
// hidden slab after GELU -> the two B fragments of W2's 64-K slice s
__device__ __forceinline__ void gelu_slab(Acc4& h, bf16x8& f0, bf16x8& f1) {
#pragma unroll
  for (int f = 0; f < 4; ++f) gelu4(h[f]);
  f0 = pack8(h[0], h[1]);
  f1 = pack8(h[2], h[3]);
}

// S chunk of W2 slab s-1 (x += h_{s-1} W2[:, s-1]^T) with the GELU of slab s in its shadow
// (tiles 0-1 in the first half, 2-3 in the second)
template <bool LAG, int NT>
__device__ __forceinline__ void run_w2_gelu(Ring& ring, const char* smem, AWin& a, const bf16x8& b0,
                                            const bf16x8& b1, Acc& x, Acc4& h, bf16x8& n0, bf16x8& n1) {
  run_chunk<LAG, CK_S, NT, 3>(
      ring, smem, a,
      [&](int k, const bf16x8& fr) {
        x[k % 12] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fr, k < 12 ? b0 : b1, x[k % 12], 0, 0, 0);
      },
      [&](int half) {
        gelu4(h[2 * half]);
        gelu4(h[2 * half + 1]);
        if (half == 0) n0 = pack8(h[0], h[1]);
        else n1 = pack8(h[2], h[3]);
      });
}

// x = LN(x) * gamma + beta over the token's 192 features (lanes l, l^16, l^32, l^48).
// The residual add is already in x: every sub-layer's output product accumulates into x.
__device__ __forceinline__ void layer_norm(Acc& x, const float* lnp) {
#ifdef NPFN_DIAG_NOLN
  return;
#endif
  const int g4 = (threadIdx.x & 63) >> 4;
  // four independent partial sums (r) instead of one 48-long dependent chain, combined in a
  // fixed order: the result depends on the token's values only, not on its slot
  float s4[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int f = 0; f < 12; ++f)
#pragma unroll
    for (int r = 0; r < 4; ++r) s4[r] += x[f][r];
  float s = (s4[0] + s4[1]) + (s4[2] + s4[3]);
  s = xor32_sum(xor16_sum(s));
  const float mean = s * (1.0f / 192.0f);
  float v4[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int f = 0; f < 12; ++f)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float d = x[f][r] - mean;
      v4[r] = fmaf(d, d, v4[r]);
    }
  float v = (v4[0] + v4[1]) + (v4[2] + v4[3]);
  v = xor32_sum(xor16_sum(v));
  const float rstd = 1.0f / sqrtf(v * (1.0f / 192.0f) + 1e-5f);
  const float nmr = -mean * rstd;
  // (x - mean) rstd gamma + beta as two FMAs per value
#pragma unroll
  for (int f = 0; f < 12; ++f) {
    const f32x4 gg = *reinterpret_cast<const f32x4*>(lnp + f * 16 + g4 * 4);
    const f32x4 bb = *reinterpret_cast<const f32x4*>(lnp + 192 + f * 16 + g4 * 4);
#pragma unroll
    for (int r = 0; r < 4; ++r) x[f][r] = fmaf(fmaf(x[f][r], rstd, nmr), gg[r], bb[r]);
  }
}

typedef __attribute__((ext_vector_type(4))) short bf16x4;
typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;

// Two 8-byte transposed reads (ds_read_b64_tr_b16) give the A operand V^T [16 dims][32 keys] of
// one key step: lane (dim i = lane & 15, g = lane >> 4) holds the keys pi(8g + j) of dim i.  In
// each 16-lane group, lane 4q + p supplies row (key) k0 + 4g + q (first read) / k0 + 16 + 4g + q
// (second read), dims 4p .. 4p+3 of the tile -- the keys are addressed per lane, so a step may
// start at any row.
// (rows t and t + 16 share the swizzle ((t >> 1) & 3), so the second read is the first + 16 rows)
__device__ __forceinline__ bf16x8 read_vt(const char* smem, int k0, int gi0) {
  const int lane = threadIdx.x & 63, g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const bf16_t* vv = reinterpret_cast<const bf16_t*>(smem + VV_OFF) + vv_idx(k0 + 4 * g + q, gi0 + p);
  const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4*)vv);
  const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4*)(vv + 16 * 64));
  return bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}

// Feature attention of head pair hp over the tile's rows, ROW-RELATIVE: the work items are
// (row, head, 16-query block) triples, spread over the 8 waves.  An item's MFMAs see only its
// row: S^T = K Q^T per 16-key block of the row (keys and queries addressed from the row's first
// slot, q pre-scaled by 1/sqrt(32) log2 e through its weights), the exact row max (a max is
// order-free), P = exp2(S - max) summed in a fixed row-relative order, and O^T = V^T P^T per
// 32-key step of the row.  So a token's attention output depends on its row's values only,
// never on where the row sits in the tile: chunked, repeated-row and multi-GPU forwards give
// the single-call results bit for bit (the rest of the layer is per token).  O^T lands in pi
// order in the query image (the item overwrites only its own queries, after reading them):
// the B fragments of Wo_f's 64-K slice hp for the token owners.
// NKB = 16-key blocks (and 16-query blocks) of a row = ceil(C / 16) <= 4; 32-key steps NST = ceil(C / 32)
template <int NKB>
__device__ __forceinline__ void feat_attn_rows_t(char* smem, int C, int nrows) {
  constexpr int nkb = NKB, nst = (NKB + 1) / 2;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // uniform: item math on the SALU
  const int col = lane & 15, g4 = lane >> 4;
  const int items = nrows * 2 * nkb;
  for (int it = wave; it < items; it += 8) {
    const int rh = it / nkb, qb = it - rh * nkb, h = rh & 1, r = rh >> 1;
    const int rs = r * C, re = rs + C;  // the row's slots [rs, re)
    const bf16_t* kh = reinterpret_cast<const bf16_t*>(smem + KH_OFF) + h * KH_ELEMS;
    bf16_t* qh = reinterpret_cast<bf16_t*>(smem + QH_OFF) + h * KH_ELEMS;
    const int qt = rs + 16 * qb + col;  // this lane's query
    const bf16x8 qf = *reinterpret_cast<const bf16x8*>(qh + kh_idx(qt, g4));
    // key row rs + 16 kb + col of the A operand: the swizzle term ((t >> 2) & 3) is the same
    // for every kb, so the blocks are one base + kb * 1 KB
    const bf16_t* kp = kh + kh_idx(rs + col, g4);
    const int lim0 = C - 4 * g4;  // this lane's D rows are keys 16 kb + 4 g4 + i of the row
    f32x4 sc[4];
    float mx = -INFINITY;
#pragma unroll
    for (int kb = 0; kb < 4; ++kb) {
      if (kb < nkb) {
        const bf16x8 ak = *reinterpret_cast<const bf16x8*>(kp + kb * 16 * 32);
        sc[kb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ak, qf, f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
        const int lim = lim0 - 16 * kb;
#pragma unroll
        for (int i = 0; i < 4; ++i) sc[kb][i] = i < lim ? sc[kb][i] : -INFINITY;  // keys of the row only
        mx = max3f(mx, sc[kb][0], sc[kb][1]);
        mx = max3f(mx, sc[kb][2], sc[kb][3]);
      } else {
        sc[kb] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
    }
    mx = xor32_max(xor16_max(mx));
    float l = 0.f;
#pragma unroll
    for (int kb = 0; kb < 4; ++kb) {
      if (kb < nkb) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          sc[kb][i] = __builtin_amdgcn_exp2f(sc[kb][i] - mx);
          l += sc[kb][i];
        }
      }
    }
    l = xor32_sum(xor16_sum(l));
    f32x4 o[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
    for (int st = 0; st < 2; ++st) {
      if (st < nst) {
        const bf16x8 bp = pack8(sc[2 * st], sc[2 * st + 1]);
#pragma unroll
        for (int d = 0; d < 2; ++d)
          o[d] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(read_vt(smem, rs + 32 * st, 8 * h + 4 * d), bp, o[d], 0, 0, 0);
      }
    }
    const float inv = __builtin_amdgcn_rcpf(l);
    if (qt < re) *reinterpret_cast<bf16x8*>(qh + kh_idx(qt, g4)) = pack8(o[0] * inv, o[1] * inv);
  }
}

__device__ __forceinline__ void feat_attn_rows(char* smem, int C, int nrows) {
  switch ((C + 15) >> 4) {
    case 1: feat_attn_rows_t<1>(smem, C, nrows); break;
    case 2: feat_attn_rows_t<2>(smem, C, nrows); break;
    case 3: feat_attn_rows_t<3>(smem, C, nrows); break;
    default: feat_attn_rows_t<4>(smem, C, nrows); break;
  }
}

__device__ __forceinline__ void store_bf16_row(bf16_t* dst, const Acc& a, int g4) {
#pragma unroll
  for (int f = 0; f < 12; ++f) {
    uint2 pk;
    pk.x = pack_bf2(a[f][0], a[f][1]);
    pk.y = pack_bf2(a[f][2], a[f][3]);
    *reinterpret_cast<uint2*>(dst + f * 16 + g4 * 4) = pk;
  }
}
// a B-fragment array (pi order) back to feature order: slots 0-3 / 4-7 of fragment m hold
// features 32m + 4g.. / 32m + 16 + 4g..
__device__ __forceinline__ void store_frag_row(bf16_t* dst, const Frag& fr, int g4) {
#pragma unroll
  for (int m = 0; m < 6; ++m) {
    const uint4 u = __builtin_bit_cast(uint4, fr[m]);
    *reinterpret_cast<uint2*>(dst + 32 * m + 4 * g4) = make_uint2(u.x, u.y);
    *reinterpret_cast<uint2*>(dst + 32 * m + 16 + 4 * g4) = make_uint2(u.z, u.w);
  }
}

}  // namespace

// Diagnostic phase clock (build with -DNPFN_ROWK_STAMPS, `make stamps`): wave 0's
// s_memtime totals per phase, summed into P.stamps[0..7]; [15] = workgroups.
// 0 prologue, 1 chunk bodies (reads + MFMAs; the MLP GELUs included: they run inside the W2
// chunks), 2 LayerNorm, 3 chunk-open vmcnt waits, 4 k/v epilogues, 5 feature attention,
// 6 stores, 7 LDS-DMA issue, 8 chunk-open barrier waits.  The compiler may move
// VALU work across a stamp, so the split is indicative.
#ifdef NPFN_ROWK_STAMPS
#define MARK(k)                                                   \
  if (P.stamps) {                                                 \
    const unsigned long long now_ = __builtin_amdgcn_s_memtime(); \
    ph[k] += now_ - tprev;                                        \
    tprev = now_;                                                 \
  }
#define MARK_FLUSH()                                                               \
  if (P.stamps && threadIdx.x == 0) {                                              \
    for (int k_ = 0; k_ < 12; ++k_) atomicAdd(&P.stamps[k_], ph[k_]);               \
    atomicAdd(&P.stamps[15], 1ull);                                                \
  }
#else
#define MARK(k)
#define MARK_FLUSH()
#endif

// one head pair of the pre phase: k (O), q (O), attention, x += o Wo_f[:, hp]^T (S, followed
// by a chunk of kind NT_)
// one head pair of the pre phase: v (O), k (O), q (O) of the pair into the LDS images, the
// row-relative attention, x += o_hp Wo_f[:, hp]^T (S, followed by a chunk of kind NT_)
#define FEAT_PAIR(NT_)                                                                            \
  {                                                                                               \
    Acc4 kq;                                                                                      \
    run_o<LAG, CK_O>(ring, smem, a, xb, kq); /* values of heads 2hp, 2hp+1: dims 16f + 4g4 + i */      \
    {                                                                                             \
      bf16_t* vv = reinterpret_cast<bf16_t*>(smem + VV_OFF);                                      \
      _Pragma("unroll") for (int f = 0; f < 4; ++f) {                                             \
        uint2 pk;                                                                                 \
        pk.x = pack_bf2(kq[f][0], kq[f][1]);                                                      \
        pk.y = pack_bf2(kq[f][2], kq[f][3]);                                                      \
        *reinterpret_cast<uint2*>(vv + vv_idx(th, 4 * f + g4)) = pk;                              \
      }                                                                                           \
    }                                                                                             \
    run_o<LAG, CK_O>(ring, smem, a, xb, kq); /* keys */                                                \
    {                                                                                             \
      bf16_t* kh = reinterpret_cast<bf16_t*>(smem + KH_OFF);                                      \
      *reinterpret_cast<bf16x8*>(kh + kh_idx(th, g4)) = pack8(kq[0], kq[1]);                      \
      *reinterpret_cast<bf16x8*>(kh + KH_ELEMS + kh_idx(th, g4)) = pack8(kq[2], kq[3]);           \
    }                                                                                             \
    MARK(4);                                                                                      \
    run_o<LAG, CK_S>(ring, smem, a, xb, kq); /* queries (weights carry 1/sqrt(32) log2 e) */           \
    {                                                                                             \
      bf16_t* qh = reinterpret_cast<bf16_t*>(smem + QH_OFF);                                      \
      *reinterpret_cast<bf16x8*>(qh + kh_idx(th, g4)) = pack8(kq[0], kq[1]);                      \
      *reinterpret_cast<bf16x8*>(qh + KH_ELEMS + kh_idx(th, g4)) = pack8(kq[2], kq[3]);           \
    }                                                                                             \
    MARK(1);                                                                                      \
    bar(); /* every wave's v, k, q of the pair in LDS */                                          \
    FEAT_ATTN();                                                                                  \
    bar(); /* every item's output in the query image */                                           \
    bf16x8 of[2];                                                                                 \
    {                                                                                             \
      const bf16_t* qh = reinterpret_cast<const bf16_t*>(smem + QH_OFF);                          \
      _Pragma("unroll") for (int j = 0; j < 2; ++j) of[j] =                                      \
          tv ? *reinterpret_cast<const bf16x8*>(qh + j * KH_ELEMS + kh_idx(th, g4)) : bf16x8{};    \
    }                                                                                             \
    MARK(5);                                                                                      \
    run_s<LAG, false, false, NT_>(ring, smem, a, of[0], of[1], x); /* x += o_hp Wo_f[:, hp]^T */        \
    MARK(1);                                                                                      \
  }
#ifndef NPFN_DIAG_NOATTN
#define FEAT_ATTN() feat_attn_rows(smem, C, nrows)
#else
#define FEAT_ATTN()
#endif

// One instance per launch kind, so that every instance is straight-line code per tile (the
// pipeline's 24 prefetched fragments stay live across it; branches made the register
// allocator spill them): TRAIN = item q | k | v out (P.out_qkv), POST = P.do_post,
// PRE = P.do_pre.
template <bool TRAIN, bool POST, bool PRE, bool LAG>
__device__ __forceinline__ void row_layer_body(const RowLayerParams& P, char* smem) {
#ifdef NPFN_ROWK_STAMPS
  unsigned long long ph[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  unsigned long long tprev = __builtin_amdgcn_s_memtime();
#endif
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int col = lane & 15, g4 = lane >> 4;
  const int th = wave * 16 + col;  // this lane's token slot
  const int nslab = P.dff / 64;
  const int64_t ntiles = P.ntiles;
  if ((int64_t)blockIdx.x >= ntiles) return;
  const char* stream = reinterpret_cast<const char*>(P.stream);
  Ring ring{stream, stream + (int64_t)P.stream_chunks * WS_BYTES, stream, (uint32_t)(uintptr_t)(smem + WS_OFF), 0};
#ifdef NPFN_ROWK_STAMPS
  ring.ph = ph;
  ring.tprev = &tprev;
#endif
  const float* lnp = reinterpret_cast<const float*>(smem + LNP_OFF);

  // persistent: the weight stream runs on across this workgroup's tiles, so the next
  // tile's first chunks are in flight while the current one finishes
  ring.issue(0);
  ring.issue(1);
  ring.issue(2);
  if (tid < 288) {  // LayerNorm parameters of this launch -> LDS (read after the first chunk's barrier)
    const int a = tid / 48, o = (tid - a * 48) * 4;
    const float* src = a == 0 ? P.ln2g : a == 1 ? P.ln2b : a == 2 ? P.ln3g : a == 3 ? P.ln3b : a == 4 ? P.ln1g : P.ln1b;
    f32x4 v = f32x4{0.f, 0.f, 0.f, 0.f};
    if (src) v = *reinterpret_cast<const f32x4*>(src + o);
    *reinterpret_cast<f32x4*>(reinterpret_cast<float*>(smem + LNP_OFF) + a * 192 + o) = v;
  }
  // the attention images start finite (pad rows are read by the last row's blocks and steps,
  // scaled by zero probabilities; they are never written)
  for (int i = tid; i < (FA_END - KH_OFF) / 16; i += 512)
    *reinterpret_cast<uint4*>(smem + KH_OFF + 16 * i) = make_uint4(0, 0, 0, 0);
  // chunk 0 landed everywhere -> its first fragments (a post launch's stream starts with the
  // Wo_i S chunks, a pre-only launch's with the first pair's v O chunk)
  constexpr int FIRST = POST ? CK_S : CK_O;
  AWin a;
  wait_vmcnt<2 * GLDS_PER_WAVE>();
  bar();
  read_first_half<FIRST>(reinterpret_cast<const bf16_t*>(smem + WS_OFF), a);
  for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
  // the tile's segment (estimator group), picked with constant indices (no scratch copy)
  RowSeg sg = P.seg[0];
#pragma unroll
  for (int i = 1; i < kRowSegs; ++i)
    if (i < P.nseg && tile >= P.seg[i].tile0) sg = P.seg[i];
  const int C = sg.C;
  const int64_t tpe = (P.R + sg.rpt - 1) / sg.rpt;   // tiles per estimator
  const int64_t lt = tile - sg.tile0;
  const int64_t te = lt / tpe;                        // estimator of this tile
  const int64_t rt = (lt - te * tpe) * sg.rpt;        // first row within the estimator
  const int64_t row0 = te * P.R + rt;
  const int nrows = (int)max((int64_t)0, min((int64_t)sg.rpt, P.R - rt));
  const bool tv = th < nrows * C;
  const int64_t gt = row0 * C + th;
  Acc x;
#pragma unroll
  for (int f = 0; f < 12; ++f)
    x[f] = tv ? *reinterpret_cast<const f32x4*>(sg.resid + gt * 192 + f * 16 + g4 * 4) : f32x4{0.f, 0.f, 0.f, 0.f};

  Frag xb;
  MARK(0);
  if constexpr (POST) {
    Frag ob;  // item-attention output in pi order
#pragma unroll
    for (int m = 0; m < 6; ++m) {
      uint4 u = make_uint4(0, 0, 0, 0);
      if (tv) {
        const uint2 lo = *reinterpret_cast<const uint2*>(sg.o_item + gt * 192 + 32 * m + 4 * g4);
        const uint2 hi = *reinterpret_cast<const uint2*>(sg.o_item + gt * 192 + 32 * m + 16 + 4 * g4);
        u = make_uint4(lo.x, lo.y, hi.x, hi.y);
      }
      ob[m] = __builtin_bit_cast(bf16x8, u);
    }
    run_s<LAG, false, false, CK_S>(ring, smem, a, ob[0], ob[1], x);  // x += o_item Wo_i^T
    run_s<LAG, false, false, CK_S>(ring, smem, a, ob[2], ob[3], x);
    run_s<LAG, false, false, CK_O>(ring, smem, a, ob[4], ob[5], x);
    MARK(1);
    layer_norm(x, lnp + 0 * 384);
    to_frag(x, xb);
    MARK(2);
    // MLP, software-pipelined over 64-wide hidden slabs: W1_0 | W1_1, W2_0 (+GELU 1) | ...
    Acc4 h;
    bf16x8 hp0, hp1;  // GELU(h_{s-1}) as W2's B fragments
    run_o<LAG, CK_O>(ring, smem, a, xb, h);
    gelu_slab(h, hp0, hp1);
#pragma unroll 1
    for (int s = 1; s < nslab - 1; ++s) {
      run_o<LAG, CK_S>(ring, smem, a, xb, h);  // h_s = x W1_s^T
      bf16x8 hn0, hn1;
      run_w2_gelu<LAG, CK_O>(ring, smem, a, hp0, hp1, x, h, hn0, hn1);  // x += GELU(h_{s-1}) W2_{s-1}^T; GELU(h_s)
      hp0 = hn0;
      hp1 = hn1;
    }
    {
      run_o<LAG, CK_S>(ring, smem, a, xb, h);  // the last slab
      bf16x8 hn0, hn1;
      run_w2_gelu<LAG, CK_S>(ring, smem, a, hp0, hp1, x, h, hn0, hn1);
      run_s<LAG, false, false, PRE ? CK_O : FIRST>(ring, smem, a, hn0, hn1, x);  // x += GELU(h_last) W2_last^T
    }
    MARK(1);
    layer_norm(x, lnp + 1 * 384);
    to_frag(x, xb);
    MARK(2);
    if constexpr (!PRE) {  // last layer: bf16 x for the decoder
      if (tv) store_bf16_row(sg.out + gt * 192, x, g4);
      MARK(6);
      continue;
    }
  } else {
    to_frag(x, xb);
  }

  // ---- pre of the next layer: head pairs; Wo_f's slice of the last pair is followed by the
  // item q chunk (S)
#pragma unroll 1
  for (int hp_i = 0; hp_i < 2; ++hp_i) FEAT_PAIR(CK_O);
  FEAT_PAIR(CK_S);
  layer_norm(x, lnp + 2 * 384);
  to_frag(x, xb);
  MARK(2);
  Acc acc;
  run_s<LAG, true, false, CK_S>(ring, smem, a, xb[0], xb[1], acc);  // item-attention q
  run_s<LAG, false, false, CK_S>(ring, smem, a, xb[2], xb[3], acc);
  run_s<LAG, false, false, TRAIN ? CK_S : FIRST>(ring, smem, a, xb[4], xb[5], acc);  // next: the next tile's first chunk, or k
  MARK(1);
  if constexpr (!TRAIN) {
    if (tv) {
      store_bf16_row(sg.out + gt * 192, acc, g4);
#pragma unroll
      for (int f = 0; f < 12; ++f) *reinterpret_cast<f32x4*>(sg.resid + gt * 192 + f * 16 + g4 * 4) = x[f];
    }
    MARK(6);
    continue;
  }
  // train side: x is final, store it now (frees 48 registers for holding q and k)
  if (tv) {
#pragma unroll
    for (int f = 0; f < 12; ++f) *reinterpret_cast<f32x4*>(sg.resid + gt * 192 + f * 16 + g4 * 4) = x[f];
  }
  Frag qb, kb;  // bf16 q, k held until the tile's stream has ended
  to_frag(acc, qb);
  run_s<LAG, true, false, CK_S>(ring, smem, a, xb[0], xb[1], acc);  // item-attention k
  run_s<LAG, false, false, CK_S>(ring, smem, a, xb[2], xb[3], acc);
  run_s<LAG, false, false, CK_S>(ring, smem, a, xb[4], xb[5], acc);
  to_frag(acc, kb);
  run_s<LAG, true, false, CK_S>(ring, smem, a, xb[0], xb[1], acc);  // item-attention v
  run_s<LAG, false, false, CK_S>(ring, smem, a, xb[2], xb[3], acc);
  run_s<LAG, false, false, FIRST>(ring, smem, a, xb[4], xb[5], acc);  // next: the next tile's first chunk
  if (tv) {
    bf16_t* o = sg.out + gt * 576;
    store_frag_row(o, qb, g4);
    store_frag_row(o + 192, kb, g4);
    store_bf16_row(o + 384, acc, g4);
  }
  MARK(6);
  }  // tiles
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // drain the wrapped-around DMA
  MARK_FLUSH();
}

template <bool TRAIN, bool POST, bool PRE>
__global__ __launch_bounds__(512, 1) void k_row_layer(RowLayerParams P) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
#if NPFN_ROWK_STAGGER
  if (__builtin_amdgcn_readfirstlane(threadIdx.x >> 6) >= 4) row_layer_body<TRAIN, POST, PRE, true>(P, smem);
  else row_layer_body<TRAIN, POST, PRE, false>(P, smem);
#else
  row_layer_body<TRAIN, POST, PRE, false>(P, smem);
#endif
}

static_assert(SMEM_BYTES <= 160 * 1024, "LDS budget");

void rowk_setup() {
  (void)hipFuncSetAttribute((const void*)k_row_layer<false, false, true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            SMEM_BYTES);
  (void)hipFuncSetAttribute((const void*)k_row_layer<false, true, true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            SMEM_BYTES);
  (void)hipFuncSetAttribute((const void*)k_row_layer<false, true, false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            SMEM_BYTES);
  (void)hipFuncSetAttribute((const void*)k_row_layer<true, false, true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            SMEM_BYTES);
  (void)hipFuncSetAttribute((const void*)k_row_layer<true, true, true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            SMEM_BYTES);
}

// whole rows per tile (128 token slots): C <= 128
int rowk_rows_per_tile(int C) { return RT / C; }

int64_t rowk_grid(int64_t ntiles) {
  static int ncu = 0;  // one persistent workgroup per CU
  if (ncu == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu <= 0) ncu = 256;
  }
  return ntiles < ncu ? ntiles : ncu;
}

// (static tile schedule only: p.tile_ctr is not read)
void launch_row_layer(const RowLayerParams& p, hipStream_t s) {
  const int64_t grid = rowk_grid(p.ntiles);
  if (grid <= 0) return;
  const dim3 g((unsigned)grid), b(512);
  if (p.out_qkv) {  // the train side never runs a post-only launch (it stops after the last item attention)
    if (p.do_post) hipLaunchKernelGGL((k_row_layer<true, true, true>), g, b, SMEM_BYTES, s, p);
    else hipLaunchKernelGGL((k_row_layer<true, false, true>), g, b, SMEM_BYTES, s, p);
  } else if (!p.do_post) {
    hipLaunchKernelGGL((k_row_layer<false, false, true>), g, b, SMEM_BYTES, s, p);
  } else if (p.do_pre) {
    hipLaunchKernelGGL((k_row_layer<false, true, true>), g, b, SMEM_BYTES, s, p);
  } else {
    hipLaunchKernelGGL((k_row_layer<false, true, false>), g, b, SMEM_BYTES, s, p);
  }
}

}  // namespace npfn
