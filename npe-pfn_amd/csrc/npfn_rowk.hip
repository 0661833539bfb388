// npfn_rowk.hip -- fused row-tile layer kernel (everything of a PerFeatureEncoderLayer
// except the item attention, which needs other rows), register-resident.
//
// One workgroup (8 waves) owns a tile of whole rows (rpt rows x C tokens <= 128
// tokens); wave w owns tokens 16w .. 16w+15, one per lane column (lane & 15).  The
// chain of the layer runs on those 16 tokens entirely in the wave's registers:
//
//   [post of layer l]  x = LN2(x + o_item Wo_i^T); for c < 4: h = GELU(x W1_c^T),
//                      x += h W2_c^T; x = LN3(x)
//   [pre of layer l+1] k, v, q = x Wk_f^T, x Wv_f^T, x Wq_f^T; feature attention over
//                      the row's C tokens (per head, K / V^T of the tile through LDS);
//                      x = LN1(x + o Wo_f^T); out = x Wq_i^T (test) or x Wqkv_i^T (train)
//
// Every GEMM is Y^T = W X^T on v_mfma_f32_16x16x32_bf16 with A = weight rows from LDS
// and B = the wave's activations.  The D tile of features 16f.. of a GEMM leaves lane
// (g = lane >> 4) features 16f + 4g + {0..3}; packing D tiles 2m and 2m+1 gives the
// B fragment of K-step m in the order
//     slot 8g + j  <->  feature 32m + pi(8g + j),  pi = j < 4 ? 4g + j : 16 + 4g + j - 4,
// so a GEMM's output is the next GEMM's input without leaving the registers, provided
// the weights' K axis is stored in the same order (npfn_engine.hip uploads a
// pi-permuted copy of every row-kernel weight).  LayerNorm over a token's 192 features
// is an in-lane sum + two lane shuffles, and every residual add is the accumulator
// input of the sub-layer's output GEMM (x is the MFMA C operand).  Only the weights and the per-head K / V^T of
// the feature attention go through LDS.
//
// Weights stream as [192][64] chunks (3 per GEMM) through a 3-slot LDS ring filled by
// LDS-DMA (global_load_lds_dwordx4; the bank swizzle is applied on the source address).
// All barriers are raw s_barrier after lgkmcnt(0): a __syncthreads() fence would drain
// the DMA queue.
//
// Weight issue.  Waves 0-3 (half A, one per SIMD) own the tile's token slots 0-63, waves
// 4-7 (half B) slots 64-127.  Rows pack the whole 128-slot tile (rpt = floor(128 / C), a
// row may straddle the halves: all eight waves write their keys before the feature
// attention's barrier); only the ping-pong variant keeps rows inside a half (rpt = 2 *
// floor(64 / C)).  Half A issues the whole weight stream.  Default (lockstep): both halves run the
// same events; at its open of chunk i A waits until chunk i has landed with a counted
// vmcnt(6) (chunk i+1 stays in flight), passes the barrier and refills the slot of chunk
// i-1, which every wave has finished, with chunk i+2 (lead 2, 3-slot ring).  This beat
// the ping-pong variant below by 1.8 % on the c2 workload (tools/ab.py, same GPU).
//
// Ping-pong halves (-DNPFN_ROWK_PINGPONG).  Both halves run the same program, but B runs one barrier behind A: B
// executes one extra barrier before its first chunk, A one after its last.  Every
// s_barrier is therefore A's event e and B's event e-1, so while one half runs an
// epilogue (LayerNorm, GELU, operand packing, feature-attention softmax) on the VALU the
// other half issues the MFMAs of a GEMM chunk on the same SIMDs, instead of all eight
// waves idling the matrix pipes through the epilogue together.  Half A issues the whole
// weight stream: at its open of chunk i it waits for chunk i (vmcnt(0): every older
// vector-memory op of A), passes the barrier and refills the slot of chunk i-2 -- which
// B, one event behind and so at least at its own open of chunk i-1, has finished -- with
// chunk i+1.  B's open of chunk i is A's next barrier, after A's wait for chunk i.  The
// two halves touch disjoint parts of the key/value images, so the feature-attention
// barriers need no cross-half ordering.
#include "npfn_common.h"
#include "npfn_kernels.h"

namespace npfn {
namespace {

constexpr int RT = 128;                              // token slots per tile (8 waves x 16)
constexpr int HT = 64;                               // token slots per half
#ifdef NPFN_ROWK_PINGPONG
constexpr int RS = HT;                               // slots a row's keys may span (its half)
#else
constexpr int RS = RT;                               // the whole tile (lockstep halves)
#endif
constexpr int NSLOT = 3;                             // weight ring depth
constexpr int WS_ELEMS = 192 * 64;                   // one [192][64] bf16 chunk
constexpr int WS_OFF = 0;
constexpr int KH_OFF = WS_OFF + NSLOT * WS_ELEMS * 2;  // 2 pairs x 2 heads x bf16 [RT][32] head keys (pi order)
constexpr int KH_ELEMS = RT * 32;
constexpr int VT_OFF = KH_OFF + 4 * KH_ELEMS * 2;      // bf16 [192][RT] values, transposed
constexpr int LNP_OFF = VT_OFF + 192 * RT * 2;         // float [6][192]: ln2 g,b | ln3 g,b | ln1 g,b
constexpr int SMEM_BYTES = LNP_OFF + 6 * 192 * 4;
constexpr int GLDS_PER_CHUNK = 6;                    // 16-B LDS-DMA instructions per half-A thread per chunk

typedef f32x4 Acc[12];   // D of a 192-feature GEMM for the wave's 16 tokens
typedef bf16x8 Frag[6];  // B operand of a K = 192 GEMM (pi order per 32-feature step)

__device__ __forceinline__ void bar() { lds_barrier(); }

// element offset of 16-byte unit `ch` of row `row` in a swizzled [rows][8 units] chunk image
__device__ __forceinline__ int wsz(int row, int ch) { return (row * 8 + (ch ^ (row & 7))) * 8; }
// head-key image [RT][32] (4 units per token row)
__device__ __forceinline__ int kh_idx(int t, int u) { return t * 32 + ((u ^ ((t >> 2) & 3)) << 3); }
// value image [192][RT]: 8-byte granule (t/4) ^ (d % 16) of row d
__device__ __forceinline__ int vt_idx(int d, int t) { return d * RT + ((((t >> 2) ^ (d & 15))) << 2) + (t & 3); }

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
__device__ __forceinline__ void zero(Acc& a) {
#pragma unroll
  for (int f = 0; f < 12; ++f) a[f] = f32x4{0.f, 0.f, 0.f, 0.f};
}

// The weight stream of one tile: P.stream_chunks [192][64] chunk images in consumption
// order (npfn_engine.hip build_rowk_streams), 3 per GEMM, K axes pi-permuted (see the file
// comment); replayed from the start for every tile.  Since every GEMM is 3 chunks, chunk c
// of every GEMM lives in ring slot c: slots and LDS addresses are compile-time constants.
struct Ring {
  const char* istart;  // stream of this launch
  const char* iend;
  const char* isrc;    // next chunk to issue (half A)
  uint32_t ws_lds;     // LDS byte address of slot 0
  bool issuer;         // half A: issues the stream and waits for it

  // next chunk of the stream -> slot SLOT: a contiguous 24 KB copy by the 4 waves of half
  // A, 1 KB per wave instruction, scalar source base + per-lane 32-bit offset.  The stream
  // wraps to the next tile's first chunk (after the last tile it lands in a slot never
  // read, and A drains it before exiting).
  template <int SLOT>
  __device__ __forceinline__ void issue() {
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t voff = (threadIdx.x & 255) * 16u;  // the lane's 16 bytes of each 4 KB piece
    const uint32_t dst = ws_lds + (uint32_t)(SLOT * WS_ELEMS * 2) + (uint32_t)wave * 1024u;
#pragma unroll
    for (int p = 0; p < GLDS_PER_CHUNK; ++p)  // piece p: 16-byte units 256 p .. 256 p + 255 (waves 0-3)
      glds16_s(isrc + p * 4096, voff, dst + (uint32_t)p * 4096u);
    isrc += WS_ELEMS * 2;
    if (isrc == iend) isrc = istart;
  }
  // open chunk c (slot c) of a GEMM.  A: wait for it, barrier, issue the next chunk into
  // slot c+1 (the slot of chunk i-2, left by both halves); B: barrier (A waited for the
  // chunk one barrier earlier).
  template <int C>
  __device__ __forceinline__ void open() {
#ifdef NPFN_ROWK_PINGPONG
    if (issuer) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    bar();
    if (issuer) issue<(C + 1) % NSLOT>();
#else  // all waves in step, chunk i+1 stays in flight, chunk i+2 refills the slot of i-1
    if (issuer) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    bar();
    if (issuer) issue<(C + 2) % NSLOT>();
#endif
  }
};

// acc += W_g X^T (INIT: acc = W_g X^T) over the three chunks of the stream's next GEMM.  SWAP:
// D = X W_g^T (rows = the wave's tokens 4g+i, cols = features) -- the layout the v^T image wants.
template <int KC, bool SWAP, bool INIT>
__device__ __forceinline__ void gemm_chunk(Ring& ring, const char* smem, const Frag& b, Acc& acc) {
  const int lane = threadIdx.x & 63;
  // row f*16 + (lane & 15) of the chunk, unit (4 ks + (lane >> 4)) ^ (lane & 7): wsz() with the
  // f-independent part hoisted (two lane offsets instead of 24 addresses)
  const int off0 = (lane & 15) * 64 + (((lane >> 4) ^ (lane & 7)) << 3);
  const int off1 = (lane & 15) * 64 + (((4 + (lane >> 4)) ^ (lane & 7)) << 3);
  ring.open<KC>();
  const bf16_t* wb = reinterpret_cast<const bf16_t*>(smem + WS_OFF) + KC * WS_ELEMS;
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) {  // K-step: 12 fragments in flight
    const bf16_t* wk = wb + (ks ? off1 : off0);
    bf16x8 a[12];
#pragma unroll
    for (int f = 0; f < 12; ++f) a[f] = *reinterpret_cast<const bf16x8*>(wk + f * 1024);
    const bool first = INIT && ks == 0;  // INIT: acc = W X^T (C = 0 on the first K-step)
#ifndef NPFN_DIAG_NOMFMA
#pragma unroll
    for (int f = 0; f < 12; ++f) {
      const f32x4 c = first ? f32x4{0.f, 0.f, 0.f, 0.f} : acc[f];
      acc[f] = SWAP ? __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[2 * KC + ks], a[f], c, 0, 0, 0)
                    : __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[f], b[2 * KC + ks], c, 0, 0, 0);
    }
#else  // diagnostic: fragments read, no matrix work
#pragma unroll
    for (int f = 0; f < 12; ++f) {
      asm volatile("" ::"v"(a[f]));
      if (first) acc[f] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
#endif
  }
}
template <bool SWAP, bool INIT>
__device__ __forceinline__ void gemm(Ring& ring, const char* smem, const Frag& b, Acc& acc) {
  gemm_chunk<0, SWAP, INIT>(ring, smem, b, acc);
  gemm_chunk<1, SWAP, false>(ring, smem, b, acc);
  gemm_chunk<2, SWAP, false>(ring, smem, b, acc);
}

// x = LN(x) * gamma + beta over the token's 192 features (lanes l, l^16, l^32, l^48).
// The residual add is already in x: every sub-layer's output GEMM accumulates into x.
__device__ __forceinline__ void layer_norm(Acc& x, const float* lnp) {
#ifdef NPFN_DIAG_NOLN
  return;
#endif
  const int g4 = (threadIdx.x & 63) >> 4;
  float s = 0.f;
#pragma unroll
  for (int f = 0; f < 12; ++f)
#pragma unroll
    for (int r = 0; r < 4; ++r) s += x[f][r];
  s = xor32_sum(xor16_sum(s));
  const float mean = s * (1.0f / 192.0f);
  float v = 0.f;
#pragma unroll
  for (int f = 0; f < 12; ++f)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float d = x[f][r] - mean;
      v += d * d;
    }
  v = xor32_sum(xor16_sum(v));
  const float rstd = 1.0f / sqrtf(v * (1.0f / 192.0f) + 1e-5f);
#pragma unroll
  for (int f = 0; f < 12; ++f) {
    const f32x4 gg = *reinterpret_cast<const f32x4*>(lnp + f * 16 + g4 * 4);
    const f32x4 bb = *reinterpret_cast<const f32x4*>(lnp + 192 + f * 16 + g4 * 4);
#pragma unroll
    for (int r = 0; r < 4; ++r) x[f][r] = (x[f][r] - mean) * rstd * gg[r] + bb[r];
  }
}

// Feature attention of the wave's 16 query tokens, two heads at a time (values already
// in the v^T image; q pre-scaled by 1/sqrt(32) log2 e).  Per head pair: every wave writes
// its tokens' keys of both heads (pi order, one 16-B store each) into the pair's key
// images (two sets, alternating); after one barrier each wave runs, for both heads
// interleaved, S^T = K Q^T per 16-key block (one MFMA: K = the 32 head dims), a masked
// online softmax down each query column (keys of the same row only) and O^T += V^T P^T
// per 32-key step, whose key order is permuted identically in A (v^T granules) and B
// (the lane's own probabilities).  O^T lands in pi order: the B fragment of Wo_f's
// K-step h.  Rows are packed from slot 0 of their span (the tile, or the half in the
// ping-pong variant), so a query's key blocks never leave the span.
__device__ void feature_attention(char* smem, const Frag& kf, const Frag& qf, Frag& of, int C) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int col = lane & 15, g4 = lane >> 4;
  const int q0 = wave * 16, q = q0 + col;
  const int hb = RS == HT ? (wave >> 2) * HT : 0, h0 = q0 - hb;  // the span's first slot; its rows start there
  const int rs = hb + ((q - hb) / C) * C;         // keys of the query's row: [rs, rs + C)
  const int kb0 = (hb + (h0 / C) * C) >> 4;
  const int kb1 = min(hb + ((h0 + 15) / C) * C + C - 1, hb + RS - 1) >> 4;
  const bf16_t* vt = reinterpret_cast<const bf16_t*>(smem + VT_OFF);
#pragma unroll
  for (int hp = 0; hp < 3; ++hp) {
    bf16_t* kh = reinterpret_cast<bf16_t*>(smem + KH_OFF) + (hp & 1) * 2 * KH_ELEMS;
#pragma unroll
    for (int j = 0; j < 2; ++j) *reinterpret_cast<bf16x8*>(kh + j * KH_ELEMS + kh_idx(q, g4)) = kf[2 * hp + j];
    bar();  // also: every wave of the half finished pair hp-2's reads of this set (before pair hp-1's barrier)
    float m[2] = {-INFINITY, -INFINITY}, l[2] = {0.f, 0.f};
    f32x4 o[2][2];
#pragma unroll
    for (int j = 0; j < 2; ++j) o[j][0] = o[j][1] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int pb = kb0 >> 1; pb <= (kb1 >> 1); ++pb) {
      f32x4 s[2][2];
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const int kb = 2 * pb + kk;
        const bool in = kb >= kb0 && kb <= kb1;
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          s[j][kk] = f32x4{0.f, 0.f, 0.f, 0.f};
          if (in) {
            const bf16x8 ak = *reinterpret_cast<const bf16x8*>(kh + j * KH_ELEMS + kh_idx(kb * 16 + col, g4));
            s[j][kk] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ak, qf[2 * hp + j], s[j][kk], 0, 0, 0);
          }
        }
      }
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        // keys of the query's row only (blocks outside [kb0, kb1] hold none of them)
        const uint32_t d0 = (uint32_t)((2 * pb + kk) * 16 + g4 * 4 - rs);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const bool keep = d0 + i < (uint32_t)C;
#pragma unroll
          for (int j = 0; j < 2; ++j) s[j][kk][i] = keep ? s[j][kk][i] : -INFINITY;
        }
      }
      float mx[2];
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        float t = max3f(m[j], s[j][0][0], s[j][0][1]);
        t = max3f(t, s[j][0][2], s[j][0][3]);
        t = max3f(t, s[j][1][0], s[j][1][1]);
        mx[j] = max3f(t, s[j][1][2], s[j][1][3]);
      }
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        mx[j] = xor32_max(xor16_max(mx[j]));
      }
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const float mref = (mx[j] == -INFINITY) ? 0.f : mx[j];  // no key of the row yet: keep l = o = 0
        const float alpha = __builtin_amdgcn_exp2f(m[j] - mref);
        l[j] *= alpha;
#pragma unroll
        for (int d = 0; d < 2; ++d) o[j][d] *= alpha;
#pragma unroll
        for (int kk = 0; kk < 2; ++kk)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            s[j][kk][i] = __builtin_amdgcn_exp2f(s[j][kk][i] - mref);
            l[j] += s[j][kk][i];
          }
        m[j] = mx[j];
      }
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const bf16x8 bp = pack8(s[j][0], s[j][1]);
#pragma unroll
        for (int d = 0; d < 2; ++d) {
          const int dim = (2 * hp + j) * 32 + d * 16 + col;
          const uint2 lo = *reinterpret_cast<const uint2*>(vt + vt_idx(dim, 32 * pb + 4 * g4));
          const uint2 hi = *reinterpret_cast<const uint2*>(vt + vt_idx(dim, 32 * pb + 16 + 4 * g4));
          const uint4 u = make_uint4(lo.x, lo.y, hi.x, hi.y);
          o[j][d] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, u), bp, o[j][d], 0, 0, 0);
        }
      }
    }
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      l[j] = xor32_sum(xor16_sum(l[j]));
      const float inv = 1.0f / l[j];
      of[2 * hp + j] = pack8(o[j][0] * inv, o[j][1] * inv);
    }
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

}  // namespace

// Diagnostic phase clock (build with -DNPFN_ROWK_STAMPS, `make stamps`): wave 0's
// s_memtime totals per phase, summed over tiles into P.stamps[0..7]; [15] = tiles.
// 0 prologue, 1 GEMMs, 2 LayerNorm, 3 GELU, 4 k/v/q epilogues, 5 feature attention, 6 stores
#ifdef NPFN_ROWK_STAMPS
#define MARK(k)                                                   \
  if (P.stamps) {                                                 \
    const unsigned long long now_ = __builtin_amdgcn_s_memtime(); \
    ph[k] += now_ - tprev;                                        \
    tprev = now_;                                                 \
  }
#define MARK_FLUSH()                                                               \
  if (P.stamps && threadIdx.x == 0) {                                              \
    for (int k_ = 0; k_ < 8; ++k_) atomicAdd(&P.stamps[k_], ph[k_]);               \
    atomicAdd(&P.stamps[15], 1ull);                                                \
  }
#else
#define MARK(k)
#define MARK_FLUSH()
#endif

__global__ __launch_bounds__(512, 1) void k_row_layer(RowLayerParams P) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
#ifdef NPFN_ROWK_STAMPS
  unsigned long long ph[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  unsigned long long tprev = __builtin_amdgcn_s_memtime();
#endif
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int col = lane & 15, g4 = lane >> 4;
  const int C = P.C;
  const int half = __builtin_amdgcn_readfirstlane(wave >> 2);  // 0: A, 1: B (one barrier behind)
  // this lane's token slot within its row span (the tile, or its half when ping-ponging)
  const int th = RS == HT ? (wave & 3) * 16 + col : wave * 16 + col;
  const int rph = RS == HT ? P.rpt >> 1 : P.rpt;                // rows per span
  const int nh = P.dff / 192;
  const int64_t tpe = (P.R + P.rpt - 1) / P.rpt;  // tiles per estimator
  const int64_t ntiles = tpe * (P.rows / P.R);
  if ((int64_t)blockIdx.x >= ntiles) return;
  const char* stream = reinterpret_cast<const char*>(P.stream);
  Ring ring{stream, stream + (int64_t)P.stream_chunks * WS_ELEMS * 2, stream, (uint32_t)(uintptr_t)(smem + WS_OFF),
            half == 0};
  const float* lnp = reinterpret_cast<const float*>(smem + LNP_OFF);

  // persistent: the weight stream runs on across this workgroup's tiles, so the next
  // tile's first chunk is in flight while the current one finishes
  if (half == 0) ring.issue<0>();  // chunk 0
#ifndef NPFN_ROWK_PINGPONG
  if (half == 0) ring.issue<1>();
#endif
  if (tid < 288) {  // LayerNorm parameters of this launch -> LDS (read after the first chunk's barrier)
    const int a = tid / 48, o = (tid - a * 48) * 4;
    const float* src = a == 0 ? P.ln2g : a == 1 ? P.ln2b : a == 2 ? P.ln3g : a == 3 ? P.ln3b : a == 4 ? P.ln1g : P.ln1b;
    f32x4 v = f32x4{0.f, 0.f, 0.f, 0.f};
    if (src) v = *reinterpret_cast<const f32x4*>(src + o);
    *reinterpret_cast<f32x4*>(reinterpret_cast<float*>(smem + LNP_OFF) + a * 192 + o) = v;
  }
#ifdef NPFN_ROWK_PINGPONG
  if (half == 1) bar();  // B: one barrier behind A from here on
#endif
  for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
  const int64_t te = tile / tpe;                      // estimator of this tile
  const int64_t rt = (tile - te * tpe) * P.rpt + (RS == HT ? half * rph : 0);  // first row within the estimator
  const int64_t row0 = te * P.R + rt;                 // first row of this span
  const int nrows = (int)max((int64_t)0, min((int64_t)rph, P.R - rt));
  const bool tv = th < nrows * C;
  const int64_t gt = row0 * C + th;
  Acc x;
#pragma unroll
  for (int f = 0; f < 12; ++f)
    x[f] = tv ? *reinterpret_cast<const f32x4*>(P.resid + gt * 192 + f * 16 + g4 * 4) : f32x4{0.f, 0.f, 0.f, 0.f};

  Frag xb;
  Acc acc;
  MARK(0);
  if (P.do_post) {
    Frag ob;  // item-attention output in pi order
#pragma unroll
    for (int m = 0; m < 6; ++m) {
      uint4 u = make_uint4(0, 0, 0, 0);
      if (tv) {
        const uint2 lo = *reinterpret_cast<const uint2*>(P.o_item + gt * 192 + 32 * m + 4 * g4);
        const uint2 hi = *reinterpret_cast<const uint2*>(P.o_item + gt * 192 + 32 * m + 16 + 4 * g4);
        u = make_uint4(lo.x, lo.y, hi.x, hi.y);
      }
      ob[m] = __builtin_bit_cast(bf16x8, u);
    }
    gemm<false, false>(ring, smem, ob, x);  // x += o_item Wo_i^T
    MARK(1);
    layer_norm(x, lnp + 0 * 384);
    to_frag(x, xb);
    MARK(2);
#pragma unroll 1
    for (int c = 0; c < nh; ++c) {
      gemm<false, true>(ring, smem, xb, acc);  // W1 rows of hidden chunk c
      MARK(1);
      Frag hf;
#ifndef NPFN_DIAG_NOGELU
#pragma unroll
      for (int f = 0; f < 12; ++f)
#pragma unroll
        for (int r = 0; r < 4; r += 2) {
          acc[f][r] = gelu_tanh(acc[f][r]);
          acc[f][r + 1] = gelu_tanh(acc[f][r + 1]);
        }
#endif
      to_frag(acc, hf);
      MARK(3);
      gemm<false, false>(ring, smem, hf, x);  // x += h_c W2_c^T
      MARK(1);
    }
    layer_norm(x, lnp + 1 * 384);
    to_frag(x, xb);
    MARK(2);
    if (!P.do_pre) {  // last layer: bf16 x for the decoder
      if (tv) store_bf16_row(P.out + gt * 192, x, g4);
      MARK(6);
      continue;
    }
  } else {
    to_frag(x, xb);
  }

  // ---- pre of the next layer
  Frag kf, qf, of;
  gemm<false, true>(ring, smem, xb, acc);  // k
  MARK(1);
  to_frag(acc, kf);
  MARK(4);
  gemm<true, true>(ring, smem, xb, acc);  // v, swapped: lane holds tokens 16w + 4g4 + {0..3} of feature 16f + col
  MARK(1);
  {
    bf16_t* vt = reinterpret_cast<bf16_t*>(smem + VT_OFF);  // read after feature attention's first barrier
#pragma unroll
    for (int f = 0; f < 12; ++f) {
      uint2 pk;
      pk.x = pack_bf2(acc[f][0], acc[f][1]);
      pk.y = pack_bf2(acc[f][2], acc[f][3]);
      *reinterpret_cast<uint2*>(vt + vt_idx(f * 16 + col, wave * 16 + 4 * g4)) = pk;
    }
  }
  MARK(4);
  gemm<false, true>(ring, smem, xb, acc);  // q
  MARK(1);
#pragma unroll
  for (int f = 0; f < 12; ++f) acc[f] *= 0.17677669529663687f * 1.4426950408889634f;  // 1/sqrt(32) log2(e): S in log2 units
  to_frag(acc, qf);
  MARK(4);
#ifndef NPFN_DIAG_NOATTN
  feature_attention(smem, kf, qf, of, C);
#else
#pragma unroll
  for (int m = 0; m < 6; ++m) of[m] = qf[m] + kf[m];
#endif
  MARK(5);
  gemm<false, false>(ring, smem, of, x);  // x += o Wo_f^T
  MARK(1);
  layer_norm(x, lnp + 2 * 384);
  to_frag(x, xb);
  MARK(2);
  gemm<false, true>(ring, smem, xb, acc);  // item-attention q
  MARK(1);
  if (!P.out_qkv) {
    if (tv) {
      store_bf16_row(P.out + gt * 192, acc, g4);
#pragma unroll
      for (int f = 0; f < 12; ++f) *reinterpret_cast<f32x4*>(P.resid + gt * 192 + f * 16 + g4 * 4) = x[f];
    }
    MARK(6);
    continue;
  }
  Acc acc_k;
  gemm<false, true>(ring, smem, xb, acc_k);  // item-attention k
  Frag qb, kb;  // bf16 q, k held until the stream has ended
  to_frag(acc, qb);
  to_frag(acc_k, kb);
  gemm<false, true>(ring, smem, xb, acc);  // item-attention v
  if (tv) {
    bf16_t* o = P.out + gt * 576;
#pragma unroll
    for (int m = 0; m < 6; ++m) {  // undo pi: slots 0-3 / 4-7 hold features 32m+4g4.. / 32m+16+4g4..
      const uint4 uq = __builtin_bit_cast(uint4, qb[m]);
      const uint4 uk = __builtin_bit_cast(uint4, kb[m]);
      *reinterpret_cast<uint2*>(o + 32 * m + 4 * g4) = make_uint2(uq.x, uq.y);
      *reinterpret_cast<uint2*>(o + 32 * m + 16 + 4 * g4) = make_uint2(uq.z, uq.w);
      *reinterpret_cast<uint2*>(o + 192 + 32 * m + 4 * g4) = make_uint2(uk.x, uk.y);
      *reinterpret_cast<uint2*>(o + 192 + 32 * m + 16 + 4 * g4) = make_uint2(uk.z, uk.w);
    }
    store_bf16_row(o + 384, acc, g4);
#pragma unroll
    for (int f = 0; f < 12; ++f) *reinterpret_cast<f32x4*>(P.resid + gt * 192 + f * 16 + g4 * 4) = x[f];
  }
  MARK(6);
  }  // tiles
  if (half == 0) {  // A: drain the wrapped-around DMA, then the barrier B's last open pairs with
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#ifdef NPFN_ROWK_PINGPONG
    bar();
#endif
  }
  MARK_FLUSH();
}

static_assert(SMEM_BYTES <= 160 * 1024, "LDS budget");

void rowk_setup() {
  (void)hipFuncSetAttribute((const void*)k_row_layer, hipFuncAttributeMaxDynamicSharedMemorySize, SMEM_BYTES);
}

// whole rows per tile (128 token slots; 64 per half in the ping-pong variant): C <= 56
int rowk_rows_per_tile(int C) { return RS == HT ? 2 * (HT / C) : RT / C; }

void launch_row_layer(const RowLayerParams& p, hipStream_t s) {
  static int ncu = 0;  // one persistent workgroup per CU
  if (ncu == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu <= 0) ncu = 256;
  }
  const int64_t tiles = (p.R + p.rpt - 1) / p.rpt * (p.rows / p.R);
  const int64_t grid = tiles < ncu ? tiles : ncu;
  if (grid > 0) hipLaunchKernelGGL(k_row_layer, dim3((unsigned)grid), dim3(512), SMEM_BYTES, s, p);
}

}  // namespace npfn
