// npfn_rowk.hip -- fused row-tile layer kernel (everything of a PerFeatureEncoderLayer
// except the item attention, which needs other rows).
//
// One workgroup (8 waves) owns a tile of whole rows (rpt rows x C tokens <= 64
// tokens).  The fp32 residual stream of the tile stays in registers and its bf16
// copy in LDS across the chain
//
//   [post of layer l]  x = LN2(x + o_item Wo_i^T); h_c = GELU(x W1_c^T) (4 chunks of
//                      192 hidden units in LDS); x = LN3(x + sum_c h_c W2_c^T)
//   [pre of layer l+1] k, v = x Wk_f^T, x Wv_f^T (LDS); q = x Wq_f^T (LDS, in the x
//                      slot once the GEMMs have read it); feature attention over the
//                      row's C tokens, a lane pair per (token, head), output in place of q;
//                      x = LN1(x + o Wo_f^T); out = x Wq_i^T (test) or x Wqkv_i^T (train)
//
// so HBM sees only the item-attention output, the residual and the next queries
// (~3 KB per token and layer instead of ~14 KB for per-sublayer kernels).
// Every GEMM of the chain is 192 output features x 192 inputs, streamed as three
// [192][64] weight chunks through a 3-slot LDS ring filled by LDS-DMA
// (global_load_lds_dwordx4, swizzle applied on the source address): chunk i+2 is
// issued right after the barrier that opens chunk i, so two chunks are always in
// flight -- also across GEMM epilogues -- and the only wait is a counted vmcnt.
// All barriers are raw s_barrier after lgkmcnt(0): a __syncthreads() fence would
// drain the DMA queue.
//
// Every GEMM is computed transposed, Y^T = W X^T on v_mfma_f32_16x16x32_bf16 (A =
// weight rows, B = token rows): a lane then holds 4 consecutive features of one
// token per 16x16 tile, so LayerNorm over features is a register sum + 2 lane
// shuffles + one 4-wave LDS exchange, and bf16 outputs are 8-byte LDS writes.
#include "npfn_common.h"
#include "npfn_kernels.h"

namespace npfn {
namespace {

constexpr int RT = 64;                       // token slots per tile
constexpr int XB_OFF = 0;                    // bf16 [RT][192] (24 chunks/row): x | o_item | q -> feature-attn output
constexpr int KV_OFF = XB_OFF + RT * 384;    // bf16 [RT][384] k|v (48 chunks/row); first [RT][192]: MLP hidden chunk
constexpr int HB_OFF = KV_OFF;
constexpr int NSLOT = 3;                     // weight ring depth
constexpr int WS_OFF = KV_OFF + RT * 768;    // bf16 NSLOT x [192][64] weight chunks
constexpr int WS_ELEMS = 192 * 64;
constexpr int LNP_OFF = WS_OFF + NSLOT * WS_ELEMS * 2;  // float [6][192] ln2 g,b | ln3 g,b | ln1 g,b
constexpr int RED_OFF = LNP_OFF + 6 * 192 * 4;          // float [RT][4] LayerNorm partials
constexpr int SMEM_BYTES = RED_OFF + RT * 4 * 4;
constexpr int TT = RT / 2 / 16;              // 16-token tiles per wave (waves: 4 along features x 2 along tokens)
constexpr int GLDS_PER_CHUNK = 3;            // 16-B LDS-DMA instructions per thread per weight chunk

// LDS-only workgroup barrier (no vmcnt drain: LDS-DMA stays in flight across it)
__device__ __forceinline__ void bar() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// 16 bytes global -> LDS per lane; lds_dst is the wave-uniform byte address of lane 0's slot
__device__ __forceinline__ void glds16(const void* gsrc, uint32_t lds_dst) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(gsrc), "s"(lds_dst)
               : "memory");
}

// element offset of 16-byte chunk `ch` of row `row` in a swizzled [rows][cpr*8] bf16 image (cpr % 8 == 0)
__device__ __forceinline__ int swz(int row, int ch, int cpr) { return (row * cpr + (ch ^ (row & 7))) * 8; }

__device__ __forceinline__ int feat_of(int wn, int nt, int lane) { return wn * 48 + nt * 16 + (lane >> 4) * 4; }
__device__ __forceinline__ int tok_of(int wt, int tt, int lane) { return wt * (RT / 2) + tt * 16 + (lane & 15); }

typedef f32x4 Acc[3][TT];

__device__ __forceinline__ void zero(Acc& a) {
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < TT; ++j) a[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
}

__device__ __forceinline__ void store_bf4(bf16_t* img, int t, int n0, int cpr, const f32x4& v) {
  uint2 pk;
  pk.x = pack_bf2(v[0], v[1]);
  pk.y = pack_bf2(v[2], v[3]);
  *reinterpret_cast<uint2*>(img + swz(t, n0 >> 3, cpr) + (n0 & 7)) = pk;
}

// The GEMM chain of one tile.  g indexes:
//   0          Wo_i                      (post)   X = item-attention output
//   1 + 2c     W1 rows [192c, 192c+192)  (post)   X = x
//   2 + 2c     W2 cols [192c, 192c+192)  (post)   X = GELU hidden chunk c
//   9, 10, 11  Wqkv_f rows k | v | q     (pre)    X = x
//   12         Wo_f                      (pre)    X = feature-attention output
//   13..15     Wq_i (rows q | k | v)     (pre)    X = x
struct Chain {
  const RowLayerParams& P;
  __device__ __forceinline__ void weight(int g, const bf16_t*& base, int& ld, int& col0) const {
    col0 = 0;
    ld = 192;
    if (g == 0) base = P.wo_i;
    else if (g <= 8) {
      const int c = (g - 1) >> 1;
      if (g & 1) { base = P.w1 + (int64_t)c * 192 * 192; }
      else { base = P.w2; ld = P.dff; col0 = c * 192; }
    } else if (g <= 11) base = P.wqkv_f + (int64_t)(g == 11 ? 0 : g - 8) * 192 * 192;
    else if (g == 12) base = P.wo_f;
    else base = P.wq_i + (int64_t)(g - 13) * 192 * 192;
  }
};

// issue chunk i of the weight stream (GEMM g_first + i/3, K columns 64*(i%3)...) into ring
// slot i % NSLOT.  Each wave instruction fills 1 KB = 8 rows of the [192][64] slot image
// lane-linearly; LDS unit cs of row n holds global unit cs ^ (n & 7) (the swz() image).
__device__ __forceinline__ void chunk_issue(const Chain& ch, int i, int g_first, uint32_t ws_lds) {
  const int g = g_first + i / 3, kc = i - (i / 3) * 3;
  const bf16_t* base;
  int ld, col0;
  ch.weight(g, base, ld, col0);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint32_t slot_lds = ws_lds + (uint32_t)((i % NSLOT) * WS_ELEMS * 2);
#pragma unroll
  for (int p = 0; p < GLDS_PER_CHUNK; ++p) {
    const int q0 = wave * 64 + p * 512;
    const int q = q0 + lane;
    const int n = q >> 3, cs = q & 7;
    glds16(base + (int64_t)n * ld + col0 + kc * 64 + ((cs ^ (n & 7)) << 3),
           __builtin_amdgcn_readfirstlane(slot_lds + (uint32_t)q0 * 16u));
  }
}

// acc += W_chunk(buf) * X[:, 64kc .. 64kc+64]^T
__device__ __forceinline__ void chunk_mfma(const char* smem, int buf, int kc, int x_off, int x_cpr, Acc& acc) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wn = wave & 3, wt = wave >> 2;
  const bf16_t* wb = reinterpret_cast<const bf16_t*>(smem + WS_OFF) + buf * WS_ELEMS;
  const bf16_t* xb = reinterpret_cast<const bf16_t*>(smem + x_off);
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) {
    bf16x8 a[3], b[TT];
#pragma unroll
    for (int nt = 0; nt < 3; ++nt) {
      const int n = wn * 48 + nt * 16 + (lane & 15);
      a[nt] = *reinterpret_cast<const bf16x8*>(wb + swz(n, kk * 4 + (lane >> 4), 8));
    }
#pragma unroll
    for (int tt = 0; tt < TT; ++tt) {
      const int t = tok_of(wt, tt, lane);
      b[tt] = *reinterpret_cast<const bf16x8*>(xb + swz(t, kc * 8 + kk * 4 + (lane >> 4), x_cpr));
    }
#pragma unroll
    for (int nt = 0; nt < 3; ++nt)
#pragma unroll
      for (int tt = 0; tt < TT; ++tt)
        acc[nt][tt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[nt], b[tt], acc[nt][tt], 0, 0, 0);
  }
}

// x = LN(x + acc) * g + b over the 192 features of each token; XB = bf16(x).
__device__ void ln_epilogue(char* smem, const Acc& acc, Acc& x, int which) {
  const float* g = reinterpret_cast<const float*>(smem + LNP_OFF) + which * 384;
  const float* bta = g + 192;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wn = wave & 3, wt = wave >> 2;
  float* red = reinterpret_cast<float*>(smem + RED_OFF);
  float s[TT];
#pragma unroll
  for (int tt = 0; tt < TT; ++tt) {
    s[tt] = 0.f;
#pragma unroll
    for (int nt = 0; nt < 3; ++nt) {
      x[nt][tt] += acc[nt][tt];
      s[tt] += x[nt][tt][0] + x[nt][tt][1] + x[nt][tt][2] + x[nt][tt][3];
    }
    s[tt] += __shfl_xor(s[tt], 16, 64);
    s[tt] += __shfl_xor(s[tt], 32, 64);
  }
  if (lane < 16) {
#pragma unroll
    for (int tt = 0; tt < TT; ++tt) red[tok_of(wt, tt, lane) * 4 + wn] = s[tt];
  }
  bar();
  float mean[TT];
#pragma unroll
  for (int tt = 0; tt < TT; ++tt) {
    const float* rr = red + tok_of(wt, tt, lane) * 4;
    mean[tt] = (rr[0] + rr[1] + rr[2] + rr[3]) * (1.0f / 192.0f);
  }
  bar();
#pragma unroll
  for (int tt = 0; tt < TT; ++tt) {
    s[tt] = 0.f;
#pragma unroll
    for (int nt = 0; nt < 3; ++nt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float d = x[nt][tt][r] - mean[tt];
        s[tt] += d * d;
      }
    s[tt] += __shfl_xor(s[tt], 16, 64);
    s[tt] += __shfl_xor(s[tt], 32, 64);
  }
  if (lane < 16) {
#pragma unroll
    for (int tt = 0; tt < TT; ++tt) red[tok_of(wt, tt, lane) * 4 + wn] = s[tt];
  }
  bar();
  bf16_t* xb = reinterpret_cast<bf16_t*>(smem + XB_OFF);
#pragma unroll
  for (int tt = 0; tt < TT; ++tt) {
    const float* rr = red + tok_of(wt, tt, lane) * 4;
    const float var = (rr[0] + rr[1] + rr[2] + rr[3]) * (1.0f / 192.0f);
    const float rstd = 1.0f / sqrtf(var + 1e-5f);
    const int t = tok_of(wt, tt, lane);
#pragma unroll
    for (int nt = 0; nt < 3; ++nt) {
      const int n0 = feat_of(wn, nt, lane);
      const f32x4 gg = *reinterpret_cast<const f32x4*>(g + n0);
      const f32x4 bb = *reinterpret_cast<const f32x4*>(bta + n0);
#pragma unroll
      for (int r = 0; r < 4; ++r) x[nt][tt][r] = (x[nt][tt][r] - mean[tt]) * rstd * gg[r] + bb[r];
      store_bf4(xb, t, n0, 24, x[nt][tt]);
    }
  }
  // no trailing barrier: the next weight chunk opens with one before XB is read
}

// Feature attention of the tile's rows: a lane pair per (token, head), 16 dims each
// (one xor-1 exchange per key); q in XB, k|v in KV, output written over the lane's own q.
__device__ void feature_attention(char* smem, int ntok, int C) {
  const bf16_t* kv = reinterpret_cast<const bf16_t*>(smem + KV_OFF);
  bf16_t* ob = reinterpret_cast<bf16_t*>(smem + XB_OFF);
  const float scale = 0.17677669529663687f;  // 1/sqrt(32)
  for (int pidx = threadIdx.x; pidx < RT * 12; pidx += 512) {
    const int half = pidx & 1;
    const int th = pidx >> 1;
    const int t = th / 6, h = th - t * 6;
    const int c0 = h * 4 + half * 2;  // first of this lane's two 16-byte chunks within a 192-wide block
    float o[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) o[j] = 0.f;
    const bool active = t < ntok;
    float q[16];
#pragma unroll
    for (int c2 = 0; c2 < 2; ++c2) {
      const bf16x8 v = *reinterpret_cast<const bf16x8*>(ob + swz(t, c0 + c2, 24));
#pragma unroll
      for (int j = 0; j < 8; ++j) q[c2 * 8 + j] = bf2f((bf16_t)v[j]) * scale;
    }
    const int base = active ? (t / C) * C : 0;
    const int nk = active ? C : 0;
    float m = -INFINITY, l = 0.f;
    for (int kj = 0; kj < C; ++kj) {
      const int kt = base + (kj < nk ? kj : 0);
      float sc = 0.f;
#pragma unroll
      for (int c2 = 0; c2 < 2; ++c2) {
        const bf16x8 v = *reinterpret_cast<const bf16x8*>(kv + swz(kt, c0 + c2, 48));
#pragma unroll
        for (int j = 0; j < 8; ++j) sc += q[c2 * 8 + j] * bf2f((bf16_t)v[j]);
      }
      sc += __shfl_xor(sc, 1, 64);
      const float mn = fmaxf(m, sc);
      const float alpha = __expf(m - mn);
      const float pp = __expf(sc - mn);
      l = l * alpha + pp;
#pragma unroll
      for (int c2 = 0; c2 < 2; ++c2) {
        const bf16x8 v = *reinterpret_cast<const bf16x8*>(kv + swz(kt, 24 + c0 + c2, 48));
#pragma unroll
        for (int j = 0; j < 8; ++j) o[c2 * 8 + j] = o[c2 * 8 + j] * alpha + pp * bf2f((bf16_t)v[j]);
      }
      m = mn;
    }
    const float inv = active ? 1.0f / l : 0.f;
#pragma unroll
    for (int c2 = 0; c2 < 2; ++c2) {
      uint4 pk;
      pk.x = pack_bf2(o[c2 * 8 + 0] * inv, o[c2 * 8 + 1] * inv);
      pk.y = pack_bf2(o[c2 * 8 + 2] * inv, o[c2 * 8 + 3] * inv);
      pk.z = pack_bf2(o[c2 * 8 + 4] * inv, o[c2 * 8 + 5] * inv);
      pk.w = pack_bf2(o[c2 * 8 + 6] * inv, o[c2 * 8 + 7] * inv);
      *reinterpret_cast<uint4*>(ob + swz(t, c0 + c2, 24)) = pk;
    }
  }
}

}  // namespace

__global__ __launch_bounds__(512, 1) void k_row_layer(RowLayerParams P) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wn = wave & 3, wt = wave >> 2;
  const int C = P.C;
  const int64_t row0 = (int64_t)blockIdx.x * P.rpt;
  const int nrows = (int)min((int64_t)P.rpt, P.rows - row0);
  const int ntok = nrows * C;
  const int64_t tok0 = row0 * C;
  bf16_t* xb = reinterpret_cast<bf16_t*>(smem + XB_OFF);
  bf16_t* hb = reinterpret_cast<bf16_t*>(smem + HB_OFF);
  bf16_t* kvb = reinterpret_cast<bf16_t*>(smem + KV_OFF);
  const uint32_t ws_lds = (uint32_t)(uintptr_t)(smem + WS_OFF);  // LDS byte address (low half of the flat address)
  const Chain chain{P};
  const int g_first = P.do_post ? 0 : 9;
  const int g_last = P.do_pre ? (P.out_qkv ? 15 : 13) : 8;
  const int nchunks = 3 * (g_last - g_first + 1);

  // diagnostic phase clock (build with -DNPFN_ROWK_STAMPS; wave 0's view): 0 prologue, 1 MFMA bodies, 2 LayerNorm, 3 GELU,
  // 4 k/v/q stores, 5 feature attention, 6 global outputs, 7 DMA wait + barrier
#ifdef NPFN_ROWK_STAMPS
  unsigned long long ph[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  unsigned long long tprev = P.stamps ? __builtin_amdgcn_s_memtime() : 0ull;
#define MARK(k)                                                   \
  if (P.stamps) {                                                 \
    const unsigned long long now_ = __builtin_amdgcn_s_memtime(); \
    ph[k] += now_ - tprev;                                        \
    tprev = now_;                                                 \
  }
#else
#define MARK(k)
#endif
  // the first two weight chunks are in flight while the tile's activations arrive
  chunk_issue(chain, 0, g_first, ws_lds);
  chunk_issue(chain, 1, g_first, ws_lds);

  {  // LayerNorm parameters of this launch -> LDS (1152 floats)
    float* lnp = reinterpret_cast<float*>(smem + LNP_OFF);
    if (tid < 288) {
      const int a = tid / 48, o = (tid - a * 48) * 4;
      const float* src = a == 0 ? P.ln2g : a == 1 ? P.ln2b : a == 2 ? P.ln3g : a == 3 ? P.ln3b : a == 4 ? P.ln1g : P.ln1b;
      f32x4 v = f32x4{0.f, 0.f, 0.f, 0.f};
      if (src) v = *reinterpret_cast<const f32x4*>(src + o);
      *reinterpret_cast<f32x4*>(lnp + a * 192 + o) = v;
    }
  }
  Acc x;
#pragma unroll
  for (int tt = 0; tt < TT; ++tt) {
    const int t = tok_of(wt, tt, lane);
#pragma unroll
    for (int nt = 0; nt < 3; ++nt) {
      const int n0 = feat_of(wn, nt, lane);
      x[nt][tt] = (t < ntok) ? *reinterpret_cast<const f32x4*>(P.resid + (tok0 + t) * 192 + n0)
                             : f32x4{0.f, 0.f, 0.f, 0.f};
    }
  }
  if (P.do_post) {
    for (int q = tid; q < RT * 24; q += 512) {
      const int t = q / 24, c = q - t * 24;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (t < ntok) v = *reinterpret_cast<const uint4*>(P.o_item + (tok0 + t) * 192 + c * 8);
      *reinterpret_cast<uint4*>(xb + swz(t, c, 24)) = v;
    }
  } else {
#pragma unroll
    for (int tt = 0; tt < TT; ++tt)
#pragma unroll
      for (int nt = 0; nt < 3; ++nt) store_bf4(xb, tok_of(wt, tt, lane), feat_of(wn, nt, lane), 24, x[nt][tt]);
  }
  MARK(0);

  Acc acc, acc2;
  for (int g = g_first; g <= g_last; ++g) {
    const bool w2 = (g >= 2 && g <= 8 && (g & 1) == 0);
    const int x_off = w2 ? HB_OFF : XB_OFF;
    if (g == 2) zero(acc2);
    if (!w2) zero(acc);
#pragma unroll 1
    for (int kc = 0; kc < 3; ++kc) {
      const int i = 3 * (g - g_first) + kc;
      // chunk i landed (own DMA: everything but the GLDS_PER_CHUNK of chunk i+1), then everyone's
      if (i + 1 < nchunks) asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      bar();
      MARK(7);
      // slot (i+2) % 3 == (i-1) % 3: every wave finished reading it before this barrier
      if (i + 2 < nchunks) chunk_issue(chain, i + 2, g_first, ws_lds);
      if (w2) chunk_mfma(smem, i % NSLOT, kc, x_off, 24, acc2);
      else chunk_mfma(smem, i % NSLOT, kc, x_off, 24, acc);
      MARK(1);
    }

    // ---- epilogue of GEMM g (two chunks of the stream stay in flight)
    if (g == 0) {
      ln_epilogue(smem, acc, x, 0);
      MARK(2);
    } else if (g <= 8 && (g & 1)) {
      // HB was last read by GEMM g-1, which every wave finished before this GEMM's first barrier
#pragma unroll
      for (int tt = 0; tt < TT; ++tt)
#pragma unroll
        for (int nt = 0; nt < 3; ++nt) {
          f32x4 v = acc[nt][tt];
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = gelu_fast(v[r]);
          store_bf4(hb, tok_of(wt, tt, lane), feat_of(wn, nt, lane), 24, v);
        }
      MARK(3);
    } else if (g < 8) {
      // W2 partial products accumulate in acc2; nothing to do
    } else if (g == 8) {
      ln_epilogue(smem, acc2, x, 1);
      MARK(2);
      if (!P.do_pre) {  // last layer: bf16 x for the decoder
        bar();
        for (int q = tid; q < RT * 24; q += 512) {
          const int t = q / 24, c = q - t * 24;
          if (t < ntok)
            *reinterpret_cast<uint4*>(P.out + (tok0 + t) * 192 + c * 8) =
                *reinterpret_cast<const uint4*>(xb + swz(t, c, 24));
        }
        MARK(6);
      }
    } else if (g == 9 || g == 10) {  // k | v -> KV (its HB part was last read by GEMM 8)
#pragma unroll
      for (int tt = 0; tt < TT; ++tt)
#pragma unroll
        for (int nt = 0; nt < 3; ++nt)
          store_bf4(kvb, tok_of(wt, tt, lane), (g - 9) * 192 + feat_of(wn, nt, lane), 48, acc[nt][tt]);
      MARK(4);
    } else if (g == 11) {  // q -> XB once every wave has finished reading x from it
      bar();
#pragma unroll
      for (int tt = 0; tt < TT; ++tt)
#pragma unroll
        for (int nt = 0; nt < 3; ++nt) store_bf4(xb, tok_of(wt, tt, lane), feat_of(wn, nt, lane), 24, acc[nt][tt]);
      bar();
      MARK(4);
      feature_attention(smem, ntok, C);
      MARK(5);
    } else if (g == 12) {
      ln_epilogue(smem, acc, x, 2);
      MARK(2);
#pragma unroll
      for (int tt = 0; tt < TT; ++tt) {
        const int t = tok_of(wt, tt, lane);
        if (t >= ntok) continue;
#pragma unroll
        for (int nt = 0; nt < 3; ++nt)
          *reinterpret_cast<f32x4*>(P.resid + (tok0 + t) * 192 + feat_of(wn, nt, lane)) = x[nt][tt];
      }
      MARK(6);
    } else {  // g >= 13: next layer's item-attention q (test) or q|k|v (train)
      const int ld = P.out_qkv ? 576 : 192;
      const int col0 = (g - 13) * 192;
#pragma unroll
      for (int tt = 0; tt < TT; ++tt) {
        const int t = tok_of(wt, tt, lane);
        if (t >= ntok) continue;
#pragma unroll
        for (int nt = 0; nt < 3; ++nt) {
          uint2 pk;
          pk.x = pack_bf2(acc[nt][tt][0], acc[nt][tt][1]);
          pk.y = pack_bf2(acc[nt][tt][2], acc[nt][tt][3]);
          *reinterpret_cast<uint2*>(P.out + (tok0 + t) * ld + col0 + feat_of(wn, nt, lane)) = pk;
        }
      }
      MARK(6);
    }
  }
#ifdef NPFN_ROWK_STAMPS
  if (P.stamps && tid == 0) {
#pragma unroll
    for (int k = 0; k < 8; ++k) atomicAdd(&P.stamps[k], ph[k]);
    atomicAdd(&P.stamps[15], 1ull);
  }
#endif
#undef MARK
}

static_assert(SMEM_BYTES <= 160 * 1024, "LDS budget");

void rowk_setup() {
  (void)hipFuncSetAttribute((const void*)k_row_layer, hipFuncAttributeMaxDynamicSharedMemorySize, SMEM_BYTES);
}

int rowk_rows_per_tile(int C) { return RT / C; }

void launch_row_layer(const RowLayerParams& p, hipStream_t s) {
  const int64_t tiles = (p.rows + p.rpt - 1) / p.rpt;
  hipLaunchKernelGGL(k_row_layer, dim3((unsigned)tiles), dim3(512), SMEM_BYTES, s, p);
}

}  // namespace npfn
