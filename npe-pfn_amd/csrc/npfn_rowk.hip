// npfn_rowk.hip -- fused row-tile layer kernel (everything of a PerFeatureEncoderLayer
// except the item attention, which needs other rows).
//
// One workgroup (8 waves) owns a tile of whole rows (rpt rows x C tokens <= 128
// tokens).  The fp32 residual stream of the tile stays in registers and its bf16
// copy in LDS across the chain
//
//   [post of layer l]  x = LN2(x + o_item Wo_i^T); h_c = GELU(x W1_c^T) (4 chunks of
//                      192 hidden units in LDS); x = LN3(x + sum_c h_c W2_c^T)
//   [pre of layer l+1] qkv = x Wqkv_f^T (LDS, all heads); feature attention over the
//                      row's C tokens, one thread per (token, head) -> o (LDS);
//                      x = LN1(x + o Wo_f^T); out = x Wq_i^T (test) or x Wqkv_i^T (train)
//
// so HBM sees only the item-attention output, the residual and the next queries
// (~3 KB per token and layer instead of ~14 KB for per-sublayer kernels).
// Every GEMM of the chain is 192 output features x 192 inputs, streamed as three
// [192][64] weight chunks through a double-buffered LDS stage shared by the 8
// waves; the load of the next chunk -- also across GEMM boundaries -- is issued
// before the current chunk's MFMAs, so epilogues overlap the weight stream.
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
constexpr int XB_OFF = 0;                    // bf16 [RT][192] x (24 chunks/row); also the feature-attention output
constexpr int QKV_OFF = XB_OFF + RT * 384;   // bf16 [RT][576] q|k|v (72 chunks/row); first [RT][192]: MLP hidden chunk
constexpr int HB_OFF = QKV_OFF;
constexpr int WS_OFF = QKV_OFF + RT * 1152;  // bf16 2 x [192][64] weight chunks
constexpr int WS_ELEMS = 192 * 64;
constexpr int RED_OFF = WS_OFF + 2 * WS_ELEMS * 2;  // float [RT][4] LayerNorm partials
constexpr int SMEM_BYTES = RED_OFF + RT * 4 * 4;
constexpr int TT = RT / 2 / 16;              // 16-token tiles per wave (waves: 4 along features x 2 along tokens)

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
//   9, 10, 11  Wqkv_f rows q | k | v     (pre)    X = x
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
    } else if (g <= 11) base = P.wqkv_f + (int64_t)(g - 9) * 192 * 192;
    else if (g == 12) base = P.wo_f;
    else base = P.wq_i + (int64_t)(g - 13) * 192 * 192;
  }
};

// chunk (g, kc) of the weight stream: [192][64] -> 3 uint4 per thread
__device__ __forceinline__ void chunk_load(const Chain& ch, int g, int kc, uint4 (&st)[3]) {
  const bf16_t* base;
  int ld, col0;
  ch.weight(g, base, ld, col0);
#pragma unroll
  for (int p = 0; p < 3; ++p) {
    const int q = threadIdx.x + p * 512;
    const int n = q >> 3, c = q & 7;
    st[p] = *reinterpret_cast<const uint4*>(base + (int64_t)n * ld + col0 + kc * 64 + c * 8);
  }
}
__device__ __forceinline__ void chunk_store(char* smem, int buf, const uint4 (&st)[3]) {
  bf16_t* d = reinterpret_cast<bf16_t*>(smem + WS_OFF) + buf * WS_ELEMS;
#pragma unroll
  for (int p = 0; p < 3; ++p) {
    const int q = threadIdx.x + p * 512;
    const int n = q >> 3, c = q & 7;
    *reinterpret_cast<uint4*>(d + swz(n, c, 8)) = st[p];
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
__device__ void ln_epilogue(char* smem, const Acc& acc, Acc& x, const float* __restrict__ g,
                            const float* __restrict__ bta) {
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
  __syncthreads();
  float mean[TT];
#pragma unroll
  for (int tt = 0; tt < TT; ++tt) {
    const float* rr = red + tok_of(wt, tt, lane) * 4;
    mean[tt] = (rr[0] + rr[1] + rr[2] + rr[3]) * (1.0f / 192.0f);
  }
  __syncthreads();
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
  __syncthreads();
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
#pragma unroll
      for (int r = 0; r < 4; ++r) x[nt][tt][r] = (x[nt][tt][r] - mean[tt]) * rstd * g[n0 + r] + bta[n0 + r];
      store_bf4(xb, t, n0, 24, x[nt][tt]);
    }
  }
  __syncthreads();
}

// Feature attention of the tile's rows: a lane pair per (token, head), 16 dims each
// (one xor-1 exchange per key); q|k|v in QKV, output into XB.
__device__ void feature_attention(char* smem, int ntok, int C) {
  const bf16_t* qkv = reinterpret_cast<const bf16_t*>(smem + QKV_OFF);
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
      const bf16x8 v = *reinterpret_cast<const bf16x8*>(qkv + swz(t, c0 + c2, 72));
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
        const bf16x8 v = *reinterpret_cast<const bf16x8*>(qkv + swz(kt, 24 + c0 + c2, 72));
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
        const bf16x8 v = *reinterpret_cast<const bf16x8*>(qkv + swz(kt, 48 + c0 + c2, 72));
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
  const Chain chain{P};
  const int g_first = P.do_post ? 0 : 9;
  const int g_last = P.do_pre ? (P.out_qkv ? 15 : 13) : 8;

  // first weight chunk in flight while the tile's activations arrive
  uint4 st[3];
  chunk_load(chain, g_first, 0, st);

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
  chunk_store(smem, 0, st);
  __syncthreads();

  Acc acc, acc2;
  bf16_t* hb = reinterpret_cast<bf16_t*>(smem + HB_OFF);
  bf16_t* qkv = reinterpret_cast<bf16_t*>(smem + QKV_OFF);
  int buf = 0;
  for (int g = g_first; g <= g_last; ++g) {
    const bool w2 = (g >= 2 && g <= 8 && (g & 1) == 0);
    const int x_off = w2 ? HB_OFF : XB_OFF;
    if (g == 2) zero(acc2);
    if (!w2) zero(acc);
#pragma unroll 1
    for (int kc = 0; kc < 3; ++kc) {
      // next chunk of the stream (past the end: re-stage the current one, unused)
      int gn = (kc < 2) ? g : g + 1;
      int kn = (kc < 2) ? kc + 1 : 0;
      if (gn > g_last) { gn = g; kn = kc; }
      chunk_load(chain, gn, kn, st);
      if (w2) chunk_mfma(smem, buf, kc, x_off, 24, acc2);
      else chunk_mfma(smem, buf, kc, x_off, 24, acc);
      chunk_store(smem, buf ^ 1, st);
      __syncthreads();
      buf ^= 1;
    }
    // ---- epilogue of GEMM g (the next GEMM's first chunk is already staged)
    if (g == 0) {
      ln_epilogue(smem, acc, x, P.ln2g, P.ln2b);
    } else if (g <= 8 && (g & 1)) {
#pragma unroll
      for (int tt = 0; tt < TT; ++tt)
#pragma unroll
        for (int nt = 0; nt < 3; ++nt) {
          f32x4 v = acc[nt][tt];
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = gelu_f(v[r]);
          store_bf4(hb, tok_of(wt, tt, lane), feat_of(wn, nt, lane), 24, v);
        }
      __syncthreads();
    } else if (g < 8) {
      // W2 partial products accumulate in acc2; nothing to do
    } else if (g == 8) {
      ln_epilogue(smem, acc2, x, P.ln3g, P.ln3b);
      if (!P.do_pre) {  // last layer: bf16 x for the decoder
        for (int q = tid; q < RT * 24; q += 512) {
          const int t = q / 24, c = q - t * 24;
          if (t < ntok)
            *reinterpret_cast<uint4*>(P.out + (tok0 + t) * 192 + c * 8) =
                *reinterpret_cast<const uint4*>(xb + swz(t, c, 24));
        }
      }
    } else if (g >= 9 && g <= 11) {
#pragma unroll
      for (int tt = 0; tt < TT; ++tt)
#pragma unroll
        for (int nt = 0; nt < 3; ++nt)
          store_bf4(qkv, tok_of(wt, tt, lane), (g - 9) * 192 + feat_of(wn, nt, lane), 72, acc[nt][tt]);
      if (g == 11) {
        __syncthreads();
        feature_attention(smem, ntok, C);
        __syncthreads();
      }
    } else if (g == 12) {
      ln_epilogue(smem, acc, x, P.ln1g, P.ln1b);
#pragma unroll
      for (int tt = 0; tt < TT; ++tt) {
        const int t = tok_of(wt, tt, lane);
        if (t >= ntok) continue;
#pragma unroll
        for (int nt = 0; nt < 3; ++nt)
          *reinterpret_cast<f32x4*>(P.resid + (tok0 + t) * 192 + feat_of(wn, nt, lane)) = x[nt][tt];
      }
    } else if (g >= 13) {
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
    }
  }
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
