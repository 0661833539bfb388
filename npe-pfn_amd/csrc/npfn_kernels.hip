// npfn_kernels.hip -- gfx950 kernels of the NPE-PFN engine.
//
// Hot path (SURVEY.md §2 "Native components", §8a rows a5-a10):
//   K1 encoder (k_encode), K2 feature attention (k_feat_attn), K3/K4 item
//   attention (k_item_attn, flash-style on MFMA 32x32x16 bf16), K5 projections
//   + MLP + residual/LayerNorm (k_gemm<EPI>, MFMA 16x16x32 bf16), K6 decoder
//   head (k_gemm) + ensemble mix (k_mix*), K7 bar sample, K8 bar NLL.
// The CPU restatement of every kernel is oracle/tabpfn_oracle.py.
#include <algorithm>
#include <type_traits>

#include <mutex>

#include <rocblas/rocblas.h>
#include <rocsolver/rocsolver.h>

#include "npfn_common.h"
#include "npfn_kernels.h"

namespace npfn {

// ============================================================ fit statistics
// One block per column of X (and one for y).  Oracle: OracleTabPFN.fit.
__global__ __launch_bounds__(256) void k_col_stats(const float* __restrict__ X, int64_t ldx,
                                                   const float* __restrict__ y, int64_t ldy,
                                                   int64_t n, int F, float* __restrict__ colstat,
                                                   float* __restrict__ ystats) {
  __shared__ double red[2][4];
  __shared__ float redf[2][4];
  const int j = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  auto block_sum2 = [&](double a, double b, double& ra, double& rb) {
    a = wave_sum_d(a);
    b = wave_sum_d(b);
    __syncthreads();
    if (lane == 0) { red[0][w] = a; red[1][w] = b; }
    __syncthreads();
    ra = red[0][0] + red[0][1] + red[0][2] + red[0][3];
    rb = red[1][0] + red[1][1] + red[1][2] + red[1][3];
  };
  if (j < F) {
    double s = 0.0, c = 0.0;
    float mn = INFINITY, mx = -INFINITY;
    for (int64_t i = tid; i < n; i += 256) {
      float v = X[i * ldx + j];
      if (isfinite(v)) { s += v; c += 1.0; mn = fminf(mn, v); mx = fmaxf(mx, v); }
    }
    double S, Cn;
    block_sum2(s, c, S, Cn);
    double mean = S / fmax(Cn, 1.0);
    double q = 0.0;
    for (int64_t i = tid; i < n; i += 256) {
      float v = X[i * ldx + j];
      if (isfinite(v)) { double dv = (double)v - mean; q += dv * dv; }
    }
    double Q, dummy;
    block_sum2(q, 0.0, Q, dummy);
    // min / max
    for (int o = 32; o > 0; o >>= 1) {
      mn = fminf(mn, __shfl_xor(mn, o, 64));
      mx = fmaxf(mx, __shfl_xor(mx, o, 64));
    }
    __syncthreads();
    if (lane == 0) { redf[0][w] = mn; redf[1][w] = mx; }
    __syncthreads();
    if (tid == 0) {
      float MN = fminf(fminf(redf[0][0], redf[0][1]), fminf(redf[0][2], redf[0][3]));
      float MX = fmaxf(fmaxf(redf[1][0], redf[1][1]), fmaxf(redf[1][2], redf[1][3]));
      colstat[3 * j + 0] = (float)mean;
      colstat[3 * j + 1] = (float)sqrt(Q / fmax(Cn - 1.0, 1.0));
      colstat[3 * j + 2] = (MX > MN) ? 1.0f : 0.0f;
    }
  } else {
    double s = 0.0;
    for (int64_t i = tid; i < n; i += 256) s += (double)y[i * ldy];
    double S, dummy;
    block_sum2(s, 0.0, S, dummy);
    double mean = S / (double)n;
    double q = 0.0;
    for (int64_t i = tid; i < n; i += 256) { double dv = (double)y[i * ldy] - mean; q += dv * dv; }
    double Q;
    block_sum2(q, 0.0, Q, dummy);
    const float ym = (float)mean;
    const float ys = (float)(sqrt(Q / (double)n) + 1e-20);
    double z = 0.0;
    for (int64_t i = tid; i < n; i += 256) z += (double)((y[i * ldy] - ym) / ys);
    double Z;
    block_sum2(z, 0.0, Z, dummy);
    if (tid == 0) {
      ystats[0] = ym;
      ystats[1] = ys;
      ystats[2] = (float)(Z / (double)n);
    }
  }
}

// ======================================================= K0 quantile preprocessing
// sklearn QuantileTransformer(output_distribution="uniform", n_quantiles=max(n//5, 2))
// restated in oracle/preprocess_oracle.py (pinned against sklearn 1.7.2):
// fit = nanpercentile at linspace(0,1,nq) + running max; transform = the two-sided
// np.interp average with x==q[0] -> 0, x==q[-1] -> 1.  All in float64, as numpy.
__host__ __device__ int quantile_count(int64_t n, int div) {
  int64_t q = n / div > 2 ? n / div : 2;
  q = q < n ? q : n;
  return (int)(q > 1 ? q : 1);
}
__device__ __forceinline__ double qt_ref(int i, int nq) {
  if (nq == 1) return 0.0;
  if (i == nq - 1) return 1.0;
  return (double)i * (1.0 / (double)(nq - 1));  // np.linspace: arange * step, last = stop
}
// np.interp(x, q, ref): j = last index with q[j] <= x
__device__ __forceinline__ double qt_interp_up(double x, const double* q, int nq) {
  if (x > q[nq - 1]) return qt_ref(nq - 1, nq);
  if (x < q[0]) return qt_ref(0, nq);
  int lo = 0, hi = nq;
  while (lo < hi) { const int m = (lo + hi) >> 1; if (q[m] <= x) lo = m + 1; else hi = m; }
  const int j = lo - 1;
  if (j == nq - 1 || q[j] == x) return qt_ref(j, nq);
  const double r0 = qt_ref(j, nq), r1 = qt_ref(j + 1, nq);
  return (r1 - r0) / (q[j + 1] - q[j]) * (x - q[j]) + r0;
}
// np.interp(-x, -q[::-1], -ref[::-1]): xp'[i] = -q[nq-1-i]; j' = #(q >= x) - 1, k = nq-1-j'
__device__ __forceinline__ double qt_interp_dn(double x, const double* q, int nq) {
  const double xn = -x;
  if (xn > -q[0]) return -qt_ref(0, nq);
  if (xn < -q[nq - 1]) return -qt_ref(nq - 1, nq);
  int lo = 0, hi = nq;  // first index with q[i] >= x
  while (lo < hi) { const int m = (lo + hi) >> 1; if (q[m] < x) lo = m + 1; else hi = m; }
  const int jp = nq - lo - 1, k = nq - 1 - jp;
  if (jp == nq - 1 || -q[k] == xn) return -qt_ref(k, nq);
  const double f0 = -qt_ref(k, nq), f1 = -qt_ref(k - 1, nq);
  const double x0 = -q[k], x1 = -q[k - 1];
  return (f1 - f0) / (x1 - x0) * (xn - x0) + f0;
}
__device__ __forceinline__ float qt_apply(float xf, const double* q, int nq) {
  const double x = (double)xf;
  double v = 0.5 * (qt_interp_up(x, q, nq) - qt_interp_dn(x, q, nq));
  if (x == q[nq - 1]) v = 1.0;
  if (x == q[0]) v = 0.0;
  return (float)v;
}

// sklearn's QuantileTransformer(subsample=10_000) fits on a row subsample when the context has
// more rows: resample(X, replace=False, n_samples=10_000, random_state=RandomState(seed)), i.e.
// indices = arange(n), RandomState.shuffle(indices), the first 10 000 (oracle
// preprocess_oracle.quantile_subsample, pinned to sklearn).  The percentiles are of the SET of
// those rows, so only the shuffle's steps i >= 10 000 matter (the later ones permute the
// first 10 000 among themselves).  One wave: MT19937 (numpy's legacy seeding, twist and
// tempering, random_interval's masked rejection), the Fisher-Yates swaps on a uint16 array in
// LDS (n <= 65 536), the first 10 000 entries out as row indices.
__global__ __launch_bounds__(64) void k_qt_subsample(int64_t n, uint32_t seed, int* __restrict__ idx) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  uint32_t* mt = reinterpret_cast<uint32_t*>(smem);          // [624] state
  uint32_t* tw = mt + 624;                                    // [624] tempered outputs of the state
  uint16_t* arr = reinterpret_cast<uint16_t*>(tw + 624);      // [n]
  const int lane = threadIdx.x;
  for (int64_t i = lane; i < n; i += 64) arr[i] = (uint16_t)i;
  if (lane == 0) {
    uint32_t v = seed;
    for (int i = 0; i < 624; ++i) {
      mt[i] = v;
      v = 1812433253u * (v ^ (v >> 30)) + (uint32_t)(i + 1);
    }
  }
  __syncthreads();
  auto step = [&](int kk, int src) -> uint32_t {
    const uint32_t y = (mt[kk] & 0x80000000u) | (mt[kk == 623 ? 0 : kk + 1] & 0x7fffffffu);
    return mt[src] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
  };
  auto twist = [&]() {  // genrand's three loops, 64 entries at a time (each chunk reads only settled entries)
    for (int k0 = 0; k0 < 227; k0 += 64) {
      const int kk = k0 + lane;
      uint32_t nv = 0;
      if (kk < 227) nv = step(kk, kk + 397);
      __syncthreads();
      if (kk < 227) mt[kk] = nv;
      __syncthreads();
    }
    for (int k0 = 227; k0 < 623; k0 += 64) {
      const int kk = k0 + lane;
      uint32_t nv = 0;
      if (kk < 623) nv = step(kk, kk - 227);
      __syncthreads();
      if (kk < 623) mt[kk] = nv;
      __syncthreads();
    }
    if (lane == 0) mt[623] = step(623, 396);
    __syncthreads();
    for (int i = lane; i < 624; i += 64) {
      uint32_t y = mt[i];
      y ^= y >> 11;
      y ^= (y << 7) & 0x9d2c5680u;
      y ^= (y << 15) & 0xefc60000u;
      y ^= y >> 18;
      tw[i] = y;
    }
    __syncthreads();
  };
  // the wave walks the shuffle in lockstep (lane 0 swaps); it refills the tempered block
  // whenever it is used up
  int pos = 624;
  for (int64_t i = n - 1; i >= kQtSubsample; --i) {
    uint32_t mask = (uint32_t)i;
    mask |= mask >> 1; mask |= mask >> 2; mask |= mask >> 4; mask |= mask >> 8; mask |= mask >> 16;
    uint32_t j;
    do {
      if (pos == 624) {
        twist();
        pos = 0;
      }
      j = tw[pos++] & mask;
    } while (j > (uint32_t)i);
    if (lane == 0) {
      const uint16_t t = arr[i];
      arr[i] = arr[j];
      arr[j] = t;
    }
  }
  __syncthreads();
  for (int t = lane; t < kQtSubsample; t += 64) idx[t] = (int)arr[t];
}

// One block per column: finite values -> LDS, bitonic sort, percentile table, then the
// statistics of the transformed train column (qstat [F][3] = mean, std ddof=1, used).  sub:
// the subsample's row indices (n > 10 000) or null (every row).  Dynamic LDS:
// max(QT_SORT_MAX floats, nq doubles) (launch_quantile_fit).
__global__ __launch_bounds__(256) void k_quantile_fit(const float* __restrict__ X, int64_t ldx, int64_t n, int F,
                                                      int div, int nqmax, const int* __restrict__ sub,
                                                      double* __restrict__ qtab, int* __restrict__ qn,
                                                      float* __restrict__ qstat) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* sv = reinterpret_cast<float*>(smem);  // [QT_SORT_MAX] values; then [nq] f64 quantiles
  __shared__ int cnt_s;
  __shared__ double red[2][4];
  __shared__ float redf[2][4];
  const int j = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  if (tid == 0) cnt_s = 0;
  __syncthreads();
  const int64_t nfit = sub ? (int64_t)kQtSubsample : n;
  for (int64_t i = tid; i < nfit; i += 256) {
    const float v = X[(sub ? (int64_t)sub[i] : i) * ldx + j];
    if (isfinite(v)) sv[atomicAdd(&cnt_s, 1)] = v;
  }
  __syncthreads();
  const int cnt = cnt_s;
  int P = 1;
  while (P < cnt) P <<= 1;
  for (int i = cnt + tid; i < P; i += 256) sv[i] = INFINITY;
  __syncthreads();
  for (int k = 2; k <= P; k <<= 1) {
    for (int jj = k >> 1; jj > 0; jj >>= 1) {
      for (int i = tid; i < P; i += 256) {
        const int ixj = i ^ jj;
        if (ixj > i) {
          const float a = sv[i], b = sv[ixj];
          if ((a > b) == ((i & k) == 0)) { sv[i] = b; sv[ixj] = a; }
        }
      }
      __syncthreads();
    }
  }
  const int nq = quantile_count(n, div);
  double* qt = qtab + (int64_t)j * nqmax;
  if (cnt == 0) {
    if (tid == 0) { qn[j] = 0; qstat[3 * j + 0] = 0.f; qstat[3 * j + 1] = 0.f; qstat[3 * j + 2] = 0.f; }
    return;
  }
  for (int i = tid; i < nq; i += 256) {
    const double pq = (qt_ref(i, nq) * 100.0) / 100.0;       // percentile(ref*100) / 100
    const double vi = (double)(cnt - 1) * pq;
    const double pf = floor(vi);
    const double g = vi - pf;
    const int i0 = (int)pf, i1 = min(i0 + 1, cnt - 1);
    const double a = (double)sv[i0], b = (double)sv[i1], dba = b - a;
    qt[i] = g >= 0.5 ? b - dba * (1.0 - g) : a + dba * g;   // numpy _lerp
  }
  __syncthreads();  // the sorted values are no longer read; qt is visible to the block
  double* qs = reinterpret_cast<double*>(smem);
  if (w == 0) {  // np.maximum.accumulate: per-lane segments, a wave scan of the segment maxima
    const int seg = (nq + 63) / 64, s0 = min(lane * seg, nq), s1 = min(s0 + seg, nq);
    double m = -INFINITY;
    for (int i = s0; i < s1; ++i) m = fmax(m, qt[i]);
    double carry = m;  // inclusive scan of the segment maxima
    for (int o = 1; o < 64; o <<= 1) {
      const double u = __shfl_up(carry, o, 64);
      if (lane >= o) carry = fmax(carry, u);
    }
    double run = __shfl_up(carry, 1, 64);
    if (lane == 0) run = -INFINITY;
    for (int i = s0; i < s1; ++i) {
      run = fmax(run, qt[i]);
      qs[i] = run;
    }
    if (lane == 0) qn[j] = nq;
  }
  __syncthreads();
  for (int i = tid; i < nq; i += 256) qt[i] = qs[i];
  // statistics of the transformed train column (oracle _fit_features on quantile estimators)
  double s = 0.0, c = 0.0;
  float mn = INFINITY, mx = -INFINITY;
  for (int64_t i = tid; i < n; i += 256) {
    const float v = X[i * ldx + j];
    if (isfinite(v)) { const float u = qt_apply(v, qs, nq); s += u; c += 1.0; mn = fminf(mn, u); mx = fmaxf(mx, u); }
  }
  s = wave_sum_d(s); c = wave_sum_d(c);
  if (lane == 0) { red[0][w] = s; red[1][w] = c; }
  __syncthreads();
  const double S = red[0][0] + red[0][1] + red[0][2] + red[0][3];
  const double Cn = red[1][0] + red[1][1] + red[1][2] + red[1][3];
  const double mean = S / fmax(Cn, 1.0);
  double q2 = 0.0;
  for (int64_t i = tid; i < n; i += 256) {
    const float v = X[i * ldx + j];
    if (isfinite(v)) { const double dv = (double)qt_apply(v, qs, nq) - mean; q2 += dv * dv; }
  }
  q2 = wave_sum_d(q2);
  for (int o = 32; o > 0; o >>= 1) {
    mn = fminf(mn, __shfl_xor(mn, o, 64));
    mx = fmaxf(mx, __shfl_xor(mx, o, 64));
  }
  __syncthreads();
  if (lane == 0) { red[0][w] = q2; redf[0][w] = mn; redf[1][w] = mx; }
  __syncthreads();
  if (tid == 0) {
    const double Q = red[0][0] + red[0][1] + red[0][2] + red[0][3];
    const float MN = fminf(fminf(redf[0][0], redf[0][1]), fminf(redf[0][2], redf[0][3]));
    const float MX = fmaxf(fmaxf(redf[1][0], redf[1][1]), fmaxf(redf[1][2], redf[1][3]));
    qstat[3 * j + 0] = (float)mean;
    qstat[3 * j + 1] = (float)sqrt(Q / fmax(Cn - 1.0, 1.0));
    qstat[3 * j + 2] = (MX > MN) ? 1.0f : 0.0f;
  }
}

// Yeo-Johnson power transform (sklearn PowerTransformer._yeo_johnson_transform), f64.
__device__ __forceinline__ double yj_apply(double x, double lam) {
  constexpr double eps = 2.220446049250313e-16;  // np.spacing(1.0)
  if (x >= 0.0) return fabs(lam) < eps ? log1p(x) : (pow(x + 1.0, lam) - 1.0) / lam;
  return fabs(lam - 2.0) > eps ? -(pow(-x + 1.0, 2.0 - lam) - 1.0) / (2.0 - lam) : -log1p(-x);
}

// One block per column: lambda = argmin of sklearn's Yeo-Johnson negative log-likelihood by
// the fixed search of oracle/preprocess_oracle.py yj_fit (grid -6:1:6, then 40 golden-section
// steps), then mean / std (ddof 1) / used of the float32-rounded transformed train column.
// 512 threads (two context values each at n = 1000): each of the 55 dependent evaluations is
// one f64 expm1 per value (log1p(|x|) hoisted out of the search) and one block reduction of
// (sum, sum of squares) -- the search is latency-bound and sits on the critical path of AR
// step 0's fit.
constexpr int PF_THREADS = 512, PF_WAVES = PF_THREADS / 64, PF_VPT = 4;
// Blocks 0 .. F-1 fit the columns of X; a block F (Y != null) fits the target column Y (the
// ensemble's target transform) in the same launch.
__global__ __launch_bounds__(PF_THREADS) void k_power_fit(const float* __restrict__ Xm, int64_t ldxm, int64_t n,
                                                          int F, double* __restrict__ plam, float* __restrict__ pstat,
                                                          const float* __restrict__ Y, int64_t ldy,
                                                          double* __restrict__ ylam, float* __restrict__ ypstat) {
  __shared__ float sv[QT_SORT_MAX];
  __shared__ double red[PF_WAVES];
  __shared__ double red2[2][PF_WAVES];
  __shared__ float redf[2][PF_WAVES];
  const bool target = (int)blockIdx.x >= F;
  const float* __restrict__ X = target ? Y : Xm + blockIdx.x;  // the block's column, stride ldx
  const int64_t ldx = target ? ldy : ldxm;
  if (target) {
    plam = ylam;
    pstat = ypstat;
  } else {
    plam += blockIdx.x;
    pstat += 3 * blockIdx.x;
  }
  constexpr int j = 0;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  // the column in row order (non-finite entries stay in place and are skipped), so every
  // thread's partial sums see the same values in the same order on every run
  // contexts of more than QT_SORT_MAX rows read the column from global memory (L2) instead
  const bool in_lds = n <= (int64_t)QT_SORT_MAX;
  auto col = [&](int64_t i) -> float { return in_lds ? sv[i] : X[i * ldx + j]; };
  float mn = INFINITY, mx = -INFINITY;
  int cl = 0;
  for (int64_t i = tid; i < n; i += PF_THREADS) {
    const float v = X[i * ldx + j];
    if (in_lds) sv[i] = v;
    if (isfinite(v)) { mn = fminf(mn, v); mx = fmaxf(mx, v); ++cl; }
  }
  auto wsum = [&](const double* r) {
    double t = 0.0;
#pragma unroll
    for (int q = 0; q < PF_WAVES; ++q) t += r[q];
    return t;
  };
  auto bsum = [&](double a) -> double {   // block sum, result in every thread
    a = wave_sum_d(a);
    __syncthreads();
    if (lane == 0) red[w] = a;
    __syncthreads();
    return wsum(red);
  };
  auto bminmax = [&](float& a, float& b) {
    for (int o = 32; o > 0; o >>= 1) { a = fminf(a, __shfl_xor(a, o, 64)); b = fmaxf(b, __shfl_xor(b, o, 64)); }
    __syncthreads();
    if (lane == 0) { redf[0][w] = a; redf[1][w] = b; }
    __syncthreads();
    a = redf[0][0];
    b = redf[1][0];
    for (int q = 1; q < PF_WAVES; ++q) { a = fminf(a, redf[0][q]); b = fmaxf(b, redf[1][q]); }
  };
  bminmax(mn, mx);
  const int cnt = (int)bsum((double)cl);
  double lam = 1.0;
  if (cnt > 0 && mx > mn) {
    double sl = 0.0;
    for (int64_t i = tid; i < n; i += PF_THREADS) {
      const float xf = col(i);
      if (isfinite(xf)) { const double x = xf; sl += (x > 0 ? 1.0 : (x < 0 ? -1.0 : 0.0)) * log1p(fabs(x)); }
    }
    const double S = bsum(sl);
    // sums shifted by the transform of the column minimum (robust to cancellation)
    const double x_shift = (double)mn;
    auto nll_of = [&](double l, double S1, double S2) -> double {
      const double var = fmax(S2 - S1 * S1 / (double)cnt, 0.0) / (double)cnt;
      if (!(var >= 2.2250738585072014e-308)) return INFINITY;
      return -(-(double)cnt / 2.0 * log(var) + (l - 1.0) * S);
    };
    // The search evaluates the transform as expm1(a L) / a with L = log1p(|x|) computed once
    // per value (a = lambda for x >= 0, 2 - lambda below): one f64 expm1 per value and
    // evaluation instead of a pow.  Up to PF_VPT values per thread keep (sign, L) in registers.
    const bool in_regs = n <= (int64_t)PF_THREADS * PF_VPT;
    double Lr[PF_VPT];
    int sg[PF_VPT];
#pragma unroll
    for (int k = 0; k < PF_VPT; ++k) {
      const int64_t i = tid + (int64_t)k * PF_THREADS;
      const float v = (in_regs && i < n) ? col(i) : NAN;
      sg[k] = isfinite(v) ? (v >= 0.f ? 1 : -1) : 0;
      Lr[k] = sg[k] ? log1p(fabs((double)v)) : 0.0;
    }
    constexpr double eps = 2.220446049250313e-16;  // np.spacing(1.0), as yj_apply
    const int s_shift = x_shift >= 0.0 ? 1 : -1;
    const double L_shift = log1p(fabs(x_shift));  // hoisted: the same value every evaluation
    auto nllf = [&](double l) -> double {
      const bool p_log = fabs(l) < eps, n_log = !(fabs(l - 2.0) > eps);
      const double ip = p_log ? 0.0 : 1.0 / l, in = n_log ? 0.0 : 1.0 / (2.0 - l);
      auto yj = [&](int sgn, double L) -> double {
        if (sgn > 0) return p_log ? L : expm1(l * L) * ip;
        return n_log ? -L : -expm1((2.0 - l) * L) * in;
      };
      const double k0 = yj(s_shift, L_shift);
      double t1 = 0.0, t2 = 0.0;
      if (in_regs) {
#pragma unroll
        for (int k = 0; k < PF_VPT; ++k)
          if (sg[k]) {
            const double d = yj(sg[k], Lr[k]) - k0;
            t1 += d; t2 += d * d;
          }
      } else {
        for (int64_t i = tid; i < n; i += PF_THREADS) {
          const float v = col(i);
          if (!isfinite(v)) continue;
          const double d = yj(v >= 0.f ? 1 : -1, log1p(fabs((double)v))) - k0;
          t1 += d; t2 += d * d;
        }
      }
      t1 = wave_sum_d(t1);
      t2 = wave_sum_d(t2);
      __syncthreads();
      if (lane == 0) { red2[0][w] = t1; red2[1][w] = t2; }
      __syncthreads();
      return nll_of(l, wsum(red2[0]), wsum(red2[1]));
    };
    int best = 0;
    double fbest = INFINITY;
    for (int g = 0; g < 13; ++g) {
      const double f = nllf(-6.0 + 1.0 * g);
      if (f < fbest) { fbest = f; best = g; }
    }
    double a = -6.0 + 1.0 * max(best - 1, 0), b = -6.0 + 1.0 * min(best + 1, 12);
    const double r = (sqrt(5.0) - 1.0) / 2.0;
    double c = b - r * (b - a), d = a + r * (b - a);
    double fc = nllf(c), fd = nllf(d);
    for (int it = 0; it < 40; ++it) {
      if (fc <= fd) { b = d; d = c; fd = fc; c = b - r * (b - a); fc = nllf(c); }
      else { a = c; c = d; fc = fd; d = a + r * (b - a); fd = nllf(d); }
    }
    lam = 0.5 * (a + b);
  }
  // statistics of the transformed column (float32 values, as the oracle's power_transform_vec)
  double s = 0.0;
  float tmn = INFINITY, tmx = -INFINITY;
  double c2 = 0.0;
  for (int64_t i = tid; i < n; i += PF_THREADS) {
    const float xv = col(i);
    if (!isfinite(xv)) continue;
    const float u = (float)yj_apply((double)xv, lam);
    if (isfinite(u)) { s += u; c2 += 1.0; tmn = fminf(tmn, u); tmx = fmaxf(tmx, u); }
  }
  const double Cn = bsum(c2);
  const double mean = bsum(s) / fmax(Cn, 1.0);
  double q2 = 0.0;
  for (int64_t i = tid; i < n; i += PF_THREADS) {
    const float xv = col(i);
    if (!isfinite(xv)) continue;
    const float u = (float)yj_apply((double)xv, lam);
    if (isfinite(u)) { const double dv = (double)u - mean; q2 += dv * dv; }
  }
  const double Q = bsum(q2);
  bminmax(tmn, tmx);
  if (tid == 0) {
    plam[j] = lam;
    pstat[3 * j + 0] = (float)mean;
    pstat[3 * j + 1] = (float)sqrt(Q / fmax(Cn - 1.0, 1.0));
    pstat[3 * j + 2] = (tmx > tmn) ? 1.0f : 0.0f;
  }
}

// Per-estimator feature tables (oracle OracleTabPFN._fit_features): the pipeline's column list
// (preprocess_oracle T_*, over the views layout), its splitmix64 Fisher-Yates shuffle
// (oracle.philox.estimator_permutation over the F_e columns), the train statistics of each
// shuffled column and the group scales sqrt(2 / used features).  One thread per estimator.
__host__ __device__ inline int pipeline_features(int t, int F, int k) {
  return t == T_QSVD ? 2 * F + k + 1 : ((t == T_PFP || t == T_RFP) ? F + 1 : F);
}
__device__ __forceinline__ int pipeline_column(int t, int i, int e, int F, int k, const ViewLayout& L) {
  switch (t) {
    case T_QUANT: return L.q_off + i;
    case T_POWER: return L.p_off + i;
    case T_QSVD:
      if (i < F) return i;
      if (i < 2 * F) return L.q_off + i - F;
      if (i < 2 * F + k) return L.s_off + i - 2 * F;
      return L.fp_off + e;
    case T_PFP: return i < F ? L.p_off + i : L.fp_off + e;
    case T_RFP: return i < F ? i : L.fp_off + e;
    default: return i;
  }
}
__global__ __launch_bounds__(64) void k_build_params(const float* __restrict__ colstat, int F, int k, int E, int Fmax,
                                                    int Gmax, uint64_t seed, const int* __restrict__ ftype, ViewLayout L,
                                                    int* __restrict__ vcol, float* __restrict__ mu,
                                                    float* __restrict__ sd, float* __restrict__ gscale,
                                                    int* __restrict__ eF) {
  // one wave per estimator: lane 0 runs the (sequential) shuffle in LDS, the lanes then write
  // the column list, its statistics and the group scales
  __shared__ int p[4096];
  const int e = blockIdx.x, lane = threadIdx.x;
  if (e >= E) return;
  const int t = ftype[e];
  const int Fe = pipeline_features(t, F, k);
  const int G = (Fe + 1) / 2;
  for (int i = lane; i < Fe; i += 64) p[i] = i;
  __syncthreads();
  if (lane == 0) {
    eF[e] = Fe;
    uint64_t st = (seed & 0xFFFFFFFFull) | ((uint64_t)(e & 0xFFFF) << 32) | ((uint64_t)(Fe & 0xFFFF) << 48);
    for (int i = Fe - 1; i > 0; --i) {
      const uint64_t out = splitmix64_next(st);
      const int jj = (int)(out % (uint64_t)(i + 1));
      const int tmp = p[i]; p[i] = p[jj]; p[jj] = tmp;
    }
  }
  __syncthreads();
  for (int i = lane; i < Fe; i += 64) {
    const int c = pipeline_column(t, p[i], e, F, k, L);
    p[i] = c;
    vcol[(int64_t)e * Fmax + i] = c;
    mu[(int64_t)e * Fmax + i] = colstat[3 * c + 0];
    sd[(int64_t)e * Fmax + i] = colstat[3 * c + 1];
  }
  __syncthreads();
  for (int g = lane; g < G; g += 64) {
    float u = 0.f;
    for (int q = 0; q < 2; ++q) {
      const int jj = 2 * g + q;
      if (jj < Fe) u += colstat[3 * p[jj] + 2];
    }
    gscale[(int64_t)e * Gmax + g] = sqrtf(2.0f / fmaxf(u, 1.0f));
  }
}

// Classifier fit (oracle OracleTabPFN.fit_classes): per-estimator class permutation
// (splitmix64 Fisher-Yates on a salted state, oracle.philox.class_permutation) and the
// test-row target value ybar_e = mean over train rows of perm_e(y).  One block.
__global__ __launch_bounds__(256) void k_class_params(const float* __restrict__ y, int64_t ldy, int64_t n, int K,
                                                      int E, uint64_t seed, int* __restrict__ cperm,
                                                      float* __restrict__ ybar_e) {
  __shared__ unsigned long long cnt[KMAX_CLS];
  const int tid = threadIdx.x;
  if (tid < KMAX_CLS) cnt[tid] = 0ull;
  __syncthreads();
  for (int64_t i = tid; i < n; i += 256) {
    const int c = min(max((int)y[i * ldy], 0), K - 1);
    atomicAdd(&cnt[c], 1ull);
  }
  __syncthreads();
  if (tid < E) {
    int p[KMAX_CLS];
    for (int i = 0; i < K; ++i) p[i] = i;
    uint64_t st = ((seed & 0xFFFFFFFFull) | ((uint64_t)(tid & 0xFFFF) << 32) | ((uint64_t)(K & 0xFFFF) << 48)) ^
                  0x5A17C1A55E5EED00ull;
    for (int i = K - 1; i > 0; --i) {
      const uint64_t out = splitmix64_next(st);
      const int jj = (int)(out % (uint64_t)(i + 1));
      const int t = p[i];
      p[i] = p[jj];
      p[jj] = t;
    }
    double sum = 0.0;
    for (int c = 0; c < K; ++c) {
      cperm[tid * KMAX_CLS + c] = p[c];
      sum += (double)cnt[c] * (double)p[c];
    }
    ybar_e[tid] = (float)(sum / (double)n);
  }
}

// Classifier head (oracle OracleTabPFN.predict_proba): per row, per estimator the K
// permuted class logits / T -> softmax, mapped back to the original labels, averaged
// over estimators (geo != 0, tabpfn's average_before_softmax [ext]: the estimators' logits
// averaged, then one softmax -- computed as the mean of each estimator's log-softmax, which
// differs from the mean logits by a per-row constant only).  One thread per row; logits
// [E][R][nout].
__global__ __launch_bounds__(256) void k_cls_mix(const logit_t* __restrict__ logits, int64_t R, int E, int nout,
                                                 int K, float invT, const int* __restrict__ cperm, int geo,
                                                 float* __restrict__ probs, int64_t ldo) {
  const int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (r >= R) return;
  float acc[KMAX_CLS];
#pragma unroll
  for (int c = 0; c < KMAX_CLS; ++c) acc[c] = 0.f;
  for (int e = 0; e < E; ++e) {
    const logit_t* lg = logits + ((int64_t)e * R + r) * nout;
    float x[KMAX_CLS], v[KMAX_CLS];
    float m = -INFINITY;
#pragma unroll
    for (int c = 0; c < KMAX_CLS; ++c) {
      x[c] = (c < K) ? (float)lg[cperm[e * KMAX_CLS + c]] * invT : -INFINITY;
      m = fmaxf(m, x[c]);
    }
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < KMAX_CLS; ++c) {
      v[c] = (c < K) ? __expf(x[c] - m) : 0.f;
      s += v[c];
    }
    if (geo) {
      const float lse = m + __logf(s);
#pragma unroll
      for (int c = 0; c < KMAX_CLS; ++c) acc[c] += (c < K) ? x[c] - lse : 0.f;
      continue;
    }
    const float inv = 1.0f / s;
#pragma unroll
    for (int c = 0; c < KMAX_CLS; ++c) acc[c] += v[c] * inv;
  }
  const float invE = 1.0f / (float)E;
  if (geo) {
    float m = -INFINITY;
#pragma unroll
    for (int c = 0; c < KMAX_CLS; ++c)
      if (c < K) m = fmaxf(m, acc[c] * invE);
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < KMAX_CLS; ++c) {
      acc[c] = (c < K) ? __expf(acc[c] * invE - m) : 0.f;
      s += acc[c];
    }
    for (int c = 0; c < K; ++c) probs[r * ldo + c] = acc[c] / s;
    return;
  }
  for (int c = 0; c < K; ++c) probs[r * ldo + c] = acc[c] * invE;
}

// ====================================================== K0 views of the table
// The preprocessed table of one forward, [R][Vw] (ViewLayout): raw | quantile | SVD | power |
// fingerprints.  Non-finite values pass through to k_encode's NaN-indicator path.
// Oracle: OracleTabPFN._features.
__global__ __launch_bounds__(256) void k_views(const float* __restrict__ X, int64_t ldx, int64_t R, ViewParams vp,
                                               float* __restrict__ views) {
  const ViewLayout& L = vp.L;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= R * L.F) return;
  const int64_t r = i / L.F;
  const int col = (int)(i - r * L.F);
  const float x = X[r * ldx + col];
  float* v = views + r * L.Vw;
  v[col] = x;
  if (L.has_q) v[L.q_off + col] = (isfinite(x) && vp.qn[col] > 0) ? qt_apply(x, vp.qtab + (int64_t)col * vp.nqmax, vp.qn[col]) : x;
  if (L.has_p) v[L.p_off + col] = isfinite(x) ? (float)yj_apply((double)x, vp.plam[col]) : x;
}

// SVD columns: (z / scale) . component_c over z = [raw | quantile] of the row, f64 (oracle
// preprocess_oracle.svd_transform).  One thread per (row, component).
__global__ __launch_bounds__(256) void k_views_svd(int64_t R, ViewParams vp, float* __restrict__ views) {
  const ViewLayout& L = vp.L;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= R * L.k) return;
  const int64_t r = i / L.k;
  const int c = (int)(i - r * L.k);
  const int m = 2 * L.F;
  const double* scale = vp.svd;
  const double* comp = vp.svd + m + (int64_t)c * m;
  const float* v = views + r * L.Vw;
  double acc = 0.0;
  for (int j = 0; j < m; ++j) {
    const float z = j < L.F ? v[j] : v[L.q_off + j - L.F];
    acc += comp[j] * ((double)z / scale[j]);
  }
  views[r * L.Vw + L.s_off + c] = (float)acc;
}

// ------------------------------------------------ fingerprint feature (SHA-256)
// tabpfn's AddFingerprintFeaturesStep [ext]: int(sha256(row bytes).hexdigest(), 16) % 10000 /
// 10000 of the row + salt (+ 1, + 2, ... for a train row whose hash an earlier train row took).
// The hashed row is the raw feature row widened to float64 (oracle preprocess_oracle.fingerprint).
__constant__ uint32_t kSha256K[64] = {
    0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u, 0xab1c5ed5u,
    0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu, 0x9bdc06a7u, 0xc19bf174u,
    0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu, 0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau,
    0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u, 0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u,
    0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu, 0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u,
    0xa2bfe8a1u, 0xa81a664bu, 0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u,
    0x19a4c116u, 0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u,
    0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u, 0xc67178f2u};

__device__ __forceinline__ uint32_t rotr32(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }

// message word gw of the padded message whose first 8F bytes are the float64 values
// (double)row[j] + salt (+ add when add > 0), little-endian, as numpy's tobytes()
__device__ __forceinline__ uint32_t fp_word(const float* row, int F, double salt, double add, int gw, int nblk) {
  const int L = 8 * F;
  if (4 * gw < L) {
    double v = __dadd_rn((double)row[gw >> 1], salt);
    if (add > 0.0) v = __dadd_rn(v, add);
    const uint64_t bits = (uint64_t)__double_as_longlong(v);
    const uint32_t half = (gw & 1) ? (uint32_t)(bits >> 32) : (uint32_t)bits;
    return __builtin_bswap32(half);
  }
  if (4 * gw == L) return 0x80000000u;
  if (gw == 16 * nblk - 1) return (uint32_t)((uint64_t)L * 8u);
  if (gw == 16 * nblk - 2) return (uint32_t)(((uint64_t)L * 8u) >> 32);
  return 0u;
}

__device__ int fp_hash(const float* row, int F, double salt, double add) {
  uint32_t H[8] = {0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au, 0x510e527fu, 0x9b05688cu, 0x1f83d9abu, 0x5be0cd19u};
  const int nblk = (8 * F + 8) / 64 + 1;
  for (int b = 0; b < nblk; ++b) {
    uint32_t w[16];
#pragma unroll
    for (int t = 0; t < 16; ++t) w[t] = fp_word(row, F, salt, add, 16 * b + t, nblk);
    uint32_t a = H[0], bb = H[1], c = H[2], d = H[3], e = H[4], f = H[5], g = H[6], h = H[7];
#pragma unroll
    for (int t = 0; t < 64; ++t) {
      uint32_t wt;
      if (t < 16) {
        wt = w[t];
      } else {
        const uint32_t w15 = w[(t + 1) & 15], w2 = w[(t + 14) & 15];
        const uint32_t s0 = rotr32(w15, 7) ^ rotr32(w15, 18) ^ (w15 >> 3);
        const uint32_t s1 = rotr32(w2, 17) ^ rotr32(w2, 19) ^ (w2 >> 10);
        wt = w[t & 15] + s0 + w[(t + 9) & 15] + s1;
        w[t & 15] = wt;
      }
      const uint32_t S1 = rotr32(e, 6) ^ rotr32(e, 11) ^ rotr32(e, 25);
      const uint32_t ch = (e & f) ^ (~e & g);
      const uint32_t t1 = h + S1 + ch + kSha256K[t] + wt;
      const uint32_t S0 = rotr32(a, 2) ^ rotr32(a, 13) ^ rotr32(a, 22);
      const uint32_t mj = (a & bb) ^ (a & c) ^ (bb & c);
      const uint32_t t2 = S0 + mj;
      h = g; g = f; f = e; e = d + t1; d = c; c = bb; bb = a; a = t1 + t2;
    }
    H[0] += a; H[1] += bb; H[2] += c; H[3] += d; H[4] += e; H[5] += f; H[6] += g; H[7] += h;
  }
  uint64_t r = 0;  // the 256-bit digest, big-endian, modulo 10000
#pragma unroll
  for (int i = 0; i < 8; ++i) r = ((r << 32) + H[i]) % (uint64_t)kFpBuckets;
  return (int)r;
}

// test rows: one thread per (row, estimator with a fingerprint column)
__global__ __launch_bounds__(256) void k_views_fp(const float* __restrict__ X, int64_t ldx, int64_t R, ViewParams vp,
                                                  float* __restrict__ views) {
  const ViewLayout& L = vp.L;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= R * L.E) return;
  const int64_t r = i / L.E;
  const int e = (int)(i - r * L.E);
  const int salt = vp.fp_salt[e];
  if (salt < 0) return;
  const int h = fp_hash(X + r * ldx, L.F, (double)salt, 0.0);
  views[r * L.Vw + L.fp_off + e] = (float)((double)h / (double)kFpBuckets);
}

// candidate layout: row k of a block of kFpBlock rows starts at g_fp_off[k] (the prefix of the
// rows' counts rounded up to 4), a block takes g_fp_off[kFpBlock]; set once by svd_setup
__device__ int g_fp_off[kFpBlock + 1];
static int h_fp_off[kFpBlock + 1];
static void fp_off_init() {
  h_fp_off[0] = 0;
  for (int k = 0; k < kFpBlock; ++k) h_fp_off[k + 1] = h_fp_off[k] + ((fp_count(k) + 3) & ~3);
}
int64_t fp_total(int64_t n) {
  if (h_fp_off[kFpBlock] == 0) fp_off_init();
  return (n / kFpBlock) * (int64_t)h_fp_off[kFpBlock] + h_fp_off[n % kFpBlock];
}
__device__ __forceinline__ int64_t fp_row_off(int64_t r) {
  return (r / kFpBlock) * (int64_t)g_fp_off[kFpBlock] + g_fp_off[r % kFpBlock];
}

// train rows, pass 1: the first fp_count(k) candidate hashes (add = 0, 1, ...) of every row,
// k = its position in its block of kFpBlock rows -- the expected number of tries grows as the
// taken set fills (about kFpBuckets / (kFpBuckets - k)), so the count does too (4x that, at
// least 4, at most kFpCap), and nearly every row finds its hash among precomputed candidates.
// htab [E][total]: row r's candidates at fp_row_off(r); thread i of an estimator finds its row
// by a binary search of the block's offsets (13 steps, the table L2-resident).
__global__ __launch_bounds__(256) void k_fp_train_hash(const float* __restrict__ X, int64_t ldx, int64_t n,
                                                       int64_t total, ViewParams vp, int* __restrict__ htab) {
  const ViewLayout& L = vp.L;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (int64_t)L.E * total) return;
  const int e = (int)(i / total);
  const int64_t j = i - (int64_t)e * total;
  const int64_t blk = j / g_fp_off[kFpBlock];
  const int jj = (int)(j - blk * g_fp_off[kFpBlock]);
  int lo = 0, hi = kFpBlock;  // the largest k with g_fp_off[k] <= jj
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (g_fp_off[mid] <= jj) lo = mid; else hi = mid;
  }
  const int a = jj - g_fp_off[lo];
  const int64_t r = blk * kFpBlock + lo;
  const int salt = vp.fp_salt[e];
  if (salt < 0 || r >= n || a >= fp_count(lo)) return;
  htab[i] = fp_hash(X + r * ldx, L.F, (double)salt, (double)a);
}

// train rows, pass 2 (one block per estimator): rows in order take their first candidate hash
// not yet taken (a 10000-bit map in LDS).  Wave 0 takes 64 rows at a time: every lane proposes
// its row's first precomputed candidate not in the map; the rows before the first lane whose
// proposal repeats an earlier lane's (or that has no free precomputed candidate) keep their
// proposals -- exactly the sequential choice, since their proposals are distinct -- and the
// next round starts at that lane's row.  A row past its precomputed candidates is hashed by
// the whole block, blockDim.x more candidates (add = a0 + thread) at a time, the first free
// one in add order kept (one wave for contexts of up to 4096 rows, 16 beyond: the slow path is
// what the last rows of a 10 000-row block need).  10 000 hash values cannot give more than 10 000 rows distinct hashes
// (tabpfn's loop would not end), so the map starts empty again every kFpBlock rows (oracle
// preprocess_oracle.fingerprint; identical to tabpfn up to 10 000 rows).
constexpr int FPR_THREADS = 1024;
// dynamic LDS of k_fp_train_resolve: the taken map [NW] | claim [kFpBuckets] (the first lane
// of a batch proposing a hash) | staged candidates: the first kFpStage of each row, 128 rows
constexpr int kFpNW = (kFpBuckets + 31) / 32;
constexpr int kFpStage = 64;
constexpr int kFpCB = 128 * kFpStage;
constexpr size_t kFpResolveSmem = (size_t)(kFpNW + kFpBuckets + kFpCB) * sizeof(int);
__global__ __launch_bounds__(FPR_THREADS) void k_fp_train_resolve(const float* __restrict__ X, int64_t ldx, int64_t n,
                                                                  int stride, int64_t total, ViewParams vp,
                                                                  const int* __restrict__ htab,
                                                                  float* __restrict__ views) {
  const ViewLayout& L = vp.L;
  const int e = blockIdx.x;
  const int salt = vp.fp_salt[e];
  if (salt < 0) return;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  uint32_t* seen = reinterpret_cast<uint32_t*>(smem);
  int* claim = reinterpret_cast<int*>(seen + kFpNW);
  int* cbuf = claim + kFpBuckets;  // 16-byte aligned: (313 + 10000) ints = 41 252 bytes, rounded below
  cbuf = reinterpret_cast<int*>((reinterpret_cast<uintptr_t>(cbuf) + 15) & ~(uintptr_t)15);
  __shared__ int s_state, s_hit[FPR_THREADS / 64];
  __shared__ int64_t s_row;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int nthr = blockDim.x, nwav = nthr >> 6;
  const int* ht = htab + (int64_t)e * total;
  auto taken = [&](int c) { return (seen[c >> 5] >> (c & 31)) & 1u; };
  auto put = [&](int64_t r, int h) {
    atomicOr(&seen[h >> 5], 1u << (h & 31));
    views[r * L.Vw + L.fp_off + e] = (float)((double)h / (double)kFpBuckets);
  };
  // a row whose first kFpStage candidates are taken, by the whole block: its other precomputed
  // candidates (one load each), then blockDim.x fresh hashes a step; every wave computes the
  // same h, so the step count -- and the barrier count -- agree
  const int sstride = min(stride, kFpStage);
  auto first_free = [&](int cc, bool ok) -> int {  // the block's first ok && free candidate, in thread order
    const uint64_t fb = __ballot(ok && !taken(cc));
    const int first = fb ? __shfl(cc, __ffsll((unsigned long long)fb) - 1, 64) : -1;  // the wave's first
    if (lane == 0) s_hit[wave] = first;
    __syncthreads();
    int h = -1;
    for (int w = 0; w < nwav; ++w)
      if (h < 0 && s_hit[w] >= 0) h = s_hit[w];
    __syncthreads();
    return h;
  };
  auto slow_row = [&](int64_t r) {
    const float* row = X + r * ldx;
    const int cnt = fp_count((int)(r % kFpBlock));
    int h = -1;
    for (int a0 = sstride; h < 0 && a0 < cnt; a0 += nthr)
      h = first_free(a0 + tid < cnt ? ht[fp_row_off(r) + a0 + tid] : 0, a0 + tid < cnt);
    for (int a0 = cnt; h < 0; a0 += nthr) h = first_free(fp_hash(row, L.F, (double)salt, (double)(a0 + tid)), true);
    if (tid == 0) put(r, h);
  };
  for (int i = tid; i < kFpBuckets; i += nthr) claim[i] = 64;  // no lane
  __syncthreads();
  if (wave != 0) {  // helpers: wait for wave 0 to hand over a slow row, or to finish
    for (;;) {
      __syncthreads();  // (A)
      if (s_state == 2) break;
      slow_row(s_row);
      __syncthreads();  // (B)
    }
    return;
  }
  // wave 0 walks the rows alone (no block barrier per batch): staging, map resets, batches
  const int rows_per_stage = kFpCB / sstride;  // >= 128
  int64_t buf0 = 0, buf1 = 0;                 // rows [buf0, buf1) have their candidates in cbuf
  int64_t r0 = 0;
  while (r0 < n) {
    if (r0 % kFpBlock == 0)
      for (int i = lane; i < kFpNW; i += 64) seen[i] = 0u;
    const int64_t seg_end = min(n, (r0 / kFpBlock + 1) * (int64_t)kFpBlock);
    if (min(r0 + 64, n) > buf1) {  // stage the next rows' first sstride candidates (16-byte pieces)
      buf0 = r0;
      buf1 = min(n, r0 + rows_per_stage);
      const int q = sstride / 4;  // staged pieces per row (sstride % 4 == 0)
      int4* dst = reinterpret_cast<int4*>(cbuf);
      for (int i = lane; i < (int)(buf1 - buf0) * q; i += 64) {
        const int rr = i / q, pc = i - rr * q;
        const int64_t r = buf0 + rr;
        // the row's own pieces (its count rounded up to 4); the scan reads no further
        if (4 * pc < fp_count((int)(r % kFpBlock))) dst[i] = reinterpret_cast<const int4*>(ht + fp_row_off(r))[pc];
      }
    }
    const int64_t r = r0 + lane;
    const bool valid = r < seg_end;
    int p = -1;
    if (valid) {  // the row's first candidate not taken, four at a time
      const int cnt = min(fp_count((int)(r % kFpBlock)), sstride);  // the staged ones; slow_row the rest
      const int4* cr = reinterpret_cast<const int4*>(cbuf + (r - buf0) * sstride);
      for (int a = 0; a < cnt && p < 0; a += 4) {
        const int4 c = cr[a >> 2];
        const bool f0 = !taken(c.x), f1 = a + 1 < cnt && !taken(c.y), f2 = a + 2 < cnt && !taken(c.z),
                   f3 = a + 3 < cnt && !taken(c.w);
        p = f0 ? c.x : f1 ? c.y : f2 ? c.z : f3 ? c.w : -1;
      }
    }
    // an earlier lane proposing the same hash: the lowest proposing lane wins the claim
    if (p >= 0) atomicMin(&claim[p], lane);
    const bool dup = p >= 0 && claim[p] < lane;
    const uint64_t badm = __ballot(valid && (p < 0 || dup));
    if (p >= 0) claim[p] = 64;  // reset for the next batch (every proposer writes the same value)
    const int nvalid = (int)min((int64_t)64, seg_end - r0);
    const int nfin = badm ? __ffsll((unsigned long long)badm) - 1 : nvalid;
    if (lane < nfin) put(r, p);
    const bool slow = nfin < nvalid && __shfl(p, nfin, 64) < 0;  // no free staged candidate
    r0 += nfin;
    if (slow) {
      if (lane == 0) {
        s_row = r0;
        s_state = 1;
      }
      __syncthreads();  // (A): the map and the row are visible to the helpers
      slow_row(r0);
      __syncthreads();  // (B)
      r0 += 1;
    }
  }
  if (lane == 0) s_state = 2;
  __syncthreads();  // (A): release the helpers
}

// ====================================================== SVD of the train views
// StandardScaler(with_mean=False) scale = population std of each of the m = 2F columns of
// Z = [raw | quantile] (1 where ~0); Gram matrix of Y = Z / scale; cyclic parallel Jacobi
// (round-robin pairs, f64); the k eigenvectors of the largest eigenvalues, each signed so its
// largest-magnitude entry is positive (sklearn svd_flip with u_based_decision=False).  Oracle:
// preprocess_oracle.svd_fit (pinned to sklearn TruncatedSVD).
//
// Two launches.  k_svd_gram (grid: upper 32x32 tiles of Z^T Z x row chunks): each block
// sums its tile over its chunk's rows, and the diagonal tiles also the shifted column sums
// sum (z - z_0), sum (z - z_0)^2 (z_0 = the column's first value, so a constant column has
// variance exactly 0); partials go to a workspace in fixed slots, so the result does not
// depend on scheduling.  k_svd_jacobi (one block of 1024 threads) adds the partials in chunk
// order, forms A = D^-1 Z^T Z D^-1 and runs the sweeps: per round the pair rotations
// (m / 2 threads), one barrier, then every 2x2 pair block of A is rotated from both sides at
// once (J_i^T B J_j, the upper blocks written with their transposes) together with the two
// columns of V per pair, one barrier.  A lives in LDS up to m = 128 (V too up to m = 64),
// beyond that in the workspace (L2).
constexpr int kSvdTile = 32;
__host__ __device__ inline int svd_tiles(int m) { return (m + kSvdTile - 1) / kSvdTile; }
__host__ __device__ inline int svd_upper_tiles(int m) { const int T = svd_tiles(m); return T * (T + 1) / 2; }
__host__ __device__ inline int svd_tile_index(int ti, int tj, int T) { return ti * T - ti * (ti - 1) / 2 + (tj - ti); }
static int svd_chunks(int64_t n, int m) {
  const int64_t by_rows = (n + 127) / 128;
  const int64_t by_grid = std::max<int64_t>(1, 512 / svd_upper_tiles(m));
  return (int)std::max<int64_t>(1, std::min<int64_t>(std::min<int64_t>(by_rows, by_grid), 16));
}
// workspace: partial tiles [chunks][upper tiles][32][32] | partial sums [chunks][m][2] |
// A, V [m][m + 1] (m > 128: A; m > 64: V)
static int svd_dual_np(int64_t n) { return (int)(n + (n & 1)); }
size_t svd_work_bytes(int64_t n, int m) {
  if (m > kSvdMaxM && n > kSvdMaxM) {  // large: tiles | psum | scl [m] | A [m][m] | D, E [m] | info
    const size_t nc = (size_t)svd_chunks(n, m);
    return (nc * svd_upper_tiles(m) * kSvdTile * kSvdTile + nc * m * 2 + (size_t)m + (size_t)m * m + 2 * (size_t)m +
            1) * sizeof(double);
  }
  if (m > kSvdMaxM) {  // dual: scl [m] | psum [n'][2] | tiles of Y Y^T | A, V [n'][n' + 1] | u out [n'][n' + 1]
    const size_t np = (size_t)svd_dual_np(std::min<int64_t>(n, kSvdMaxM));
    return ((size_t)m + 2 * np + (size_t)svd_upper_tiles((int)np) * kSvdTile * kSvdTile + 3 * np * (np + 1)) *
           sizeof(double);
  }
  const size_t nc = (size_t)svd_chunks(n, m);
  return (nc * svd_upper_tiles(m) * kSvdTile * kSvdTile + nc * m * 2 + 2 * (size_t)m * (m + 1)) * sizeof(double);
}

__global__ __launch_bounds__(256) void k_svd_gram(const float* __restrict__ views, int64_t n, ViewLayout L, int nchunk,
                                                  double* __restrict__ part, double* __restrict__ psum) {
  __shared__ double za[kSvdTile][kSvdTile + 1];
  __shared__ double zb[kSvdTile][kSvdTile + 1];
  const int m = 2 * L.F, T = svd_tiles(m);
  int ti = 0, u = blockIdx.x;
  while (u >= T - ti) { u -= T - ti; ++ti; }
  const int tj = ti + u;
  const int c = blockIdx.y;
  const int64_t r0 = n * c / nchunk, r1 = n * (c + 1) / nchunk;
  const int tid = threadIdx.x;
  auto col = [&](int64_t r, int j) -> double {
    if (j >= m) return 0.0;
    const float* v = views + r * L.Vw;
    return (double)(j < L.F ? v[j] : v[L.q_off + j - L.F]);
  };
  const int a = tid >> 3, b0 = (tid & 7) * 4;  // this thread's entries (a, b0 .. b0 + 3) of the tile
  double g[4] = {0.0, 0.0, 0.0, 0.0};
  const bool diag = ti == tj;
  const int sc = tid;                          // diagonal tiles: threads < 32 sum column ti * 32 + sc
  const double z0 = (diag && sc < kSvdTile) ? col(0, ti * kSvdTile + sc) : 0.0;
  double s1 = 0.0, s2 = 0.0;
  for (int64_t rb = r0; rb < r1; rb += kSvdTile) {
    const int rows = (int)min((int64_t)kSvdTile, r1 - rb);
    __syncthreads();
    for (int i = tid; i < kSvdTile * kSvdTile; i += 256) {
      const int rr = i >> 5, j = i & 31;
      za[rr][j] = rr < rows ? col(rb + rr, ti * kSvdTile + j) : 0.0;
      zb[rr][j] = rr < rows ? col(rb + rr, tj * kSvdTile + j) : 0.0;
    }
    __syncthreads();
    for (int rr = 0; rr < rows; ++rr) {
      const double x = za[rr][a];
#pragma unroll
      for (int q = 0; q < 4; ++q) g[q] = fma(x, zb[rr][b0 + q], g[q]);
    }
    if (diag && sc < kSvdTile)
      for (int rr = 0; rr < rows; ++rr) {
        const double d = za[rr][sc] - z0;
        s1 += d;
        s2 = fma(d, d, s2);
      }
  }
  double* pt = part + ((int64_t)c * svd_upper_tiles(m) + blockIdx.x) * (kSvdTile * kSvdTile);
#pragma unroll
  for (int q = 0; q < 4; ++q) pt[a * kSvdTile + b0 + q] = g[q];
  if (diag && sc < kSvdTile && ti * kSvdTile + sc < m) {
    psum[((int64_t)c * m + ti * kSvdTile + sc) * 2 + 0] = s1;
    psum[((int64_t)c * m + ti * kSvdTile + sc) * 2 + 1] = s2;
  }
}

constexpr int SVJ_THREADS = 1024;
// LDS head of k_svd_jacobi: scl, sgn [512] | rot c, s [256] | red [32] (doubles) | sel [512] (ints).  A
// round's pairs follow from the round number (svj_pair), so no index arrays sit in the chain.
constexpr size_t kSvjHead = (512 * 2 + 256 * 2 + 32) * sizeof(double) + 512 * sizeof(int);

// scale = population std from the shifted sums (partials added in chunk order), A = the Gram
// matrix of Y = Z / scale from the partial tiles, V = I
__device__ __forceinline__ void svj_fill(const double* __restrict__ part, const double* __restrict__ psum, int nchunk,
                                         int64_t n, int m, double* scl, double* A, double* V, int ld) {
  const int tid = threadIdx.x;
  const int T = svd_tiles(m), NT = svd_upper_tiles(m);
  for (int j = tid; j < m; j += SVJ_THREADS) {
    double s1 = 0.0, s2 = 0.0;
    for (int c = 0; c < nchunk; ++c) {
      s1 += psum[((int64_t)c * m + j) * 2 + 0];
      s2 += psum[((int64_t)c * m + j) * 2 + 1];
    }
    const double mu = s1 / (double)n;
    const double sd = sqrt(fmax(s2 / (double)n - mu * mu, 0.0));
    scl[j] = sd < 10.0 * 2.220446049250313e-16 ? 1.0 : sd;
  }
  __syncthreads();
  for (int i = tid; i < m * m; i += SVJ_THREADS) {
    const int a = i / m, b = i - a * m;
    const int ta = a / kSvdTile, tb = b / kSvdTile;
    const int t = ta <= tb ? svd_tile_index(ta, tb, T) : svd_tile_index(tb, ta, T);
    const int e = ta <= tb ? (a % kSvdTile) * kSvdTile + (b % kSvdTile) : (b % kSvdTile) * kSvdTile + (a % kSvdTile);
    double g = 0.0;
    for (int c = 0; c < nchunk; ++c) g += part[((int64_t)c * NT + t) * (kSvdTile * kSvdTile) + e];
    A[a * ld + b] = g / (scl[a] * scl[b]);
    V[a * ld + b] = a == b ? 1.0 : 0.0;
  }
  __syncthreads();
}

// pair i of round `round` of the cyclic round-robin ordering (m even), p < q
__device__ __forceinline__ void svj_pair(int i, int round, int m, int& p, int& q) {
  int xr = i - 1 + round, yr = m - 2 - i + round;  // both in [0, 2 (m - 1)): one wrap each
  xr -= xr >= m - 1 ? m - 1 : 0;
  yr -= yr >= m - 1 ? m - 1 : 0;
  const int x = i == 0 ? 0 : 1 + xr;
  const int y = 1 + yr;
  p = min(x, y);
  q = max(x, y);
}

// the rotation annihilating A[p][q] (classic Jacobi, f64)
__device__ __forceinline__ void svj_rot(double apq, double app, double aqq, double& c, double& sn) {
  c = 1.0;
  sn = 0.0;
  if (fabs(apq) > 1e-300 && fabs(apq) > 1e-18 * sqrt(fabs(app * aqq))) {
    const double tau = (aqq - app) / (2.0 * apq);
    const double t = (tau >= 0.0 ? 1.0 : -1.0) / (fabs(tau) + sqrt(1.0 + tau * tau));
    c = 1.0 / sqrt(1.0 + t * t);
    sn = t * c;
  }
}

// J_i^T B J_j of the 2x2 pair block B = A[{pi, qi}][{pj, qj}]: rows with rotation i, then
// columns with rotation j; n[2 x + y] = new A[x ? qi : pi][y ? qj : pj]
__device__ __forceinline__ void svj_block(const double* A, int ld, int pi, int qi, int pj, int qj, double ci,
                                          double si, double cj, double sj, double (&nv)[4]) {
  const double a_pp = A[pi * ld + pj], a_pq = A[pi * ld + qj], a_qp = A[qi * ld + pj], a_qq = A[qi * ld + qj];
  const double r_pp = ci * a_pp - si * a_qp, r_pq = ci * a_pq - si * a_qq;
  const double r_qp = si * a_pp + ci * a_qp, r_qq = si * a_pq + ci * a_qq;
  nv[0] = cj * r_pp - sj * r_pq;
  nv[1] = sj * r_pp + cj * r_pq;
  nv[2] = cj * r_qp - sj * r_qq;
  nv[3] = sj * r_qp + cj * r_qq;
}

// top-k eigenvalues, descending (ties: lower index first): column i's rank among the diagonal;
// each selected eigenvector signed so its largest-magnitude entry is positive
__device__ __forceinline__ void svj_output(const double* A, const double* V, int ld, int m, int k, const double* scl,
                                           double* sgn, int* sel, double* __restrict__ out) {
  const int tid = threadIdx.x;
  for (int i = tid; i < m; i += SVJ_THREADS) {
    const double d = A[i * ld + i];
    int rank = 0;
    for (int j = 0; j < m; ++j) {
      const double e = A[j * ld + j];
      rank += (e > d || (e == d && j < i)) ? 1 : 0;
    }
    sel[i] = rank < k ? rank + 1 : 0;
    double sg = 1.0;
    if (sel[i]) {
      int am = 0;
      for (int j = 1; j < m; ++j)
        if (fabs(V[j * ld + i]) > fabs(V[am * ld + i])) am = j;
      sg = V[am * ld + i] < 0.0 ? -1.0 : 1.0;
    }
    sgn[i] = sg;
    out[i] = scl[i];
  }
  __syncthreads();
  for (int u = tid; u < m * m; u += SVJ_THREADS) {
    const int j = u / m, i = u - j * m;  // V[j][i] of column i
    const int c = sel[i] - 1;
    if (c >= 0) out[m + (int64_t)c * m + j] = sgn[i] * V[j * ld + i];
  }
}

template <bool ALDS, bool VLDS>
__global__ __launch_bounds__(SVJ_THREADS) void k_svd_jacobi(const double* __restrict__ part,
                                                            const double* __restrict__ psum, int nchunk, int64_t n,
                                                            int m, int k, double* __restrict__ gA,
                                                            double* __restrict__ gV, double* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  double* scl = reinterpret_cast<double*>(smem);
  double* sgn = scl + 512;
  double* rc = sgn + 512;
  double* rs = rc + 256;
  double* red = rs + 256;
  int* sel = reinterpret_cast<int*>(red + 32);
  double* lds_mat = reinterpret_cast<double*>(smem + kSvjHead);
  const int ld = m + 1;
  double* A = ALDS ? lds_mat : gA;
  double* V = VLDS ? lds_mat + (size_t)m * ld : gV;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  auto bsum = [&](double v) -> double {
    v = wave_sum_d(v);
    __syncthreads();
    if (lane == 0) red[w] = v;
    __syncthreads();
    double t = 0.0;
#pragma unroll
    for (int i = 0; i < SVJ_THREADS / 64; ++i) t += red[i];
    return t;
  };
  svj_fill(part, psum, nchunk, n, m, scl, A, V, ld);
  const int half = m / 2;
  // the round's work items on power-of-two grids (shift / mask decode, no division): pair
  // blocks (i, j), j >= i, of a P2 x P2 grid, and V's (row, pair) of an m x P2 grid
  int lg = 0;
  while ((1 << lg) < half) ++lg;
  const int P2 = 1 << lg;
  const int nblk = P2 * P2;
  // when the round's pair blocks (i <= j < half) and V's (row, pair) units together fit the
  // workgroup (m <= 40), each thread owns one unit for the whole fit, decoded once, and the
  // block and V updates of a round run side by side instead of one loop after the other
  const int nbu = half * (half + 1) / 2, nvu = m * half;
  const bool one = nbu + nvu <= SVJ_THREADS;
  int ui = -1, uj = -1, urow = -1;  // this thread's block (ui, uj) or V unit (urow, ui)
  if (one) {
    if (tid < nbu) {
      int u = tid, i = 0;
      while (u >= half - i) {
        u -= half - i;
        ++i;
      }
      ui = i;
      uj = i + u;
    } else if (tid < nbu + nvu) {
      urow = (tid - nbu) / half;
      ui = tid - nbu - urow * half;
    }
  }
  const int max_sweeps = m <= 64 ? 12 : 16;
  for (int sweep = 0; sweep < max_sweeps; ++sweep) {
    // converged (off-diagonal mass under 1e-28 of the diagonal's): further rotations are
    // identities to f64 precision
    if (sweep >= 3) {
      double off = 0.0, dia = 0.0;
      for (int i = tid; i < m * m; i += SVJ_THREADS) {
        const int a = i / m, b = i - a * m;
        const double v = A[a * ld + b] * A[a * ld + b];
        if (a == b) dia += v; else off += v;
      }
      const double offs = bsum(off), dias = bsum(dia);
      if (offs <= 1e-28 * dias) break;
    }
    for (int round = 0; round < m - 1; ++round) {
      if (tid < half) {
        int p, q;
        svj_pair(tid, round, m, p, q);
        double c, sn;
        svj_rot(A[p * ld + q], A[p * ld + p], A[q * ld + q], c, sn);
        rc[tid] = c; rs[tid] = sn;
      }
      __syncthreads();
      // A <- J^T A J, one 2x2 pair block (i, j), i <= j, per unit (the transpose block written
      // alongside); V <- V J
      auto block = [&](int i, int j) {
        int pi, qi, pj, qj;  // the pairs from the round number (no LDS lookup in the chain)
        svj_pair(i, round, m, pi, qi);
        svj_pair(j, round, m, pj, qj);
        double nv[4];
        svj_block(A, ld, pi, qi, pj, qj, rc[i], rs[i], rc[j], rs[j], nv);
        A[pi * ld + pj] = nv[0]; A[pi * ld + qj] = nv[1]; A[qi * ld + pj] = nv[2]; A[qi * ld + qj] = nv[3];
        if (i != j) { A[pj * ld + pi] = nv[0]; A[qj * ld + pi] = nv[1]; A[pj * ld + qi] = nv[2]; A[qj * ld + qi] = nv[3]; }
      };
      auto vrot = [&](int row, int i) {
        int p, q;
        svj_pair(i, round, m, p, q);
        const double c = rc[i], sn = rs[i];
        const double vp = V[row * ld + p], vq = V[row * ld + q];
        V[row * ld + p] = c * vp - sn * vq;
        V[row * ld + q] = sn * vp + c * vq;
      };
      if (one) {
        if (uj >= 0) block(ui, uj);
        else if (urow >= 0) vrot(urow, ui);
      } else {
        for (int u = tid; u < nblk; u += SVJ_THREADS) {
          const int i = u >> lg, j = u & (P2 - 1);
          if (j >= i && j < half) block(i, j);
        }
        for (int u = tid; u < (m << lg); u += SVJ_THREADS) {
          const int row = u >> lg, i = u & (P2 - 1);
          if (i < half) vrot(row, i);
        }
      }
      __syncthreads();
    }
  }
  svj_output(A, V, ld, m, k, scl, sgn, sel, out);
}

// ---- dual form (wide tables: m = 2F > kSvdMaxM, n <= kSvdMaxM rows).  The nonzero eigenvalues
// of Y^T Y and Y Y^T are the same, and v = Y^T u / |Y^T u| maps an eigenvector u of the n x n
// matrix Y Y^T to the Gram matrix's eigenvector of the same eigenvalue.  So: the column scales
// (k_svd_colscale, the shifted sums of k_svd_gram in row order), the upper 32 x 32 tiles of
// Y Y^T in k_svd_gram's partial-tile format (k_svd_dual_gram; one chunk), the same Jacobi on the
// n' x n' matrix (n' = n rounded up to even, a zero padding row; the fake partial sums s1 = 0,
// s2 = n' make its scales 1), and per component v = Y^T u normalised and signed as svd_flip
// (k_svd_dual_out: largest-magnitude entry, first index on ties, made positive).
__device__ __forceinline__ double svd_z(const float* __restrict__ views, const ViewLayout& L, int64_t r, int j) {
  const float* v = views + r * L.Vw;
  return (double)(j < L.F ? v[j] : v[L.q_off + j - L.F]);
}

__global__ __launch_bounds__(256) void k_svd_colscale(const float* __restrict__ views, int64_t n, ViewLayout L,
                                                      int np, double* __restrict__ scl, double* __restrict__ psum) {
  const int m = 2 * L.F;
  const int j = blockIdx.x * 256 + threadIdx.x;
  if (j < np) {
    psum[2 * j + 0] = 0.0;
    psum[2 * j + 1] = (double)np;
  }
  if (j >= m) return;
  const double z0 = svd_z(views, L, 0, j);
  double s1 = 0.0, s2 = 0.0;
  for (int64_t r = 0; r < n; ++r) {
    const double d = svd_z(views, L, r, j) - z0;
    s1 += d;
    s2 = fma(d, d, s2);
  }
  const double mu = s1 / (double)n;
  const double sd = sqrt(fmax(s2 / (double)n - mu * mu, 0.0));
  scl[j] = sd < 10.0 * 2.220446049250313e-16 ? 1.0 : sd;
}

__global__ __launch_bounds__(256) void k_svd_dual_gram(const float* __restrict__ views, int64_t n, ViewLayout L,
                                                       const double* __restrict__ scl, int np,
                                                       double* __restrict__ part) {
  __shared__ double za[kSvdTile][kSvdTile + 1];
  __shared__ double zb[kSvdTile][kSvdTile + 1];
  const int m = 2 * L.F, T = svd_tiles(np);
  int ti = 0, u = blockIdx.x;
  while (u >= T - ti) { u -= T - ti; ++ti; }
  const int tj = ti + u;
  const int tid = threadIdx.x;
  const int a = tid >> 3, b0 = (tid & 7) * 4;  // this thread's entries (a, b0 .. b0 + 3) of the tile
  double g[4] = {0.0, 0.0, 0.0, 0.0};
  for (int j0 = 0; j0 < m; j0 += kSvdTile) {
    __syncthreads();
    for (int i = tid; i < kSvdTile * kSvdTile; i += 256) {
      const int rr = i >> 5, jj = i & 31, j = j0 + jj;
      const int64_t ra = ti * kSvdTile + rr, rb = tj * kSvdTile + rr;
      za[rr][jj] = (j < m && ra < n) ? svd_z(views, L, ra, j) / scl[j] : 0.0;
      zb[rr][jj] = (j < m && rb < n) ? svd_z(views, L, rb, j) / scl[j] : 0.0;
    }
    __syncthreads();
    for (int jj = 0; jj < kSvdTile; ++jj) {
      const double x = za[a][jj];
#pragma unroll
      for (int q = 0; q < 4; ++q) g[q] = fma(x, zb[b0 + q][jj], g[q]);
    }
  }
  double* pt = part + (int64_t)blockIdx.x * (kSvdTile * kSvdTile);
#pragma unroll
  for (int q = 0; q < 4; ++q) pt[a * kSvdTile + b0 + q] = g[q];
}

// one block per component c: uo = the Jacobi's output over n' ([n'] ones | [k][n'] u vectors)
__global__ __launch_bounds__(256) void k_svd_dual_out(const float* __restrict__ views, int64_t n, ViewLayout L,
                                                      const double* __restrict__ scl, int np,
                                                      const double* __restrict__ uo, double* __restrict__ out) {
  __shared__ double u[kSvdMaxM];
  __shared__ double rsum[4], rbest[4], rval[4];
  __shared__ int ridx[4];
  const int m = 2 * L.F, c = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  for (int i = tid; i < np; i += 256) u[i] = uo[np + (int64_t)c * np + i];
  if (c == 0)
    for (int j = tid; j < m; j += 256) out[j] = scl[j];
  __syncthreads();
  double* v = out + m + (int64_t)c * m;
  double ss = 0.0, best = -1.0, bval = 0.0;
  int bi = 0x7fffffff;
  for (int j = tid; j < m; j += 256) {
    double acc = 0.0;
    for (int64_t r = 0; r < n; ++r) acc = fma(svd_z(views, L, r, j) / scl[j], u[r], acc);
    v[j] = acc;
    ss = fma(acc, acc, ss);
    if (fabs(acc) > best) {  // j increases: the first index of this thread's maximum is kept
      best = fabs(acc);
      bi = j;
      bval = acc;
    }
  }
  ss = wave_sum_d(ss);
  for (int o = 32; o > 0; o >>= 1) {
    const double ob = __shfl_xor(best, o), ov = __shfl_xor(bval, o);
    const int oi = __shfl_xor(bi, o);
    if (ob > best || (ob == best && oi < bi)) {
      best = ob;
      bi = oi;
      bval = ov;
    }
  }
  if (lane == 0) {
    rsum[w] = ss;
    rbest[w] = best;
    rval[w] = bval;
    ridx[w] = bi;
  }
  __syncthreads();
  const double tot = (rsum[0] + rsum[1]) + (rsum[2] + rsum[3]);
  double gb = rbest[0], gv = rval[0];
  int gi = ridx[0];
  for (int q = 1; q < 4; ++q)
    if (rbest[q] > gb || (rbest[q] == gb && ridx[q] < gi)) {
      gb = rbest[q];
      gi = ridx[q];
      gv = rval[q];
    }
  const double f = (gv < 0.0 ? -1.0 : 1.0) / sqrt(tot);
  for (int j = tid; j < m; j += 256) v[j] *= f;
}


// ======================================== target transform of the ensemble mode
// (one block) ystats[3..5] = stats of float(YJ(y; lambda)); the translated borders
// YJ^-1(bz * s_t + m_t), repaired (tabpfn _cancel_nan_borders [ext]), and per common border
// (bz * s_y + m_y) its source bucket, share and flag (oracle preprocess_oracle.translation_table).
__device__ __forceinline__ double yj_inverse(double t, double lam) {
  constexpr double eps = 2.220446049250313e-16;
  if (t >= 0.0) return fabs(lam) < eps ? exp(t) - 1.0 : pow(t * lam + 1.0, 1.0 / lam) - 1.0;
  return fabs(lam - 2.0) > eps ? 1.0 - pow(-(2.0 - lam) * t + 1.0, 1.0 / (2.0 - lam)) : 1.0 - exp(-t);
}

__global__ __launch_bounds__(256) void k_target_tf(const float* __restrict__ y, int64_t ldy, int64_t n,
                                                   const float* __restrict__ bz, int nb,
                                                   const double* __restrict__ ylam, float* __restrict__ ystats,
                                                   TransEntry* __restrict__ tab, uint8_t* __restrict__ tcancel) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* frm = reinterpret_cast<float*>(smem);                       // [nb + 1]
  uint8_t* broken = reinterpret_cast<uint8_t*>(frm + nb + 1);        // [nb + 1]
  __shared__ double red[4];
  __shared__ int lohi[2];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const double lam = *ylam;
  auto bsum = [&](double a) -> double {
    a = wave_sum_d(a);
    __syncthreads();
    if (lane == 0) red[w] = a;
    __syncthreads();
    return red[0] + red[1] + red[2] + red[3];
  };
  double s1 = 0.0;
  for (int64_t i = tid; i < n; i += 256) s1 += (double)(float)yj_apply((double)y[i * ldy], lam);
  const double mean = bsum(s1) / (double)n;
  double s2 = 0.0;
  for (int64_t i = tid; i < n; i += 256) {
    const double d = (double)(float)yj_apply((double)y[i * ldy], lam) - mean;
    s2 += d * d;
  }
  const float tm = (float)mean;
  const float ts = (float)(sqrt(bsum(s2) / (double)n) + 1e-20);
  double z = 0.0;
  for (int64_t i = tid; i < n; i += 256) z += (double)(((float)yj_apply((double)y[i * ldy], lam) - tm) / ts);
  const double zbar = bsum(z) / (double)n;
  if (tid == 0) {
    ystats[3] = tm;
    ystats[4] = ts;
    ystats[5] = (float)zbar;
  }
  // source borders in f64 as numpy: (bz * ts) + tm, then the inverse transform; broken ones marked
  for (int b = tid; b <= nb; b += 256) {
    const double v = yj_inverse(__dadd_rn(__dmul_rn((double)bz[b], (double)ts), (double)tm), lam);
    const bool bad = !isfinite(v) || v > 1e3 || v < -1e3;
    broken[b] = bad ? 1 : 0;
    frm[b] = bad ? 0.f : (float)v;
  }
  __syncthreads();
  if (tid == 0) {
    int lo = 0, hi = nb;
    while (lo <= nb && broken[lo]) ++lo;
    while (hi >= 0 && broken[hi]) --hi;
    lohi[0] = lo;
    lohi[1] = hi;
  }
  __syncthreads();
  const int lo = lohi[0], hi = lohi[1];
  if (lo > nb) {  // every border broke: translation impossible, leave the bars as they are
    for (int b = tid; b <= nb; b += 256) tab[b] = TransEntry{min(b, nb - 1), b == nb ? 1.f : 0.f};
    for (int b = tid; b < nb; b += 256) tcancel[b] = 0;
    return;
  }
  // repair in f64 as the oracle, then round to f32: b[:lo] = b[lo], b[0] = b[1] - 1; b[hi+1:] = b[hi], b[-1] = b[-2] + 1
  // (frm holds the f32 rounding of good borders; the fills copy them, the +-1 ends round their sums)
  if (tid == 0) {
    const double vlo = (double)yj_inverse(__dadd_rn(__dmul_rn((double)bz[lo], (double)ts), (double)tm), lam);
    const double vhi = (double)yj_inverse(__dadd_rn(__dmul_rn((double)bz[hi], (double)ts), (double)tm), lam);
    for (int b = 0; b < lo; ++b) frm[b] = (float)vlo;
    if (lo > 0) frm[0] = (float)(vlo - 1.0);
    for (int b = hi + 1; b <= nb; ++b) frm[b] = (float)vhi;
    if (hi < nb) frm[nb] = (float)(vhi + 1.0);
  }
  __syncthreads();
  for (int b = tid; b < nb; b += 256) tcancel[b] = (broken[b] | broken[b + 1]) ? 1 : 0;
  for (int b = tid; b <= nb; b += 256) {
    const float to = __fadd_rn(__fmul_rn(bz[b], ystats[1]), ystats[0]);
    int l = 0, h = nb + 1;  // searchsorted(frm, to, left)
    while (l < h) {
      const int md = (l + h) >> 1;
      if (frm[md] < to) l = md + 1; else h = md;
    }
    const int idx = min(max(l - 1, 0), nb - 1);
    const float wd = __fsub_rn(frm[idx + 1], frm[idx]);
    float sh = __fdiv_rn(__fsub_rn(to, frm[idx]), wd);
    sh = fminf(fmaxf(sh, 0.f), 1.f);
    tab[b] = TransEntry{idx, to <= frm[0] ? -1.f : (to >= frm[nb] ? 2.f : sh)};
  }
}

// ================================================================ K1 encoder
// tokens [E][R][C][d]: resid fp32 + bf16 copy.  One wave per token; features come from the
// views table through the estimator's shuffled column list (k_build_params).
// U32: the launch's tokens < 2^32, so (estimator, row, token) come from FastDiv (the 64-bit
// divisions bound the kernel: r04 ran it at ~2 TB/s of stores); else 64-bit division.
#ifndef NPFN_ENC_SPEC  // 1: feature loads ahead of Fe (r05: k_encode 3.53 -> 3.37 ms, bitwise equal,
#define NPFN_ENC_SPEC 1  // profiles/r05/ab_encode_spec_r05bd.txt); 0: loads behind the j < Fe test
#endif
template <bool U32>
__device__ __forceinline__ void encode_token(int64_t tok, const float* __restrict__ ytr, int64_t ldy, int64_t R,
                                             const DevFit& fp, const float* __restrict__ encw,
                                             const float* __restrict__ yencw, const float* __restrict__ pos,
                                             float* __restrict__ resid, bf16_t* __restrict__ resid_bf,
                                             const FastDiv& divC, const FastDiv& divR) {
  const int lane = threadIdx.x & 63;
  const int C = fp.C;
  int c, ei;
  int64_t r;
  if constexpr (U32) {  // tok is wave-uniform: the decomposition runs once per wave
    uint32_t cu, ru;
    const uint32_t rr = divC.divmod((uint32_t)tok, cu);
    ei = (int)divR.divmod(rr, ru);
    c = (int)cu;
    r = ru;
  } else {
    c = (int)(tok % C);
    const int64_t rr = tok / C;
    r = rr % R;
    ei = (int)(rr / R);
  }
  const int e = fp.e0 + fp.es * ei;  // global estimator index (tables, preprocessing view)
  float a0, a1, a2, a3;
  const bool target = (c == fp.G);
  // the output weights and positional row are loaded before the feature gather's dependent chain
  // (eF / vcol -> views), so their latency overlaps it
  float w[3][4], pw[3];
  {
    const int cp = target ? 0 : c;
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      const int dd = lane + 64 * q;
      if (!target) {
        const float4 w4 = *reinterpret_cast<const float4*>(encw + dd * 4);
        w[q][0] = w4.x; w[q][1] = w4.y; w[q][2] = w4.z; w[q][3] = w4.w;
      } else {
        const float2 w2 = *reinterpret_cast<const float2*>(yencw + dd * 2);
        w[q][0] = w2.x; w[q][1] = w2.y; w[q][2] = w[q][3] = 0.f;
      }
      pw[q] = target ? 0.f : pos[cp * 192 + dd];
    }
  }
  if (!target) {
    float v[2], ind[2];
    const int Fe = fp.eF[e];
#if NPFN_ENC_SPEC
    // the feature loads are issued before Fe is known (index clamped into the tables, the
    // view column into the row), so the chain is (eF | vcol, mu, sd) -> views, not eF -> vcol -> views
    float xs[2], ms[2], ss[2];
    {
      const int64_t eb = (int64_t)e * fp.Fmax;
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int jj = min(2 * c + q, fp.Fmax - 1);
        const int vc = min(max(fp.vcol[eb + jj], 0), fp.Vw - 1);
        xs[q] = fp.views[r * fp.Vw + vc];
        ms[q] = fp.mu[eb + jj];
        ss[q] = fp.sd[eb + jj];
      }
    }
#endif
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int j = 2 * c + q;
      v[q] = 0.f; ind[q] = 0.f;
      if (j < Fe) {
#if NPFN_ENC_SPEC
        float x = xs[q];
        const float m = ms[q];
        const float s = ss[q];
#else
        float x = fp.views[r * fp.Vw + fp.vcol[(int64_t)e * fp.Fmax + j]];
        const float m = fp.mu[(int64_t)e * fp.Fmax + j];
        const float s = fp.sd[(int64_t)e * fp.Fmax + j];
#endif
        if (!isfinite(x)) {
          ind[q] = isnan(x) ? -2.0f : (x > 0.f ? 2.0f : 4.0f);
          x = m;
        }
        float xn = (x - m) / (s + 1e-16f);
        xn = fminf(fmaxf(xn, -100.f), 100.f);
        v[q] = xn * fp.gscale[(int64_t)e * fp.Gmax + c];
      }
    }
    a0 = v[0]; a1 = v[1]; a2 = ind[0]; a3 = ind[1];
  } else if (fp.ncls > 0) {  // classifier: permuted label index / train mean of it
    if (ytr != nullptr) {
      const int cl = min(max((int)ytr[r * ldy], 0), fp.ncls - 1);
      a0 = (float)fp.cperm[e * KMAX_CLS + cl];
      a1 = 0.f;
    } else {
      a0 = fp.ybar_e[e];
      a1 = -2.0f;
    }
    a2 = a3 = 0.f;
  } else {
    const int tt = fp.ett[e];
    const float* st = fp.ystats + 3 * tt;
    if (ytr != nullptr) {
      float yv = ytr[r * ldy];
      if (tt) yv = (float)yj_apply((double)yv, *fp.ylam);
      a0 = (yv - st[0]) / st[1];
      a1 = 0.f;
    } else {
      a0 = st[2];
      a1 = -2.0f;
    }
    a2 = a3 = 0.f;
  }
  const int64_t base = tok * 192;
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    const int dd = lane + 64 * q;
    float o;
    // explicit fma order: w0 a0 + w1 a1 + w2 a2 + w3 a3 + pos as the contracted expression
    // evaluates (the first product fused onto the rounded second)
    const float s01 = __fmaf_rn(w[q][0], a0, w[q][1] * a1);
    if (!target) {
      o = __fmaf_rn(w[q][3], a3, __fmaf_rn(w[q][2], a2, s01)) + pw[q];
    } else {
      o = s01;
    }
    resid[base + dd] = o;
    if (resid_bf) resid_bf[base + dd] = f2bf(o);  // null: the fused path (k_row_layer reads resid)
  }
}

// One wave per token, one workgroup per 4 tokens (r05: a grid-stride form with 4096 / 1024
// workgroups was 41 % slower -- fewer stores in flight -- profiles/r05/ab_encode_grid_r05w.txt;
// one 16-byte store per lane on lanes 0..47 instead of three 4-byte stores per lane, bitwise
// equal, 12 % slower -- profiles/r05/ab_encode_wide_store_r05ad.txt; the output weights and
// positional row loaded before the feature gather's dependent chain: 4.10 -> 3.65 ms per c2 call,
// bitwise equal once the fma order is written out -- profiles/r05/ab_encode_preload_r05as.txt)
template <bool U32>
__global__ __launch_bounds__(256) void k_encode(const float* __restrict__ ytr, int64_t ldy, int64_t R, DevFit fp,
                                                const float* __restrict__ encw, const float* __restrict__ yencw,
                                                const float* __restrict__ pos, float* __restrict__ resid,
                                                bf16_t* __restrict__ resid_bf, FastDiv divC, FastDiv divR) {
  const int64_t tok = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (tok < (int64_t)fp.E * R * fp.C)
    encode_token<U32>(tok, ytr, ldy, R, fp, encw, yencw, pos, resid, resid_bf, divC, divR);
}

// ========================================================== K5 GEMM + epilogues
// C[M,N] = A[M,K] (bf16, row stride lda) x W[N,K]^T (bf16), fp32 accumulation.
// Tile 64 x 192, BK 64, 4 waves (2x2, 32 x 96 per wave), MFMA 16x16x32 bf16,
// register-staged double-buffered LDS with a 16-byte XOR swizzle.
// MT = rows per tile: 64 (4 waves) or 128 (8 waves, the decoder head: half the weight-tile
// traffic per flop).  Waves tile the block as (MT/32) x 2 of 32 x 96.
#ifndef NPFN_GEMM_STAGED
#define NPFN_GEMM_STAGED 1
#endif
constexpr bool kGemmStagedF32 = NPFN_GEMM_STAGED != 0;
// WM = rows per wave (32, or 64 for the decoder head: 4 A + 6 B fragment reads per 24 MFMAs
// instead of 2 + 6 per 12 -- the same per-element K order, so the same bits).
template <int EPI, int MT = 64, int WM = 32>
__global__ __launch_bounds__((MT / WM) * 128) void k_gemm(const bf16_t* __restrict__ A, int64_t lda,
                                                          const bf16_t* __restrict__ W, int64_t M, int N, int K,
                                                          EpiParams p) {
  static_assert(MT == 64 || MT == 128 || MT == 256, "k_gemm: MT must be 64, 128 or 256");
  static_assert(WM == 32 || WM == 64, "k_gemm: WM must be 32 or 64");
  static_assert(EPI != EPI_LN || (MT == 64 && WM == 32), "k_gemm: the LayerNorm epilogue assumes 64-row tiles");
  constexpr int NT = (MT / WM) * 128;            // threads: (MT / WM) x 2 waves
  constexpr int IM = WM / 16;                    // 16-row MFMA blocks per wave
  constexpr int NA = MT * 8 / NT;                // A-tile uint4 per thread (MT rows x 8)
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16_t* As = reinterpret_cast<bf16_t*>(smem);  // [2][MT*64]
  bf16_t* Bs = As + 2 * MT * 64;                 // [2][192*64]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int64_t m0 = (int64_t)blockIdx.x * MT;
  const int n0 = blockIdx.y * 192;
  f32x4 acc[IM][6];
#pragma unroll
  for (int i = 0; i < IM; ++i)
#pragma unroll
    for (int j = 0; j < 6; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  constexpr int NB = (1536 + NT - 1) / NT;       // B-tile uint4 per thread (192 rows x 8)
  uint4 ra[NA], rb[NB];
  auto gload = [&](int k0) {
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const int q = tid + i * NT, row = q >> 3, kc = q & 7;
      const int64_t gm = m0 + row;
      // (r05: loading row min(gm, M - 1) without the branch, same for W: decoder GEMM 6.6 -> 24.5 ms,
      // bitwise equal; profiles/r05/ab_gemm_clamp_r05bb.txt)
      ra[i] = (gm < M) ? *reinterpret_cast<const uint4*>(A + gm * lda + k0 + kc * 8) : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      const int q = tid + i * NT, row = q >> 3, kc = q & 7;
      const int gn = n0 + row;
      rb[i] = (gn < N && q < 1536) ? *reinterpret_cast<const uint4*>(W + (int64_t)gn * K + k0 + kc * 8) : make_uint4(0, 0, 0, 0);
    }
  };
  auto sstore = [&](int buf) {
    bf16_t* a = As + buf * (MT * 64);
    bf16_t* b = Bs + buf * 12288;
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const int q = tid + i * NT, row = q >> 3, kc = q & 7;
      *reinterpret_cast<uint4*>(a + row * 64 + ((kc ^ (row & 7)) << 3)) = ra[i];
    }
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      const int q = tid + i * NT, row = q >> 3, kc = q & 7;
      if (NT * NB == 1536 || q < 1536) *reinterpret_cast<uint4*>(b + row * 64 + ((kc ^ (row & 7)) << 3)) = rb[i];
    }
  };
  const int nk = K >> 6;
  gload(0);
  sstore(0);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < nk) gload((kt + 1) * 64);
    const bf16_t* a = As + buf * (MT * 64);
    const bf16_t* b = Bs + buf * 12288;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int kc = kk * 4 + (lane >> 4);
      bf16x8 af[IM], bfr[6];
#pragma unroll
      for (int im = 0; im < IM; ++im) {
        const int row = wm * WM + im * 16 + (lane & 15);
        af[im] = *reinterpret_cast<const bf16x8*>(a + row * 64 + ((kc ^ (row & 7)) << 3));
      }
#pragma unroll
      for (int in = 0; in < 6; ++in) {
        const int n = wn * 96 + in * 16 + (lane & 15);
        bfr[in] = *reinterpret_cast<const bf16x8*>(b + n * 64 + ((kc ^ (n & 7)) << 3));
      }
#pragma unroll
      for (int im = 0; im < IM; ++im)
#pragma unroll
        for (int in = 0; in < 6; ++in)
          acc[im][in] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[im], bfr[in], acc[im][in], 0, 0, 0);
    }
    if (kt + 1 < nk) sstore(buf ^ 1);
    __syncthreads();
  }

  if constexpr (EPI == EPI_LN) {
    // out = LN(resid + acc) * g + b ; N == 192, gridDim.y == 1
    float* tile = reinterpret_cast<float*>(smem);  // [64][196]
#pragma unroll
    for (int im = 0; im < 2; ++im)
#pragma unroll
      for (int in = 0; in < 6; ++in)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int row = wm * 32 + im * 16 + (lane >> 4) * 4 + i;
          const int col = wn * 96 + in * 16 + (lane & 15);
          tile[row * 196 + col] = acc[im][in][i];
        }
    __syncthreads();
    for (int rr = 0; rr < 16; ++rr) {
      const int row = wave * 16 + rr;
      const int64_t gm = m0 + row;
      if (gm >= M) break;
      float v[3];
      float s = 0.f;
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        const int col = lane + 64 * q;
        v[q] = tile[row * 196 + col] + p.resid[gm * 192 + col];
        s += v[q];
      }
      const float mean = wave_sum(s) * (1.0f / 192.0f);
      float s2 = 0.f;
#pragma unroll
      for (int q = 0; q < 3; ++q) { v[q] -= mean; s2 += v[q] * v[q]; }
      const float var = wave_sum(s2) * (1.0f / 192.0f);
      const float rstd = 1.0f / sqrtf(var + 1e-5f);
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        const int col = lane + 64 * q;
        const float o = v[q] * rstd * p.ln_g[col] + p.ln_b[col];
        p.resid[gm * 192 + col] = o;
        p.resid_bf[gm * 192 + col] = f2bf(o);
      }
    }
  } else if (EPI == EPI_LOGIT && MT >= 128 && kGemmStagedF32) {
    // decoder logits: the accumulators go through LDS in two 64-row halves so that every
    // store is a 16-byte piece of a contiguous 768-byte row segment (the MFMA layout would
    // store 4-byte columns of 4 rows per instruction)
    float* tile = reinterpret_cast<float*>(smem);  // [64][196] (the K loop's buffers are free)
    const int ncol = min(192, N - n0);
    constexpr int RPW = 64 / (NT / 64);  // rows of the half each wave stores
#pragma unroll
    for (int half = 0; half < MT / 64; ++half) {  // 64-row pieces of the tile
      if (half) __syncthreads();  // the previous piece's rows are stored
      if ((wm * WM) / 64 == half) {
#pragma unroll
        for (int im = 0; im < IM; ++im)
#pragma unroll
          for (int in = 0; in < 6; ++in)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              const int row = (wm * WM) % 64 + im * 16 + (lane >> 4) * 4 + i;
              const int col = wn * 96 + in * 16 + (lane & 15);
              tile[row * 196 + col] = acc[im][in][i];
            }
      }
      __syncthreads();
      // wave w stores rows w*RPW .. of the half: lanes 0..47 one float4 each
      if (lane < 48 && lane * 4 < ncol) {
        const int c4 = lane * 4;
        f32x4 bias4;
#pragma unroll
        for (int i = 0; i < 4; ++i) bias4[i] = (p.bias != nullptr && c4 + i < ncol) ? p.bias[n0 + c4 + i] : 0.f;
#pragma unroll
        for (int rr = 0; rr < RPW; ++rr) {
          const int row = wave * RPW + rr;
          const int64_t gm = m0 + half * 64 + row;
          if (gm >= M) break;
          const f32x4 v = *reinterpret_cast<const f32x4*>(tile + row * 196 + c4) + bias4;
          logit_t* dst = p.out_l + gm * p.ldo + n0 + c4;
          typedef logit_t lg4 __attribute__((ext_vector_type(4)));
          if (c4 + 4 <= ncol && ((p.ldo | n0) & 3) == 0) {
            *reinterpret_cast<lg4*>(dst) = __builtin_convertvector(v, lg4);
          } else {
            for (int i = 0; i < 4 && c4 + i < ncol; ++i) dst[i] = (logit_t)v[i];
          }
        }
      }
    }
  } else {
#pragma unroll
    for (int im = 0; im < IM; ++im)
#pragma unroll
      for (int in = 0; in < 6; ++in) {
        const int col = n0 + wn * 96 + in * 16 + (lane & 15);
        if (col >= N) continue;
        const float bias = (p.bias != nullptr) ? p.bias[col] : 0.f;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int64_t row = m0 + wm * WM + im * 16 + (lane >> 4) * 4 + i;
          if (row >= M) continue;
          float v = acc[im][in][i] + bias;
          if constexpr (EPI == EPI_BF16_GELU) v = gelu_fast(v);
          if constexpr (EPI == EPI_LOGIT) {
            p.out_l[row * p.ldo + col] = (logit_t)v;
          } else {
            p.out_bf[row * p.ldo + col] = f2bf(v);
          }
        }
      }
  }
}

// ===================================================== K2 feature attention
// One wave per row: the row's C tokens attend to each other (6 heads x 32).
// qkv [rows][C][576] bf16 -> out [rows][C][192] bf16.
__global__ __launch_bounds__(64) void k_feat_attn(const bf16_t* __restrict__ qkv,
                                                  bf16_t* __restrict__ out, int64_t rows, int C,
                                                  float scale) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16_t* s = reinterpret_cast<bf16_t*>(smem);
  const int64_t row = blockIdx.x;
  const int lane = threadIdx.x;
  const bf16_t* src = qkv + row * (int64_t)C * 576;
  const int nchunk = C * 576 / 8;
  for (int i = lane; i < nchunk; i += 64)
    reinterpret_cast<uint4*>(s)[i] = reinterpret_cast<const uint4*>(src)[i];
  __syncthreads();
  for (int pidx = lane; pidx < C * 6; pidx += 64) {
    const int t = pidx / 6, h = pidx - t * 6;
    float q[32], o[32];
    const bf16_t* qp = s + t * 576 + h * 32;
#pragma unroll
    for (int dd = 0; dd < 32; ++dd) { q[dd] = bf2f(qp[dd]) * scale; o[dd] = 0.f; }
    float m = -INFINITY, l = 0.f;
    for (int t2 = 0; t2 < C; ++t2) {
      const bf16_t* kp = s + t2 * 576 + 192 + h * 32;
      const bf16_t* vp = s + t2 * 576 + 384 + h * 32;
      float sc = 0.f;
#pragma unroll
      for (int dd = 0; dd < 32; ++dd) sc += q[dd] * bf2f(kp[dd]);
      const float mn = fmaxf(m, sc);
      const float alpha = __expf(m - mn);
      const float pp = __expf(sc - mn);
      l = l * alpha + pp;
#pragma unroll
      for (int dd = 0; dd < 32; ++dd) o[dd] = o[dd] * alpha + pp * bf2f(vp[dd]);
      m = mn;
    }
    const float inv = 1.0f / l;
    bf16_t* op = out + (row * C + t) * 192 + h * 32;
#pragma unroll
    for (int dd = 0; dd < 32; dd += 2)
      *reinterpret_cast<uint32_t*>(op + dd) = pack_bf2(o[dd] * inv, o[dd + 1] * inv);
  }
}

// Long rows (wide tables, C > kFeatAttnMaxC): one block per (row, head) with the head's K | V of
// the row in LDS ([C][64] bf16, 128 B per token); thread t runs queries t, t + 256, ... with
// k_feat_attn's arithmetic (same score sum order, online softmax over keys 0 .. C - 1).
__global__ __launch_bounds__(256) void k_feat_attn_wide(const bf16_t* __restrict__ qkv, bf16_t* __restrict__ out,
                                                        int64_t rows, int C, float scale) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16_t* kv = reinterpret_cast<bf16_t*>(smem);
  const int64_t row = blockIdx.x / 6;
  const int h = (int)(blockIdx.x - row * 6);
  const bf16_t* src = qkv + row * (int64_t)C * 576;
  for (int i = threadIdx.x; i < C * 8; i += 256) {  // per token: 4 x 16 B of K, then 4 x 16 B of V
    const int t = i >> 3, j = i & 7;
    reinterpret_cast<uint4*>(kv)[i] =
        *reinterpret_cast<const uint4*>(src + (int64_t)t * 576 + (j < 4 ? 192 : 384) + h * 32 + (j & 3) * 8);
  }
  __syncthreads();
  for (int t = threadIdx.x; t < C; t += 256) {
    float q[32], o[32];
    const bf16_t* qp = src + (int64_t)t * 576 + h * 32;
#pragma unroll
    for (int dd = 0; dd < 32; ++dd) { q[dd] = bf2f(qp[dd]) * scale; o[dd] = 0.f; }
    float m = -INFINITY, l = 0.f;
    for (int t2 = 0; t2 < C; ++t2) {
      const bf16_t* kp = kv + t2 * 64;
      const bf16_t* vp = kp + 32;
      float sc = 0.f;
#pragma unroll
      for (int dd = 0; dd < 32; ++dd) sc += q[dd] * bf2f(kp[dd]);
      const float mn = fmaxf(m, sc);
      const float alpha = __expf(m - mn);
      const float pp = __expf(sc - mn);
      l = l * alpha + pp;
#pragma unroll
      for (int dd = 0; dd < 32; ++dd) o[dd] = o[dd] * alpha + pp * bf2f(vp[dd]);
      m = mn;
    }
    const float inv = 1.0f / l;
    bf16_t* op = out + (row * C + t) * 192 + h * 32;
#pragma unroll
    for (int dd = 0; dd < 32; dd += 2)
      *reinterpret_cast<uint32_t*>(op + dd) = pack_bf2(o[dd] * inv, o[dd + 1] * inv);
  }
}

// ===================================================== K3/K4 item attention
// Packed K/V cache per (e, c, head): tiles of 32 keys, 2048 bf16 per tile:
//   K: [s 0..1][h2 0..1][key 0..31][8]  = K[key][16s + 8h2 + j]
//   V: [s][h2][d 0..31][8]              = V[16s + 8(j>>2) + 4h2 + (j&3)][d]
// so that every MFMA operand fragment is one contiguous 1 KiB wave load.
// One wave per 32-key tile of one (e, c, head) stream, 4 tiles per block.  k: each output chunk
// is 16 contiguous bytes of a key's row (2 per lane).  v: the tile's 32 keys x 32 dims are
// read as 16-byte row pieces into an LDS image (2 per lane) and every output chunk (8 keys of one
// dim) is gathered from there -- not 8 scattered 2-byte global loads.  Keys >= n are zeros.
// U32: the launch's tiles < 2^32 -- (estimator, column, head, tile) from FastDiv; else 64-bit
template <bool U32>
__global__ __launch_bounds__(256) void k_kv_pack(const bf16_t* __restrict__ qkv, int64_t n, int C,
                                                 int E, int ntile, bf16_t* __restrict__ kvc, int c_lo,
                                                 FastDiv divT, FastDiv divNC) {
  __shared__ bf16_t vimg[4][32][40];  // per wave: [key][dim], rows padded to 80 bytes
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t tile = (int64_t)blockIdx.x * 4 + wave;
  const int nc = C - c_lo;  // the columns packed: [c_lo, C)
  if (tile >= (int64_t)E * nc * 6 * ntile) return;  // wave-uniform
  int t, h, c, e;
  // tile = ((e * nc + c) * ntile + t) * 6 + h: the 6 heads of one key tile are neighbouring waves, so a
  // key row's K|V bytes are read close together in time (r05: head-slowest order 6.05 -> 5.68 ms per c2 call)
  // (2 or 6 waves per block instead of 4: 5.76 / 5.79 vs 5.70 ms, profiles/r05/ab_kv_waves_r05av.txt)
  if constexpr (U32) {
    uint32_t tu, cu;
    const uint32_t rest = (uint32_t)tile / 6u;  // a constant divisor: the compiler's multiply-shift
    h = (int)((uint32_t)tile - rest * 6u);
    const uint32_t rest2 = divT.divmod(rest, tu);
    e = (int)divNC.divmod(rest2, cu);
    t = (int)tu;
    c = c_lo + (int)cu;
  } else {
    int64_t rest = tile;
    h = (int)(rest % 6); rest /= 6;
    t = (int)(rest % ntile); rest /= ntile;
    c = c_lo + (int)(rest % nc); rest /= nc;
    e = (int)rest;
  }
  bf16_t* dst = kvc + ((((int64_t)e * C + c) * 6 + h) * ntile + t) * 2048;
  auto row = [&](int key) { return qkv + (((int64_t)e * n + (int64_t)t * 32 + key) * C + c) * 576; };
  const bool ok0 = (int64_t)t * 32 + (lane & 31) < n;
#pragma unroll
  for (int i = 0; i < 2; ++i) {  // k chunks ch = lane + 64 i: s = ch >> 6, h2 = (ch >> 5) & 1, key = ch & 31
    const int ch = lane + 64 * i, s = ch >> 6, h2 = (ch >> 5) & 1;
    uint4 v = make_uint4(0, 0, 0, 0);
    if (ok0) v = *reinterpret_cast<const uint4*>(row(ch & 31) + 192 + h * 32 + 16 * s + 8 * h2);
    *reinterpret_cast<uint4*>(dst + ch * 8) = v;
  }
#pragma unroll
  for (int i = 0; i < 2; ++i) {  // v rows: key = lane & 31, dims 8 (2 i + (lane >> 5)) .. + 7
    const int q = 2 * i + (lane >> 5);
    uint4 v = make_uint4(0, 0, 0, 0);
    if (ok0) v = *reinterpret_cast<const uint4*>(row(lane & 31) + 384 + h * 32 + 8 * q);
    *reinterpret_cast<uint4*>(&vimg[wave][lane & 31][8 * q]) = v;
  }
  // (LDS instructions of one wave complete in order: the image is complete for every lane here)
#pragma unroll
  for (int i = 0; i < 2; ++i) {  // v chunks cv = lane + 64 i: [s][h2][d][8], key 16 s + 8 (j >> 2) + 4 h2 + (j & 3)
    const int cv = lane + 64 * i, s = cv >> 6, h2 = (cv >> 5) & 1, d = cv & 31;
    bf16_t tmp[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) tmp[j] = vimg[wave][16 * s + 8 * (j >> 2) + 4 * h2 + (j & 3)][d];
    *reinterpret_cast<uint4*>(dst + 1024 + cv * 8) = *reinterpret_cast<const uint4*>(tmp);
  }
}

// Flash-style item attention with the key on the MFMA row ("swapped" QK^T):
// S^T = K Q^T and O^T += V^T P^T on v_mfma_f32_32x32x16_bf16, so the softmax
// over keys is lane-local, and P^T feeds the PV MFMA as its B operand straight from the
// accumulator registers.  Each step takes two 32-key tiles (64 keys) behind one barrier:
// per 32-query set 4 independent QK^T MFMAs, 32 exp2, 4 PV MFMAs and the row sums as packed
// f32 adds on the VALU (as ones^T P^T MFMAs they took a third of the matrix pipe and were
// 2.2 % slower); the 1/sqrt(32) and log2(e) scale is folded into q.
//
// Reference-free softmax.  softmax(s) = exp2(s - c) / sum exp2(s - c) for ANY constant c;
// the online max only keeps exp2 inside the float range.  With head dim 32 the max is a
// third of the VALU issue of a step (hd 32 gives each score only 128 MFMA flops), so the
// first pass takes c = 0: P = exp2(s) straight from the QK^T accumulator, no max, no
// rescale.  That is exact (bf16 P and f32 sums are relative-precision formats, so the scale
// changes no rounding that matters) as long as every exp2 stays finite and the sum is neither
// tiny nor huge (each query checks 2^-100 <= l <= 2^100 at the end).  Against a uniform score
// level -- the case that broke it at moderately scaled scores (r04) -- the first step also takes
// each query's max over its first 32 keys: a query whose max lies outside [kIaShiftLo,
// kIaShiftHi] gets that max + 60 as its own reference c, and a query set holding such a query
// subtracts its lanes' references from every score from then on (a wave-uniform branch per set;
// exactly S - 0 = S for the set's other queries, so a row's result never depends on its
// wave-mates).  Its sum is then >= 2^-60 (its max key) and only a spread of more than ~160
// log2 units (e^110) between the first 32 keys' max and the others' fails.  What still fails
// re-runs with the classic online softmax (IA_ONLINE: running max subtracted from S, rescale
// deferred until the max grows by 2^8 -- cdna guide T13), whose result only the failing queries
// take.  The padding keys of the last step (packed as K = V = 0) are masked to P = 0 in both
// passes.  The first and the last step are instances of their own, so the steady-state loop
// carries neither the max nor the mask.
// One wave = kIaQs sets of 32 query rows of one (estimator, column, head); 4 waves / block.
// The sets share every K/V fragment read, barrier and DMA of a step, and their independent
// MFMA -> exp2 -> MFMA chains interleave (the kernel is bound by VALU issue and dependency
// waits, not by the matrix pipe).
constexpr float kDeferLog2 = 8.0f;
// first-step max (log2 units) above / below which a query gets its own reference
// (r05 stress sweeps, profiles/r05/ia_stress_*: hi 16 / lo -64 / margin 60 keep the fallback under
// 0.01 % of rows at score scale x16 and c2 at 0.91x of its clean rate at x48)
constexpr float kIaShiftHi = 16.0f, kIaShiftLo = -64.0f, kIaShiftMargin = 60.0f;

constexpr int kIaPairs = 3;  // K/V ring depth in 64-key steps (one in flight beside the one read; r02: 4 equal)
#ifndef NPFN_IA_QSETS
#define NPFN_IA_QSETS 2
#endif
constexpr int kIaQs = NPFN_IA_QSETS;
static_assert(kIaQs >= 1 && kIaQs <= 4, "1 to 4 query sets per wave");

enum { IA_FIRST = 0, IA_ONLINE = 2 };

// MODE IA_FIRST: every set; out: cref (the lane's reference, 0 where its first-32-key max lies
// inside the band).  IA_ONLINE: only the sets with todo (wave-uniform); a wave with none still
// streams its share of the K/V ring and meets every barrier, but issues no math.
template <int MODE>
__device__ __forceinline__ void item_attn_pass(bf16_t (*ring)[2048], const bf16_t* kvseg, uint32_t seg_lds,
                                               int ntile, int64_t n, const bf16x8 (&qf)[kIaQs][2],
                                               f32x16 (&o)[kIaQs], float (&lsum)[kIaQs],
                                               const bool (&todo)[kIaQs], float (&cref)[kIaQs]) {
  constexpr bool ONLINE = MODE == IA_ONLINE, SEL = MODE != IA_FIRST;
  bool any_todo = !SEL;
#pragma unroll
  for (int qs = 0; qs < kIaQs; ++qs) any_todo |= todo[qs];
  const int lane = threadIdx.x & 63, h2 = lane >> 5;
  f32x2 lacc2[kIaQs][2];  // the lane's partial row sums (its 16 keys of a tile)
#pragma unroll
  for (int qs = 0; qs < kIaQs; ++qs) {
    lacc2[qs][0] = f32x2{0.f, 0.f};
    lacc2[qs][1] = f32x2{0.f, 0.f};
  }
  const int npair = ntile >> 1;  // ntile is a multiple of 2 (npfn_engine.hip fit_prep)
  // step p = tiles 2p, 2p+1 into ring slots 2 slot(p) +{0, 1}: exactly 2 DMAs per step, one step
  // behind each barrier, the ring kIaPairs steps deep
  auto slot_of = [](int p) { return p % kIaPairs; };
  auto issue_pair = [&](int p) {
    const uint32_t dst = seg_lds + (uint32_t)(slot_of(p) * 8192);
    glds16(kvseg + (int64_t)(2 * p) * 2048, dst);
    glds16(kvseg + (int64_t)(2 * p + 1) * 2048, dst + 4096u);
  };
  issue_pair(0);
  if (npair > 1) issue_pair(1);
#pragma unroll
  for (int qs = 0; qs < kIaQs; ++qs)
#pragma unroll
    for (int i = 0; i < 16; ++i) o[qs][i] = 0.f;
  // ONLINE: m = running max (log2 domain) of this lane's query; P = exp2(S - m) (the rare
  // fallback subtracts on the VALU: no bias accumulators, so the kernel's register count is
  // the first pass's)
  float m[kIaQs];
#pragma unroll
  for (int qs = 0; qs < kIaQs; ++qs) m[qs] = -INFINITY;
  const f32x16 zero = {};
  const bool ragged = (int64_t)ntile * 32 != n;  // the cache holds padding keys (any tile quantum)
  bool shifted[kIaQs];  // IA_FIRST: the set holds a lane with a reference (wave-uniform)
#pragma unroll
  for (int qs = 0; qs < kIaQs; ++qs) shifted[qs] = false;
  auto step = [&](int p, auto first_c, auto last_c) {
    constexpr bool FIRST = decltype(first_c)::value, LAST = decltype(last_c)::value;
    // step p landed for this wave (p+1 may stay in flight), then for all waves
    if (p + 1 < npair) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    lds_barrier();
    // refill the slots every wave finished with (step p-1's) with step p+2
    if (p + 2 < npair) issue_pair(p + 2);
    if (SEL && !any_todo) return;
    const bf16_t* ta = &ring[2 * slot_of(p)][lane * 8];
    const bf16_t* tb = ta + 2048;
    const bf16x8 ka0 = *reinterpret_cast<const bf16x8*>(ta);
    const bf16x8 ka1 = *reinterpret_cast<const bf16x8*>(ta + 512);
    const bf16x8 kb0 = *reinterpret_cast<const bf16x8*>(tb);
    const bf16x8 kb1 = *reinterpret_cast<const bf16x8*>(tb + 512);
    f32x16 sa[kIaQs], sb[kIaQs];
#pragma unroll
    for (int qs = 0; qs < kIaQs; ++qs) {
      if (SEL && !todo[qs]) continue;
      sa[qs] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ka0, qf[qs][0], zero, 0, 0, 0);
      sb[qs] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kb0, qf[qs][0], zero, 0, 0, 0);
    }
#pragma unroll
    for (int qs = 0; qs < kIaQs; ++qs) {
      if (SEL && !todo[qs]) continue;
      sa[qs] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ka1, qf[qs][1], sa[qs], 0, 0, 0);
      sb[qs] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kb1, qf[qs][1], sb[qs], 0, 0, 0);
    }
    const bf16x8 va0 = *reinterpret_cast<const bf16x8*>(ta + 1024);
    const bf16x8 va1 = *reinterpret_cast<const bf16x8*>(ta + 1536);
    const bf16x8 vb0 = *reinterpret_cast<const bf16x8*>(tb + 1024);
    const bf16x8 vb1 = *reinterpret_cast<const bf16x8*>(tb + 1536);
    if constexpr (MODE == IA_FIRST && FIRST) {  // the lane's reference: its query's max over the first 32 keys
#pragma unroll
      for (int qs = 0; qs < kIaQs; ++qs) {
        float tmax = fmaxf(sa[qs][0], sa[qs][15]);  // compiler-visible first read (MFMA hazard)
#pragma unroll
        for (int i = 1; i < 15; i += 2) tmax = max3f(tmax, sa[qs][i], sa[qs][i + 1]);
        tmax = xor32_max(tmax);
        // headroom: the reference sits kIaShiftMargin above that max, so the lane's sum stays >=
        // 2^-kIaShiftMargin (>> 2^-100) and the other keys may exceed the max by ~100 + the margin;
        // a key more than ~66 log2 units under the max (flushed by exp2) weighs < 2^-66 of it
        cref[qs] = (tmax > kIaShiftHi || tmax < kIaShiftLo) ? tmax + kIaShiftMargin : 0.f;
        shifted[qs] = __ballot(cref[qs] != 0.f) != 0ull;
      }
    }
    if constexpr (LAST) {
      if (ragged) {  // the last step holds the padding keys (< 64 of them): P = 0 for them
        // the lane's keys of tile a are p 64 + 4 h2 + off_i (off_i = (i & 3) + 8 (i >> 2)), of
        // tile b 32 more; rem = the lane's real keys left in tile a's numbering
        const int rem = (int)(n - ((int64_t)p * 64 + 4 * h2));
        const bool a_pad = (int64_t)p * 64 + 32 > n;  // wave-uniform: tile a holds padding (b is all padding)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int off = (i & 3) + 8 * (i >> 2);
#pragma unroll
          for (int qs = 0; qs < kIaQs; ++qs) {
            if (a_pad) {
              if (off >= rem) sa[qs][i] = -INFINITY;
              sb[qs][i] = -INFINITY;
            } else if (off + 32 >= rem) {
              sb[qs][i] = -INFINITY;
            }
          }
        }
      }
    }
#pragma unroll
    for (int qs = 0; qs < kIaQs; ++qs) {
      if (SEL && !todo[qs]) continue;
      if constexpr (ONLINE) {
        // the first reads of the QK^T accumulators are compiler-visible fmaxf: the hazard
        // recognizer puts the MFMA read-after-write wait states in front of them (it cannot
        // see into max3f's asm, which read stale registers when it came first)
        float tmax = fmaxf(fmaxf(sa[qs][0], sb[qs][0]), fmaxf(sa[qs][15], sb[qs][15]));
#pragma unroll
        for (int i = 1; i < 15; ++i) tmax = max3f(tmax, sa[qs][i], sb[qs][i]);
        tmax = xor32_max(tmax);  // step max of the lane's query
        // only the queries whose max grew past the deferral margin move their reference; the
        // others scale by exactly 1, so a query's result never depends on its wave-mates
        const bool up = tmax > m[qs] + kDeferLog2;
        if (__ballot(up) != 0ull) {
          const float alpha = up ? __builtin_amdgcn_exp2f(m[qs] - tmax) : 1.0f;
#pragma unroll
          for (int i = 0; i < 16; ++i) o[qs][i] *= alpha;
          lacc2[qs][0] *= alpha;
          lacc2[qs][1] *= alpha;
          m[qs] = up ? tmax : m[qs];
        }
        const float mref = m[qs] == -INFINITY ? 0.f : m[qs];  // no finite key yet: P = 0 either way
#pragma unroll
        for (int i = 0; i < 16; ++i) { sa[qs][i] -= mref; sb[qs][i] -= mref; }
      } else if (shifted[qs]) {  // S - cref (exactly S where cref = 0)
#pragma unroll
        for (int i = 0; i < 16; ++i) { sa[qs][i] -= cref[qs]; sb[qs][i] -= cref[qs]; }
      }
      // P = exp2(S) in f32; the row sums on the VALU (packed adds of the lane's keys, the
      // lane-pair sum at the end), the PV products on the matrix pipe from bf16 P
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        sa[qs][i] = __builtin_amdgcn_exp2f(sa[qs][i]);
        sb[qs][i] = __builtin_amdgcn_exp2f(sb[qs][i]);
      }
      uint4 pa0, pa1, pb0, pb1;  // bf16 P^T fragments, two keys per word
      pa0.x = pack_bf2(sa[qs][0], sa[qs][1]);   pa0.y = pack_bf2(sa[qs][2], sa[qs][3]);
      pa0.z = pack_bf2(sa[qs][4], sa[qs][5]);   pa0.w = pack_bf2(sa[qs][6], sa[qs][7]);
      pa1.x = pack_bf2(sa[qs][8], sa[qs][9]);   pa1.y = pack_bf2(sa[qs][10], sa[qs][11]);
      pa1.z = pack_bf2(sa[qs][12], sa[qs][13]); pa1.w = pack_bf2(sa[qs][14], sa[qs][15]);
      pb0.x = pack_bf2(sb[qs][0], sb[qs][1]);   pb0.y = pack_bf2(sb[qs][2], sb[qs][3]);
      pb0.z = pack_bf2(sb[qs][4], sb[qs][5]);   pb0.w = pack_bf2(sb[qs][6], sb[qs][7]);
      pb1.x = pack_bf2(sb[qs][8], sb[qs][9]);   pb1.y = pack_bf2(sb[qs][10], sb[qs][11]);
      pb1.z = pack_bf2(sb[qs][12], sb[qs][13]); pb1.w = pack_bf2(sb[qs][14], sb[qs][15]);
      o[qs] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(va0, __builtin_bit_cast(bf16x8, pa0), o[qs], 0, 0, 0);
      o[qs] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(va1, __builtin_bit_cast(bf16x8, pa1), o[qs], 0, 0, 0);
      o[qs] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vb0, __builtin_bit_cast(bf16x8, pb0), o[qs], 0, 0, 0);
      o[qs] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vb1, __builtin_bit_cast(bf16x8, pb1), o[qs], 0, 0, 0);
      // register pairs of the exp outputs (aligned: the accumulators' 16 registers), so every
      // add is a v_pk_add_f32.  (r05: the sums as one v_dot2c_f32_bf16 per bf16 P word were
      // 2.2 % faster but farther from the oracle at peaked scores -- x16: TV 0.049 against the
      // f32 sums' 0.032 -- so the f32 sums stay; profiles/r05/ab_ia_dot2_r05aa.txt; as 32 scalar
      // v_add_f32 instead of 16 packed: item attention +1.1 %, profiles/r05/ab_ia_scalar_add_r05ab.txt)
#define NPFN_IA_RSUM(i)                                                              \
  {                                                                                  \
    f32x2 t = __builtin_shufflevector(sa[qs], sa[qs], i, i + 1);                     \
    t += __builtin_shufflevector(sb[qs], sb[qs], i, i + 1);                          \
    lacc2[qs][((i) >> 1) & 1] += t;                                                  \
  }
      NPFN_IA_RSUM(0) NPFN_IA_RSUM(2) NPFN_IA_RSUM(4) NPFN_IA_RSUM(6)
      NPFN_IA_RSUM(8) NPFN_IA_RSUM(10) NPFN_IA_RSUM(12) NPFN_IA_RSUM(14)
#undef NPFN_IA_RSUM
    }
  };
  using T_ = std::true_type;
  using F_ = std::false_type;
  if (npair == 1) {
    step(0, T_{}, T_{});
  } else {
    step(0, T_{}, F_{});
    for (int p = 1; p < npair - 1; ++p) step(p, F_{}, F_{});
    step(npair - 1, F_{}, T_{});
  }
#pragma unroll
  for (int qs = 0; qs < kIaQs; ++qs) {
    const f32x2 t = lacc2[qs][0] + lacc2[qs][1];
    lsum[qs] = t[0] + t[1];
    lsum[qs] += __shfl_xor(lsum[qs], 32, 64);
  }
}

// resident blocks per CU the item attention is compiled for (3: <= 168 VGPRs).  r06: 3 query sets
// per wave at 2 blocks per CU (256 VGPRs, 84 B of scratch) ran k_item_attn 122.5 -> 131.9 ms per c2
// call (profiles/r06/ab_ia_qsets3_r06w.txt); 2 sets at 3 blocks stay
#ifndef NPFN_IA_MINB
#define NPFN_IA_MINB 3
#endif
__global__ __launch_bounds__(256, NPFN_IA_MINB) void k_item_attn(IaParams P, float scale_log2, int force_online) {
  constexpr bool kAll[kIaQs] = {};  // first pass: every set (todo is read by the later passes only)
  // K/V tiles of this (estimator, column, head) stream through an LDS ring shared by the
  // block's 4 waves (128 kIaQs queries): per tile one 1 KB LDS-DMA per wave instead of 4 KB of
  // fragment loads per wave, then 4 ds_read_b128 per wave.
  __shared__ __attribute__((aligned(16))) bf16_t ring[2 * kIaPairs][2048];
  // the block's segment (estimator group), picked with constant indices (no scratch copy)
  IaSeg sg = P.seg[0];
#pragma unroll
  for (int i = 1; i < kIaSegs; ++i)
    if (i < P.nseg && (int)blockIdx.y >= P.seg[i].y0) sg = P.seg[i];
  const bf16_t* __restrict__ q = sg.q;
  const bf16_t* __restrict__ kvc = sg.kvc;
  bf16_t* __restrict__ out = sg.out;
  const int64_t ldq = P.ldq, R = P.R, n = P.n;
  const int C = sg.C, ntile = P.ntile;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int qi = lane & 31, h2 = lane >> 5;
  const int ech = (int)blockIdx.y - sg.y0;  // (e * ncol + c - c_lo) * 6 + h within the segment
  const int h = ech % 6;
  const int ec = ech / 6;
  const int ncol = C - sg.c_lo;
  const int c = sg.c_lo + ec % ncol;
  const int e = ec / ncol;
  const int kvi = (e * C + c) * 6 + h;      // the triple's K/V stream in the cache
  bool valid[kIaQs];
  int64_t qrow[kIaQs];
  bf16x8 qf[kIaQs][2];
#pragma unroll
  for (int qs = 0; qs < kIaQs; ++qs) {
    const int64_t r = (int64_t)blockIdx.x * (128 * kIaQs) + wave * (32 * kIaQs) + 32 * qs + qi;
    valid[qs] = r < R;
    qrow[qs] = ((int64_t)e * R + (valid[qs] ? r : 0)) * C + c;
    const bf16_t* qp = q + qrow[qs] * ldq + h * 32 + 8 * h2;
    const bf16x8 z = {0, 0, 0, 0, 0, 0, 0, 0};
    qf[qs][0] = valid[qs] ? *reinterpret_cast<const bf16x8*>(qp) : z;
    qf[qs][1] = valid[qs] ? *reinterpret_cast<const bf16x8*>(qp + 16) : z;
    // fold the softmax scale (1/sqrt(32) * log2 e) into q: S = K (cs q)^T is then already in
    // the log2 domain (one extra bf16 rounding of q, 2^-9 relative)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      qf[qs][0][j] = (short)f2bf(bf2f((bf16_t)qf[qs][0][j]) * scale_log2);
      qf[qs][1][j] = (short)f2bf(bf2f((bf16_t)qf[qs][1][j]) * scale_log2);
    }
  }
  // tile t, segment `wave` (k0 | k1 | v0 | v1, 1 KB each): wave-uniform source, lane-linear image
  const bf16_t* kvseg = kvc + (int64_t)kvi * ntile * 2048 + wave * 512 + lane * 8;
  const uint32_t ring_lds = (uint32_t)(uintptr_t)&ring[0][0];
  const uint32_t seg_lds = __builtin_amdgcn_readfirstlane(ring_lds + (uint32_t)wave * 1024u);
  f32x16 o[kIaQs];
  float lsum[kIaQs];
  auto store = [&](int qs) {
    bf16_t* op = out + qrow[qs] * 192 + h * 32;
    const float inv = 1.0f / lsum[qs];
    // dims 8g + 4h2 + i; v_permlane32_swap pairs groups g, g+1 of the two half waves, so the
    // lower half stores dims 8g + [0, 8) and the upper one 8g + [8, 16) as one 16-byte store
#pragma unroll
    for (int g = 0; g < 4; g += 2) {
      const uint32_t a0 = pack_bf2(o[qs][4 * g + 0] * inv, o[qs][4 * g + 1] * inv);
      const uint32_t a1 = pack_bf2(o[qs][4 * g + 2] * inv, o[qs][4 * g + 3] * inv);
      const uint32_t b0 = pack_bf2(o[qs][4 * g + 4] * inv, o[qs][4 * g + 5] * inv);
      const uint32_t b1 = pack_bf2(o[qs][4 * g + 6] * inv, o[qs][4 * g + 7] * inv);
      const auto r0 = __builtin_amdgcn_permlane32_swap(a0, b0, false, false);
      const auto r1 = __builtin_amdgcn_permlane32_swap(a1, b1, false, false);
      *reinterpret_cast<uint4*>(op + 8 * g + 8 * h2) = make_uint4(r0[0], r1[0], r0[1], r1[1]);
    }
  };
  // every query keeps the result of its own checks (the block only decides whether a later pass
  // runs at all), so a row's output never depends on which rows share its block; a failing row
  // is counted by cause (sum overflow / underflow) in P.fb
  auto range_ok = [](float l) { return l >= 0x1p-100f && l <= 0x1p100f; };  // false also for NaN / inf
  float cref[kIaQs] = {};
  item_attn_pass<IA_FIRST>(ring, kvseg, seg_lds, ntile, n, qf, o, lsum, kAll, cref);
  bool pend[kIaQs], todo[kIaQs];  // pend: the lane's result is still open
#pragma unroll
  for (int qs = 0; qs < kIaQs; ++qs) {
    pend[qs] = valid[qs] && (!range_ok(lsum[qs]) || force_online);
    if (valid[qs] && !pend[qs]) store(qs);
  }
  bool any_bad = false;
  int nbad = 0, nover = 0, nunder = 0;
#pragma unroll
  for (int qs = 0; qs < kIaQs; ++qs) {
    const uint64_t bm = __ballot(pend[qs]);
    todo[qs] = bm != 0ull;  // the set's online rerun, decided per wave
    nbad += __popcll(bm) / 2;  // two lanes (h2 = 0, 1) per query row
    nover += __popcll(__ballot(pend[qs] && !(lsum[qs] <= 0x1p100f))) / 2;
    nunder += __popcll(__ballot(pend[qs] && lsum[qs] < 0x1p-100f)) / 2;
    any_bad |= todo[qs];
  }
  // fb: [blocks, rows, rows by overflow, rows by underflow] that took the online pass (the rest
  // of the rows: forced by npfn_debug_item_attn_online)
  if (P.fb && lane == 0 && nbad) {
    atomicAdd(P.fb + 1, (unsigned long long)nbad);
    if (nover) atomicAdd(P.fb + 2, (unsigned long long)nover);
    if (nunder) atomicAdd(P.fb + 3, (unsigned long long)nunder);
  }
  if (__syncthreads_or(any_bad)) {
    if (P.fb && threadIdx.x == 0) atomicAdd(P.fb, 1ull);
    item_attn_pass<IA_ONLINE>(ring, kvseg, seg_lds, ntile, n, qf, o, lsum, todo, cref);
#pragma unroll
    for (int qs = 0; qs < kIaQs; ++qs)
      if (pend[qs]) store(qs);
  }
}

// ================================================== K6-K8 bar distribution
// Block-wide helpers for 256 threads.
__device__ __forceinline__ float block_reduce_sum(float v, float* red) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  v = wave_sum(v);
  __syncthreads();
  if (lane == 0) red[w] = v;
  __syncthreads();
  return red[0] + red[1] + red[2] + red[3];
}
__device__ __forceinline__ float block_reduce_max(float v, float* red) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  v = wave_max(v);
  __syncthreads();
  if (lane == 0) red[w] = v;
  __syncthreads();
  return fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
}

// Ensemble mix: p[b] = mean_e q_e[b] for one query row, left in LDS, where q_e =
// softmax(logits_e / T) -- or, for a target-transformed estimator of the ensemble mode, that
// softmax (bars cancelled by the border repair removed) translated from the estimator's
// inverse-transformed borders to the common ones (translate_across_borders).
// Fast path (n_bars % 4 == 0, n_bars <= 256 * 4 * kMixV4): one pass over each estimator's
// logits -- the row lives in registers as float4 (bar 4 (256 j + tid) + i), the block max
// and sum come from one merged (max, sum) reduction behind a single barrier, and every
// thread accumulates its probabilities in registers: HBM-streaming, E barriers per row.
constexpr int kMixV4 = 8;
#ifndef NPFN_MIX_HOIST
#define NPFN_MIX_HOIST 1
#endif
constexpr bool kMixHoist = NPFN_MIX_HOIST != 0;

__device__ __forceinline__ void ms_merge(float& m, float& s, float m2, float s2) {
  const float M = fmaxf(m, m2);
  if (M == -INFINITY) return;  // both empty
  s = s * __expf(m - M) + s2 * __expf(m2 - M);
  m = M;
}

// exclusive prefix sum of in[0..nb) into out (both LDS), 256 threads, contiguous segments
__device__ void block_excl_scan(const float* in, float* out, int nb, float* scan) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int per = (nb + 255) / 256;
  const int b0 = min(tid * per, nb), b1 = min(b0 + per, nb);
  float local = 0.f;
  for (int b = b0; b < b1; ++b) local += in[b];
  const float incl = wave_incl_scan_dpp(local);
  if (lane == 63) scan[w] = incl;
  __syncthreads();
  float base = 0.f;
#pragma unroll
  for (int k = 0; k < 4; ++k)
    if (k < w) base += scan[k];
  float c = base + incl - local;
  for (int b = b0; b < b1; ++b) {
    out[b] = c;
    c += in[b];
  }
  __syncthreads();
}

// cdf of a translated estimator at common border b from its probabilities and their exclusive
// prefix sums, pc[i] = (p_i, cum_i) in LDS: cum + p * share of the source bucket, 0 / 1 beyond
// the source range, and 0 / 1 at the first / last border (translate_probs_across_borders [ext])
__device__ __forceinline__ float trans_left_e(const float2* pc, const TransEntry t, int b, int nb) {
  if (b == 0) return 0.f;
  if (b == nb) return 1.f;
  if (t.share < 0.f) return 0.f;
  if (t.share > 1.5f) return 1.f;
  const float2 v = pc[t.idx];
  return fminf(fmaxf(v.y + v.x * t.share, 0.f), 1.f);
}

// Fast path: thread t owns the contiguous bars [t PB, t PB + PB) (PB = 4 * nv <= 4 * NV; NV =
// the register arrays' size, a template parameter so that the default 5000 bars (nv = 5) do
// not pay for the largest case's registers),
// held as nv float4 in registers; one merged (max, sum) block reduction per estimator.  A
// translated estimator additionally scans its probabilities in registers, publishes (p, cum)
// through LDS (pc, [nb] float2) and gathers the cdf at its PB + 1 common borders.
template <int NV>
__device__ void mix_row_fast(const logit_t* __restrict__ logits, int64_t R, int64_t r, int E, int nb,
                             float invT, const MixTrans& tr, float* __restrict__ p, float* red /* [2][8] */,
                             float2* pc, float* scan) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int nv = (nb + 1023) / 1024;   // float4 per thread
  const int b0 = tid * 4 * nv;
  f32x4 acc[NV];
#pragma unroll
  for (int j = 0; j < NV; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // NPFN_MIX_HOIST: the translation entries of the thread's borders b0 .. b0 + PB loaded once
  // for all the row's translated estimators (they depend on the fit only; +42 VGPRs, 2 instead
  // of 4 resident blocks per CU), else read per translated estimator
  TransEntry te[kMixHoist ? 4 * NV + 1 : 1];
  // the thread's border-repair cancel flags (4 bytes per float4), fit-only too: loaded once, not per
  // translated estimator (r05: k_mix_sample 7.03 -> 6.50 ms, profiles/r05/ab_mix_cancel_hoist_r05az.txt)
  uint32_t cmask[NV];
  if (kMixHoist && tr.ett != nullptr) {
#pragma unroll
    for (int k = 0; k <= 4 * NV; ++k) {
      const int b = b0 + k;
      te[k] = (k <= 4 * nv && b <= nb) ? tr.tab[b] : TransEntry{0, 0.f};
    }
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      const int b = b0 + 4 * j;
      cmask[j] = (j < nv && b < nb) ? *reinterpret_cast<const uint32_t*>(tr.tcancel + b) : 0u;
    }
  }
  // the next estimator's logits are loaded while this one is reduced / translated (+4 NV VGPRs;
  // r05: k_mix_sample -10 %; two ahead spilled in r04)
  typedef logit_t lg4 __attribute__((ext_vector_type(4)));
  lg4 nx[NV];
  auto load_raw = [&](int e) {
    const logit_t* lg = logits + ((int64_t)e * R + r) * nb;
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      const int b = b0 + 4 * j;
      if (j < nv && b < nb) nx[j] = *reinterpret_cast<const lg4*>(lg + b);
    }
  };
  load_raw(0);
  for (int e = 0; e < E; ++e) {  // (r05: ett as a bit mask read once: 6.55 -> 6.69 ms, not kept -- ab_mix_ett_mask_r05ba.txt)
    const bool trans = tr.ett != nullptr && tr.ett[e];
    f32x4 v[NV];
#pragma unroll
    for (int j = 0; j < NV; ++j) v[j] = __builtin_convertvector(nx[j], f32x4);
    if (e + 1 < E) load_raw(e + 1);
    float ml = -INFINITY;
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      const int b = b0 + 4 * j;
      if (j < nv && b < nb) {
        v[j] = v[j] * invT;
        if (trans) {
          const uint32_t cm = kMixHoist ? cmask[j] : *reinterpret_cast<const uint32_t*>(tr.tcancel + b);
#pragma unroll
          for (int i = 0; i < 4; ++i)
            if ((cm >> (8 * i)) & 0xffu) v[j][i] = -INFINITY;
        }
        ml = fmaxf(ml, fmaxf(fmaxf(v[j][0], v[j][1]), fmaxf(v[j][2], v[j][3])));
      } else {
        v[j] = f32x4{-INFINITY, -INFINITY, -INFINITY, -INFINITY};
      }
    }
    float sl = 0.f;
    const float mref = (ml == -INFINITY) ? 0.f : ml;  // a thread with no mass keeps v = 0, s = 0
#pragma unroll
    for (int j = 0; j < NV; ++j)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        v[j][i] = __expf(v[j][i] - mref);
        sl += v[j][i];
      }
    // the wave's (max, sum): the max first (DPP / permlane, no LDS), then each lane's sum
    // rescaled to it once and summed the same way
    const float m = wave_max_dpp(ml);
    const float sm = wave_sum_dpp(ml == -INFINITY ? 0.f : sl * __expf(ml - m));
    float* rb = red + (e & 1) * 8;  // alternate buffers: one barrier per estimator
    if (lane == 0) {
      rb[w] = m;
      rb[4 + w] = sm;
    }
    __syncthreads();
    float M = rb[0], S = rb[4];
#pragma unroll
    for (int k = 1; k < 4; ++k) ms_merge(M, S, rb[k], rb[4 + k]);
    if (!trans) {
      if (tr.geo) {  // average_before_softmax: mean of the log probabilities
        // the exact log-softmax, x / T - M - log S, from the logits re-read (L2) -- not log of the
        // flushed probability, which is -inf below FLT_MIN and would zero that bar of the mixture
        const float lS = __logf(S), invE = 1.0f / (float)E;
        const logit_t* lg = logits + ((int64_t)e * R + r) * nb;
#pragma unroll
        for (int j = 0; j < NV; ++j) {
          const int b = b0 + 4 * j;
          if (j < nv && b < nb)
#pragma unroll
            for (int i = 0; i < 4; ++i) acc[j][i] += ((float)lg[b + i] * invT - M - lS) * invE;
        }
        continue;
      }
      const float sc = (ml == -INFINITY) ? 0.f : __expf(ml - M) / (S * (float)E);
#pragma unroll
      for (int j = 0; j < NV; ++j) acc[j] += v[j] * sc;
      continue;
    }
    // translated estimator: normalized probabilities, exclusive prefix sums (registers, then
    // across threads), (p, cum) to LDS, cdf at the thread's borders b0 .. b0 + PB
    const float sc = (ml == -INFINITY) ? 0.f : __expf(ml - M) / S;
    float run = 0.f;
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      v[j] *= sc;
#pragma unroll
      for (int i = 0; i < 4; ++i) run += v[j][i];
    }
    const float incl = wave_incl_scan_dpp(run);
    if (lane == 63) scan[w] = incl;
    __syncthreads();
    float c = incl - run;
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (k < w) c += scan[k];
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      const int b = b0 + 4 * j;
      if (j < nv && b < nb)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          pc[b + i] = make_float2(v[j][i], c);
          c += v[j][i];
        }
    }
    __syncthreads();
    const float invE = 1.0f / (float)E;
    float left = trans_left_e(pc, kMixHoist ? te[0] : tr.tab[min(b0, nb)], min(b0, nb), nb);
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      const int b = b0 + 4 * j;
      if (j < nv && b < nb)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float right = trans_left_e(pc, kMixHoist ? te[(4 * j + i + 1) % (kMixHoist ? 4 * NV + 1 : 1)]
                                                         : tr.tab[b + i + 1], b + i + 1, nb);
          const float q = fmaxf(right - left, 0.f);
          acc[j][i] += (tr.geo ? __logf(q) : q) * invE;
          left = right;
        }
    }
    __syncthreads();  // pc / scan are rewritten by the next translated estimator
  }
  if (tr.geo) {  // softmax of the mean log probabilities (tabpfn's average_before_softmax [ext])
    float mx = -INFINITY;
#pragma unroll
    for (int j = 0; j < NV; ++j)
      if (j < nv && b0 + 4 * j < nb) mx = fmaxf(mx, fmaxf(fmaxf(acc[j][0], acc[j][1]), fmaxf(acc[j][2], acc[j][3])));
    mx = block_reduce_max(mx, red);
    float sm = 0.f;
#pragma unroll
    for (int j = 0; j < NV; ++j)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        acc[j][i] = (j < nv && b0 + 4 * j < nb && mx != -INFINITY) ? __expf(acc[j][i] - mx) : 0.f;
        sm += acc[j][i];
      }
    sm = block_reduce_sum(sm, red);
    const float inv = sm > 0.f ? 1.0f / sm : 0.f;
#pragma unroll
    for (int j = 0; j < NV; ++j) acc[j] *= inv;
  }
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    const int b = b0 + 4 * j;
    if (j < nv && b < nb)  // scalar stores: the dynamic LDS base need not be 16-byte aligned here
#pragma unroll
      for (int i = 0; i < 4; ++i) p[b + i] = acc[j][i];
  }
  __syncthreads();
}

__device__ void mix_row(const logit_t* __restrict__ logits, int64_t R, int64_t r, int E, int nb,
                        float invT, const MixTrans& tr, float* __restrict__ p, float* red, float2* pc,
                        float* scan) {
  const int tid = threadIdx.x;
  for (int b = tid; b < nb; b += 256) p[b] = 0.f;
  float* pe = reinterpret_cast<float*>(pc);  // [nb] probabilities, then [nb] prefix sums
  float* cum = pe + nb;
  for (int e = 0; e < E; ++e) {
    const logit_t* lg = logits + ((int64_t)e * R + r) * nb;
    const bool trans = tr.ett != nullptr && tr.ett[e];
    auto lv = [&](int b) -> float { return (trans && tr.tcancel[b]) ? -INFINITY : (float)lg[b] * invT; };
    float mx = -INFINITY;
    for (int b = tid; b < nb; b += 256) mx = fmaxf(mx, lv(b));
    mx = block_reduce_max(mx, red);
    float s = 0.f;
    for (int b = tid; b < nb; b += 256) s += __expf(lv(b) - mx);
    s = block_reduce_sum(s, red);
    if (!trans) {
      if (tr.geo) {  // the exact log-softmax (no flush of tiny probabilities to log 0)
        const float ls = __logf(s);
        for (int b = tid; b < nb; b += 256) p[b] += (lv(b) - mx - ls) / (float)E;
        continue;
      }
      const float sc = 1.0f / (s * (float)E);
      for (int b = tid; b < nb; b += 256) p[b] += __expf(lv(b) - mx) * sc;
      continue;
    }
    const float sc = 1.0f / s;
    for (int b = tid; b < nb; b += 256) pe[b] = __expf(lv(b) - mx) * sc;
    __syncthreads();
    block_excl_scan(pe, cum, nb, scan);
    auto left = [&](int b) -> float {
      if (b == 0) return 0.f;
      if (b == nb) return 1.f;
      const TransEntry t = tr.tab[b];
      if (t.share < 0.f) return 0.f;
      if (t.share > 1.5f) return 1.f;
      return fminf(fmaxf(cum[t.idx] + pe[t.idx] * t.share, 0.f), 1.f);
    };
    for (int b = tid; b < nb; b += 256) {
      const float q = fmaxf(left(b + 1) - left(b), 0.f);
      p[b] += (tr.geo ? __logf(q) : q) / (float)E;
    }
    __syncthreads();
  }
  __syncthreads();
  if (tr.geo) {  // softmax of the mean log probabilities
    float m2 = -INFINITY;
    for (int b = tid; b < nb; b += 256) m2 = fmaxf(m2, p[b]);
    m2 = block_reduce_max(m2, red);
    float s2 = 0.f;
    for (int b = tid; b < nb; b += 256) {
      p[b] = m2 == -INFINITY ? 0.f : __expf(p[b] - m2);
      s2 += p[b];
    }
    s2 = block_reduce_sum(s2, red);
    const float inv = s2 > 0.f ? 1.0f / s2 : 0.f;
    for (int b = tid; b < nb; b += 256) p[b] *= inv;
    __syncthreads();
  }
}

// Sample one row from probabilities p[0..nb) (unnormalized; divided by their
// sum exactly as softmax(log p) would): returns theta and writes bucket.
// Also returns the log density of theta (full-support NLL form).
__device__ void bar_sample_row(const float* __restrict__ p, const float* __restrict__ bz, float bscale,
                               float bshift, int nb, float u, float* red, float* scan,
                               float& theta_out, float& logp_out) {
  const int tid = threadIdx.x;
  const int per = (nb + 255) / 256;
  const int b0 = tid * per;
  const int b1 = min(b0 + per, nb);
  float local = 0.f;
  for (int b = b0; b < b1; ++b) local += p[b];
  // block exclusive scan of the per-thread sums: inclusive scan inside the wave by
  // shuffles, wave totals through LDS (one barrier)
  const int lane = tid & 63, w = tid >> 6;
  float incl = wave_incl_scan_dpp(local);
  if (lane == 63) scan[w] = incl;
  __syncthreads();
  float base = 0.f, total = 0.f;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const float t = scan[k];
    if (k < w) base += t;
    total += t;
  }
  incl += base;
  const float excl = incl - local;
  __shared__ int s_idx;
  __shared__ float s_cprev;
  __shared__ int s_lastnz;
  if (tid == 0) { s_idx = 0x7fffffff; s_cprev = 0.f; s_lastnz = 0; }
  __syncthreads();
  // Each thread walks its bars with a serial cumulative sum started at the scan prefix and
  // reports its first bar with mass whose cumulative reaches u*total; the lowest index wins
  // (torch.searchsorted(cumsum, u, side='left') semantics, never a zero-mass bar).
  const float ut = u * total;
  int found = -1;
  float cfound = 0.f;
  {
    float c = excl;
    for (int b = b0; b < b1; ++b) {
      const float cn = c + p[b];
      if (p[b] > 0.f && cn >= ut) { found = b; cfound = c; break; }
      c = cn;
    }
  }
  int lastnz = -1;
  for (int b = b1 - 1; b >= b0; --b)
    if (p[b] > 0.f) { lastnz = b; break; }
  if (found >= 0) atomicMin(&s_idx, found);
  if (lastnz >= 0) atomicMax(&s_lastnz, lastnz);
  __syncthreads();
  if (found >= 0 && found == s_idx) s_cprev = cfound;
  __syncthreads();
  if (tid == 0) {
    int idx = s_idx;
    float cprev = s_cprev;
    if (idx == 0x7fffffff) {  // u beyond the rounded total: the last bar with mass
      idx = s_lastnz;
      cprev = total - p[idx];
    }
    const float left = bz[idx] * bscale + bshift;
    const float right = bz[idx + 1] * bscale + bshift;
    const float pn = p[idx] / total;
    // fraction of the bar below u, clamped to [0, 1] so rounding between the block scan and
    // the serial prefix can never push a draw outside its bar
    const float frac = fminf(fmaxf((u - cprev / total) / pn, 0.f), 1.f);
    const float th = left + (right - left) * frac;
    theta_out = th;
    // NLL of th (re-bucketed like map_to_bucket_idx): searchsorted(borders, th, left) = the
    // first i with b[i] >= th.  th lies in [b[idx], b[idx + 1]] (up to rounding), so walk to it
    // from idx + 1 instead of a 13-load binary search; the borders are non-decreasing, so the
    // walk ends at the same index (r05: bz[0], bz[1], bz[nb - 1], bz[nb] loaded ahead of the scan
    // and the walk reusing left / right: bitwise equal, mix 7.09 -> 7.14 ms, not kept --
    // profiles/r05/ab_mix_tail_borders_r05aw.txt)
    int lo = idx + 1;
    while (lo > 0 && bz[lo - 1] * bscale + bshift >= th) --lo;
    while (lo <= nb && bz[lo] * bscale + bshift < th) ++lo;
    int j = lo - 1;
    const float bfirst = bz[0] * bscale + bshift;
    const float blast = bz[nb] * bscale + bshift;
    if (th == bfirst) j = 0;
    if (th == blast) j = nb - 1;
    j = min(max(j, 0), nb - 1);
    const float bj = bz[j] * bscale + bshift, bj1 = bz[j + 1] * bscale + bshift;
    const double w = (double)bj1 - (double)bj;
    double lp = log((double)p[j] / (double)total) - log(w);
    if (j == 0) {
      const double w0 = w;
      const double s0 = w0 / NPFN_HALFNORMAL_MEDIAN;
      const double vv = fmax((double)(bz[1] * bscale + bshift) - (double)th, 1e-8);
      lp += log(sqrt(2.0 / M_PI) / s0) - vv * vv / (2.0 * s0 * s0) + log(w0);
    }
    if (j == nb - 1) {
      const double s1 = w / NPFN_HALFNORMAL_MEDIAN;
      const double vv = fmax((double)th - (double)(bz[nb - 1] * bscale + bshift), 1e-8);
      lp += log(sqrt(2.0 / M_PI) / s1) - vv * vv / (2.0 * s1 * s1) + log(w);
    }
    logp_out = (float)lp;
  }
}

// resident blocks per CU the k_mix_* kernels are compiled for: 3 (3 waves per SIMD, <= 168
// VGPRs; the fast path needs 175 at 2 blocks and takes 168 + 32 B of scratch at 3).  The per-row
// chain of reductions / scans / barriers is latency-bound, so the third block pays: r06 with the
// DPP reductions, k_mix_sample 6.66 (bf16-era shuffles, 2 blocks) -> 6.11 (DPP, 2) -> 5.21 ms per c2
// call (DPP, 3; profiles/r06/ab_mix_dpp_minb3_r06k.txt).  4 would cap them at 128 and spill ~170
// of the fast path's registers to scratch (r04)
#ifndef NPFN_MIX_MINB
#define NPFN_MIX_MINB 3
#endif
// dynamic LDS of the k_mix_* kernels: [64 B reduction scratch | p | pc] (pc = (probability,
// prefix sum) pairs of a translated estimator, only with target-border translation).  The fast
// path keeps p in registers until after its last estimator (whose pc reads end at a barrier),
// so there p overlays pc: half the LDS, twice the resident blocks per CU.
#define NPFN_MIX_SMEM_VIEW                                                     \
  extern __shared__ __attribute__((aligned(16))) char smem[];                 \
  float* p = reinterpret_cast<float*>(smem + 64);                             \
  float* red = reinterpret_cast<float*>(smem);                                \
  float2* pc = reinterpret_cast<float2*>(smem + 64 + (NV > 0 ? 0 : (((size_t)nb * 4 + 15) & ~(size_t)15))); \
  __shared__ float scan4[4];
#define NPFN_MIX_ROW()                                                        \
  if constexpr (NV > 0) mix_row_fast<NV>(logits, R, r, E, nb, invT, tr, p, red, pc, scan4); \
  else mix_row(logits, R, r, E, nb, invT, tr, p, red, pc, scan4);

// predict(): logits_out[r][b] = log(mean_e q_e[b])
template <int NV>  // 0: generic path, else the fast path with NV float4 per thread
__global__ __launch_bounds__(256, NPFN_MIX_MINB) void k_mix_log(const logit_t* __restrict__ logits, int64_t R, int E,
                                                 int nb, float invT, MixTrans tr, float* __restrict__ out,
                                                 int64_t ldo) {
  NPFN_MIX_SMEM_VIEW
  const int64_t r = blockIdx.x;
  NPFN_MIX_ROW()
  for (int b = threadIdx.x; b < nb; b += 256) out[r * ldo + b] = __logf(p[b]);
}

// Fused AR step: mix -> sample -> NLL -> write theta into the feature buffer.
template <int NV>  // 0: generic path, else the fast path with NV float4 per thread
__global__ __launch_bounds__(256, NPFN_MIX_MINB) void k_mix_sample(const logit_t* __restrict__ logits, int64_t R, int E,
                                                    int nb, float invT, MixTrans tr, const float* __restrict__ bz,
                                                    const float* __restrict__ ystats, uint64_t seed,
                                                    uint64_t counter, int64_t row_offset, uint64_t philox_row0,
                                                    float* __restrict__ feat, int64_t ldf, int col,
                                                    float* __restrict__ logp_acc, float log_eps) {
  NPFN_MIX_SMEM_VIEW
  __shared__ float scan[256];
  const int64_t r = blockIdx.x;
  NPFN_MIX_ROW()
  const float u = philox_uniform(seed, counter, philox_row0 + (uint64_t)(row_offset + r));
  float th = 0.f, lp = 0.f;
  bar_sample_row(p, bz, ystats[1], ystats[0], nb, u, red, scan, th, lp);
  if (threadIdx.x == 0) {
    feat[(row_offset + r) * ldf + col] = th;
    if (logp_acc != nullptr) logp_acc[row_offset + r] += (lp == -INFINITY) ? log_eps : lp;
  }
}

// Mixture p of each row (what k_mix_sample samples from), written once per distinct query row.
template <int NV>  // 0: generic path, else the fast path with NV float4 per thread
__global__ __launch_bounds__(256, NPFN_MIX_MINB) void k_mix_prob(const logit_t* __restrict__ logits, int64_t R, int E, int nb,
                                                  float invT, MixTrans tr, float* __restrict__ p_out) {
  NPFN_MIX_SMEM_VIEW
  const int64_t r = blockIdx.x;
  NPFN_MIX_ROW()
  for (int b = threadIdx.x; b < nb; b += 256) p_out[r * nb + b] = p[b];
}

// The sampling half of k_mix_sample for draws whose query rows repeat: row r draws from the
// mixture of its distinct row, p_rows[(row_offset + r) / per], loaded into the same LDS slot
// k_mix_sample leaves it in, so the draw and its log density are bit for bit those of
// k_mix_sample over the repeated rows.
__global__ __launch_bounds__(256) void k_group_sample(const float* __restrict__ p_rows, int64_t per, int nb,
                                                      const float* __restrict__ bz, const float* __restrict__ ystats,
                                                      uint64_t seed, uint64_t counter, int64_t row_offset,
                                                      uint64_t philox_row0, float* __restrict__ feat, int64_t ldf,
                                                      int col, float* __restrict__ logp_acc, float log_eps) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* p = reinterpret_cast<float*>(smem + 64);
  float* red = reinterpret_cast<float*>(smem);
  __shared__ float scan[256];
  const int64_t r = blockIdx.x;
  const float* src = p_rows + ((row_offset + r) / per) * (int64_t)nb;
  for (int b = threadIdx.x; b < nb; b += 256) p[b] = src[b];
  __syncthreads();
  const float u = philox_uniform(seed, counter, philox_row0 + (uint64_t)(row_offset + r));
  float th = 0.f, lp = 0.f;
  bar_sample_row(p, bz, ystats[1], ystats[0], nb, u, red, scan, th, lp);
  if (threadIdx.x == 0) {
    feat[(row_offset + r) * ldf + col] = th;
    if (logp_acc != nullptr) logp_acc[row_offset + r] += (lp == -INFINITY) ? log_eps : lp;
  }
}

// Full-support bar log density of th under the mixture p[0..nb) (unnormalized, divided by its
// block sum), borders bz * bs + bsh; every thread calls it, thread 0's result is the one used.
__device__ float bar_logp_row(const float* __restrict__ p, int nb, const float* __restrict__ bz, float bs, float bsh,
                              float th, float* red) {
  float tot = 0.f;
  for (int b = threadIdx.x; b < nb; b += 256) tot += p[b];
  tot = block_reduce_sum(tot, red);
  if (threadIdx.x != 0) return 0.f;
  int lo = 0, hi = nb + 1;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (bz[mid] * bs + bsh < th) lo = mid + 1; else hi = mid;
  }
  int j = lo - 1;
  if (th == bz[0] * bs + bsh) j = 0;
  if (th == bz[nb] * bs + bsh) j = nb - 1;
  j = min(max(j, 0), nb - 1);
  const double w = (double)(bz[j + 1] * bs + bsh) - (double)(bz[j] * bs + bsh);
  double lp = log((double)p[j] / (double)tot) - log(w);
  if (j == 0) {
    const double s0 = w / NPFN_HALFNORMAL_MEDIAN;
    const double vv = fmax((double)(bz[1] * bs + bsh) - (double)th, 1e-8);
    lp += log(sqrt(2.0 / M_PI) / s0) - vv * vv / (2.0 * s0 * s0) + log(w);
  }
  if (j == nb - 1) {
    const double s1 = w / NPFN_HALFNORMAL_MEDIAN;
    const double vv = fmax((double)th - (double)(bz[nb - 1] * bs + bsh), 1e-8);
    lp += log(sqrt(2.0 / M_PI) / s1) - vv * vv / (2.0 * s1 * s1) + log(w);
  }
  return (float)lp;
}

// Teacher-forced step: NLL of the given target column.
template <int NV>  // 0: generic path, else the fast path with NV float4 per thread
__global__ __launch_bounds__(256, NPFN_MIX_MINB) void k_mix_nll(const logit_t* __restrict__ logits, int64_t R, int E, int nb,
                                                 float invT, MixTrans tr, const float* __restrict__ bz,
                                                 const float* __restrict__ ystats, int64_t row_offset,
                                                 const float* __restrict__ feat, int64_t ldf, int col,
                                                 float* __restrict__ logp_acc, float log_eps) {
  NPFN_MIX_SMEM_VIEW
  const int64_t r = blockIdx.x;
  NPFN_MIX_ROW()
  const float th = feat[(row_offset + r) * ldf + col];
  const float lpf = bar_logp_row(p, nb, bz, ystats[1], ystats[0], th, red);
  if (threadIdx.x == 0) logp_acc[row_offset + r] += (lpf == -INFINITY) ? log_eps : lpf;
}

// k_mix_nll for repeated query rows: row r's mixture is p_rows[(row_offset + r) / per]
// (k_mix_prob), loaded where k_mix_nll leaves it -- the same log density bit for bit.
__global__ __launch_bounds__(256) void k_group_nll(const float* __restrict__ p_rows, int64_t per, int nb,
                                                   const float* __restrict__ bz, const float* __restrict__ ystats,
                                                   int64_t row_offset, const float* __restrict__ feat, int64_t ldf,
                                                   int col, float* __restrict__ logp_acc, float log_eps) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* p = reinterpret_cast<float*>(smem + 64);
  float* red = reinterpret_cast<float*>(smem);
  const int64_t r = blockIdx.x;
  const float* src = p_rows + ((row_offset + r) / per) * (int64_t)nb;
  for (int b = threadIdx.x; b < nb; b += 256) p[b] = src[b];
  __syncthreads();
  const float th = feat[(row_offset + r) * ldf + col];
  const float lpf = bar_logp_row(p, nb, bz, ystats[1], ystats[0], th, red);
  if (threadIdx.x == 0) logp_acc[row_offset + r] += (lpf == -INFINITY) ? log_eps : lpf;
}

// Generic criterion.sample(logits): softmax(logits row) -> inverse CDF.
__global__ __launch_bounds__(256) void k_bar_sample(const float* __restrict__ logits, const float* __restrict__ borders,
                                                    int64_t R, int nb, uint64_t seed, uint64_t counter,
                                                    float* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* p = reinterpret_cast<float*>(smem);
  __shared__ float red[4];
  __shared__ float scan[256];
  const int64_t r = blockIdx.x;
  const float* lg = logits + r * nb;
  float mx = -INFINITY;
  for (int b = threadIdx.x; b < nb; b += 256) mx = fmaxf(mx, lg[b]);
  mx = block_reduce_max(mx, red);
  for (int b = threadIdx.x; b < nb; b += 256) p[b] = __expf(lg[b] - mx);
  __syncthreads();
  const float u = philox_uniform(seed, counter, (uint64_t)r);
  float th = 0.f, lp = 0.f;
  bar_sample_row(p, borders, 1.0f, 0.0f, nb, u, red, scan, th, lp);
  if (threadIdx.x == 0) out[r] = th;
}

// Generic criterion(logits, y): full-support bar NLL.
__global__ __launch_bounds__(256) void k_bar_nll(const float* __restrict__ logits, const float* __restrict__ b,
                                                 const float* __restrict__ y, int64_t R, int nb,
                                                 float* __restrict__ out) {
  __shared__ float red[4];
  const int64_t r = blockIdx.x;
  const float* lg = logits + r * nb;
  float mx = -INFINITY;
  for (int k = threadIdx.x; k < nb; k += 256) mx = fmaxf(mx, lg[k]);
  mx = block_reduce_max(mx, red);
  float s = 0.f;
  for (int k = threadIdx.x; k < nb; k += 256) s += __expf(lg[k] - mx);
  s = block_reduce_sum(s, red);
  if (threadIdx.x == 0) {
    const float th = y[r];
    int lo = 0, hi = nb + 1;
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (b[mid] < th) lo = mid + 1; else hi = mid;
    }
    int j = lo - 1;
    if (th == b[0]) j = 0;
    if (th == b[nb]) j = nb - 1;
    j = min(max(j, 0), nb - 1);
    const double w = (double)b[j + 1] - (double)b[j];
    double lp = ((double)lg[j] - (double)mx - log((double)s)) - log(w);
    if (j == 0) {
      const double s0 = w / NPFN_HALFNORMAL_MEDIAN;
      const double vv = fmax((double)b[1] - (double)th, 1e-8);
      lp += log(sqrt(2.0 / M_PI) / s0) - vv * vv / (2.0 * s0 * s0) + log(w);
    }
    if (j == nb - 1) {
      const double s1 = w / NPFN_HALFNORMAL_MEDIAN;
      const double vv = fmax((double)th - (double)b[nb - 1], 1e-8);
      lp += log(sqrt(2.0 / M_PI) / s1) - vv * vv / (2.0 * s1 * s1) + log(w);
    }
    out[r] = (float)(-lp);
  }
}

__global__ void k_borders(const float* __restrict__ bz, const float* __restrict__ ystats, int nb,
                          float* __restrict__ out) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i <= nb) out[i] = bz[i] * ystats[1] + ystats[0];
}

// ======================================================= small utilities
__global__ void k_copy_cols(const float* __restrict__ src, int64_t lds, float* __restrict__ dst,
                            int64_t ldd, int64_t rows, int cols, int dst_col0, int64_t per) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= rows * cols) return;
  const int64_t r = i / cols;
  const int c = (int)(i - r * cols);
  dst[r * ldd + dst_col0 + c] = src[(r / per) * lds + c];
}

__global__ void k_fill(float* __restrict__ dst, int64_t n, float v) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n) dst[i] = v;
}

__global__ void k_box_support(const float* __restrict__ th, int64_t n, int dim, const float* __restrict__ lo,
                              const float* __restrict__ hi, uint8_t* __restrict__ mask) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  bool ok = true;
  for (int j = 0; j < dim; ++j) {
    const float v = th[i * dim + j];
    ok = ok && (v >= lo[j]) && (v <= hi[j]);
  }
  mask[i] = ok ? 1 : 0;
}

// ------------------------------------------------------------- launchers
static inline unsigned blocks_for(int64_t n, int b) { return (unsigned)((n + b - 1) / b); }

void launch_col_stats(const float* X, int64_t ldx, const float* y, int64_t ldy, int64_t n, int F,
                      float* colstat, float* ystats, hipStream_t s) {
  hipLaunchKernelGGL(k_col_stats, dim3(F + 1), dim3(256), 0, s, X, ldx, y, ldy, n, F, colstat, ystats);
}
void launch_build_params(const float* colstat, int F, int k, int E, int Fmax, int Gmax, uint64_t seed,
                         const int* ftype, ViewLayout L, int* vcol, float* mu, float* sd, float* gscale, int* eF,
                         hipStream_t s) {
  hipLaunchKernelGGL(k_build_params, dim3(E), dim3(64), 0, s, colstat, F, k, E, Fmax, Gmax, seed, ftype, L, vcol, mu,
                     sd, gscale, eF);
}
void launch_power_fit(const float* X, int64_t ldx, int64_t n, int F, double* plam, float* pstat, hipStream_t s,
                      const float* y, int64_t ldy, double* ylam, float* ypstat) {
  const int blocks = F + (y ? 1 : 0);
  if (blocks <= 0) return;
  hipLaunchKernelGGL(k_power_fit, dim3(blocks), dim3(PF_THREADS), 0, s, X, ldx, n, F, plam, pstat, y, ldy, ylam,
                     ypstat);
}
void launch_quantile_fit(const float* X, int64_t ldx, int64_t n, int F, int div, int nqmax, const int* sub,
                         double* qtab, int* qn, float* qstat, hipStream_t s) {
  const size_t lds = std::max<size_t>((size_t)QT_SORT_MAX * sizeof(float), (size_t)nqmax * sizeof(double));
  hipLaunchKernelGGL(k_quantile_fit, dim3(F), dim3(256), lds, s, X, ldx, n, F, div, nqmax, sub, qtab, qn, qstat);
}
void launch_qt_subsample(int64_t n, uint32_t seed, int* idx, hipStream_t s) {
  const size_t lds = 2 * 624 * sizeof(uint32_t) + (size_t)n * sizeof(uint16_t);
  hipLaunchKernelGGL(k_qt_subsample, dim3(1), dim3(64), lds, s, n, seed, idx);
}
void launch_views_base(const float* X, int64_t ldx, int64_t R, const ViewParams& vp, float* views, hipStream_t s) {
  if (R <= 0) return;
  hipLaunchKernelGGL(k_views, dim3(blocks_for(R * vp.L.F, 256)), dim3(256), 0, s, X, ldx, R, vp, views);
}
void launch_views_svd(int64_t R, const ViewParams& vp, float* views, hipStream_t s) {
  if (R <= 0 || vp.L.k <= 0) return;
  hipLaunchKernelGGL(k_views_svd, dim3(blocks_for(R * vp.L.k, 256)), dim3(256), 0, s, R, vp, views);
}
void launch_views_fp_test(const float* X, int64_t ldx, int64_t R, const ViewParams& vp, float* views, hipStream_t s) {
  if (R <= 0 || !vp.L.has_fp) return;
  hipLaunchKernelGGL(k_views_fp, dim3(blocks_for(R * vp.L.E, 256)), dim3(256), 0, s, X, ldx, R, vp, views);
}
int fp_stride(int64_t n) {  // a multiple of 4 (the resolve stages 16-byte pieces)
  const int c = n <= 0 ? kFpMin : fp_count((int)(std::min<int64_t>(n, kFpBlock) - 1));
  return (c + 3) & ~3;
}
void launch_fp_train(const float* X, int64_t ldx, int64_t n, const ViewParams& vp, int* htab, float* views,
                     hipStream_t s) {
  if (n <= 0 || !vp.L.has_fp) return;
  const int st = fp_stride(n);
  const int64_t total = fp_total(n);
  hipLaunchKernelGGL(k_fp_train_hash, dim3(blocks_for((int64_t)vp.L.E * total, 256)), dim3(256), 0, s, X, ldx, n, total,
                     vp, htab);
  hipLaunchKernelGGL(k_fp_train_resolve, dim3(vp.L.E), dim3(n <= 4096 ? 64 : FPR_THREADS), kFpResolveSmem + 16, s, X,
                     ldx, n, st, total, vp, htab, views);
}
void svd_setup() {
  if (h_fp_off[kFpBlock] == 0) fp_off_init();
  (void)hipMemcpyToSymbol(HIP_SYMBOL(g_fp_off), h_fp_off, sizeof(h_fp_off));
  (void)hipFuncSetAttribute((const void*)k_fp_train_resolve, hipFuncAttributeMaxDynamicSharedMemorySize,
                            kFpResolveSmem + 16);
  (void)hipFuncSetAttribute((const void*)k_quantile_fit, hipFuncAttributeMaxDynamicSharedMemorySize,
                            std::max<int>(QT_SORT_MAX * sizeof(float), kQtSubsample * sizeof(double)));
  (void)hipFuncSetAttribute((const void*)k_qt_subsample, hipFuncAttributeMaxDynamicSharedMemorySize,
                            2 * 624 * sizeof(uint32_t) + kQtSubsampleMaxRows * sizeof(uint16_t));
  const size_t big = kSvjHead + (size_t)128 * 129 * sizeof(double);
  (void)hipFuncSetAttribute((const void*)k_svd_jacobi<true, false>, hipFuncAttributeMaxDynamicSharedMemorySize, big);
  (void)hipFuncSetAttribute((const void*)k_svd_jacobi<true, true>, hipFuncAttributeMaxDynamicSharedMemorySize, big);
}
// ---- large form (wide tables: m = 2F > kSvdMaxM and n > kSvdMaxM): the same Gram tiles and
// shifted sums (k_svd_gram), the scaled Gram matrix A = D^-1 Z^T Z D^-1 assembled densely
// (k_svd_assemble: svj_fill's arithmetic over the whole grid), its eigen-decomposition by
// rocSOLVER's dsyevd (a plain library eigensolver: a one-block Jacobi is O(m^3) per sweep on one
// CU), and the top-k eigenvectors signed as svd_flip (k_svd_select).
__global__ __launch_bounds__(256) void k_svd_scale(const double* __restrict__ psum, int nchunk, int64_t n, int m,
                                                   double* __restrict__ scl) {
  const int j = blockIdx.x * 256 + threadIdx.x;
  if (j >= m) return;
  double s1 = 0.0, s2 = 0.0;
  for (int c = 0; c < nchunk; ++c) {
    s1 += psum[((int64_t)c * m + j) * 2 + 0];
    s2 += psum[((int64_t)c * m + j) * 2 + 1];
  }
  const double mu = s1 / (double)n;
  const double sd = sqrt(fmax(s2 / (double)n - mu * mu, 0.0));
  scl[j] = sd < 10.0 * 2.220446049250313e-16 ? 1.0 : sd;
}
__global__ __launch_bounds__(256) void k_svd_assemble(const double* __restrict__ part, int nchunk, int m,
                                                      const double* __restrict__ scl, double* __restrict__ A) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (int64_t)m * m) return;
  const int a = (int)(i / m), b = (int)(i - (int64_t)a * m);
  const int T = svd_tiles(m), NT = svd_upper_tiles(m);
  const int ta = a / kSvdTile, tb = b / kSvdTile;
  const int t = ta <= tb ? svd_tile_index(ta, tb, T) : svd_tile_index(tb, ta, T);
  const int e = ta <= tb ? (a % kSvdTile) * kSvdTile + (b % kSvdTile) : (b % kSvdTile) * kSvdTile + (a % kSvdTile);
  double g = 0.0;
  for (int c = 0; c < nchunk; ++c) g += part[((int64_t)c * NT + t) * (kSvdTile * kSvdTile) + e];
  A[i] = g / (scl[a] * scl[b]);
}
// one block per component c: eigenvector m - 1 - c of dsyevd's ascending order (column-major:
// component i at A[i + j m]), its largest-magnitude entry (first index on ties) made positive
__global__ __launch_bounds__(256) void k_svd_select(const double* __restrict__ A, int m, const double* __restrict__ scl,
                                                    double* __restrict__ out) {
  __shared__ double rbest[4], rval[4];
  __shared__ int ridx[4];
  const int c = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const double* v = A + (int64_t)(m - 1 - c) * m;
  if (c == 0)
    for (int j = tid; j < m; j += 256) out[j] = scl[j];
  double best = -1.0, bval = 0.0;
  int bi = 0x7fffffff;
  for (int j = tid; j < m; j += 256)
    if (fabs(v[j]) > best) {
      best = fabs(v[j]);
      bval = v[j];
      bi = j;
    }
  for (int o = 32; o > 0; o >>= 1) {
    const double ob = __shfl_xor(best, o), ov = __shfl_xor(bval, o);
    const int oi = __shfl_xor(bi, o);
    if (ob > best || (ob == best && oi < bi)) {
      best = ob;
      bval = ov;
      bi = oi;
    }
  }
  if (lane == 0) {
    rbest[w] = best;
    rval[w] = bval;
    ridx[w] = bi;
  }
  __syncthreads();
  double gb = rbest[0], gv = rval[0];
  int gi = ridx[0];
  for (int q = 1; q < 4; ++q)
    if (rbest[q] > gb || (rbest[q] == gb && ridx[q] < gi)) {
      gb = rbest[q];
      gv = rval[q];
      gi = ridx[q];
    }
  const double sg = gv < 0.0 ? -1.0 : 1.0;
  for (int j = tid; j < m; j += 256) out[m + (int64_t)c * m + j] = sg * v[j];
}
// rocBLAS handles for the eigensolver, one per device (created on first use on that device, under
// a lock; bound to the caller's stream at each call), so two engines on two devices of one process
// never share a handle bound to the other device's stream.
static rocblas_handle svd_solver() {
  static std::mutex mu;
  static rocblas_handle hs[64] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
  std::lock_guard<std::mutex> lk(mu);
  if (!hs[dev] && rocblas_create_handle(&hs[dev]) != rocblas_status_success) hs[dev] = nullptr;
  return hs[dev];
}

// the Jacobi over an m x m matrix given as partial tiles (LDS-resident A up to 128, V up to 64)
static void launch_svj(const double* part, const double* psum, int nc, int64_t n, int m, int k, double* gA, double* gV,
                       double* out, hipStream_t s) {
  const size_t mat = (size_t)m * (m + 1) * sizeof(double);
  if (m <= 64)
    hipLaunchKernelGGL((k_svd_jacobi<true, true>), dim3(1), dim3(SVJ_THREADS), kSvjHead + 2 * mat, s, part, psum, nc, n,
                       m, k, gA, gV, out);
  else if (m <= 128)
    hipLaunchKernelGGL((k_svd_jacobi<true, false>), dim3(1), dim3(SVJ_THREADS), kSvjHead + mat, s, part, psum, nc, n,
                       m, k, gA, gV, out);
  else
    hipLaunchKernelGGL((k_svd_jacobi<false, false>), dim3(1), dim3(SVJ_THREADS), kSvjHead, s, part, psum, nc, n, m, k,
                       gA, gV, out);
}
int launch_svd_fit(const float* views, int64_t n, ViewLayout L, void* work, double* out, hipStream_t s) {
  const int m = 2 * L.F;
  if (m < 2 || L.k < 1 || L.k > m || n < 1) return -1;
  if (m > kSvdMaxM && n > kSvdMaxM) {  // large: the dense scaled Gram matrix through dsyevd
    if (m > kSvdLargeMaxM) return -1;
    rocblas_handle hs = svd_solver();
    if (!hs || rocblas_set_stream(hs, s) != rocblas_status_success) return -1;
    const int nc = svd_chunks(n, m), NT = svd_upper_tiles(m);
    double* part = static_cast<double*>(work);
    double* psum = part + (size_t)nc * NT * kSvdTile * kSvdTile;
    double* scl = psum + (size_t)nc * m * 2;
    double* A = scl + m;
    double* D = A + (size_t)m * m;
    double* E = D + m;
    rocblas_int* info = reinterpret_cast<rocblas_int*>(E + m);
    hipLaunchKernelGGL(k_svd_gram, dim3((unsigned)NT, (unsigned)nc), dim3(256), 0, s, views, n, L, nc, part, psum);
    hipLaunchKernelGGL(k_svd_scale, dim3(blocks_for(m, 256)), dim3(256), 0, s, psum, nc, n, m, scl);
    hipLaunchKernelGGL(k_svd_assemble, dim3(blocks_for((int64_t)m * m, 256)), dim3(256), 0, s, part, nc, m, scl, A);
    if (rocsolver_dsyevd(hs, rocblas_evect_original, rocblas_fill_upper, m, A, m, D, E, info) !=
        rocblas_status_success)
      return -1;
    // dsyevd's convergence flag, checked before its vectors are used: a failed solve ends the fit
    // with an error instead of selecting components from an unconverged matrix (this wide-table
    // path runs only past 256 features and 512 context rows; the eigensolve itself dominates the
    // stream wait)
    rocblas_int hinfo = 0;
    if (hipMemcpyAsync(&hinfo, info, sizeof(hinfo), hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
      return -1;
    if (hinfo != 0) return -2;
    hipLaunchKernelGGL(k_svd_select, dim3((unsigned)L.k), dim3(256), 0, s, A, m, scl, out);
    return 0;
  }
  if (m > kSvdMaxM) {  // the n x n dual (wide tables)
    if (n > kSvdMaxM || L.k > n) return -1;
    const int np = svd_dual_np(n), NT = svd_upper_tiles(np);
    double* scl = static_cast<double*>(work);
    double* psum = scl + m;
    double* part = psum + 2 * (size_t)np;
    double* gA = part + (size_t)NT * kSvdTile * kSvdTile;
    double* gV = gA + (size_t)np * (np + 1);
    double* uo = gV + (size_t)np * (np + 1);
    hipLaunchKernelGGL(k_svd_colscale, dim3(blocks_for(std::max(m, np), 256)), dim3(256), 0, s, views, n, L, np, scl,
                       psum);
    hipLaunchKernelGGL(k_svd_dual_gram, dim3((unsigned)NT), dim3(256), 0, s, views, n, L, scl, np, part);
    launch_svj(part, psum, 1, np, np, L.k, gA, gV, uo, s);
    hipLaunchKernelGGL(k_svd_dual_out, dim3((unsigned)L.k), dim3(256), 0, s, views, n, L, scl, np, uo, out);
    return 0;
  }
  const int nc = svd_chunks(n, m), NT = svd_upper_tiles(m);
  double* part = static_cast<double*>(work);
  double* psum = part + (size_t)nc * NT * kSvdTile * kSvdTile;
  double* gA = psum + (size_t)nc * m * 2;
  double* gV = gA + (size_t)m * (m + 1);
  hipLaunchKernelGGL(k_svd_gram, dim3((unsigned)NT, (unsigned)nc), dim3(256), 0, s, views, n, L, nc, part, psum);
  launch_svj(part, psum, nc, n, m, L.k, gA, gV, out, s);
  return 0;
}
void launch_target_tf(const float* y, int64_t ldy, int64_t n, const float* bz, int nb, double* ylam, float* ystats,
                      TransEntry* tab, uint8_t* tcancel, float* pscratch, hipStream_t s, bool fit_lambda) {
  if (fit_lambda) launch_power_fit(nullptr, 0, n, 0, nullptr, nullptr, s, y, ldy, ylam, pscratch);  // the target's lambda
  hipLaunchKernelGGL(k_target_tf, dim3(1), dim3(256), (size_t)(nb + 1) * 5, s, y, ldy, n, bz, nb, ylam, ystats, tab,
                     tcancel);
}
void launch_encode(const float* ytr, int64_t ldy, int64_t R, const DevFit& fp, const float* encw,
                   const float* yencw, const float* pos, float* resid, bf16_t* resid_bf, hipStream_t s) {
  const int64_t tokens = (int64_t)fp.E * R * fp.C;
  if (tokens <= 0) return;
  const unsigned grid = (unsigned)blocks_for(tokens, 4);
  if (tokens < (int64_t(1) << 32) && R < (int64_t(1) << 32))
    hipLaunchKernelGGL(k_encode<true>, dim3(grid), dim3(256), 0, s, ytr, ldy, R, fp, encw, yencw, pos, resid, resid_bf,
                       FastDiv((uint32_t)fp.C), FastDiv((uint32_t)R));
  else
    hipLaunchKernelGGL(k_encode<false>, dim3(grid), dim3(256), 0, s, ytr, ldy, R, fp, encw, yencw, pos, resid, resid_bf,
                       FastDiv(), FastDiv());
}
static constexpr size_t kGemmSmem = 2 * (64 * 64 + 192 * 64) * sizeof(bf16_t);  // 64 KiB
// decoder-head rows per wave: 32 (8 waves per 128-row tile) or 64 (4 waves, 4 A + 6 B fragment
// reads per 24 MFMAs instead of 2 + 6 per 12).  r06, bitwise equal: WM 64 7.30 ms, WM 64 on
// 256-row tiles 8.57 ms, against 6.66 ms per c2 call at 32 (profiles/r06/ab_decoder_wm64_r06s.txt):
// the head GEMM is not bound by its LDS reads; the occupancy the wider wave tile costs is what counts
#ifndef NPFN_DEC_WM
#define NPFN_DEC_WM 32
#endif
#ifndef NPFN_DEC_MT
#define NPFN_DEC_MT 128
#endif
static constexpr size_t kGemmSmem128 = 2 * (NPFN_DEC_MT * 64 + 192 * 64) * sizeof(bf16_t);  // 80 KiB at 128
void gemm_setup() {
  (void)hipFuncSetAttribute((const void*)k_feat_attn, hipFuncAttributeMaxDynamicSharedMemorySize,
                            kFeatAttnMaxC * 576 * sizeof(bf16_t));
  (void)hipFuncSetAttribute((const void*)k_feat_attn_wide, hipFuncAttributeMaxDynamicSharedMemorySize,
                            kWideMaxC * 64 * sizeof(bf16_t));
  (void)hipFuncSetAttribute((const void*)k_gemm<EPI_LOGIT, NPFN_DEC_MT, NPFN_DEC_WM>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, kGemmSmem128);
  (void)hipFuncSetAttribute((const void*)k_gemm<EPI_LOGIT, NPFN_DEC_MT>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            kGemmSmem128);
  (void)hipFuncSetAttribute((const void*)k_gemm<EPI_BF16>, hipFuncAttributeMaxDynamicSharedMemorySize, kGemmSmem);
  (void)hipFuncSetAttribute((const void*)k_gemm<EPI_BF16_GELU>, hipFuncAttributeMaxDynamicSharedMemorySize, kGemmSmem);
  (void)hipFuncSetAttribute((const void*)k_gemm<EPI_LOGIT>, hipFuncAttributeMaxDynamicSharedMemorySize, kGemmSmem);
  (void)hipFuncSetAttribute((const void*)k_gemm<EPI_LN>, hipFuncAttributeMaxDynamicSharedMemorySize, kGemmSmem);
}
// decoder-head tile size: 128 rows unless NPFN_GEMM_MT64=1 (A/B switch)
static bool gemm_mt128() {
  static const bool v = [] { const char* e = getenv("NPFN_GEMM_MT64"); return !(e && e[0] == '1'); }();
  return v;
}
void launch_gemm(int epi, const bf16_t* A, int64_t lda, const bf16_t* W, int64_t M, int N, int K,
                 const EpiParams& p, hipStream_t s) {
  dim3 grid(blocks_for(M, 64), (unsigned)((N + 191) / 192));
  switch (epi) {
    case EPI_BF16: hipLaunchKernelGGL(k_gemm<EPI_BF16>, grid, dim3(256), kGemmSmem, s, A, lda, W, M, N, K, p); break;
    case EPI_BF16_GELU: hipLaunchKernelGGL(k_gemm<EPI_BF16_GELU>, grid, dim3(256), kGemmSmem, s, A, lda, W, M, N, K, p); break;
    case EPI_LOGIT:
      if (gemm_mt128()) {
        dim3 g128(blocks_for(M, NPFN_DEC_MT), grid.y);
        hipLaunchKernelGGL((k_gemm<EPI_LOGIT, NPFN_DEC_MT, NPFN_DEC_WM>), g128, dim3((NPFN_DEC_MT / NPFN_DEC_WM) * 128),
                           kGemmSmem128, s, A, lda, W, M, N, K, p);
      } else {
        hipLaunchKernelGGL(k_gemm<EPI_LOGIT>, grid, dim3(256), kGemmSmem, s, A, lda, W, M, N, K, p);
      }
      break;
    case EPI_LN: hipLaunchKernelGGL(k_gemm<EPI_LN>, grid, dim3(256), kGemmSmem, s, A, lda, W, M, N, K, p); break;
  }
}
void launch_feat_attn(const bf16_t* qkv, bf16_t* out, int64_t rows, int C, hipStream_t s) {
  if (C > kFeatAttnMaxC) {
    hipLaunchKernelGGL(k_feat_attn_wide, dim3((unsigned)(rows * 6)), dim3(256), (size_t)C * 64 * sizeof(bf16_t), s,
                       qkv, out, rows, C, 0.17677669529663687f /* 1/sqrt(32) */);
    return;
  }
  const size_t smem = (size_t)C * 576 * sizeof(bf16_t);
  hipLaunchKernelGGL(k_feat_attn, dim3((unsigned)rows), dim3(64), smem, s, qkv, out, rows, C,
                     0.17677669529663687f /* 1/sqrt(32) */);
}
void launch_kv_pack(const bf16_t* qkv, int64_t n, int C, int E, int ntile, bf16_t* kvc, hipStream_t s, int c_lo) {
  const int64_t tiles = (int64_t)E * (C - c_lo) * 6 * ntile;
  if (tiles <= 0) return;
  if (tiles < (int64_t(1) << 32))
    hipLaunchKernelGGL(k_kv_pack<true>, dim3(blocks_for(tiles, 4)), dim3(256), 0, s, qkv, n, C, E, ntile, kvc, c_lo,
                       FastDiv((uint32_t)ntile), FastDiv((uint32_t)(C - c_lo)));
  else
    hipLaunchKernelGGL(k_kv_pack<false>, dim3(blocks_for(tiles, 4)), dim3(256), 0, s, qkv, n, C, E, ntile, kvc, c_lo,
                       FastDiv(), FastDiv());
}
// npfn_debug_item_attn_online: every block also runs the online-softmax pass (tests of the fallback)
int g_item_attn_online = 0;
void set_item_attn_online(int on) { g_item_attn_online = on ? 1 : 0; }
// npfn_debug_item_attn_scale: multiplies every item-attention score (stress runs of the fallback)
float g_item_attn_scale = 1.0f;
void set_item_attn_scale(float s) { g_item_attn_scale = s; }
int64_t item_attn_blocks(const IaParams& p) { return (int64_t)blocks_for(p.R, 128 * kIaQs) * p.ny; }

void launch_item_attn(const IaParams& p, hipStream_t s) {
  if (p.R <= 0 || p.ny <= 0) return;
  dim3 grid(blocks_for(p.R, 128 * kIaQs), (unsigned)p.ny);
  const float scale_log2 = 0.17677669529663687f * 1.4426950408889634f * g_item_attn_scale;
  hipLaunchKernelGGL(k_item_attn, grid, dim3(256), 0, s, p, scale_log2, g_item_attn_online);
}
void launch_class_params(const float* y, int64_t ldy, int64_t n, int K, int E, uint64_t seed, int* cperm,
                         float* ybar_e, hipStream_t s) {
  hipLaunchKernelGGL(k_class_params, dim3(1), dim3(256), 0, s, y, ldy, n, K, E, seed, cperm, ybar_e);
}
void launch_cls_mix(const logit_t* logits, int64_t R, int E, int nout, int K, float invT, const int* cperm, int geo,
                    float* probs, int64_t ldo, hipStream_t s) {
  if (R <= 0) return;
  hipLaunchKernelGGL(k_cls_mix, dim3((unsigned)((R + 255) / 256)), dim3(256), 0, s, logits, R, E, nout, K, invT,
                     cperm, geo, probs, ldo);
}
static bool mix_fast(int nb) { return nb % 4 == 0 && nb <= 256 * 4 * kMixV4; }

static size_t mix_smem(int nb, const MixTrans& tr) {
  const size_t pb = ((size_t)nb * 4 + 15) & ~(size_t)15, pcb = tr.ett ? (size_t)nb * 8 : 0;
  return 64 + (mix_fast(nb) ? std::max(pb, pcb) : pb + pcb);  // fast path: p overlays pc
}

// k_mix_* instance for nb bars: the fast path with register arrays for 5 float4 per thread
// (up to 5120 bars: the default 5000 at 2 waves / SIMD more than the 8-float4 instance), or
// 8 (up to 8192 bars), or the generic path
#define NPFN_MIX_LAUNCH(KERNEL, nb, tr, s, ...)                                                       \
  do {                                                                                                \
    const dim3 g_((unsigned)R), b_(256);                                                              \
    const size_t sm_ = mix_smem(nb, tr);                                                              \
    if (!mix_fast(nb)) hipLaunchKernelGGL(KERNEL<0>, g_, b_, sm_, s, __VA_ARGS__);                    \
    else if ((nb + 1023) / 1024 <= 5) hipLaunchKernelGGL(KERNEL<5>, g_, b_, sm_, s, __VA_ARGS__);     \
    else hipLaunchKernelGGL(KERNEL<kMixV4>, g_, b_, sm_, s, __VA_ARGS__);                             \
  } while (0)

void launch_mix_log(const logit_t* logits, int64_t R, int E, int nb, float invT, const MixTrans& tr, float* out,
                    int64_t ldo, hipStream_t s) {
  if (R <= 0) return;
  NPFN_MIX_LAUNCH(k_mix_log, nb, tr, s, logits, R, E, nb, invT, tr, out, ldo);
}
void launch_mix_sample(const logit_t* logits, int64_t R, int E, int nb, float invT, const MixTrans& tr,
                       const float* bz, const float* ystats, uint64_t seed, uint64_t counter, int64_t row_offset,
                       uint64_t philox_row0, float* feat, int64_t ldf, int col, float* logp_acc, float log_eps,
                       hipStream_t s) {
  if (R <= 0) return;
  NPFN_MIX_LAUNCH(k_mix_sample, nb, tr, s, logits, R, E, nb, invT, tr, bz, ystats, seed, counter, row_offset,
                  philox_row0, feat, ldf, col, logp_acc, log_eps);
}
void launch_mix_prob(const logit_t* logits, int64_t R, int E, int nb, float invT, const MixTrans& tr, float* p_out,
                     hipStream_t s) {
  if (R <= 0) return;
  NPFN_MIX_LAUNCH(k_mix_prob, nb, tr, s, logits, R, E, nb, invT, tr, p_out);
}
void launch_group_sample(const float* p_rows, int64_t per, int64_t R, int nb, const float* bz, const float* ystats,
                         uint64_t seed, uint64_t counter, int64_t row_offset, uint64_t philox_row0, float* feat,
                         int64_t ldf, int col, float* logp_acc, float log_eps, hipStream_t s) {
  if (R <= 0) return;
  hipLaunchKernelGGL(k_group_sample, dim3((unsigned)R), dim3(256), 64 + (size_t)nb * 4, s, p_rows, per, nb, bz, ystats,
                     seed, counter, row_offset, philox_row0, feat, ldf, col, logp_acc, log_eps);
}
void launch_group_nll(const float* p_rows, int64_t per, int64_t R, int nb, const float* bz, const float* ystats,
                      int64_t row_offset, const float* feat, int64_t ldf, int col, float* logp_acc, float log_eps,
                      hipStream_t s) {
  if (R <= 0) return;
  hipLaunchKernelGGL(k_group_nll, dim3((unsigned)R), dim3(256), 64 + (size_t)nb * 4, s, p_rows, per, nb, bz, ystats,
                     row_offset, feat, ldf, col, logp_acc, log_eps);
}
void launch_mix_nll(const logit_t* logits, int64_t R, int E, int nb, float invT, const MixTrans& tr, const float* bz,
                    const float* ystats, int64_t row_offset, const float* feat, int64_t ldf, int col,
                    float* logp_acc, float log_eps, hipStream_t s) {
  if (R <= 0) return;
  NPFN_MIX_LAUNCH(k_mix_nll, nb, tr, s, logits, R, E, nb, invT, tr, bz, ystats, row_offset, feat, ldf, col, logp_acc,
                  log_eps);
}
void launch_bar_sample(const float* logits, const float* borders, int64_t R, int nb, uint64_t seed,
                       uint64_t counter, float* out, hipStream_t s) {
  hipLaunchKernelGGL(k_bar_sample, dim3((unsigned)R), dim3(256), (size_t)nb * 4, s, logits, borders, R, nb,
                     seed, counter, out);
}
void launch_bar_nll(const float* logits, const float* borders, const float* y, int64_t R, int nb, float* out,
                    hipStream_t s) {
  hipLaunchKernelGGL(k_bar_nll, dim3((unsigned)R), dim3(256), 0, s, logits, borders, y, R, nb, out);
}
void launch_borders(const float* bz, const float* ystats, int nb, float* out, hipStream_t s) {
  hipLaunchKernelGGL(k_borders, dim3(blocks_for(nb + 1, 256)), dim3(256), 0, s, bz, ystats, nb, out);
}
void launch_copy_cols(const float* src, int64_t lds, float* dst, int64_t ldd, int64_t rows, int cols,
                      int dst_col0, hipStream_t s, int64_t per) {
  if (rows * cols == 0) return;
  hipLaunchKernelGGL(k_copy_cols, dim3(blocks_for(rows * cols, 256)), dim3(256), 0, s, src, lds, dst, ldd, rows,
                     cols, dst_col0, per);
}
void launch_fill(float* dst, int64_t n, float v, hipStream_t s) {
  if (n == 0) return;
  hipLaunchKernelGGL(k_fill, dim3(blocks_for(n, 256)), dim3(256), 0, s, dst, n, v);
}
void launch_box_support(const float* th, int64_t n, int dim, const float* lo, const float* hi, uint8_t* mask,
                        hipStream_t s) {
  if (n == 0) return;
  hipLaunchKernelGGL(k_box_support, dim3(blocks_for(n, 256)), dim3(256), 0, s, th, n, dim, lo, hi, mask);
}

}  // namespace npfn
