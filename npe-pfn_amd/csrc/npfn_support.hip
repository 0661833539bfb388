// npfn_support.hip -- K9/K10 stream compaction, K11 SIR resampling and K12
// standardized-Euclidean context filter (SURVEY.md §2 native-components table).
#include <hip/hip_runtime.h>

#include <cfloat>
#include <string>

#include "npfn.h"
#include "npfn_common.h"
#include "npfn_kernels.h"

namespace {

// K9: ordered stream compaction of rows with mask != 0 (accept_reject_sampler.py:54-59).
// Single workgroup: rows are consumed in 1024-row chunks in order, so the output
// keeps the input order exactly like `candidates[are_accepted]`.
__global__ __launch_bounds__(1024) void k_compact(const float* __restrict__ src, const uint8_t* __restrict__ mask,
                                                  int64_t n, int dim, float* __restrict__ dst,
                                                  int64_t* __restrict__ count) {
  __shared__ int wsum[16];
  __shared__ long long base;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  if (tid == 0) base = 0;
  __syncthreads();
  for (int64_t c0 = 0; c0 < n; c0 += 1024) {
    const int64_t i = c0 + tid;
    const bool flag = (i < n) && mask[i] != 0;
    const unsigned long long bal = __ballot(flag);
    const int rank = __popcll(bal & ((1ull << lane) - 1ull));
    if (lane == 0) wsum[w] = __popcll(bal);
    __syncthreads();
    int pre = 0, tot = 0;
    for (int q = 0; q < 16; ++q) {
      if (q < w) pre += wsum[q];
      tot += wsum[q];
    }
    if (flag) {
      const int64_t o = base + pre + rank;
      for (int j = 0; j < dim; ++j) dst[o * dim + j] = src[i * dim + j];
    }
    __syncthreads();
    if (tid == 0) base += tot;
    __syncthreads();
  }
  if (tid == 0) *count = base;
}

// K12 step 1: column mean / unbiased std (torch.mean / torch.std, support_posterior.py:358-359)
__global__ __launch_bounds__(256) void k_colmeanstd(const float* __restrict__ x, int64_t n, int dim,
                                                    float* __restrict__ ms) {
  __shared__ double red[4];
  const int j = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  double s = 0.0;
  for (int64_t i = tid; i < n; i += 256) s += x[i * dim + j];
  s = wave_sum_d(s);
  if (lane == 0) red[w] = s;
  __syncthreads();
  const double mean = (red[0] + red[1] + red[2] + red[3]) / (double)n;
  __syncthreads();
  double q = 0.0;
  for (int64_t i = tid; i < n; i += 256) {
    const double dv = x[i * dim + j] - mean;
    q += dv * dv;
  }
  q = wave_sum_d(q);
  if (lane == 0) red[w] = q;
  __syncthreads();
  if (tid == 0) {
    ms[2 * j] = (float)mean;
    ms[2 * j + 1] = (float)sqrt((red[0] + red[1] + red[2] + red[3]) / (double)(n > 1 ? n - 1 : 1));
  }
}

// K12 step 2: key = (bits(dist) << 32) | row, padded with UINT64_MAX to a power of two
__global__ void k_dist_keys(const float* __restrict__ x, int64_t n, int dim, const float* __restrict__ obs,
                            const float* __restrict__ ms, int64_t npow, unsigned long long* __restrict__ keys) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= npow) return;
  if (i >= n) {
    keys[i] = ~0ull;
    return;
  }
  float acc = 0.f;
  for (int j = 0; j < dim; ++j) {
    const float m = ms[2 * j], sd = ms[2 * j + 1];
    const float xs = (x[i * dim + j] - m) / sd;
    const float os = (obs[j] - m) / sd;
    const float df = xs - os;
    acc += df * df;
  }
  const float dist = sqrtf(acc);
  unsigned int bits = __float_as_uint(dist);
  if (dist != dist) bits = 0xffffffffu;  // NaN last
  keys[i] = ((unsigned long long)bits << 32) | (unsigned long long)(uint32_t)i;
}

__global__ void k_bitonic_step(unsigned long long* __restrict__ keys, int64_t npow, int64_t k, int64_t j) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= npow) return;
  const int64_t ixj = i ^ j;
  if (ixj <= i) return;
  const unsigned long long a = keys[i], b = keys[ixj];
  const bool up = (i & k) == 0;
  if ((a > b) == up) {
    keys[i] = b;
    keys[ixj] = a;
  }
}

__global__ void k_take_idx(const unsigned long long* __restrict__ keys, int64_t k, int64_t* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < k) out[i] = (int64_t)(keys[i] & 0xffffffffull);
}

// K11: SIR resampling step (support_posterior.py:216-241).  One wave per group of k
// proposals: log ratio lw = nan_to_num(lpr - lq, nan=-inf) with lpr := -inf where
// lq < thr (:220-223); ESS = 1 / sum_i exp(lw_i - lse)^2 with lse = max + log(sum
// exp(lw - max)) in fp32 as torch.logsumexp forms it (:228-232); the pick is the inverse
// CDF of softmax(lw) at u = Philox(seed, counter, group) (the reference's Categorical draw,
// :234-235), found by a wave-level prefix sum in fp64; the picked row is gathered (:236-241).
// HBM-bound: 8 B per proposal read once per pass (3 passes, L2-resident for k <= 4096).
__device__ __forceinline__ float sir_log_ratio(float lpr, float lq, float thr) {
  const float d = (lq < thr ? -INFINITY : lpr) - lq;
  if (d != d) return -INFINITY;
  return fminf(fmaxf(d, -FLT_MAX), FLT_MAX);
}

__global__ __launch_bounds__(256) void k_sir_select(const float* __restrict__ lpr, const float* __restrict__ lq,
                                                    const float* __restrict__ thr_p, int64_t groups, int k,
                                                    uint64_t seed, uint64_t counter, int64_t group_offset,
                                                    const float* __restrict__ theta, int dim,
                                                    int64_t* __restrict__ pick, float* __restrict__ ess,
                                                    float* __restrict__ theta_out) {
  const int lane = threadIdx.x & 63;
  const int64_t g = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (g >= groups) return;  // wave-uniform
  const float thr = *thr_p;
  const float* a = lpr + g * k;
  const float* b = lq + g * k;
  float m = -INFINITY;
  for (int i = lane; i < k; i += 64) m = fmaxf(m, sir_log_ratio(a[i], b[i], thr));
  m = wave_max(m);
  int sel = 0;
  float ess_g = __builtin_nanf("");  // every ratio NaN: torch's probabilities are NaN
  if (m != -INFINITY) {
    double s = 0.0;
    for (int i = lane; i < k; i += 64) s += (double)expf(sir_log_ratio(a[i], b[i], thr) - m);
    s = wave_sum_d(s);
    const float lse = m + logf((float)s);
    double q = 0.0;
    for (int i = lane; i < k; i += 64) {
      const double p = (double)expf(sir_log_ratio(a[i], b[i], thr) - lse);
      q += p * p;
    }
    q = wave_sum_d(q);
    ess_g = (float)(1.0 / q);
    // first i with sum_{j <= i} e_j > u * s
    const double target = (double)philox_uniform(seed, counter, (uint64_t)(group_offset + g)) * s;
    double base = 0.0;
    int last = 0;
    sel = -1;
    for (int c0 = 0; c0 < k; c0 += 64) {
      const int i = c0 + lane;
      const double e = i < k ? (double)expf(sir_log_ratio(a[i], b[i], thr) - m) : 0.0;
      double incl = e;
#pragma unroll
      for (int off = 1; off < 64; off <<= 1) {
        const double t = __shfl_up(incl, off, 64);
        if (lane >= off) incl += t;
      }
      const unsigned long long hit = __ballot(base + incl > target);
      if (hit) {
        sel = c0 + __ffsll((long long)hit) - 1;
        break;
      }
      const unsigned long long nz = __ballot(e > 0.0);
      if (nz) last = c0 + 63 - __clzll((long long)nz);
      base += __shfl(incl, 63, 64);
    }
    if (sel < 0) sel = last;  // u * s rounded past the total: last proposal with mass
  }
  if (lane == 0) {
    pick[g] = sel;
    ess[g] = ess_g;
  }
  if (theta_out)
    for (int j = lane; j < dim; j += 64) theta_out[g * dim + j] = theta[(g * k + sel) * dim + j];
}

int fail(int code, const std::string& msg) { return npfn::set_error(code, msg.c_str()); }

int launch_status(const char* what) {
  const hipError_t e = hipGetLastError();
  if (e == hipSuccess) return NPFN_OK;
  return fail(NPFN_EHIP, std::string(what) + ": " + hipGetErrorString(e));
}

}  // namespace

extern "C" {

int npfn_compact_rows(const float* src, const uint8_t* mask, int64_t n_rows, int32_t dim, float* dst,
                      int64_t* count_out, void* stream) {
  if (!src || !mask || !dst || !count_out) return fail(NPFN_EINVAL, "compact_rows: null pointer");
  if (dim < 1 || n_rows < 0) return fail(NPFN_EINVAL, "compact_rows: need dim >= 1 and n_rows >= 0");
  hipLaunchKernelGGL(k_compact, dim3(1), dim3(1024), 0, (hipStream_t)stream, src, mask, n_rows, dim, dst,
                     count_out);
  return launch_status("compact_rows: k_compact launch");
}

int npfn_filter_stdeuclid(const float* x, int64_t n_rows, int32_t dim, const float* obs, int64_t k,
                          int64_t* idx_out, void* stream) {
  if (!x || !obs || !idx_out) return fail(NPFN_EINVAL, "filter_stdeuclid: null pointer");
  if (dim < 1 || n_rows < 1 || k < 0 || k > n_rows)
    return fail(NPFN_EINVAL, "filter_stdeuclid: need dim >= 1, n_rows >= 1 and 0 <= k <= n_rows");
  if (n_rows > 0xffffffffll) return fail(NPFN_EINVAL, "filter_stdeuclid: more than 2^32 rows");
  hipStream_t s = (hipStream_t)stream;
  int64_t npow = 1;
  while (npow < n_rows) npow <<= 1;
  float* ms = nullptr;
  unsigned long long* keys = nullptr;
  if (hipMallocAsync((void**)&ms, sizeof(float) * 2 * dim, s) != hipSuccess) {
    (void)hipGetLastError();
    return fail(NPFN_ENOMEM, "filter_stdeuclid: hipMallocAsync of the column statistics failed");
  }
  if (hipMallocAsync((void**)&keys, sizeof(unsigned long long) * npow, s) != hipSuccess) {
    (void)hipGetLastError();
    (void)hipFreeAsync(ms, s);
    return fail(NPFN_ENOMEM, "filter_stdeuclid: hipMallocAsync of " + std::to_string(npow) + " sort keys failed");
  }
  hipLaunchKernelGGL(k_colmeanstd, dim3(dim), dim3(256), 0, s, x, n_rows, dim, ms);
  const unsigned nb = (unsigned)((npow + 255) / 256);
  hipLaunchKernelGGL(k_dist_keys, dim3(nb), dim3(256), 0, s, x, n_rows, dim, obs, ms, npow, keys);
  for (int64_t kk = 2; kk <= npow; kk <<= 1)
    for (int64_t j = kk >> 1; j > 0; j >>= 1)
      hipLaunchKernelGGL(k_bitonic_step, dim3(nb), dim3(256), 0, s, keys, npow, kk, j);
  if (k > 0) hipLaunchKernelGGL(k_take_idx, dim3((unsigned)((k + 255) / 256)), dim3(256), 0, s, keys, k, idx_out);
  (void)hipFreeAsync(keys, s);
  (void)hipFreeAsync(ms, s);
  return launch_status("filter_stdeuclid: kernel launch");
}

int npfn_sir_select(const float* lpr, const float* lq, const float* thr, int64_t n_groups, int32_t k,
                    uint64_t seed, uint64_t counter, int64_t group_offset, const float* theta, int32_t dim,
                    int64_t* pick_out, float* ess_out, float* theta_out, void* stream) {
  if (!lpr || !lq || !thr || !pick_out || !ess_out) return fail(NPFN_EINVAL, "sir_select: null pointer");
  if (n_groups < 0 || k < 1 || group_offset < 0)
    return fail(NPFN_EINVAL, "sir_select: need n_groups >= 0, k >= 1 and group_offset >= 0");
  if (theta_out && (!theta || dim < 1)) return fail(NPFN_EINVAL, "sir_select: theta_out needs theta and dim >= 1");
  if (n_groups == 0) return NPFN_OK;
  if ((n_groups + 3) / 4 > 0x7fffffffll) return fail(NPFN_EINVAL, "sir_select: too many groups for one launch");
  hipLaunchKernelGGL(k_sir_select, dim3((unsigned)((n_groups + 3) / 4)), dim3(256), 0, (hipStream_t)stream, lpr,
                     lq, thr, n_groups, (int)k, seed, counter, group_offset, theta, theta_out ? (int)dim : 0,
                     pick_out, ess_out, theta_out);
  return launch_status("sir_select: k_sir_select launch");
}

}  // extern "C"
