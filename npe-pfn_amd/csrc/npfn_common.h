// npfn_common.h -- shared device helpers for the gfx950 NPE-PFN engine.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

typedef uint16_t bf16_t;  // raw bf16 bits
typedef __attribute__((ext_vector_type(8))) short bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(16))) float f32x16;

#define NPFN_WAVE 64

__device__ __forceinline__ float bf2f(bf16_t h) { return __uint_as_float(((uint32_t)h) << 16); }

typedef __bf16 bf16x2_hw __attribute__((ext_vector_type(2)));

// n / d and n % d for a 32-bit unsigned n and a divisor fixed at launch (multiply-high, add,
// shift -- Granlund-Montgomery with the 33-bit magic m' = 2^32 + m -- instead of the compiler's
// integer division sequence; exhaustive for every n < 2^32: (n + mulhi(n, m)) >> s, s =
// ceil(log2 d), m = floor(2^32 (2^s - d) / d) + 1).  For index decompositions of a launch's
// units: k_encode's (estimator, row, token) and k_kv_pack's (estimator, column, head, tile)
// were bound by their 64-bit divisions.
struct FastDiv {
  uint32_t d = 1, m = 1, s = 0;
  FastDiv() = default;
  __host__ explicit FastDiv(uint32_t dd) : d(dd) {
    while ((1ull << s) < dd) ++s;
    m = (uint32_t)(((1ull << 32) * ((1ull << s) - dd)) / dd + 1);
  }
  __device__ __forceinline__ uint32_t div(uint32_t n) const {
    return (uint32_t)(((uint64_t)__umulhi(n, m) + n) >> s);
  }
  __device__ __forceinline__ uint32_t divmod(uint32_t n, uint32_t& r) const {
    const uint32_t q = div(n);
    r = n - q * d;
    return q;
  }
};

// round-to-nearest-even float -> bf16 via v_cvt_pk_bf16_f32 (NaN stays NaN)
__device__ __forceinline__ bf16_t f2bf(float f) { return __builtin_bit_cast(bf16_t, (__bf16)f); }

__device__ __forceinline__ uint32_t pack_bf2(float a, float b) {
  bf16x2_hw v = {(__bf16)a, (__bf16)b};
  return __builtin_bit_cast(uint32_t, v);
}

// Cross-half-row / cross-half-wave combines without an LDS round trip: v_permlane16_swap /
// v_permlane32_swap (gfx950) of x with itself hands every lane {own, partner} (lane ^ 16,
// resp. lane ^ 32) in some order; + and max are commutative, so both partners get the
// bitwise-same result.
__device__ __forceinline__ float xor16_sum(float x) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ float xor32_sum(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
// (the max as one asm v_max_f32: fmaxf puts a canonicalising v_max x, x in front of each
// operand; the operands come from the permlane, never straight from an MFMA)
__device__ __forceinline__ float vmax_f32(float a, float b) {
  float r;
  asm("v_max_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ float xor16_max(float x) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return vmax_f32(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float xor32_max(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return vmax_f32(__uint_as_float(r[0]), __uint_as_float(r[1]));
}

// max(a, b, c) as one v_max3_f32, in asm so that no canonicalising v_max x, x is put in
// front of each MFMA-produced operand (plain fmaxf chains on accumulators get one per input).
// The hazard recognizer does not look into asm: an MFMA result must first be read by a
// compiler-visible VALU op (which gets the read-after-write wait states), never by max3f.
__device__ __forceinline__ float max3f(float a, float b, float c) {
  float r;
  asm("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
// Wave-wide max / sum / inclusive scan through DPP row operations and the gfx950 permlane
// swaps -- VALU-only, no LDS round trip (a __shfl_xor / __shfl_up is a ds_bpermute: ~100+ cycles
// of latency per step of a dependent chain).  Every lane gets the max / sum.  The sum's order
// differs from wave_sum's butterfly: the callers (the ensemble mix and the bar sampler) are not
// pinned bit for bit to it.
template <int CTRL, int ROW_MASK = 0xF, bool BOUND = false>
__device__ __forceinline__ float dppf(float old, float x) {
  return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(old), __float_as_int(x), CTRL, ROW_MASK, 0xF, BOUND));
}
__device__ __forceinline__ float wave_max_dpp(float v) {
  v = vmax_f32(v, dppf<0xB1>(v, v));   // quad_perm [1, 0, 3, 2]: lane ^ 1
  v = vmax_f32(v, dppf<0x4E>(v, v));   // quad_perm [2, 3, 0, 1]: lane ^ 2
  v = vmax_f32(v, dppf<0x141>(v, v));  // row_half_mirror: the other quad of the 8
  v = vmax_f32(v, dppf<0x140>(v, v));  // row_mirror: the other half of the row of 16
  return xor32_max(xor16_max(v));
}
__device__ __forceinline__ float wave_sum_dpp(float v) {
  v += dppf<0xB1>(v, v);
  v += dppf<0x4E>(v, v);
  v += dppf<0x141>(v, v);
  v += dppf<0x140>(v, v);
  return xor32_sum(xor16_sum(v));
}
// inclusive prefix sum over the wave's 64 lanes: row_shr 1, 2, 4, 8 within each row of 16 (a
// lane without a source adds 0), then row_bcast 15 / 31 carry the rows' totals forward
__device__ __forceinline__ float wave_incl_scan_dpp(float v) {
  v += dppf<0x111, 0xF, true>(0.f, v);  // row_shr:1
  v += dppf<0x112, 0xF, true>(0.f, v);  // row_shr:2
  v += dppf<0x114, 0xF, true>(0.f, v);  // row_shr:4
  v += dppf<0x118, 0xF, true>(0.f, v);  // row_shr:8
  v += dppf<0x142, 0xA>(0.f, v);        // row_bcast:15 into rows 1 and 3
  v += dppf<0x143, 0xC>(0.f, v);        // row_bcast:31 into rows 2 and 3
  return v;
}

__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Philox4x32-10 (Salmon et al. SC'11); same as oracle/philox.py.
__device__ __forceinline__ uint32_t philox_x0(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                                              uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    uint64_t p0 = (uint64_t)0xD2511F53u * c0;
    uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
    uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
    c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
    k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
  return c0;
}

// u(seed, counter, row) in [0,1) with 24 random bits -- oracle.philox.uniforms
__device__ __forceinline__ float philox_uniform(uint64_t seed, uint64_t counter, uint64_t row) {
  uint32_t x = philox_x0((uint32_t)row, (uint32_t)(row >> 32), (uint32_t)counter,
                         (uint32_t)(counter >> 32), (uint32_t)seed, (uint32_t)(seed >> 32));
  return (float)(x >> 8) * 5.9604644775390625e-08f;  // 2^-24
}

__device__ __forceinline__ uint64_t splitmix64_next(uint64_t& s) {
  s += 0x9E3779B97F4A7C15ull;
  uint64_t z = s;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// GELU, exact (erf) form, as nn.GELU()
__device__ __forceinline__ float gelu_f(float x) { return 0.5f * x * (1.0f + erff(x * 0.7071067811865476f)); }

// GELU(x) = x * Phi(x) with Phi from the Abramowitz-Stegun 7.1.26 erfc form
// (|erf error| <= 1.5e-7, far below the bf16 rounding of the stored activation):
// Phi(x) = 1 - h (x >= 0) or h (x < 0), h = 0.5 * t * P(t) * exp(-x^2/2), t = 1/(1 + p|x|/sqrt2).
__device__ __forceinline__ float gelu_fast(float x) {
  const float z = fabsf(x) * 0.7071067811865476f;
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, z, 1.0f));
  float poly = fmaf(1.061405429f, t, -1.453152027f);
  poly = fmaf(poly, t, 1.421413741f);
  poly = fmaf(poly, t, -0.284496736f);
  poly = fmaf(poly, t, 0.254829592f);
  const float h = 0.5f * t * poly * __builtin_amdgcn_exp2f(-z * z * 1.4426950408889634f);
  return x * (x >= 0.f ? 1.0f - h : h);
}

typedef __attribute__((ext_vector_type(2))) float f32x2;

// gelu_fast on two values: the polynomial and products run as packed fp32
// (v_pk_fma_f32 / v_pk_mul_f32), only rcp, exp2 and the sign select are per value.
__device__ __forceinline__ f32x2 gelu_fast2(f32x2 x) {
  const f32x2 ax = {fabsf(x.x), fabsf(x.y)};
  const f32x2 den = ax * (0.3275911f * 0.7071067811865476f) + 1.0f;
  const f32x2 t = {__builtin_amdgcn_rcpf(den.x), __builtin_amdgcn_rcpf(den.y)};
  f32x2 poly = t * 1.061405429f + -1.453152027f;
  poly = poly * t + 1.421413741f;
  poly = poly * t + -0.284496736f;
  poly = poly * t + 0.254829592f;
  const f32x2 arg = x * x * (-0.5f * 1.4426950408889634f);
  const f32x2 e = {__builtin_amdgcn_exp2f(arg.x), __builtin_amdgcn_exp2f(arg.y)};
  const f32x2 h = (t * 0.5f) * poly * e;
  const f32x2 phi = {x.x >= 0.f ? 1.0f - h.x : h.x, x.y >= 0.f ? 1.0f - h.y : h.y};
  return x * phi;
}

// GELU in the tanh form, 0.5 x (1 + tanh(sqrt(2/pi) (x + 0.044715 x^3))) = x - x / (e^{2y} + 1):
// 7 VALU (2 transcendental) per value against 16 for gelu_fast.  |gelu_tanh - GELU_erf| <=
// 4.8e-4 (at x = -2.7, where GELU = -0.0094); the row kernel stores the result in bf16,
// whose rounding (2^-9 relative) exceeds that error for |GELU| >= 0.25.
__device__ __forceinline__ float gelu_tanh(float x) {
  const float z = x * fmaf(x * x, 0.1029432395800235f, 2.302208198144325f);  // 2 log2(e) y
  const float r = __builtin_amdgcn_rcpf(__builtin_amdgcn_exp2f(z) + 1.0f);
  return fmaf(-x, r, x);
}

#define NPFN_HALFNORMAL_MEDIAN 0.6744897501960817

// LDS-only workgroup barrier: lgkmcnt(0) + s_barrier, no vmcnt drain, so LDS-DMA
// (glds16) stays in flight across it (a __syncthreads() fence would wait for it).
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// LDS-DMA with a scalar base: lane i copies 16 bytes from sbase + voff_i (voff a per-lane
// 32-bit byte offset) to lds_dst + 16 i; no 64-bit per-lane address arithmetic.
// sbase and lds_dst must be wave-uniform; readfirstlane makes that explicit to the compiler
// (an SGPR operand it could not prove uniform would otherwise be a VGPR pair: invalid).
__device__ __forceinline__ void glds16_s(const void* sbase, uint32_t voff, uint32_t lds_dst) {
  const uint64_t a = (uint64_t)(uintptr_t)sbase;
  // readfirstlane returns int: widen through uint32_t, or a low word >= 2^31 sign-extends
  // into the high word and the address is garbage
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)a);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(a >> 32));
  const uint64_t sa = ((uint64_t)hi << 32) | (uint64_t)lo;
  const uint32_t sl = (uint32_t)__builtin_amdgcn_readfirstlane((int)lds_dst);
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(voff), "s"(sa), "s"(sl)
               : "memory");
}

// LDS-DMA: 16 bytes global -> LDS per lane (global_load_lds_dwordx4); lds_dst is the
// wave-uniform LDS byte address of lane 0's 16 bytes, lane i lands at lds_dst + 16 i.
// Not tracked by the compiler's waitcnt bookkeeping: wait with a counted vmcnt.
__device__ __forceinline__ void glds16(const void* gsrc, uint32_t lds_dst) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(gsrc), "s"(lds_dst)
               : "memory");
}
