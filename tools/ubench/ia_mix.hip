// Throughput ceiling of k_item_attn's per-step instruction mix on gfx950 (no dependencies between
// the matrix and vector work, no memory): per loop body and wave 16 v_mfma_f32_32x32x16_bf16 on
// 4 independent accumulators, 64 v_exp_f32, 32 v_cvt_pk_bf16_f32, 32 v_pk_add_f32 -- the
// compiled first-pass step of k_item_attn (two 32-query sets).  Variants drop one part, or put
// the exps on the plain VALU path (v_fma_f32), so the cycles show which pipe bounds the mix and
// whether the matrix, transcendental and plain-vector work overlap.  8 waves per block (two per
// SIMD, the kernel's occupancy is 3), cycles from s_memtime: the block's span / steps per SIMD.
// hipcc --offload-arch=gfx950 -O3 tools/ubench/ia_mix.hip -o /tmp/ia_mix && /tmp/ia_mix
// (-DIA_MIX_AGPR: the MFMA accumulators in AccVGPRs, through inline asm)
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef __attribute__((ext_vector_type(8))) short bf16x8;
typedef __attribute__((ext_vector_type(16))) float f32x16;

#define EXP8 \
  asm volatile("v_exp_f32 %0, %0\n\tv_exp_f32 %1, %1\n\tv_exp_f32 %2, %2\n\tv_exp_f32 %3, %3\n\t"       \
               "v_exp_f32 %4, %4\n\tv_exp_f32 %5, %5\n\tv_exp_f32 %6, %6\n\tv_exp_f32 %7, %7"           \
               : "+v"(e0), "+v"(e1), "+v"(e2), "+v"(e3), "+v"(e4), "+v"(e5), "+v"(e6), "+v"(e7))
#define FMA8 \
  asm volatile("v_fma_f32 %0, %0, %0, %0\n\tv_fma_f32 %1, %1, %1, %1\n\tv_fma_f32 %2, %2, %2, %2\n\t" \
               "v_fma_f32 %3, %3, %3, %3\n\tv_fma_f32 %4, %4, %4, %4\n\tv_fma_f32 %5, %5, %5, %5\n\t" \
               "v_fma_f32 %6, %6, %6, %6\n\tv_fma_f32 %7, %7, %7, %7"                                 \
               : "+v"(e0), "+v"(e1), "+v"(e2), "+v"(e3), "+v"(e4), "+v"(e5), "+v"(e6), "+v"(e7))
#define CVT4 \
  asm volatile("v_cvt_pk_bf16_f32 %0, %0, %0\n\tv_cvt_pk_bf16_f32 %1, %1, %1\n\t"                     \
               "v_cvt_pk_bf16_f32 %2, %2, %2\n\tv_cvt_pk_bf16_f32 %3, %3, %3"                         \
               : "+v"(c0), "+v"(c1), "+v"(c2), "+v"(c3))
#define PKADD4 \
  asm volatile("v_pk_add_f32 %0, %0, %0\n\tv_pk_add_f32 %1, %1, %1\n\t"                               \
               "v_pk_add_f32 %2, %2, %2\n\tv_pk_add_f32 %3, %3, %3"                                   \
               : "+v"(d0), "+v"(d1), "+v"(d2), "+v"(d3))

// V: 0 full mix, 1 MFMA only, 2 vector only, 3 mix with the exps as v_fma_f32, 4 exps only,
// 5 MFMA + exps, 6 MFMA + plain vector (cvt + pk_add)
template <int V>
__global__ __launch_bounds__(1024) void k(unsigned long long* out, float seed) {
  float e0 = seed, e1 = seed + 1, e2 = seed + 2, e3 = seed + 3, e4 = seed + 4, e5 = seed + 5, e6 = seed + 6,
        e7 = seed + 7;
  float c0 = seed, c1 = seed, c2 = seed, c3 = seed;
  double d0 = seed, d1 = seed, d2 = seed, d3 = seed;
  bf16x8 a = {1, 2, 3, 4, 5, 6, 7, 8};
  bf16x8 b = {8, 7, 6, 5, 4, 3, 2, 1};
  f32x16 acc[4] = {};
  const int iters = 512;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int m = 0; m < 4; ++m) {  // a quarter of the step: 4 MFMA, 16 exp, 8 cvt, 8 pk_add
      if constexpr (V != 2 && V != 4) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
#ifdef IA_MIX_AGPR  // accumulators in the AccVGPR file (the MFMA's C/D off the ArchVGPR ports)
          asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(acc[j]) : "v"(a), "v"(b));
#else
          acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc[j], 0, 0, 0);
#endif
        }
      }
      if constexpr (V == 0 || V == 2 || V == 4 || V == 5) { EXP8; EXP8; }
      if constexpr (V == 3) { FMA8; FMA8; }
      if constexpr (V == 0 || V == 2 || V == 3 || V == 6) { CVT4; CVT4; PKADD4; PKADD4; }
    }
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  float s = e0 + e1 + e2 + e3 + e4 + e5 + e6 + e7 + c0 + c1 + c2 + c3 + (float)(d0 + d1 + d2 + d3);
  for (int j = 0; j < 4; ++j) s += acc[j][0] + acc[j][15];
  if ((threadIdx.x & 63) == 0) {
    out[2 * (threadIdx.x >> 6)] = t0;
    out[2 * (threadIdx.x >> 6) + 1] = t1 + (unsigned long long)(s * 0.f);
  }
}

template <int V>
double run(unsigned long long* d, int waves) {
  hipLaunchKernelGGL(k<V>, dim3(1), dim3(64 * waves), 0, 0, d, 0.5f);
  hipDeviceSynchronize();
  unsigned long long h[32];
  hipMemcpy(h, d, 2 * waves * 8, hipMemcpyDeviceToHost);
  unsigned long long a = h[0], b = h[1];
  for (int i = 0; i < waves; ++i) {
    a = h[2 * i] < a ? h[2 * i] : a;
    b = h[2 * i + 1] > b ? h[2 * i + 1] : b;
  }
  return (double)(b - a) / (512.0 * (waves / 4));  // the block's span per step and SIMD
}


// The row kernel's shape: v_mfma_f32_16x16x32_bf16 (16 cycles) with N plain VALU ops
// (v_pk_add_f32 / v_cvt_pk_bf16_f32, independent of the MFMAs) per MFMA.
typedef __attribute__((ext_vector_type(4))) float f32x4;
template <int N>
__global__ __launch_bounds__(1024) void k16(unsigned long long* out, float seed) {
  float c0 = seed, c1 = seed, c2 = seed, c3 = seed;
  double d0 = seed, d1 = seed, d2 = seed, d3 = seed;
  bf16x8 a = {1, 2, 3, 4, 5, 6, 7, 8};
  bf16x8 b = {8, 7, 6, 5, 4, 3, 2, 1};
  f32x4 acc[8] = {};
  const int iters = 512;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if constexpr (N >= 0) acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc[j], 0, 0, 0);
      if constexpr (N == -1 || N >= 4) { CVT4; }
      if constexpr (N == -1 || N >= 8) { PKADD4; }
    }
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  float s = c0 + c1 + c2 + c3 + (float)(d0 + d1 + d2 + d3);
  for (int j = 0; j < 8; ++j) s += acc[j][0];
  if ((threadIdx.x & 63) == 0) {
    out[2 * (threadIdx.x >> 6)] = t0;
    out[2 * (threadIdx.x >> 6) + 1] = t1 + (unsigned long long)(s * 0.f);
  }
}
template <int N>
double run16(unsigned long long* d, int waves) {
  hipLaunchKernelGGL(k16<N>, dim3(1), dim3(64 * waves), 0, 0, d, 0.5f);
  hipDeviceSynchronize();
  unsigned long long h[32];
  hipMemcpy(h, d, 2 * waves * 8, hipMemcpyDeviceToHost);
  unsigned long long a = h[0], b = h[1];
  for (int i = 0; i < waves; ++i) {
    a = h[2 * i] < a ? h[2 * i] : a;
    b = h[2 * i + 1] > b ? h[2 * i + 1] : b;
  }
  return (double)(b - a) / (512.0 * 8 * (waves / 4));  // per MFMA slot and SIMD
}

int main() {
  unsigned long long* d;
  hipMalloc(&d, 64 * 8);
  const char* names[] = {"full mix (16 mfma, 64 exp, 32 cvt, 32 pk_add)", "mfma only", "vector only",
                         "mix, exps as v_fma_f32", "exps only", "mfma + exps", "mfma + cvt + pk_add"};
  for (int w : {4, 8, 12}) {
    run<0>(d, w);
    double c[7] = {run<0>(d, w), run<1>(d, w), run<2>(d, w), run<3>(d, w), run<4>(d, w), run<5>(d, w), run<6>(d, w)};
    printf("waves per block %d (%d per SIMD): s_memtime cycles per step of work and SIMD (block span)\n", w, w / 4);
    for (int i = 0; i < 7; ++i) printf("  %-48s %8.1f\n", names[i], c[i]);
  }
  for (int w : {8, 12}) {
    run16<0>(d, w);
    printf("16x16x32 MFMA, waves per block %d: cycles per MFMA slot and SIMD: mfma only %.1f, +4 plain %.1f, "
           "+8 plain %.1f, 8 plain only %.1f\n", w, run16<0>(d, w), run16<4>(d, w), run16<8>(d, w), run16<-1>(d, w));
  }
  return 0;
}
