// Issue cost of candidate VALU instructions on gfx950, one wave per SIMD: 16 independent
// instructions per loop body (8 registers, two rounds), cycles from s_memtime.
// hipcc --offload-arch=gfx950 -O3 tools/ubench/valu_cost.hip -o /tmp/valu_cost && /tmp/valu_cost
#include <hip/hip_runtime.h>
#include <stdio.h>

#define BODY8(ins)                                                                          \
  asm volatile(ins " %0, %0\n\t" ins " %1, %1\n\t" ins " %2, %2\n\t" ins " %3, %3\n\t" ins \
               " %4, %4\n\t" ins " %5, %5\n\t" ins " %6, %6\n\t" ins " %7, %7"           \
               : "+v"(r0), "+v"(r1), "+v"(r2), "+v"(r3), "+v"(r4), "+v"(r5), "+v"(r6), "+v"(r7))
#define BODY8_3(ins)                                                                                  \
  asm volatile(ins " %0, %0, %0, %0\n\t" ins " %1, %1, %1, %1\n\t" ins " %2, %2, %2, %2\n\t" ins      \
               " %3, %3, %3, %3\n\t" ins " %4, %4, %4, %4\n\t" ins " %5, %5, %5, %5\n\t" ins         \
               " %6, %6, %6, %6\n\t" ins " %7, %7, %7, %7"                                        \
               : "+v"(r0), "+v"(r1), "+v"(r2), "+v"(r3), "+v"(r4), "+v"(r5), "+v"(r6), "+v"(r7))
#define BODY8_2(ins)                                                                                          \
  asm volatile(ins " %0, %0, %0\n\t" ins " %1, %1, %1\n\t" ins " %2, %2, %2\n\t" ins " %3, %3, %3\n\t" ins \
               " %4, %4, %4\n\t" ins " %5, %5, %5\n\t" ins " %6, %6, %6\n\t" ins " %7, %7, %7"            \
               : "+v"(r0), "+v"(r1), "+v"(r2), "+v"(r3), "+v"(r4), "+v"(r5), "+v"(r6), "+v"(r7))
#define BODY8_64_3(ins)                                                                               \
  asm volatile(ins " %0, %0, %0, %0\n\t" ins " %1, %1, %1, %1\n\t" ins " %2, %2, %2, %2\n\t" ins      \
               " %3, %3, %3, %3\n\t"                                                                  \
               : "+v"(d0), "+v"(d1), "+v"(d2), "+v"(d3))

template <int K>
__global__ void k(unsigned long long* out, float seed) {
  float r0 = seed, r1 = seed + 1, r2 = seed + 2, r3 = seed + 3, r4 = seed + 4, r5 = seed + 5, r6 = seed + 6,
        r7 = seed + 7;
  double d0 = seed, d1 = seed + 1, d2 = seed + 2, d3 = seed + 3;
  const int iters = 1024;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) {
    if constexpr (K == 0) { BODY8("v_exp_f32"); BODY8("v_exp_f32"); }
    if constexpr (K == 1) { BODY8("v_exp_f16"); BODY8("v_exp_f16"); }
    if constexpr (K == 2) { BODY8("v_rcp_f16"); BODY8("v_rcp_f16"); }
    if constexpr (K == 3) { BODY8_3("v_fma_f32"); BODY8_3("v_fma_f32"); }
    if constexpr (K == 4) { BODY8_3("v_pk_fma_f16"); BODY8_3("v_pk_fma_f16"); }
    if constexpr (K == 5) { BODY8_2("v_pk_mul_f16"); BODY8_2("v_pk_mul_f16"); }
    if constexpr (K == 6) { BODY8_64_3("v_pk_fma_f32"); BODY8_64_3("v_pk_fma_f32"); BODY8_64_3("v_pk_fma_f32"); BODY8_64_3("v_pk_fma_f32"); }
    if constexpr (K == 7) { BODY8_2("v_cvt_pk_bf16_f32"); BODY8_2("v_cvt_pk_bf16_f32"); }
    if constexpr (K == 8) { BODY8_2("v_cvt_pkrtz_f16_f32"); BODY8_2("v_cvt_pkrtz_f16_f32"); }
    if constexpr (K == 9) { BODY8("v_rcp_f32"); BODY8("v_rcp_f32"); }
    if constexpr (K == 10) { BODY8_2("v_mul_f32"); BODY8_2("v_mul_f32"); }
    if constexpr (K == 11) { BODY8_2("v_pk_add_f16"); BODY8_2("v_pk_add_f16"); }
    if constexpr (K == 12) { BODY8("v_cvt_f32_f16"); BODY8("v_cvt_f32_f16"); }
    if constexpr (K == 13) { BODY8_2("v_pk_max_f16"); BODY8_2("v_pk_max_f16"); }
    if constexpr (K == 14) { BODY8("v_exp_legacy_f32"); BODY8("v_exp_legacy_f32"); }
    if constexpr (K == 15) { BODY8("v_sqrt_f16"); BODY8("v_sqrt_f16"); }
    if constexpr (K == 16) { BODY8("v_log_f16"); BODY8("v_log_f16"); }
    if constexpr (K == 17) { BODY8_3("v_fma_mix_f32"); BODY8_3("v_fma_mix_f32"); }
    if constexpr (K == 18) { BODY8_3("v_max3_f32"); BODY8_3("v_max3_f32"); }
    if constexpr (K == 19) { BODY8_3("v_dot2_f32_bf16"); BODY8_3("v_dot2_f32_bf16"); }
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if ((threadIdx.x & 63) == 0)
    out[blockIdx.x * 4 + (threadIdx.x >> 6)] =
        (t1 - t0) + (unsigned long long)(r0 + r1 + r2 + r3 + r4 + r5 + r6 + r7 + (float)(d0 + d1 + d2 + d3)) * 0ull;
}

template <int K>
double run(unsigned long long* d, int waves) {
  hipLaunchKernelGGL(k<K>, dim3(1), dim3(64 * waves), 0, 0, d, 0.5f);
  hipDeviceSynchronize();
  unsigned long long h[8];
  hipMemcpy(h, d, 8 * 8, hipMemcpyDeviceToHost);
  double m = 0;
  for (int i = 0; i < waves; ++i) m += h[i];
  return m / waves / (1024.0 * 16);
}

int main() {
  unsigned long long* d;
  hipMalloc(&d, 64 * 8);
  const char* names[] = {"v_exp_f32", "v_exp_f16", "v_rcp_f16", "v_fma_f32", "v_pk_fma_f16", "v_pk_mul_f16",
                         "v_pk_fma_f32(64b)", "v_cvt_pk_bf16_f32", "v_cvt_pkrtz_f16_f32", "v_rcp_f32",
                         "v_mul_f32", "v_pk_add_f16", "v_cvt_f32_f16", "v_pk_max_f16", "v_exp_legacy_f32",
                         "v_sqrt_f16", "v_log_f16", "v_fma_mix_f32", "v_max3_f32", "v_dot2_f32_bf16"};
  double c[20];
  for (int w : {1, 4, 8}) {
    run<0>(d, w);
    c[0] = run<0>(d, w); c[1] = run<1>(d, w); c[2] = run<2>(d, w); c[3] = run<3>(d, w);
    c[4] = run<4>(d, w); c[5] = run<5>(d, w); c[6] = run<6>(d, w); c[7] = run<7>(d, w);
    c[8] = run<8>(d, w); c[9] = run<9>(d, w); c[10] = run<10>(d, w); c[11] = run<11>(d, w);
    c[12] = run<12>(d, w); c[13] = run<13>(d, w); c[14] = run<14>(d, w); c[15] = run<15>(d, w);
    c[16] = run<16>(d, w); c[17] = run<17>(d, w); c[18] = run<18>(d, w); c[19] = run<19>(d, w);
    printf("waves per block %d (one per SIMD up to 4): cycles per wave-instruction\n", w);
    for (int i = 0; i < 20; ++i) printf("  %-22s %.2f\n", names[i], c[i]);
  }
  return 0;
}
