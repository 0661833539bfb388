// Microbenchmark: per-chunk cost of a register-resident row GEMM fed by the LDS-DMA
// weight ring.  WAVES waves each own TB 16-token blocks (B fragments stay in VGPRs);
// per [192][64] weight chunk every wave reads all 12x2 A fragments (ds_read_b128,
// swizzled image) and issues 12*2*TB v_mfma_f32_16x16x32_bf16.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)
typedef __attribute__((ext_vector_type(8))) short bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;

__device__ __forceinline__ void glds16(const void* gsrc, uint32_t lds_dst) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(gsrc), "s"(lds_dst) : "memory");
}
__device__ __forceinline__ void bar() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

template <int WAVES, int TB, int NSLOT, int LEAD, int MODE, int DMA = 1>
__global__ __launch_bounds__(WAVES * 64, 1) void k_gemm_ring(const uint4* __restrict__ w, int nchunk_layer, int iters,
                                                              float* sink, int do_mfma) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int NT = WAVES * 64;
  constexpr int PER = 24 * 1024 / (NT * 16);
  const uint32_t base = (uint32_t)(uintptr_t)smem;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  auto issue = [&](int i) {
    const uint4* src = w + (size_t)(i % nchunk_layer) * (24 * 64);
    const uint32_t slot = base + (uint32_t)((i % NSLOT) * 24 * 1024);
#pragma unroll
    for (int p = 0; p < PER; ++p) {
      const int q0 = wave * 64 + p * NT;
      glds16(src + q0 + lane, __builtin_amdgcn_readfirstlane(slot + q0 * 16));
    }
  };
  bf16x8 b[TB][2];
#pragma unroll
  for (int t = 0; t < TB; ++t)
#pragma unroll
    for (int k = 0; k < 2; ++k)
#pragma unroll
      for (int j = 0; j < 8; ++j) b[t][k][j] = (short)(0x3f80 + lane + t + k + j);
  f32x4 acc[TB][12];
#pragma unroll
  for (int t = 0; t < TB; ++t)
#pragma unroll
    for (int f = 0; f < 12; ++f) acc[t][f] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int n = iters * nchunk_layer;
  if (DMA) for (int i = 0; i < LEAD; ++i) issue(i);
  for (int i = 0; i < n; ++i) {
    if (!DMA) {
    } else if (i + LEAD - 1 < n) {
      if constexpr (LEAD == 2) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(PER) : "memory");
      if constexpr (LEAD == 3) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(2 * PER) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    bar();
    if (DMA && i + LEAD < n) issue(i + LEAD);
    const short* ws = reinterpret_cast<const short*>(smem + (i % NSLOT) * 24 * 1024);
    const int off0 = (lane & 15) * 64 + (((lane >> 4) ^ (lane & 7)) << 3);
    const int off1 = (lane & 15) * 64 + (((4 + (lane >> 4)) ^ (lane & 7)) << 3);
    if constexpr (MODE == 0) {
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        bf16x8 a[12];
#pragma unroll
        for (int f = 0; f < 12; ++f) a[f] = *reinterpret_cast<const bf16x8*>(ws + (ks ? off1 : off0) + f * 1024);
#pragma unroll
        for (int f = 0; f < 12; ++f)
#pragma unroll
          for (int t = 0; t < TB; ++t)
            acc[t][f] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[f], b[t][ks], acc[t][f], 0, 0, 0);
      }
    } else if constexpr (MODE == 1) {
#pragma unroll
      for (int hk = 0; hk < 4; ++hk) {
        const int ks = hk >> 1, f0 = (hk & 1) * 6;
        bf16x8 a[6];
#pragma unroll
        for (int f = 0; f < 6; ++f) a[f] = *reinterpret_cast<const bf16x8*>(ws + (ks ? off1 : off0) + (f0 + f) * 1024);
#pragma unroll
        for (int f = 0; f < 6; ++f)
#pragma unroll
          for (int t = 0; t < TB; ++t)
            acc[t][f0 + f] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[f], b[t][ks], acc[t][f0 + f], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
      }
    } else {
      bf16x8 a[2][6];
#pragma unroll
      for (int f = 0; f < 6; ++f) a[0][f] = *reinterpret_cast<const bf16x8*>(ws + off0 + f * 1024);
#pragma unroll
      for (int hk = 0; hk < 4; ++hk) {
        const int ks = hk >> 1, f0 = (hk & 1) * 6;
        if (hk < 3) {
          const int nk = (hk + 1) >> 1, nf0 = ((hk + 1) & 1) * 6;
#pragma unroll
          for (int f = 0; f < 6; ++f) a[(hk + 1) & 1][f] = *reinterpret_cast<const bf16x8*>(ws + (nk ? off1 : off0) + (nf0 + f) * 1024);
        }
#pragma unroll
        for (int f = 0; f < 6; ++f)
#pragma unroll
          for (int t = 0; t < TB; ++t)
            acc[t][f0 + f] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[hk & 1][f], b[t][ks], acc[t][f0 + f], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  }
  float s = 0.f;
#pragma unroll
  for (int t = 0; t < TB; ++t)
#pragma unroll
    for (int f = 0; f < 12; ++f) s += acc[t][f][0] + acc[t][f][1] + acc[t][f][2] + acc[t][f][3];
  if (s == 1234.5f) sink[0] = s;
}

template <int WAVES, int TB, int NSLOT, int LEAD, int MODE, int DMA = 1>
int run(const char* name, const uint4* w, float* sink, int do_mfma) {
  auto k = k_gemm_ring<WAVES, TB, NSLOT, LEAD, MODE, DMA>;
  const int smem = NSLOT * 24 * 1024;
  CHK(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, smem));
  const int nchunk_layer = (1 << 20) / (24 * 1024);
  const int iters = 20, nblk = 256;
  hipEvent_t a, b;
  CHK(hipEventCreate(&a)); CHK(hipEventCreate(&b));
  hipLaunchKernelGGL(k, dim3(nblk), dim3(WAVES * 64), smem, 0, w, nchunk_layer, 2, sink, do_mfma);
  CHK(hipEventRecord(a));
  hipLaunchKernelGGL(k, dim3(nblk), dim3(WAVES * 64), smem, 0, w, nchunk_layer, iters, sink, do_mfma);
  CHK(hipEventRecord(b));
  CHK(hipEventSynchronize(b));
  float ms; CHK(hipEventElapsedTime(&ms, a, b));
  const double chunks = (double)iters * nchunk_layer;
  const int tokens = WAVES * TB * 16;
  const double flops = (double)nblk * chunks * 2.0 * 192 * 64 * tokens;
  printf("%-40s tokens/tile=%3d  per-chunk %6.0f ns  %6.1f TF/s  ns/token-chunk %5.2f\n", name, tokens,
         ms * 1e6 / chunks, do_mfma ? flops / ms / 1e9 : 0.0, ms * 1e6 / chunks / tokens);
  return 0;
}

int main() {
  uint4* w; float* sink;
  CHK(hipMalloc(&w, 1 << 20)); CHK(hipMalloc(&sink, 4));
  {  // random bf16 operands (zero operands run at a higher clock, MI355X_MICROARCH.md)
    static uint16_t hw[1 << 19];
    uint32_t st = 12345u;
    for (int i = 0; i < (1 << 19); ++i) {
      st = st * 1664525u + 1013904223u;
      hw[i] = (uint16_t)(0x3c00 + ((st >> 16) & 0x7ff)) ^ (uint16_t)((st >> 31) << 15);
    }
    CHK(hipMemcpy(w, hw, 1 << 20, hipMemcpyHostToDevice));
  }
  run<8, 1, 3, 2, 0>("8x1 ring3 2 groups of 12", w, sink, 1);
  run<4, 2, 3, 2, 0>("4x2 ring3 2 groups of 12", w, sink, 1);
  run<4, 2, 3, 2, 1>("4x2 ring3 4 groups of 6", w, sink, 1);
  run<8, 2, 3, 2, 2>("8x2 ring3 pipelined", w, sink, 1);
  run<8, 1, 3, 2, 0, 0>("8x1 NO DMA 2 groups of 12", w, sink, 1);
  run<8, 1, 3, 2, 2, 0>("8x1 NO DMA pipelined", w, sink, 1);
  run<8, 1, 3, 2, 0, 0>("8x1 NO DMA reads only", w, sink, 0);
  run<4, 2, 3, 2, 2>("4x2 ring3 pipelined", w, sink, 1);
  run<4, 2, 3, 2, 2, 0>("4x2 NO DMA pipelined", w, sink, 1);
  run<4, 2, 3, 2, 0, 0>("4x2 NO DMA reads only", w, sink, 0);
  return 0;
}
