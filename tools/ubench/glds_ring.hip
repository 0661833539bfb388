// Microbenchmark: L2 -> LDS weight-stream rate of the row kernel's LDS-DMA ring
// (no MFMA).  Every workgroup streams the same 1 MB "layer" of [192][64] bf16
// chunks (L2-resident after the first pass) through an NSLOT ring, LEAD chunks
// ahead, one barrier per chunk; optional consumer ds_reads of the whole chunk per wave.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <vector>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

__device__ __forceinline__ void glds16(const void* gsrc, uint32_t lds_dst) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(gsrc), "s"(lds_dst) : "memory");
}
__device__ __forceinline__ void bar() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

template <int NSLOT, int LEAD, int CHUNK_KB, int READS>
__global__ __launch_bounds__(512, 1) void k_ring(const uint4* __restrict__ w, int nchunk_layer, int iters, float* sink) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int PER = CHUNK_KB * 1024 / (512 * 16);  // glds per thread per chunk
  const uint32_t base = (uint32_t)(uintptr_t)smem;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  auto issue = [&](int i) {
    const uint4* src = w + (size_t)(i % nchunk_layer) * (CHUNK_KB * 64);
    const uint32_t slot = base + (uint32_t)((i % NSLOT) * CHUNK_KB * 1024);
#pragma unroll
    for (int p = 0; p < PER; ++p) {
      const int q0 = wave * 64 + p * 512;
      glds16(src + q0 + lane, __builtin_amdgcn_readfirstlane(slot + q0 * 16));
    }
  };
  const int n = iters * nchunk_layer;
  for (int i = 0; i < LEAD; ++i) issue(i);
  float acc = 0.f;
  for (int i = 0; i < n; ++i) {
    if (i + LEAD - 1 < n) {
      if constexpr (LEAD == 2) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(PER) : "memory");
      if constexpr (LEAD == 3) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(2 * PER) : "memory");
      if constexpr (LEAD == 1) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    bar();
    if (i + LEAD < n) issue(i + LEAD);
    if (READS) {
      const uint4* sl = reinterpret_cast<const uint4*>(smem + (i % NSLOT) * CHUNK_KB * 1024);
#pragma unroll 4
      for (int r = 0; r < READS; ++r) {
        uint4 v = sl[(r * 64 + lane) % (CHUNK_KB * 64)];
        acc += __uint_as_float(v.x & 0x3f800000u);
      }
    }
  }
  if (acc == 1234.5f) sink[0] = acc;
}

template <int NSLOT, int LEAD, int CHUNK_KB, int READS>
int run(const char* name, const uint4* w, float* sink, int nblk) {
  auto k = k_ring<NSLOT, LEAD, CHUNK_KB, READS>;
  const int smem = NSLOT * CHUNK_KB * 1024;
  CHK(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, smem));
  const int nchunk_layer = (1 << 20) / (CHUNK_KB * 1024);
  const int iters = 20;
  hipEvent_t a, b;
  CHK(hipEventCreate(&a)); CHK(hipEventCreate(&b));
  hipLaunchKernelGGL(k, dim3(nblk), dim3(512), smem, 0, w, nchunk_layer, 2, sink);
  CHK(hipEventRecord(a));
  hipLaunchKernelGGL(k, dim3(nblk), dim3(512), smem, 0, w, nchunk_layer, iters, sink);
  CHK(hipEventRecord(b));
  CHK(hipEventSynchronize(b));
  float ms; CHK(hipEventElapsedTime(&ms, a, b));
  const double bytes = (double)nblk * iters * (1 << 20);
  printf("%-34s blocks=%4d  %8.3f ms  chip %7.1f GB/s  per-CU %6.1f GB/s  per-chunk %6.0f ns\n", name, nblk, ms,
         bytes / ms / 1e6, bytes / ms / 1e6 / 256, ms * 1e6 / (iters * nchunk_layer) * (nblk > 256 ? 256.0 / nblk : 1.0));
  return 0;
}

int main() {
  uint4* w; float* sink;
  CHK(hipMalloc(&w, 1 << 20)); CHK(hipMemset(w, 0, 1 << 20)); CHK(hipMalloc(&sink, 4));
  for (int nb : {256, 1024}) {
    run<3, 2, 24, 0>("ring3 lead2 24KB", w, sink, nb);
    run<4, 3, 24, 0>("ring4 lead3 24KB", w, sink, nb);
    run<2, 1, 24, 0>("ring2 lead1 24KB", w, sink, nb);
    run<6, 3, 16, 0>("ring6 lead3 16KB", w, sink, nb);
    run<3, 2, 24, 24>("ring3 lead2 24KB +1x reads", w, sink, nb);
    run<3, 2, 24, 48>("ring3 lead2 24KB +2x reads", w, sink, nb);
  }
  return 0;
}
