// Numerics of the row kernel's packed-f16 GELU (npfn_rowk2.hip gelu_pk16, NPFN_GELU_F16) against
// the erf GELU in double, over x in [-12, 12]: max abs error and max rel error where |GELU| > 0.25.
// hipcc --offload-arch=gfx950 -O3 -Inpe-pfn_amd/csrc tools/ubench/gelu16_check.hip -o tools/ubench/gelu16_check
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <vector>
#include "npfn_gelu16.h"
typedef __attribute__((ext_vector_type(4))) float f32x4;
__global__ void k(const float* in, float* out, int n) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (8 * i + 7 >= n) return;
  const f32x4 lo = *reinterpret_cast<const f32x4*>(in + 8 * i), hi = *reinterpret_cast<const f32x4*>(in + 8 * i + 4);
  const uint4 u = npfn::gelu_pk16_u4(lo, hi);
  const uint32_t w[4] = {u.x, u.y, u.z, u.w};
  for (int j = 0; j < 4; ++j) {
    const npfn::h16x2 v = __builtin_bit_cast(npfn::h16x2, w[j]);
    out[8 * i + 2 * j] = (float)v[0];
    out[8 * i + 2 * j + 1] = (float)v[1];
  }
}
int main() {
  const int n = 1 << 20;
  std::vector<float> x(n), y(n);
  for (int i = 0; i < n; ++i) x[i] = -12.f + 24.f * i / n;
  float *dx, *dy;
  hipMalloc(&dx, n * 4);
  hipMalloc(&dy, n * 4);
  hipMemcpy(dx, x.data(), n * 4, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(n / 2048), dim3(256), 0, 0, dx, dy, n);
  hipMemcpy(y.data(), dy, n * 4, hipMemcpyDeviceToHost);
  double ea = 0, er = 0, xa = 0;
  int bad = 0;
  for (int i = 0; i < n; ++i) {
    const double g = x[i] * 0.5 * (1.0 + erf(x[i] / sqrt(2.0)));
    if (!isfinite(y[i])) { ++bad; continue; }
    const double d = fabs(y[i] - g);
    if (d > ea) { ea = d; xa = x[i]; }
    if (fabs(g) > 0.25) er = fmax(er, d / fabs(g));
  }
  printf("packed-f16 GELU on [-12, 12]: max abs err %.3e (at x = %.3f), max rel err (|GELU| > 0.25) %.3e, non-finite %d\n",
         ea, xa, er, bad);
  for (float t : {-4.f, -2.7f, -1.f, -0.3f, 0.f, 0.5f, 1.f, 3.f, 6.f}) {
    int i = (int)((t + 12.f) / 24.f * n);
    printf("  x %.4f  f16 %.6f  erf %.6f\n", x[i], y[i], x[i] * 0.5 * (1.0 + erf(x[i] / sqrt(2.0))));
  }
  return bad != 0;
}
