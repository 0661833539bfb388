// npfn_gelu16.h -- the row kernel's packed-f16 GELU (NPFN_GELU_F16, npfn_rowk2.hip run_w2_gelu),
// in its own header so that tools/ubench/gelu16_check.hip checks these exact instructions.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace npfn {

typedef _Float16 h16x2 __attribute__((ext_vector_type(2)));

// Packed-f16 GELU (NPFN_GELU_F16): the same tanh form as gelu_tanh, x * s with s = e / (1 + e),
// e = 2^z, z = x (a x^2 + b), on half2 pairs -- v_pk_mul / v_pk_fma / v_pk_min / v_pk_add_f16 for
// the polynomial and the products, v_exp_f16 / v_rcp_f16 per half (no packed transcendental;
// the high half written in place through SDWA, so no repacking).  z is clamped at 15 so that e
// stays finite (s = 1 - 3e-5 there).  The result is the W2 product's fp16 B fragment.
// v_exp_f16 / v_rcp_f16 of the 8 halves of 4 half2 (the low halves first, then each high half
// written in place through SDWA: the PRESERVE read of a register that a transcendental has just
// written is a forwarding hazard the compiler does not see inside asm -- one instruction after
// it the low half read back as 0 on some lanes -- so three other transcendentals sit between)
#define NPFN_H2X4_TRANS(OP)                                                                               \
  asm(OP "_e32 %0, %4\n\t" OP "_e32 %1, %5\n\t" OP "_e32 %2, %6\n\t" OP "_e32 %3, %7\n\t"          \
      OP "_sdwa %0, %4 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1\n\t"                      \
      OP "_sdwa %1, %5 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1\n\t"                      \
      OP "_sdwa %2, %6 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1\n\t"                      \
      OP "_sdwa %3, %7 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1"                            \
      : "=&v"(r[0]), "=&v"(r[1]), "=&v"(r[2]), "=&v"(r[3])                                                 \
      : "v"(u[0]), "v"(u[1]), "v"(u[2]), "v"(u[3]))
__device__ __forceinline__ void exp2_h2x4(h16x2 (&v)[4]) {
  uint32_t u[4], r[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) u[i] = __builtin_bit_cast(uint32_t, v[i]);
  NPFN_H2X4_TRANS("v_exp_f16");
#pragma unroll
  for (int i = 0; i < 4; ++i) v[i] = __builtin_bit_cast(h16x2, r[i]);
}
__device__ __forceinline__ void rcp_h2x4(h16x2 (&v)[4]) {
  uint32_t u[4], r[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) u[i] = __builtin_bit_cast(uint32_t, v[i]);
  NPFN_H2X4_TRANS("v_rcp_f16");
#pragma unroll
  for (int i = 0; i < 4; ++i) v[i] = __builtin_bit_cast(h16x2, r[i]);
}
// GELU of two D tiles (8 hidden values of the lane) as one fp16 B fragment, in pack8's order:
// uint4 of half2 (lo[0], lo[1]), (lo[2], lo[3]), (hi[0], hi[1]), (hi[2], hi[3])
template <class F4>
__device__ __forceinline__ uint4 gelu_pk16_u4(const F4& lo, const F4& hi) {
  const h16x2 a = {(_Float16)0.1029432395800235f, (_Float16)0.1029432395800235f};
  const h16x2 b = {(_Float16)2.302208198144325f, (_Float16)2.302208198144325f};
  const h16x2 c15 = {(_Float16)15.f, (_Float16)15.f}, one = {(_Float16)1.f, (_Float16)1.f};
  const h16x2 x[4] = {h16x2{(_Float16)lo[0], (_Float16)lo[1]}, h16x2{(_Float16)lo[2], (_Float16)lo[3]},
                      h16x2{(_Float16)hi[0], (_Float16)hi[1]}, h16x2{(_Float16)hi[2], (_Float16)hi[3]}};
  h16x2 e[4], d[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) e[i] = __builtin_elementwise_min(x[i] * (x[i] * x[i] * a + b), c15);
  exp2_h2x4(e);
#pragma unroll
  for (int i = 0; i < 4; ++i) d[i] = e[i] + one;
  rcp_h2x4(d);
  uint32_t o[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) o[i] = __builtin_bit_cast(uint32_t, x[i] * (e[i] * d[i]));
  return make_uint4(o[0], o[1], o[2], o[3]);
}

}  // namespace npfn
