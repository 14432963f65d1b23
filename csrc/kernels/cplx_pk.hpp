// Complex fp32 arithmetic on CDNA's packed-f32 VALU (gfx950).
//
// A complex value lives in an even-aligned VGPR pair, exactly the layout of
// v_pk_{add,mul,fma}_f32: one packed instruction does both lanes' work at the
// full 64 FLOP/clk/SIMD rate, where the plain f32 VALU (v_add_f32, v_fma_f32)
// runs at half of it.  The op_sel / op_sel_hi / neg_lo / neg_hi source
// modifiers do the complex-specific swizzles for free:
//   * a + (-i) b = (a.x + b.y, a.y - b.x): one v_pk_add_f32 with b's halves
//     swapped and the high lane negated,
//   * a * w = a.x (w.x, w.y) + a.y (-w.y, w.x): one v_pk_mul_f32 (a.x
//     broadcast) and one v_pk_fma_f32 (a.y broadcast, w swapped, low lane
//     negated) -- 2 instructions instead of 4.
// The compiler's SLP vectoriser finds the adds but emits a v_mov per swizzle
// (the dft<64> microkernel: 644 packed + 332 moves vs 1050 scalar f32 ops;
// these helpers: 544 packed, no moves), so the forms are written out.
// Every lane result is one IEEE fp32 add / mul / fma, as in the scalar forms;
// only the association of the complex product differs (fma(a.y, -w.y, a.x w.x)).
#pragma once

#include <hip/hip_runtime.h>

namespace psoup {
namespace pk {

typedef float v2f __attribute__((ext_vector_type(2)));
__device__ __forceinline__ v2f tv(float2 a) { return __builtin_bit_cast(v2f, a); }
__device__ __forceinline__ float2 tf(v2f a) { return __builtin_bit_cast(float2, a); }

// Plain adds / subtracts as vector arithmetic: the compiler emits the same
// v_pk_add_f32 (neg modifiers for the subtract) and, seeing them, can
// schedule independent work between dependent packed ops (gfx950 needs one
// wait state there, an s_nop when nothing else is ready); the swizzled forms
// below stay inline asm.
__device__ __forceinline__ float2 add(float2 a, float2 b) { return tf(tv(a) + tv(b)); }
__device__ __forceinline__ float2 sub(float2 a, float2 b) { return tf(tv(a) - tv(b)); }
// a + (-i) b = (a.x + b.y, a.y - b.x)
__device__ __forceinline__ float2 add_mi(float2 a, float2 b) {
  v2f d;
  asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0] neg_hi:[0,1]" : "=v"(d) : "v"(tv(a)), "v"(tv(b)));
  return tf(d);
}
// a - (-i) b = (a.x - b.y, a.y + b.x)
__device__ __forceinline__ float2 sub_mi(float2 a, float2 b) {
  v2f d;
  asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0] neg_lo:[0,1]" : "=v"(d) : "v"(tv(a)), "v"(tv(b)));
  return tf(d);
}
// a * w
__device__ __forceinline__ float2 mul(float2 a, float2 w) {
  v2f t, d;
  asm("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[0,1]" : "=v"(t) : "v"(tv(a)), "v"(tv(w)));
  asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,1,0] op_sel_hi:[1,0,1] neg_lo:[0,1,0]"
      : "=v"(d)
      : "v"(tv(a)), "v"(tv(w)), "v"(t));
  return tf(d);
}
// a * s (real s)
__device__ __forceinline__ float2 scale(float2 a, float s) {
  v2f d;
  const v2f ss = {s, s};
  asm("v_pk_mul_f32 %0, %1, %2" : "=v"(d) : "v"(tv(a)), "v"(ss));
  return tf(d);
}
// a * W_8 = r2 (a.x + a.y, a.y - a.x)
__device__ __forceinline__ float2 mul_w8(float2 a) {
  v2f d;
  asm("v_pk_add_f32 %0, %1, %1 op_sel:[0,1] op_sel_hi:[1,0] neg_hi:[0,1]" : "=v"(d) : "v"(tv(a)));
  return scale(tf(d), 0.70710678118654752440f);
}
// a * W_8^3 = r2 (a.y - a.x, -(a.x + a.y))
__device__ __forceinline__ float2 mul_w83(float2 a) {
  v2f d;
  asm("v_pk_add_f32 %0, %1, %1 op_sel:[1,0] op_sel_hi:[0,1] neg_lo:[0,1] neg_hi:[1,1]" : "=v"(d) : "v"(tv(a)));
  return scale(tf(d), 0.70710678118654752440f);
}

}  // namespace pk
}  // namespace psoup
