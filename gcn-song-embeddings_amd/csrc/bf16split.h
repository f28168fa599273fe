// Exact three-piece bf16 split of fp32 operands for the split-bf16 MFMA
// products (gemm.hip, aggw.hip, split_planes_kernel).
//
// x = H + M + L with H, M, L bf16: H = RN(x), M = RN(x - H), L = RN(x - H - M);
// both differences are exact in fp32, so |x - (H + M + L)| <= 2^-9 |x - H - M|
// <= 2^-26 |x| (the pieces have the exponent range of fp32).  Per pair of
// elements: three v_cvt_pk_bf16_f32, two packed fp32 subtractions
// (v_pk_add_f32) and four shifts / masks back to fp32.  (M and L by truncation,
// one conversion per pair, measured 0-3 % faster but doubles the dropped
// products' bound to 2^-25; the reference-init gradient check of
// test_gpu_fly.py, whose head-bias gradient cancels to ~1e-4, then exceeded
// its 2e-4 bound.)  Every user of these helpers splits bitwise identically, so
// a pre-split operand gives the same products as the in-register split.
#pragma once
#include <hip/hip_runtime.h>

namespace ps {

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f32x2 bf2_to_f2(unsigned p) {
  return f32x2{__uint_as_float(p << 16), __uint_as_float(p & 0xffff0000u)};
}
__device__ __forceinline__ void split_pair(f32x2 x, unsigned& H, unsigned& M, unsigned& L) {
  H = __builtin_bit_cast(unsigned, __builtin_convertvector(x, bf16x2));
  const f32x2 r = x - bf2_to_f2(H);
  M = __builtin_bit_cast(unsigned, __builtin_convertvector(r, bf16x2));
  const f32x2 s = r - bf2_to_f2(M);
  L = __builtin_bit_cast(unsigned, __builtin_convertvector(s, bf16x2));
}
__device__ __forceinline__ void split3(const float4& a, const float4& b, bf16x8& H, bf16x8& M, bf16x8& L) {
  const f32x2 x[4] = {{a.x, a.y}, {a.z, a.w}, {b.x, b.y}, {b.z, b.w}};
  unsigned hh[4], mm[4], ll[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) split_pair(x[j], hh[j], mm[j], ll[j]);
  const u32x4 h{hh[0], hh[1], hh[2], hh[3]}, m{mm[0], mm[1], mm[2], mm[3]}, l{ll[0], ll[1], ll[2], ll[3]};
  H = __builtin_bit_cast(bf16x8, h);
  M = __builtin_bit_cast(bf16x8, m);
  L = __builtin_bit_cast(bf16x8, l);
}

}  // namespace ps
