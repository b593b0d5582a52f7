// Shared device helpers of the fused f16x3 attention kernels (stw_x3.hip, stw64_x3.hip):
// the MFMA fragment types, the compiler-visible hi / lo split, the f16x3 product, the
// half-wave reductions and the attention operand of one k-step in either arithmetic
// (f16x3 hi / lo, or bf16 for EXTDM_PRECISION_BF16_ATTN).
#pragma once
#include "kernels.h"

namespace extdm {
namespace attn_ops {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf8 __attribute__((ext_vector_type(8)));
// s <- exp2(s c - m) over NT accumulator tiles, returning the lane's sum: the exponent argument and
// the running sum as packed pairs (16 v_pk_fma + 16 v_pk_add per 32 values instead of 64 VALU)
template <int NT>
__device__ __forceinline__ float exp2_sum(f32x16* s, float c, float m) {
  const f2 c2 = splat(c), m2 = splat(-m);
  f2 acc = splat(0.f);
#pragma unroll
  for (int kt = 0; kt < NT; ++kt)
#pragma unroll
    for (int r = 0; r < 16; r += 2) {
      f2 a = pk_fma(pair(s[kt][r], s[kt][r + 1]), c2, m2);
      a.x = __builtin_amdgcn_exp2f(a.x);
      a.y = __builtin_amdgcn_exp2f(a.y);
      s[kt][r] = a.x;
      s[kt][r + 1] = a.y;
      acc += a;
    }
  return acc.x + acc.y;
}

// row of accumulator register r in a 32x32 MFMA tile, lane half h
__device__ __forceinline__ int dof(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

// hi = fp16(v), lo = fp16(v - hi) of an opaque v (split_src, kernels.h): the probabilities and
// scaled q / k / v are products, whose two fp16 roundings hipcc would otherwise lower
// differently. CHECK: OR |v| >= 65504 (fp16 overflow of hi) into bad.
// Compiler-visible split2m (3 VALU per pair) rather than the split2 asm: these splits read MFMA
// results and feed MFMAs, and only compiler-visible VALU gets its MFMA hazard waits.
template <bool CHECK = true>
__device__ __forceinline__ void split8(const float* v, h8& hi, h8& lo, int& bad) {
  float m = 0.f;
#pragma unroll
  for (int e = 0; e < 8; e += 2) {
    const float w0 = split_src(v[e]), w1 = split_src(v[e + 1]);
    if (CHECK) m = fmaxf(fmaxf(m, fabsf(w0)), fabsf(w1));
    f16x2_t ph, pl;
    split2m(w0, w1, ph, pl);
    hi[e] = ph.x; hi[e + 1] = ph.y;
    lo[e] = pl.x; lo[e + 1] = pl.y;
  }
  if (CHECK) bad |= m >= 65504.f;
}

__device__ __forceinline__ f32x16 mma3(const h8& ah, const h8& al, const h8& bh, const h8& bl, f32x16 c) {
  c = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bh, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bl, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh, c, 0, 0, 0);
  return c;
}

// Reductions across the two half-waves (lane ^ 32) without LDS: v_permlane32_swap of v with
// itself leaves the partner's value in r[1] of the lower lanes and in r[0] of the upper lanes
// (own value in the other), so r[0] op r[1] is the pair's result in both halves (commutative:
// bitwise equal).
__device__ __forceinline__ float xh_sum(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ float xh_max(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}

// The attention operand of one k-step (8 values per lane): f16x3 hi / lo (fp32-faithful), or
// bf16 (BF16_ATTN: round-to-nearest-even, one MFMA). put / get: its 16-B LDS slots at stride 64.
template <bool BF> struct Op;
template <> struct Op<false> {
  static constexpr int SLOTS = 2;
  h8 hi, lo;
  __device__ void set(const float* v, int& bad) { split8<false>(v, hi, lo, bad); }
  __device__ void put(h8* p) const { p[0] = hi; p[64] = lo; }
  __device__ void get(const h8* p) { hi = p[0]; lo = p[64]; }
  __device__ void zero() {
#pragma unroll
    for (int e = 0; e < 8; ++e) { hi[e] = (_Float16)0.f; lo[e] = (_Float16)0.f; }
  }
};
template <> struct Op<true> {
  static constexpr int SLOTS = 1;
  bf8 v;
  __device__ void set(const float* x, int&) {
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = (__bf16)x[e];
  }
  __device__ void put(h8* p) const { p[0] = __builtin_bit_cast(h8, v); }
  __device__ void get(const h8* p) { v = __builtin_bit_cast(bf8, p[0]); }
  __device__ void zero() {
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = (__bf16)0.f;
  }
};
__device__ __forceinline__ f32x16 mmo(const Op<false>& a, const Op<false>& b, f32x16 c) {
  return mma3(a.hi, a.lo, b.hi, b.lo, c);
}
__device__ __forceinline__ f32x16 mmo(const Op<true>& a, const Op<true>& b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.v, b.v, c, 0, 0, 0);
}

}  // namespace attn_ops
}  // namespace extdm
