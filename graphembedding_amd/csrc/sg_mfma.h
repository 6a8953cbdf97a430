// sg_mfma.h — CDNA4 register-level helpers shared by the fused pair kernels
// (sg_fast.hip, sg_fast32.hip): f32 / bf16 MFMA tiles, the split-bf16 parts,
// DPP and permlane cross-lane sums.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace sgk {

typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ f4 mfma4(float a, float b, f4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// ---- split-bf16 gW0 product ---------------------------------------------------
// v_mfma_f32_16x16x4_f32 runs on the vector FP32 datapath (it never overlaps VALU
// on gfx950, scripts/mfma_coexec.hip).  The one-hot operand of gW0 = Xᵀ·gZ0 is
// exact in bf16, so gZ0 is carried as x = h + m + l (three bf16 parts, each residual
// exact in f32, split3 below) and the product runs on
// v_mfma_f32_16x16x32_bf16: 1.0 × part is exact, accumulation is f32.
typedef __bf16 bf8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf2v __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint32_t pk_bf16(float a, float b) {   // v_cvt_pk_bf16_f32 (RNE)
  const bf2v v = {(__bf16)a, (__bf16)b};
  return __builtin_bit_cast(uint32_t, v);
}
// (x0, x1) -> packed bf16 pairs of the h, m, l parts (x = h + m + l + e).
// Truncating parts: h = x with the low 16 mantissa bits cleared (one AND), r = x - h and
// r - m exact in f32, and the bf16 pairs are the high halves of (x0, x1) and of the
// residuals, packed by v_perm_b32.  |e| < 2^-21 |x| (RNE parts: 2^-24), at 4 ANDs, 4 subs
// and 3 perms per pair of values instead of 3 v_cvt_pk_bf16_f32 (twice the issue cost of
// a plain VALU op on gfx950, scripts/valu_rates.hip), 4 unpacks and 4 subs.
__device__ __forceinline__ uint32_t hi16x2(uint32_t a, uint32_t b) {   // hi16(a) | hi16(b) << 16
  return __builtin_amdgcn_perm(b, a, 0x07060302u);
}
// SG_SPLIT_PK = 1: the two residual subtractions of each level as one v_pk_add_f32.  It
// measured +0.1% in round 2; on the round-5 kernels the packed operands cost register
// copies (11 v_mov_b32 in the (2, 2) class loop of sg_fast) and the plain subtractions run
// C2 at 558.5 / 561.7 against 550.9 / 552.6 M pairs/s (profiles/r05_k, same box).  Both
// forms compute the same IEEE subtractions: the parts are bitwise the same.
#ifndef SG_SPLIT_PK
#define SG_SPLIT_PK 0
#endif
__device__ __forceinline__ void split3(float x0, float x1, uint32_t &h, uint32_t &m, uint32_t &l) {
  const uint32_t u0 = __float_as_uint(x0), u1 = __float_as_uint(x1);
  h = hi16x2(u0, u1);
#if SG_SPLIT_PK   // the two residual subtractions of each level as one v_pk_add_f32
  const f2 r = f2{x0, x1} - f2{__uint_as_float(u0 & 0xFFFF0000u), __uint_as_float(u1 & 0xFFFF0000u)};
  const float r0 = r.x, r1 = r.y;
#else
  const float r0 = x0 - __uint_as_float(u0 & 0xFFFF0000u), r1 = x1 - __uint_as_float(u1 & 0xFFFF0000u);
#endif
  const uint32_t v0 = __float_as_uint(r0), v1 = __float_as_uint(r1);
  m = hi16x2(v0, v1);
#if SG_SPLIT_PK
  const f2 t = f2{r0, r1} - f2{__uint_as_float(v0 & 0xFFFF0000u), __uint_as_float(v1 & 0xFFFF0000u)};
  const float s0 = t.x, s1 = t.y;
#else
  const float s0 = r0 - __uint_as_float(v0 & 0xFFFF0000u), s1 = r1 - __uint_as_float(v1 & 0xFFFF0000u);
#endif
  l = hi16x2(__float_as_uint(s0), __float_as_uint(s1));
}
__device__ __forceinline__ f4 mfbf(uint4 a, uint4 b, f4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf8, a),
                                                  __builtin_bit_cast(bf8, b), c, 0, 0, 0);
}
// v_mfma_f32_16x16x16_bf16: 4 k-slots per lane (k = 4 (lane / 16) + e), two dwords per
// operand, so a part that pairs with several others needs no duplicate registers
typedef short s4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ f4 mfbf16(uint2 a, uint2 b, f4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(__builtin_bit_cast(s4, a),
                                                    __builtin_bit_cast(s4, b), c, 0, 0, 0);
}

// relu(x) = max(x, 0) as one v_max_i32 on the bits (an f32 with the sign bit set is a
// negative int32, +0 and positive floats order as their bit patterns): fmaxf(x, 0)
// compiles to two v_max_f32 in the kernels' IEEE mode (the first quiets a signalling
// NaN), and LLVM folds v_med3_f32(x, 0, inf) back into that.  -0 maps to +0.
__device__ __forceinline__ float relu_bits(float x) {
  return __int_as_float(max(__float_as_int(x), 0));
}

// DPP lane move with bound_ctrl (no "old" operand to materialise), so the
// compiler can fold it into the consuming VALU op (v_add_f32_dpp).
template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), CTRL,
                                                            0xF, 0xF, true));
}


// x[l] + x[l ^ 16] and x[l] + x[l ^ 32]: gfx950 v_permlane16/32_swap leave x[l]
// and its partner in the two registers (either order), one add completes the sum
__device__ __forceinline__ float xsum16(float x) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false,
                                                  false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ float xsum32(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false,
                                                  false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// Sum over the 16 lanes of a DPP row; result in every lane of the row.
__device__ __forceinline__ float row_sum16(float v) {
  v += dpp<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dpp<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dpp<0x141>(v);  // row_half_mirror
  v += dpp<0x140>(v);  // row_mirror
  return v;
}

// row_sum16 of N independent values, step-interleaved: a DPP read of a VGPR written by
// the previous VALU instruction needs two wait states (s_nop 1 in a lone chain); with
// N >= 3 chains advanced in lockstep the other chains' adds fill them
// (the inputs are made opaque first: a product x = a·b would otherwise be folded into the
// first step as fma(a, b, dpp(x)), a v_mov_b32_dpp + v_fmac_f32 instead of one
// v_add_f32_dpp)
template <int N>
__device__ __forceinline__ void row_sum16_n(float (&v)[N]) {
#pragma unroll
  for (int i = 0; i < N; ++i) asm("" : "+v"(v[i]));
#pragma unroll
  for (int i = 0; i < N; ++i) v[i] += dpp<0xB1>(v[i]);
#pragma unroll
  for (int i = 0; i < N; ++i) v[i] += dpp<0x4E>(v[i]);
#pragma unroll
  for (int i = 0; i < N; ++i) v[i] += dpp<0x141>(v[i]);
#pragma unroll
  for (int i = 0; i < N; ++i) v[i] += dpp<0x140>(v[i]);
}

}  // namespace sgk
