// Cross-lane reductions on VALU lane moves (DPP, v_permlane{16,32}_swap) instead of
// __shfl_xor, which compiles to ds_bpermute: an LDS-queue round trip per level, in the
// dependent chains of every softmax and row reduction.  Each helper adds (or maxes) the
// same operand pairs as the xor butterfly it replaces, so results are bitwise equal
// (IEEE + and max are commutative).
#pragma once

#include "common.h"

namespace mocr {

template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}
// sum over aligned groups of L lanes (L = 8, 16, 32, 64): quad_perm xor 1, xor 2, then
// row_half_mirror / row_mirror, which pair each lane with one of the other half's
// lanes, all of which hold the same partial sum by then (== __shfl_xor by 4, 8), then
// the other 16-lane row / 32-lane half by v_permlane{16,32}_swap
template <int L>
__device__ __forceinline__ float row_sum(float s) {
  static_assert(L == 8 || L == 16 || L == 32 || L == 64, "row_sum: 8, 16, 32 or 64 lanes");
  s += dpp<0xB1>(s);
  s += dpp<0x4E>(s);
  s += dpp<0x141>(s);
  if constexpr (L >= 16) s += dpp<0x140>(s);
  if constexpr (L >= 32) {
    float a = s, b = s;
    asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1" : "+v"(a), "+v"(b));
    s = a + b;
  }
  if constexpr (L == 64) {
    float a = s, b = s;
    asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %1" : "+v"(a), "+v"(b));
    s = a + b;
  }
  return s;
}
// d * d rounded on its own: never contracted into the add that consumes it, so a LayerNorm
// slice's M2 has the same bits whichever epilogue shape sums it (row_sum<16> over 16 lanes,
// or 4 values in a lane and then 4 lanes: the same pairs)
__device__ __forceinline__ float sq_rn(float d) {
#pragma clang fp contract(off)
  return d * d;
}
// max over aligned groups of 8 lanes (row_sum<8>'s moves)
__device__ __forceinline__ float row_max8(float s) {
  s = fmaxf(s, dpp<0xB1>(s));
  s = fmaxf(s, dpp<0x4E>(s));
  return fmaxf(s, dpp<0x141>(s));
}
// x[lane ^ 16] and x[lane ^ 32] via v_permlane{16,32}_swap (VALU, no LDS queue).  The
// swap exchanges halves between two registers, so both start as copies of x and their
// sum / max is symmetric in the pair.  Inline asm: the builtin with one value for both
// operands returned the same register twice (hardware-checked, tools/lane_ops_test.hip);
// s_nop 1 covers the VALU-write -> permlane-read hazard.
__device__ __forceinline__ void swap16(float& a, float& b) {
  asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1" : "+v"(a), "+v"(b));
}
__device__ __forceinline__ void swap32(float& a, float& b) {
  asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %1" : "+v"(a), "+v"(b));
}
__device__ __forceinline__ float xmax16_32(float x) {
  float a = x, b = x;
  swap16(a, b);
  x = fmaxf(a, b);
  a = x;
  b = x;
  swap32(a, b);
  return fmaxf(a, b);
}
__device__ __forceinline__ float xsum16_32(float x) {
  float a = x, b = x;
  swap16(a, b);
  x = a + b;
  a = x;
  b = x;
  swap32(a, b);
  return a + b;
}
// over lanes i, i^8, i^16, i^32 .. (the 8 lane groups of a wave): row_ror:8 pairs i with
// i ^ 8 inside each 16-lane row
__device__ __forceinline__ float xsum8_16_32(float x) { return xsum16_32(x + dpp<0x128>(x)); }
__device__ __forceinline__ float xmax8_16_32(float x) { return xmax16_32(fmaxf(x, dpp<0x128>(x))); }

// x of lane ^ MASK, for the fixed (mean, M2) merge trees of the decode kernels' LayerNorm
// statistics, whose level MASK runs after levels 1 .. MASK / 2: MASK = 1, 2 by quad_perm;
// 4 and 8 by row_half_mirror / row_mirror, which return a lane of the partner quad / half
// row, all of whose lanes hold the same value by then (so == __shfl_xor); 16, 32 by
// __shfl_xor (ds_bpermute).
template <int MASK>
__device__ __forceinline__ float lane_partner(float x) {
  if constexpr (MASK == 1) return dpp<0xB1>(x);
  else if constexpr (MASK == 2) return dpp<0x4E>(x);
  else if constexpr (MASK == 4) return dpp<0x141>(x);
  else if constexpr (MASK == 8) return dpp<0x140>(x);
  else return __shfl_xor(x, MASK, 64);
}

}  // namespace mocr
