// Shared MFMA / LDS helpers for the CDNA4 flash-attention kernels (K3).
//
// MFMA: v_mfma_f32_32x32x16_bf16 (one wave computes a 32x32 fp32 tile, K = 16).
// Operand lane maps (cdna_hip_programming.md §3), lane l, r = l & 31, h = l >> 5:
//   A[row r][k = 8h + j]          (j = 0..7 of the 8-element fragment)
//   B[k = 8h + j][col r]
//   C/D reg i: row = (i & 3) + 8 * (i >> 2) + 4h, col = r
// An fp32 accumulator X reused as the B operand (sum over X's rows) takes registers 8s..8s+7
// for k-step s; element j then carries row 16s + 8(j>>2) + 4h + (j&3) of X, so the A operand
// must supply those k's: with A held row-major in LDS that is exactly what a
// ds_read_b64_tr_b16 of 4 consecutive rows delivers (T10 transposed read).
#pragma once
#include "common.h"

namespace lta {
namespace attn {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

template <typename T> struct Frag;
template <> struct Frag<__hip_bfloat16> { typedef bf16x8 type; };
template <> struct Frag<__half> { typedef f16x8 type; };

__device__ __forceinline__ f32x16 mfma(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x16 mfma(f16x8 a, f16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
}

template <typename F>
__device__ __forceinline__ F load_frag(const void* p) {
  return *reinterpret_cast<const F*>(p);
}

// Two transposed 4x16 LDS reads (rows row0..row0+3 and row0+8..row0+11 of a row-major 16-bit
// tile) assembled into one 8-element A fragment; `lds_base` points at the first row,
// `stride` is the row stride in elements, `col0` the first column of this 16-lane group.
template <typename F>
__device__ __forceinline__ F tr_frag(const __attribute__((address_space(3))) short* base, int row0, int col0, int stride,
                                     int lane16) {
  const int q = lane16 >> 2, p = lane16 & 3;
  const __attribute__((address_space(3))) short* p0 = base + (row0 + q) * stride + col0 + 4 * p;
  const __attribute__((address_space(3))) short* p1 = p0 + 8 * stride;
  s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)p0);
  s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)p1);
  union {
    struct { s16x4 a, b; } s;
    F f;
  } u;
  u.s.a = lo;
  u.s.b = hi;
  return u.f;
}

__device__ __forceinline__ void pack_frag(bf16x8& f, const f32x16& x, int s) {
#pragma unroll
  for (int j = 0; j < 8; ++j) f[j] = (__bf16)x[8 * s + j];
}
__device__ __forceinline__ void pack_frag(f16x8& f, const f32x16& x, int s) {
#pragma unroll
  for (int j = 0; j < 8; ++j) f[j] = (_Float16)x[8 * s + j];
}

__device__ __forceinline__ int acc_row(int i, int h) { return (i & 3) + 8 * (i >> 2) + 4 * h; }

}  // namespace attn
}  // namespace lta
