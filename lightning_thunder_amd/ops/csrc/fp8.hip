// K8 support: OCP fp8 (e4m3fn / e5m2) casts for the FP8 linear path on CDNA4, and a probe of the
// block-scaled MFMA operand layout (v_mfma_scale_f32_16x16x128_f8f6f4) used by the fp8 GEMM.
// (reference: TransformerEngine quantizers behind thunder/executors/transformer_engineex.py)
//
// cast:            y = sat(x * scale) in fp8, amax(|x|) folded into amax_out (delayed scaling:
//                  the amax feeds the *next* step's scale, so one pass over x suffices)
// cast_transpose:  the same, plus the transposed fp8 copy the backward GEMMs read (dgrad needs
//                  W^T, wgrad needs X^T and dY^T; all three GEMMs then run on the one NT kernel)
#include <cstdio>
#include <cstdlib>

#include "common.h"
#include "fp8_cvt.h"

using namespace lta;

namespace {

typedef int v8i __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint8_t to_e4m3(float v) {
  // saturating round-to-nearest-even to OCP e4m3fn (max 448)
  v = fminf(fmaxf(v, -448.f), 448.f);
  return (uint8_t)(__builtin_amdgcn_cvt_pk_fp8_f32(v, 0.f, 0, false) & 0xff);
}
__device__ __forceinline__ uint8_t to_e5m2(float v) {
  v = fminf(fmaxf(v, -57344.f), 57344.f);
  return (uint8_t)(__builtin_amdgcn_cvt_pk_bf8_f32(v, 0.f, 0, false) & 0xff);
}

// scale = fmax / amax_in (device scalar written by lta_amax); block 0 publishes it to scale_out
__device__ __forceinline__ float dev_scale(const float* amax_in, float fmax, float* scale_out) {
  const float s = fmax / fmaxf(*amax_in, 1e-12f);
  if (scale_out != nullptr && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) *scale_out = s;
  return s;
}

// 8 consecutive elements as fp32 (one 16-B load for bf16, two for fp32)
template <typename T>
__device__ __forceinline__ void load8(const T* p, float (&o)[8]) {
  if constexpr (sizeof(T) == 2) {
    const Vec16<T> a = load16(p);
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = to_f32(a.v[j]);
  } else {
    const Vec16<T> a = load16(p), b = load16(p + 4);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      o[j] = to_f32(a.v[j]);
      o[4 + j] = to_f32(b.v[j]);
    }
  }
}

template <typename T>
__global__ __launch_bounds__(256) void amax_kernel(const T* __restrict__ x, int64_t n, float* __restrict__ amax) {
  float m = 0.f;
  const int64_t nv = n / 8;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nv; i += (int64_t)gridDim.x * blockDim.x) {
    float v[8];
    load8(x + i * 8, v);
#pragma unroll
    for (int j = 0; j < 8; ++j) m = fmaxf(m, fabsf(v[j]));
  }
  // one atomic per workgroup: same-address atomics serialise in L2 (MI355X_MICROARCH.md §atomics)
  __shared__ float red[4];
  m = wave_max(m);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) atomic_max_pos(amax, fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3])));
}

template <typename T, bool E5M2, int U = 2>
__global__ __launch_bounds__(256) void cast_kernel(const T* __restrict__ x, uint8_t* __restrict__ y, int64_t n,
                                                   const float* __restrict__ amax_in, float fmax,
                                                   float* __restrict__ scale_out, float* __restrict__ amax) {
  const float s = dev_scale(amax_in, fmax, scale_out);
  float m = 0.f;
  const int64_t nv = n / 8, stride = (int64_t)gridDim.x * blockDim.x;
  // U 8-element vectors per thread and iteration (all loads issued before the first conversion),
  // two elements per hardware conversion (cvt4)
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + (U - 1) * stride < nv; i += U * stride) {
    float v[U][8];
#pragma unroll
    for (int u = 0; u < U; ++u) load8(x + (i + u * stride) * 8, v[u]);
#pragma unroll
    for (int u = 0; u < U; ++u) {
#pragma unroll
      for (int j = 0; j < 8; ++j) m = fmaxf(m, fabsf(v[u][j]));
      const uint32_t lo = cvt4<E5M2>(v[u][0] * s, v[u][1] * s, v[u][2] * s, v[u][3] * s);
      const uint32_t hi = cvt4<E5M2>(v[u][4] * s, v[u][5] * s, v[u][6] * s, v[u][7] * s);
      *reinterpret_cast<uint2*>(y + (i + u * stride) * 8) = make_uint2(lo, hi);
    }
  }
  for (; i < nv; i += stride) {
    float v[8];
    load8(x + i * 8, v);
#pragma unroll
    for (int j = 0; j < 8; ++j) m = fmaxf(m, fabsf(v[j]));
    const uint32_t lo = cvt4<E5M2>(v[0] * s, v[1] * s, v[2] * s, v[3] * s);
    const uint32_t hi = cvt4<E5M2>(v[4] * s, v[5] * s, v[6] * s, v[7] * s);
    *reinterpret_cast<uint2*>(y + i * 8) = make_uint2(lo, hi);
  }
  if (amax != nullptr) {  // one atomic per workgroup
    __shared__ float red[4];
    m = wave_max(m);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) atomic_max_pos(amax, fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3])));
  }
}

// x [R, C] row-major -> y [R, C] and yt [C, R] (64x64 tiles through LDS).  A capped grid loops over
// the tiles so the amax (delayed scaling) costs one atomic per workgroup, not one per tile-wave:
// same-address atomics serialise (MI355X_MICROARCH.md, global atomics contention row).
template <typename T, bool E5M2>
__global__ __launch_bounds__(256) void cast_transpose_kernel(const T* __restrict__ x, uint8_t* __restrict__ y,
                                                             uint8_t* __restrict__ yt, int R, int C,
                                                             const float* __restrict__ amax_in, float fmax,
                                                             float* __restrict__ scale_out, float* __restrict__ amax) {
  __shared__ uint8_t tile[64][64 + 4];
  __shared__ float red[4];
  const float s = dev_scale(amax_in, fmax, scale_out);
  const int tr = threadIdx.x / 8, tc = (threadIdx.x % 8) * 8;  // 32 rows x 8 chunks of 8 per pass
  const int tiles_c = C / 64, ntiles = tiles_c * (R / 64);
  float m = 0.f;
  for (int tile_id = blockIdx.x; tile_id < ntiles; tile_id += gridDim.x) {
    const int r0 = (tile_id / tiles_c) * 64, c0 = (tile_id % tiles_c) * 64;
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      const int r = tr + 32 * p;
      float v[8];
      load8(x + (int64_t)(r0 + r) * C + c0 + tc, v);
#pragma unroll
      for (int j = 0; j < 8; ++j) m = fmaxf(m, fabsf(v[j]));
      // two elements per hardware conversion, written straight into the packed words
      const uint32_t lo = cvt4<E5M2>(v[0] * s, v[1] * s, v[2] * s, v[3] * s);
      const uint32_t hi = cvt4<E5M2>(v[4] * s, v[5] * s, v[6] * s, v[7] * s);
      *reinterpret_cast<uint32_t*>(&tile[r][tc]) = lo;  // rows are 4-byte aligned (stride 68)
      *reinterpret_cast<uint32_t*>(&tile[r][tc + 4]) = hi;
      if (y != nullptr) *reinterpret_cast<uint2*>(y + (int64_t)(r0 + r) * C + c0 + tc) = make_uint2(lo, hi);
    }
    __syncthreads();
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      const int c = tr + 32 * p;  // output row = input column
      uint32_t lo = 0, hi = 0;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const uint32_t q = tile[tc + j][c];
        if (j < 4) lo |= q << (8 * j);
        else hi |= q << (8 * (j - 4));
      }
      *reinterpret_cast<uint2*>(yt + (int64_t)(c0 + c) * R + r0 + tc) = make_uint2(lo, hi);
    }
    __syncthreads();  // the tile is rewritten by the next iteration
  }
  if (amax != nullptr) {
    m = wave_max(m);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) atomic_max_pos(amax, fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3])));
  }
}

// 128 x 128 tiles (R, C % 128): every output row segment — y's 128 columns and y^T's 128 rows — is a
// full 128-B line (the 64 x 64 tile above writes half lines, and y^T's half lines from neighbouring
// tiles meet only in L2: 3.8-4.4 TB/s on the 12288- / 22016-column shapes).  All eight 16-B loads of
// a thread are issued before the first conversion.
template <typename T, bool E5M2>
__global__ __launch_bounds__(256) void cast_transpose128_kernel(const T* __restrict__ x, uint8_t* __restrict__ y,
                                                                uint8_t* __restrict__ yt, int R, int C,
                                                                const float* __restrict__ amax_in, float fmax,
                                                                float* __restrict__ scale_out,
                                                                float* __restrict__ amax) {
  __shared__ uint8_t tile[128][128 + 8];
  __shared__ float red[4];
  const float s = dev_scale(amax_in, fmax, scale_out);
  const int tr = threadIdx.x >> 4, tc = (threadIdx.x & 15) * 8;  // 16 rows x 16 chunks of 8 per pass
  const int tiles_c = C / 128, ntiles = tiles_c * (R / 128);
  float m = 0.f;
  for (int tile_id = blockIdx.x; tile_id < ntiles; tile_id += gridDim.x) {
    const int r0 = (tile_id / tiles_c) * 128, c0 = (tile_id % tiles_c) * 128;
    float v[8][8];
#pragma unroll
    for (int p = 0; p < 8; ++p) load8(x + (int64_t)(r0 + tr + 16 * p) * C + c0 + tc, v[p]);
#pragma unroll
    for (int p = 0; p < 8; ++p) {
      const int r = tr + 16 * p;
#pragma unroll
      for (int j = 0; j < 8; ++j) m = fmaxf(m, fabsf(v[p][j]));
      const uint32_t lo = cvt4<E5M2>(v[p][0] * s, v[p][1] * s, v[p][2] * s, v[p][3] * s);
      const uint32_t hi = cvt4<E5M2>(v[p][4] * s, v[p][5] * s, v[p][6] * s, v[p][7] * s);
      *reinterpret_cast<uint2*>(&tile[r][tc]) = make_uint2(lo, hi);  // rows 8-byte aligned (stride 136)
      if (y != nullptr) *reinterpret_cast<uint2*>(y + (int64_t)(r0 + r) * C + c0 + tc) = make_uint2(lo, hi);
    }
    __syncthreads();
#pragma unroll
    for (int p = 0; p < 8; ++p) {
      const int c = tr + 16 * p;  // output row = input column; 8 input rows tc .. tc + 7 per thread
      uint32_t lo = 0, hi = 0;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const uint32_t q = tile[tc + j][c];
        if (j < 4) lo |= q << (8 * j);
        else hi |= q << (8 * (j - 4));
      }
      *reinterpret_cast<uint2*>(yt + (int64_t)(c0 + c) * R + r0 + tc) = make_uint2(lo, hi);
    }
    __syncthreads();  // the tile is rewritten by the next iteration
  }
  if (amax != nullptr) {
    m = wave_max(m);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) atomic_max_pos(amax, fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3])));
  }
}

// ---------------------------------------------------------------------------------------------
// MXFP8 (OCP microscaling): blocks of 32 consecutive elements along the GEMM reduction dim share one
// E8M0 scale X = 2^ceil(log2(amax_block / fp8_max)) (the OCP floor(log2 amax) - emax choice
// saturates blocks whose amax mantissa exceeds 1.75; rounding the exponent up never clips);
// elements are x / X in fp8.  One 64x64 tile pass emits both orientations the training GEMMs read:
// q [R, C] with scales s [R, C/32] (blocks along C) and q^T [C, R] with s^T [C, R/32] (blocks along
// R), so fprop, dgrad and wgrad all reduce over 32-blocks of their own K.
// ---------------------------------------------------------------------------------------------
template <bool E5M2>
__device__ __forceinline__ uint32_t mx_exp(float amax) {
  // biased E8M0 exponent of the block scale: the smallest 2^s with amax / 2^s <= fp8 max
  // (fp8 max = 1.75 * 2^emax), so no element saturates; amax == 0 -> 2^-127 (the block is zeros)
  if (!(amax > 0.f)) return 0u;
  const uint32_t bits = __float_as_uint(amax);
  const int e = (int)((bits >> 23) & 0xff) - 127;        // floor(log2(amax)) for a normal amax
  const bool above = (bits & 0x7fffff) > 0x600000u;     // mantissa > 1.75
  const int s = e - (E5M2 ? 15 : 8) + (above ? 1 : 0);
  return (uint32_t)min(max(s + 127, 0), 254);
}

template <bool E5M2>
__device__ __forceinline__ uint32_t mx_q(float v, float inv) {
  return E5M2 ? to_e5m2(v * inv) : to_e4m3(v * inv);
}

__device__ __forceinline__ float e8m0_inv(uint32_t be) {
  // 2^-(be - 127) exactly (be in [0, 254])
  const int f = 254 - (int)be;  // float exponent field of 2^(127 - be)
  return __uint_as_float(f > 0 ? (uint32_t)f << 23 : 0x00400000u);  // be = 254: 2^-127 (subnormal)
}

template <typename T, bool E5M2>
__global__ __launch_bounds__(256) void mx_cast_transpose_kernel(const T* __restrict__ x, uint8_t* __restrict__ q,
                                                                uint8_t* __restrict__ sq, uint8_t* __restrict__ qt,
                                                                uint8_t* __restrict__ sqt, int R, int C) {
  __shared__ float tile[64][65];
  const int r0 = blockIdx.y * 64, c0 = blockIdx.x * 64;
  const int t = threadIdx.x, tr = t >> 2, tq = t & 3;  // row (or column) tr, 16-element segment tq
  // ---- rowwise: thread owns x[r0+tr][c0 + 16 tq .. +16]; blocks of 32 = segments (0,1), (2,3) ----
  float v[16];
  {
    const T* src = x + (int64_t)(r0 + tr) * C + c0 + tq * 16;
    float a[8], b[8];
    load8(src, a);
    load8(src + 8, b);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      v[j] = a[j];
      v[8 + j] = b[j];
    }
  }
  float m = 0.f;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    m = fmaxf(m, fabsf(v[j]));
    tile[tr][tq * 16 + j] = v[j];
  }
  m = fmaxf(m, __shfl_xor(m, 1));
  {
    const uint32_t be = mx_exp<E5M2>(m);
    const float inv = e8m0_inv(be);
    uint32_t w[4] = {0, 0, 0, 0};
#pragma unroll
    for (int j = 0; j < 16; ++j) w[j >> 2] |= mx_q<E5M2>(v[j], inv) << (8 * (j & 3));
    *reinterpret_cast<uint4*>(q + (int64_t)(r0 + tr) * C + c0 + tq * 16) = make_uint4(w[0], w[1], w[2], w[3]);
    if ((tq & 1) == 0) sq[(int64_t)(r0 + tr) * (C / 32) + c0 / 32 + (tq >> 1)] = (uint8_t)be;
  }
  __syncthreads();
  // ---- columnwise: thread owns column c0+tr, rows r0 + 16 tq .. +16 -> q^T[c0+tr][r0 + 16 tq ..] ----
  m = 0.f;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    v[j] = tile[tq * 16 + j][tr];
    m = fmaxf(m, fabsf(v[j]));
  }
  m = fmaxf(m, __shfl_xor(m, 1));
  {
    const uint32_t be = mx_exp<E5M2>(m);
    const float inv = e8m0_inv(be);
    uint32_t w[4] = {0, 0, 0, 0};
#pragma unroll
    for (int j = 0; j < 16; ++j) w[j >> 2] |= mx_q<E5M2>(v[j], inv) << (8 * (j & 3));
    *reinterpret_cast<uint4*>(qt + (int64_t)(c0 + tr) * R + r0 + tq * 16) = make_uint4(w[0], w[1], w[2], w[3]);
    if ((tq & 1) == 0) sqt[(int64_t)(c0 + tr) * (R / 32) + r0 / 32 + (tq >> 1)] = (uint8_t)be;
  }
}

// ---------------------------------------------------------------------------------------------
// MXFP4: blocks of 32 consecutive elements along the last dim share an E8M0 scale
// X = 2^ceil-variant(log2(amax / 6)) (as MXFP8 above: the exponent is rounded up when amax's
// mantissa exceeds 1.5, so no element saturates); elements x / X round to nearest-even e2m1
// {0, .5, 1, 1.5, 2, 3, 4, 6} and are packed two per byte, low nibble first.  One thread per
// block: 64 B of bf16 in, 16 B + 1 scale byte out.
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t e2m1_code(float v) {
  const float a = fabsf(v);
  uint32_t c = a <= 0.25f ? 0u : a < 0.75f ? 1u : a <= 1.25f ? 2u : a < 1.75f ? 3u
             : a <= 2.5f ? 4u : a < 3.5f ? 5u : a <= 5.f ? 6u : 7u;
  return c | (v < 0.f && c != 0u ? 8u : 0u);
}

__device__ __forceinline__ uint32_t mx4_exp(float amax) {
  if (!(amax > 0.f)) return 0u;
  const uint32_t bits = __float_as_uint(amax);
  const int e = (int)((bits >> 23) & 0xff) - 127;
  const bool above = (bits & 0x7fffff) > 0x400000u;  // mantissa > 1.5 (e2m1 max = 1.5 * 2^2)
  return (uint32_t)min(max(e - 2 + (above ? 1 : 0) + 127, 0), 254);
}

template <typename T>
__global__ __launch_bounds__(256) void mx4_cast_kernel(const T* __restrict__ x, uint8_t* __restrict__ q,
                                                       uint8_t* __restrict__ sq, int64_t nblocks) {
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= nblocks) return;
  const T* src = x + b * 32;
  float v[32];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    float a[8];
    load8(src + 8 * i, a);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[8 * i + j] = a[j];
  }
  float m = 0.f;
#pragma unroll
  for (int j = 0; j < 32; ++j) m = fmaxf(m, fabsf(v[j]));
  const uint32_t be = mx4_exp(m);
  const float inv = e8m0_inv(be);
  uint32_t w[4] = {0, 0, 0, 0};
#pragma unroll
  for (int j = 0; j < 32; ++j) w[j >> 3] |= e2m1_code(v[j] * inv) << (4 * (j & 7));
  *reinterpret_cast<uint4*>(q + b * 16) = make_uint4(w[0], w[1], w[2], w[3]);
  sq[b] = (uint8_t)be;
}

// one wave, 16x16x128 block-scaled MFMA with per-lane E8M0 scale registers (scale-operand probe)
__global__ void mfma_scale_probe_kernel(const v8i* __restrict__ a, const v8i* __restrict__ b,
                                        const int* __restrict__ sa, const int* __restrict__ sb,
                                        f32x4* __restrict__ c) {
  const int l = threadIdx.x;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  acc = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a[l], b[l], acc, 0, 0, 0, sa[l], 0, sb[l]);
  c[l] = acc;
}

// one wave: C = A . B^T for a 16x16x128 tile from raw per-lane registers (layout probe)
__global__ void mfma_probe_kernel(const v8i* __restrict__ a, const v8i* __restrict__ b, f32x4* __restrict__ c,
                                  int fmt_a, int fmt_b) {
  const int l = threadIdx.x;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  if (fmt_a == 0 && fmt_b == 0)
    acc = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a[l], b[l], acc, 0, 0, 0, 0x7f7f7f7f, 0, 0x7f7f7f7f);
  else if (fmt_a == 1 && fmt_b == 0)
    acc = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a[l], b[l], acc, 1, 0, 0, 0x7f7f7f7f, 0, 0x7f7f7f7f);
  else if (fmt_a == 4 && fmt_b == 4)  // fp4 e2m1 x fp4 e2m1: 16 operand bytes per lane
    acc = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a[l], b[l], acc, 4, 4, 0, 0x7f7f7f7f, 0, 0x7f7f7f7f);
  else if (fmt_a == 0 && fmt_b == 4)  // fp8 e4m3 x fp4 e2m1
    acc = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a[l], b[l], acc, 0, 4, 0, 0x7f7f7f7f, 0, 0x7f7f7f7f);
  else if (fmt_a == 4 && fmt_b == 0)
    acc = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a[l], b[l], acc, 4, 0, 0, 0x7f7f7f7f, 0, 0x7f7f7f7f);
  c[l] = acc;
}

}  // namespace

// grid / unroll of the plain cast: LTA_CAST_CFG = "<max workgroups>,<vectors per thread>" (A/B hook,
// scripts/fp8_cast_bench.py); the default is the measured fastest of that sweep
static int g_cast_wgs = 512, g_cast_u = 4;
static bool g_cast_cfg_read = false;
template <typename T, bool E5>
static void launch_cast(const void* x, void* y, int64_t n, const void* amax_in, float fmax, void* scale_out,
                        void* amax, hipStream_t s) {
  if (!g_cast_cfg_read) {
    g_cast_cfg_read = true;
    if (const char* e = std::getenv("LTA_CAST_CFG")) {
      int w = 0, u = 0;
      if (sscanf(e, "%d,%d", &w, &u) == 2 && w > 0 && (u == 1 || u == 2 || u == 4 || u == 8)) g_cast_wgs = w, g_cast_u = u;
    }
  }
  dim3 grid((unsigned)std::min<int64_t>((n / 8 + 255) / 256, g_cast_wgs)), block(256);
#define LTA_CAST(UU)                                                                                               \
  hipLaunchKernelGGL((cast_kernel<T, E5, UU>), grid, block, 0, s, (const T*)x, (uint8_t*)y, n, (const float*)amax_in, \
                     fmax, (float*)scale_out, (float*)amax)
  if (g_cast_u == 4) LTA_CAST(4);
  else if (g_cast_u == 8) LTA_CAST(8);
  else if (g_cast_u == 1) LTA_CAST(1);
  else LTA_CAST(2);
#undef LTA_CAST
}

template <typename T, bool E5>
static void launch_cast_t(const void* x, void* y, void* yt, int R, int C, const void* amax_in, float fmax,
                          void* scale_out, void* amax, hipStream_t s) {
  // 128 x 128 tiles only where they measured faster (profiles/fp8_cast_transpose_ab.json, round 3:
  // 4096x12288 46 -> 38 us, 4096x22016 98 -> 80, 32000x4096 130 -> 113; but 4096x4096 12.8 -> 17.7 and
  // 4096x11008 30 -> 35: fewer, larger tiles leave too few loads in flight on the smaller shapes)
  if (R % 128 == 0 && C % 128 == 0 && (C >= 12288 || R >= 16384) && std::getenv("LTA_CAST_T64") == nullptr) {
    dim3 grid((unsigned)std::min<int64_t>((int64_t)(C / 128) * (R / 128), 1024)), block(256);
    hipLaunchKernelGGL((cast_transpose128_kernel<T, E5>), grid, block, 0, s, (const T*)x, (uint8_t*)y, (uint8_t*)yt,
                       R, C, (const float*)amax_in, fmax, (float*)scale_out, (float*)amax);
    return;
  }
  dim3 grid((unsigned)std::min<int64_t>((int64_t)(C / 64) * (R / 64), 1024)), block(256);
  hipLaunchKernelGGL((cast_transpose_kernel<T, E5>), grid, block, 0, s, (const T*)x, (uint8_t*)y, (uint8_t*)yt, R, C,
                     (const float*)amax_in, fmax, (float*)scale_out, (float*)amax);
}

// A/B hook of the plain cast's grid cap / unroll (scripts/fp8_cast_bench.py); returns the previous cap
LTA_EXPORT int lta_fp8_cast_set_cfg(int wgs, int u) {
  g_cast_cfg_read = true;
  const int old = g_cast_wgs;
  if (wgs > 0 && (u == 1 || u == 2 || u == 4 || u == 8)) g_cast_wgs = wgs, g_cast_u = u;
  return old;
}

// amax_out (zero-initialised by the caller) = max(amax_out, max |x|)
LTA_EXPORT int lta_amax(int in_dtype, const void* x, int64_t n, void* amax_out, hipStream_t s) {
  if (n % 8) return -2;
  dim3 grid((unsigned)std::min<int64_t>((n / 8 + 255) / 256, 512)), block(256);
  if (in_dtype == kBF16)
    hipLaunchKernelGGL(amax_kernel<__hip_bfloat16>, grid, block, 0, s, (const __hip_bfloat16*)x, n, (float*)amax_out);
  else if (in_dtype == kF32)
    hipLaunchKernelGGL(amax_kernel<float>, grid, block, 0, s, (const float*)x, n, (float*)amax_out);
  else
    return -1;
  return (int)hipGetLastError();
}

// y = fp8(x * s), s = fmax / *amax_in (written to *scale_out); e5m2 if `e5m2` else e4m3fn.
// amax_out (may be null) additionally receives max |x| (delayed-scaling history).
LTA_EXPORT int lta_fp8_cast(int in_dtype, int e5m2, const void* x, void* y, int64_t n, const void* amax_in, float fmax,
                            void* scale_out, void* amax, hipStream_t s) {
  if (n % 8) return -2;
  if (in_dtype == kBF16) {
    if (e5m2) launch_cast<__hip_bfloat16, true>(x, y, n, amax_in, fmax, scale_out, amax, s);
    else launch_cast<__hip_bfloat16, false>(x, y, n, amax_in, fmax, scale_out, amax, s);
  } else if (in_dtype == kF32) {
    if (e5m2) launch_cast<float, true>(x, y, n, amax_in, fmax, scale_out, amax, s);
    else launch_cast<float, false>(x, y, n, amax_in, fmax, scale_out, amax, s);
  } else {
    return -1;
  }
  return (int)hipGetLastError();
}

// x [R, C] -> y [R, C] (optional) and yt [C, R]; R, C multiples of 64.
LTA_EXPORT int lta_fp8_cast_transpose(int in_dtype, int e5m2, const void* x, void* y, void* yt, int R, int C,
                                      const void* amax_in, float fmax, void* scale_out, void* amax, hipStream_t s) {
  if (R % 64 || C % 64) return -2;
  if (in_dtype == kBF16) {
    if (e5m2) launch_cast_t<__hip_bfloat16, true>(x, y, yt, R, C, amax_in, fmax, scale_out, amax, s);
    else launch_cast_t<__hip_bfloat16, false>(x, y, yt, R, C, amax_in, fmax, scale_out, amax, s);
  } else if (in_dtype == kF32) {
    if (e5m2) launch_cast_t<float, true>(x, y, yt, R, C, amax_in, fmax, scale_out, amax, s);
    else launch_cast_t<float, false>(x, y, yt, R, C, amax_in, fmax, scale_out, amax, s);
  } else {
    return -1;
  }
  return (int)hipGetLastError();
}

// x [R, C] -> q [R, C] + s [R, C/32] and q^T [C, R] + s^T [C, R/32] (MXFP8); R, C multiples of 64.
LTA_EXPORT int lta_mx_cast_transpose(int in_dtype, int e5m2, const void* x, void* q, void* s, void* qt, void* st, int R,
                                     int C, hipStream_t stream) {
  if (R % 64 || C % 64) return -2;
  dim3 grid(C / 64, R / 64), block(256);
#define LTA_MX(T, E5)                                                                                             \
  hipLaunchKernelGGL((mx_cast_transpose_kernel<T, E5>), grid, block, 0, stream, (const T*)x, (uint8_t*)q,          \
                     (uint8_t*)s, (uint8_t*)qt, (uint8_t*)st, R, C)
  if (in_dtype == kBF16) {
    if (e5m2) LTA_MX(__hip_bfloat16, true);
    else LTA_MX(__hip_bfloat16, false);
  } else if (in_dtype == kF32) {
    if (e5m2) LTA_MX(float, true);
    else LTA_MX(float, false);
  } else {
    return -1;
  }
#undef LTA_MX
  return (int)hipGetLastError();
}

// x [R, C] (C % 32 == 0, contiguous) -> q [R, C/2] packed e2m1 + s [R, C/32] E8M0 (MXFP4).
LTA_EXPORT int lta_mxfp4_cast(int in_dtype, const void* x, void* q, void* s, int64_t numel, hipStream_t stream) {
  if (numel % 32) return -2;
  const int64_t nb = numel / 32;
  dim3 grid((unsigned)((nb + 255) / 256)), block(256);
  if (in_dtype == kBF16)
    hipLaunchKernelGGL(mx4_cast_kernel<__hip_bfloat16>, grid, block, 0, stream, (const __hip_bfloat16*)x,
                       (uint8_t*)q, (uint8_t*)s, nb);
  else if (in_dtype == kF32)
    hipLaunchKernelGGL(mx4_cast_kernel<float>, grid, block, 0, stream, (const float*)x, (uint8_t*)q, (uint8_t*)s, nb);
  else
    return -1;
  return (int)hipGetLastError();
}

LTA_EXPORT int lta_fp8_mfma_scale_probe(const void* a, const void* b, const void* sa, const void* sb, void* c,
                                        hipStream_t s) {
  hipLaunchKernelGGL(mfma_scale_probe_kernel, dim3(1), dim3(64), 0, s, (const v8i*)a, (const v8i*)b, (const int*)sa,
                     (const int*)sb, (f32x4*)c);
  return (int)hipGetLastError();
}

// layout probe: 64 lanes x 32 B of A and B, result 64 lanes x 4 fp32
LTA_EXPORT int lta_fp8_mfma_probe(const void* a, const void* b, void* c, int fmt_a, int fmt_b, hipStream_t s) {
  hipLaunchKernelGGL(mfma_probe_kernel, dim3(1), dim3(64), 0, s, (const v8i*)a, (const v8i*)b, (f32x4*)c, fmt_a, fmt_b);
  return (int)hipGetLastError();
}
