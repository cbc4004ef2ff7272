// K8 support: OCP fp8 (e4m3fn / e5m2) casts for the FP8 linear path on CDNA4, and a probe of the
// block-scaled MFMA operand layout (v_mfma_scale_f32_16x16x128_f8f6f4) used by the fp8 GEMM.
// (reference: TransformerEngine quantizers behind thunder/executors/transformer_engineex.py)
//
// cast:            y = sat(x * scale) in fp8, amax(|x|) folded into amax_out (delayed scaling:
//                  the amax feeds the *next* step's scale, so one pass over x suffices)
// cast_transpose:  the same, plus the transposed fp8 copy the backward GEMMs read (dgrad needs
//                  W^T, wgrad needs X^T and dY^T; all three GEMMs then run on the one NT kernel)
#include "common.h"

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

__device__ __forceinline__ void atomic_max_pos(float* addr, float v) {
  // |x| >= 0: IEEE order == unsigned int order
  atomicMax(reinterpret_cast<unsigned int*>(addr), __float_as_uint(v));
}

// scale = fmax / amax_in (device scalar written by lta_amax); block 0 publishes it to scale_out
__device__ __forceinline__ float dev_scale(const float* amax_in, float fmax, float* scale_out) {
  const float s = fmax / fmaxf(*amax_in, 1e-12f);
  if (scale_out != nullptr && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) *scale_out = s;
  return s;
}

template <typename T>
__global__ __launch_bounds__(256) void amax_kernel(const T* __restrict__ x, int64_t n, float* __restrict__ amax) {
  float m = 0.f;
  const int64_t nv = n / 8;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nv; i += (int64_t)gridDim.x * blockDim.x) {
    const Vec16<T> v = load16(x + i * 8);
#pragma unroll
    for (int j = 0; j < 8; ++j) m = fmaxf(m, fabsf(to_f32(v.v[j])));
  }
  // one atomic per workgroup: same-address atomics serialise in L2 (MI355X_MICROARCH.md §atomics)
  __shared__ float red[4];
  m = wave_max(m);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) atomic_max_pos(amax, fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3])));
}

template <typename T, bool E5M2>
__global__ __launch_bounds__(256) void cast_kernel(const T* __restrict__ x, uint8_t* __restrict__ y, int64_t n,
                                                   const float* __restrict__ amax_in, float fmax,
                                                   float* __restrict__ scale_out, float* __restrict__ amax) {
  const float s = dev_scale(amax_in, fmax, scale_out);
  float m = 0.f;
  const int64_t nv = n / 8;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nv; i += (int64_t)gridDim.x * blockDim.x) {
    const Vec16<T> v = load16(x + i * 8);
    uint32_t lo = 0, hi = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float f = to_f32(v.v[j]);
      m = fmaxf(m, fabsf(f));
      const uint32_t q = E5M2 ? to_e5m2(f * s) : to_e4m3(f * s);
      if (j < 4) lo |= q << (8 * j);
      else hi |= q << (8 * (j - 4));
    }
    *reinterpret_cast<uint2*>(y + i * 8) = make_uint2(lo, hi);
  }
  m = wave_max(m);
  if ((threadIdx.x & 63) == 0 && amax != nullptr) atomic_max_pos(amax, m);
}

// x [R, C] row-major -> y [R, C] and yt [C, R] (64x64 tiles through LDS)
template <typename T, bool E5M2>
__global__ __launch_bounds__(256) void cast_transpose_kernel(const T* __restrict__ x, uint8_t* __restrict__ y,
                                                             uint8_t* __restrict__ yt, int R, int C,
                                                             const float* __restrict__ amax_in, float fmax,
                                                             float* __restrict__ scale_out, float* __restrict__ amax) {
  __shared__ uint8_t tile[64][64 + 4];
  const float s = dev_scale(amax_in, fmax, scale_out);
  const int r0 = blockIdx.y * 64, c0 = blockIdx.x * 64;
  const int tr = threadIdx.x / 8, tc = (threadIdx.x % 8) * 8;  // 32 rows x 8 chunks of 8 per pass
  float m = 0.f;
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    const int r = tr + 32 * p;
    const Vec16<T> v = load16(x + (int64_t)(r0 + r) * C + c0 + tc);
    uint32_t lo = 0, hi = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float f = to_f32(v.v[j]);
      m = fmaxf(m, fabsf(f));
      const uint32_t q = E5M2 ? to_e5m2(f * s) : to_e4m3(f * s);
      tile[r][tc + j] = (uint8_t)q;
      if (j < 4) lo |= q << (8 * j);
      else hi |= q << (8 * (j - 4));
    }
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
  m = wave_max(m);
  if ((threadIdx.x & 63) == 0 && amax != nullptr) atomic_max_pos(amax, m);
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
  c[l] = acc;
}

}  // namespace

template <typename T, bool E5>
static void launch_cast(const void* x, void* y, int64_t n, const void* amax_in, float fmax, void* scale_out,
                        void* amax, hipStream_t s) {
  dim3 grid((unsigned)std::min<int64_t>((n / 8 + 255) / 256, 4096)), block(256);
  hipLaunchKernelGGL((cast_kernel<T, E5>), grid, block, 0, s, (const T*)x, (uint8_t*)y, n, (const float*)amax_in, fmax,
                     (float*)scale_out, (float*)amax);
}

template <typename T, bool E5>
static void launch_cast_t(const void* x, void* y, void* yt, int R, int C, const void* amax_in, float fmax,
                          void* scale_out, void* amax, hipStream_t s) {
  dim3 grid(C / 64, R / 64), block(256);
  hipLaunchKernelGGL((cast_transpose_kernel<T, E5>), grid, block, 0, s, (const T*)x, (uint8_t*)y, (uint8_t*)yt, R, C,
                     (const float*)amax_in, fmax, (float*)scale_out, (float*)amax);
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

// layout probe: 64 lanes x 32 B of A and B, result 64 lanes x 4 fp32
LTA_EXPORT int lta_fp8_mfma_probe(const void* a, const void* b, void* c, int fmt_a, int fmt_b, hipStream_t s) {
  hipLaunchKernelGGL(mfma_probe_kernel, dim3(1), dim3(64), 0, s, (const v8i*)a, (const v8i*)b, (f32x4*)c, fmt_a, fmt_b);
  return (int)hipGetLastError();
}
