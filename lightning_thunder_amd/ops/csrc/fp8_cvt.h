// OCP fp8 conversion helpers shared by the cast kernels (fp8.hip) and the producer kernels that emit
// fp8 as their own output (RMSNorm forward, SwiGLU forward: the FP8 linear's input cast fused into
// the kernel that produces the activation).
#pragma once

#include "common.h"

namespace lta {

// four saturated values -> one word of four OCP fp8 (e4m3fn or e5m2), two per conversion instruction
template <bool E5M2>
__device__ __forceinline__ uint32_t cvt4(float a, float b, float c, float d) {
  const float mx = E5M2 ? 57344.f : 448.f;
  a = __builtin_amdgcn_fmed3f(a, -mx, mx);
  b = __builtin_amdgcn_fmed3f(b, -mx, mx);
  c = __builtin_amdgcn_fmed3f(c, -mx, mx);
  d = __builtin_amdgcn_fmed3f(d, -mx, mx);
  if constexpr (E5M2) {
    const int w = __builtin_amdgcn_cvt_pk_bf8_f32(a, b, 0, false);
    return (uint32_t)__builtin_amdgcn_cvt_pk_bf8_f32(c, d, w, true);
  } else {
    const int w = __builtin_amdgcn_cvt_pk_fp8_f32(a, b, 0, false);
    return (uint32_t)__builtin_amdgcn_cvt_pk_fp8_f32(c, d, w, true);
  }
}

__device__ __forceinline__ void atomic_max_pos(float* addr, float v) {
  // |x| >= 0: IEEE order == unsigned int order
  atomicMax(reinterpret_cast<unsigned int*>(addr), __float_as_uint(v));
}

// delayed scaling: s = fmax / amax_in (the amax history's max, a device scalar); block (0, 0)
// publishes it to scale_out (the GEMM's dequantisation scale)
__device__ __forceinline__ float fp8_scale(const float* amax_in, float fmax, float* scale_out) {
  const float s = fmax / fmaxf(*amax_in, 1e-12f);
  if (scale_out != nullptr && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) *scale_out = s;
  return s;
}

// the workgroup's max |value| into *amax (one atomic per workgroup; NW waves)
template <int NW>
__device__ __forceinline__ void fp8_amax_out(float m, float* amax, float* red) {
  m = wave_max(m);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = red[0];
#pragma unroll
    for (int i = 1; i < NW; ++i) t = fmaxf(t, red[i]);
    atomic_max_pos(amax, t);
  }
}

}  // namespace lta
