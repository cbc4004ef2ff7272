// Greedy sampling: row-wise argmax over the vocabulary (the decode loop's `logits[:, -1].argmax(-1)`).
// PyTorch's generic reduction takes ~40 us for one 128k-wide bf16 row on MI355X; one 1024-thread
// workgroup per row with 16-byte loads (8 x bf16 per lane, 8 independent loads in flight per
// lane) needs a fraction of that.  Ties resolve to the smallest index and NaN wins, as
// torch.argmax does.
#include "common.h"

namespace lta {
namespace {

constexpr int kThreads = 1024;

struct Best {
  float v;
  int64_t i;
};

__device__ __forceinline__ bool better(float v, int64_t i, float bv, int64_t bi) {
  const bool vn = v != v, bn = bv != bv;
  if (vn || bn) return vn && (!bn || i < bi);
  return v > bv || (v == bv && i < bi);
}

template <typename T>
__global__ __launch_bounds__(kThreads) void argmax_rows_kernel(const T* __restrict__ x, int64_t* __restrict__ out,
                                                               int64_t V, int64_t ld) {
  constexpr int NV = Vec16<T>::N;
  __shared__ float sv[kThreads / 64];
  __shared__ int64_t si[kThreads / 64];
  const T* row = x + blockIdx.x * ld;
  float bv = -INFINITY;
  int64_t bi = V;  // sentinel larger than every index
  const int64_t nvec = V / NV;
  constexpr int G = 8;  // vectors loaded per lane before the compares: 8 x 16 B in flight
  for (int64_t c0 = threadIdx.x; c0 < nvec; c0 += (int64_t)G * kThreads) {
    Vec16<T> p[G];
#pragma unroll
    for (int u = 0; u < G; ++u)
      if (c0 + u * kThreads < nvec) p[u] = load16(row + (c0 + u * kThreads) * NV);
#pragma unroll
    for (int u = 0; u < G; ++u) {
      const int64_t c = c0 + u * kThreads;
      if (c < nvec) {
#pragma unroll
        for (int e = 0; e < NV; ++e) {
          const float v = to_f32(p[u].v[e]);
          if (better(v, c * NV + e, bv, bi)) {
            bv = v;
            bi = c * NV + e;
          }
        }
      }
    }
  }
  for (int64_t j = nvec * NV + threadIdx.x; j < V; j += kThreads) {
    const float v = to_f32(row[j]);
    if (better(v, j, bv, bi)) {
      bv = v;
      bi = j;
    }
  }
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    const float ov = __shfl_xor(bv, off, 64);
    const int64_t oi = __shfl_xor(bi, off, 64);
    if (better(ov, oi, bv, bi)) {
      bv = ov;
      bi = oi;
    }
  }
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) {
    sv[w] = bv;
    si[w] = bi;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int u = 1; u < kThreads / 64; ++u)
      if (better(sv[u], si[u], bv, bi)) {
        bv = sv[u];
        bi = si[u];
      }
    out[blockIdx.x] = bi < V ? bi : 0;
  }
}

}  // namespace
}  // namespace lta

// x: R rows of V logits (row stride ld elements; rows 16-byte aligned, ld % 8 == 0) -> out[R] int64.
LTA_EXPORT int lta_argmax_rows(int dtype, const void* x, void* out, int R, int64_t V, int64_t ld, void* stream) {
  using namespace lta;
  if (R < 1 || V < 1) return (int)hipErrorInvalidValue;
  hipStream_t s = (hipStream_t)stream;
  if (dtype == kBF16)
    hipLaunchKernelGGL(argmax_rows_kernel<__hip_bfloat16>, dim3(R), dim3(kThreads), 0, s, (const __hip_bfloat16*)x,
                       (int64_t*)out, V, ld);
  else if (dtype == kF16)
    hipLaunchKernelGGL(argmax_rows_kernel<__half>, dim3(R), dim3(kThreads), 0, s, (const __half*)x, (int64_t*)out, V,
                       ld);
  else if (dtype == kF32)
    hipLaunchKernelGGL(argmax_rows_kernel<float>, dim3(R), dim3(kThreads), 0, s, (const float*)x, (int64_t*)out, V, ld);
  else
    return (int)hipErrorInvalidValue;
  return (int)hipGetLastError();
}
