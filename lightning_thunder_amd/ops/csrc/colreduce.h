// Column sum of fp32 partial rows -> T (the second pass of the normalisation backwards' weight /
// bias gradients; deterministic, no float atomics).  Shared by csrc/rmsnorm.hip and csrc/layernorm.hip.
#pragma once
#include "common.h"

namespace {

using namespace lta;

// A 256-thread block owns 32 columns, 8 lanes x float4 per row and 32 row groups, each thread
// keeping 8 independent loads in flight, one LDS pass to combine the row groups.  Needs cols % 4 == 0.
template <typename T>
__global__ __launch_bounds__(256) void column_reduce_v4_kernel(const float* __restrict__ partial,
                                                                    T* __restrict__ out, int nblocks, int cols) {
  __shared__ float4 sm[32][8];  // 256 threads: 8 column quads x 32 row groups
  const int cl = threadIdx.x & 7, rg = threadIdx.x >> 3;
  const int col = blockIdx.x * 32 + cl * 4;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  if (col < cols) {
    int b = rg;
    for (; b + 7 * 32 < nblocks; b += 8 * 32) {
      float4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = *reinterpret_cast<const float4*>(partial + (int64_t)(b + u * 32) * cols + col);
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        acc.x += v[u].x;
        acc.y += v[u].y;
        acc.z += v[u].z;
        acc.w += v[u].w;
      }
    }
    for (; b < nblocks; b += 32) {
      const float4 v = *reinterpret_cast<const float4*>(partial + (int64_t)b * cols + col);
      acc.x += v.x;
      acc.y += v.y;
      acc.z += v.z;
      acc.w += v.w;
    }
  }
  sm[rg][cl] = acc;
  __syncthreads();
  if (threadIdx.x < 32) {
    const int c = threadIdx.x >> 2, e = threadIdx.x & 3;
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < 32; ++i) t += reinterpret_cast<const float*>(&sm[i][c])[e];
    const int oc = blockIdx.x * 32 + threadIdx.x;
    if (oc < cols) out[oc] = from_f32<T>(t);
  }
}


}  // namespace
