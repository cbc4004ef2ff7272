// K5: LayerNorm forward/backward for CDNA4 (gfx950) — GPT-2 / GPT-NeoX / Pythia style models.
// (reference: cuDNN layer norm executor thunder/executors/cudnn_layernormex.py:30-382, and the
// decomposition thunder/torch/__init__.py layer_norm)
//
// Forward: one 256-thread workgroup per row, the row cached in registers (16-B vector loads),
// mean and variance by two register passes (no E[x^2]-E[x]^2 cancellation), per-row fp32
// mean / rstd saved for the backward.
// Backward: several rows per workgroup; dW and dB partial sums stay in registers and are
// written as one fp32 partial row per workgroup, then reduced column-wise by a second kernel
// (deterministic, no float atomics).
#include "common.h"

using namespace lta;

namespace {

constexpr int kThreads = 256;
constexpr int kWaves = kThreads / 64;

template <typename T, int CHUNKS>
__global__ __launch_bounds__(kThreads) void layernorm_fwd_kernel(const T* __restrict__ x, const T* __restrict__ w,
                                                                 const T* __restrict__ b, T* __restrict__ y,
                                                                 float* __restrict__ mean_out,
                                                                 float* __restrict__ rstd_out, int cols, float eps) {
  constexpr int V = Vec16<T>::N;
  __shared__ float smem[kWaves];
  const int64_t row = blockIdx.x;
  const T* xr = x + row * cols;
  Vec16<T> xv[CHUNKS];
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < CHUNKS; ++c) {
    const int idx = (c * kThreads + threadIdx.x) * V;
    if (idx < cols) {
      xv[c] = load16(xr + idx);
#pragma unroll
      for (int j = 0; j < V; ++j) s += to_f32(xv[c].v[j]);
    }
  }
  const float mean = block_sum<kWaves>(s, smem) / (float)cols;
  float ss = 0.f;
#pragma unroll
  for (int c = 0; c < CHUNKS; ++c) {
    const int idx = (c * kThreads + threadIdx.x) * V;
    if (idx < cols) {
#pragma unroll
      for (int j = 0; j < V; ++j) {
        const float d = to_f32(xv[c].v[j]) - mean;
        ss += d * d;
      }
    }
  }
  const float rstd = rsqrtf(block_sum<kWaves>(ss, smem) / (float)cols + eps);
  if (threadIdx.x == 0) {
    mean_out[row] = mean;
    rstd_out[row] = rstd;
  }
#pragma unroll
  for (int c = 0; c < CHUNKS; ++c) {
    const int idx = (c * kThreads + threadIdx.x) * V;
    if (idx < cols) {
      Vec16<T> o, wv, bv;
      if (w) wv = load16(w + idx);
      if (b) bv = load16(b + idx);
#pragma unroll
      for (int j = 0; j < V; ++j) {
        float v = (to_f32(xv[c].v[j]) - mean) * rstd;
        if (w) v *= to_f32(wv.v[j]);
        if (b) v += to_f32(bv.v[j]);
        o.v[j] = from_f32<T>(v);
      }
      store16(y + row * cols + idx, o);
    }
  }
}

template <typename T>
__global__ __launch_bounds__(kThreads) void layernorm_fwd_generic(const T* __restrict__ x, const T* __restrict__ w,
                                                                  const T* __restrict__ b, T* __restrict__ y,
                                                                  float* __restrict__ mean_out,
                                                                  float* __restrict__ rstd_out, int cols, float eps) {
  __shared__ float smem[kWaves];
  const int64_t row = blockIdx.x;
  const T* xr = x + row * cols;
  float s = 0.f;
  for (int i = threadIdx.x; i < cols; i += kThreads) s += to_f32(xr[i]);
  const float mean = block_sum<kWaves>(s, smem) / (float)cols;
  float ss = 0.f;
  for (int i = threadIdx.x; i < cols; i += kThreads) {
    const float d = to_f32(xr[i]) - mean;
    ss += d * d;
  }
  const float rstd = rsqrtf(block_sum<kWaves>(ss, smem) / (float)cols + eps);
  if (threadIdx.x == 0) {
    mean_out[row] = mean;
    rstd_out[row] = rstd;
  }
  for (int i = threadIdx.x; i < cols; i += kThreads) {
    float v = (to_f32(xr[i]) - mean) * rstd;
    if (w) v *= to_f32(w[i]);
    if (b) v += to_f32(b[i]);
    y[row * cols + i] = from_f32<T>(v);
  }
}

// partials: [nblocks][2][cols] (dW row then dB row)
template <typename T>
__global__ __launch_bounds__(kThreads) void layernorm_bwd_kernel(const T* __restrict__ dy, const T* __restrict__ x,
                                                                 const T* __restrict__ w, const float* __restrict__ mean,
                                                                 const float* __restrict__ rstd, T* __restrict__ dx,
                                                                 float* __restrict__ partial, int64_t rows, int cols,
                                                                 int rows_per_block) {
  __shared__ float smem[kWaves];
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
  const int64_t r1 = min(rows, r0 + rows_per_block);
  float* pw = partial ? partial + (int64_t)blockIdx.x * 2 * cols : nullptr;
  if (pw) {
    for (int i = threadIdx.x; i < 2 * cols; i += kThreads) pw[i] = 0.f;
  }
  for (int64_t row = r0; row < r1; ++row) {
    const float mu = mean[row], rs = rstd[row];
    float a1 = 0.f, a2 = 0.f;  // sum(g*w), sum(g*w*xhat)
    for (int i = threadIdx.x; i < cols; i += kThreads) {
      const float xh = (to_f32(x[row * cols + i]) - mu) * rs;
      const float gw = to_f32(dy[row * cols + i]) * (w ? to_f32(w[i]) : 1.f);
      a1 += gw;
      a2 += gw * xh;
    }
    a1 = block_sum<kWaves>(a1, smem) / (float)cols;
    a2 = block_sum<kWaves>(a2, smem) / (float)cols;
    for (int i = threadIdx.x; i < cols; i += kThreads) {
      const float xh = (to_f32(x[row * cols + i]) - mu) * rs;
      const float g = to_f32(dy[row * cols + i]);
      const float gw = g * (w ? to_f32(w[i]) : 1.f);
      dx[row * cols + i] = from_f32<T>(rs * (gw - a1 - xh * a2));
      if (pw) {
        pw[i] += g * xh;
        pw[cols + i] += g;
      }
    }
  }
}

template <typename T>
__global__ __launch_bounds__(kThreads) void ln_column_reduce_kernel(const float* __restrict__ partial,
                                                                    T* __restrict__ dw, T* __restrict__ db, int nblocks,
                                                                    int cols) {
  __shared__ float sm[kWaves][2][64];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int col = blockIdx.x * 64 + lane;
  float aw = 0.f, ab = 0.f;
  if (col < cols) {
    for (int b = wid; b < nblocks; b += kWaves) {
      aw += partial[(int64_t)b * 2 * cols + col];
      ab += partial[(int64_t)b * 2 * cols + cols + col];
    }
  }
  sm[wid][0][lane] = aw;
  sm[wid][1][lane] = ab;
  __syncthreads();
  if (wid == 0 && col < cols) {
    float tw = 0.f, tb = 0.f;
#pragma unroll
    for (int i = 0; i < kWaves; ++i) {
      tw += sm[i][0][lane];
      tb += sm[i][1][lane];
    }
    if (dw) dw[col] = from_f32<T>(tw);
    if (db) db[col] = from_f32<T>(tb);
  }
}

template <typename T>
int launch_fwd(const void* x, const void* w, const void* b, void* y, void* mean, void* rstd, int64_t rows, int cols,
               float eps, hipStream_t s) {
  constexpr int V = Vec16<T>::N;
  const int chunks = (cols + kThreads * V - 1) / (kThreads * V);
  dim3 grid((unsigned)rows), block(kThreads);
  const T *X = (const T*)x, *W = (const T*)w, *B = (const T*)b;
  T* Y = (T*)y;
  const bool aligned = !((uintptr_t)x % 16) && !((uintptr_t)y % 16) && !(w && (uintptr_t)w % 16) && !(b && (uintptr_t)b % 16);
  if (cols % V != 0 || chunks > 8 || !aligned) {
    hipLaunchKernelGGL((layernorm_fwd_generic<T>), grid, block, 0, s, X, W, B, Y, (float*)mean, (float*)rstd, cols, eps);
  } else {
    switch (chunks) {
#define LTA_CASE(C)                                                                                                    \
  case C:                                                                                                              \
    hipLaunchKernelGGL((layernorm_fwd_kernel<T, C>), grid, block, 0, s, X, W, B, Y, (float*)mean, (float*)rstd, cols, \
                       eps);                                                                                           \
    break;
      LTA_CASE(1) LTA_CASE(2) LTA_CASE(3) LTA_CASE(4) LTA_CASE(5) LTA_CASE(6) LTA_CASE(7) LTA_CASE(8)
#undef LTA_CASE
    }
  }
  return (int)hipGetLastError();
}

template <typename T>
int launch_bwd(const void* dy, const void* x, const void* w, const void* mean, const void* rstd, void* dx, void* dw,
               void* db, void* ws, int64_t rows, int cols, int nblocks, hipStream_t s) {
  const int rpb = (int)((rows + nblocks - 1) / nblocks);
  float* P = (dw || db) ? (float*)ws : nullptr;
  hipLaunchKernelGGL((layernorm_bwd_kernel<T>), dim3((unsigned)nblocks), dim3(kThreads), 0, s, (const T*)dy,
                     (const T*)x, (const T*)w, (const float*)mean, (const float*)rstd, (T*)dx, P, rows, cols, rpb);
  if (P) {
    hipLaunchKernelGGL((ln_column_reduce_kernel<T>), dim3((unsigned)((cols + 63) / 64)), dim3(kThreads), 0, s, P,
                       (T*)dw, (T*)db, nblocks, cols);
  }
  return (int)hipGetLastError();
}

}  // namespace

LTA_EXPORT int lta_layernorm_fwd(int dtype, const void* x, const void* w, const void* b, void* y, void* mean,
                                 void* rstd, int64_t rows, int64_t cols, float eps, hipStream_t stream) {
  switch (dtype) {
    case kBF16: return launch_fwd<__hip_bfloat16>(x, w, b, y, mean, rstd, rows, (int)cols, eps, stream);
    case kF16: return launch_fwd<__half>(x, w, b, y, mean, rstd, rows, (int)cols, eps, stream);
    case kF32: return launch_fwd<float>(x, w, b, y, mean, rstd, rows, (int)cols, eps, stream);
  }
  return -1;
}

LTA_EXPORT int lta_layernorm_bwd(int dtype, const void* dy, const void* x, const void* w, const void* mean,
                                 const void* rstd, void* dx, void* dw, void* db, void* workspace, int64_t rows,
                                 int64_t cols, int nblocks, hipStream_t stream) {
  switch (dtype) {
    case kBF16: return launch_bwd<__hip_bfloat16>(dy, x, w, mean, rstd, dx, dw, db, workspace, rows, (int)cols, nblocks, stream);
    case kF16: return launch_bwd<__half>(dy, x, w, mean, rstd, dx, dw, db, workspace, rows, (int)cols, nblocks, stream);
    case kF32: return launch_bwd<float>(dy, x, w, mean, rstd, dx, dw, db, workspace, rows, (int)cols, nblocks, stream);
  }
  return -1;
}
