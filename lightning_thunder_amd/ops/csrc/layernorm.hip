// K5: LayerNorm forward/backward for CDNA4 (gfx950) — GPT-2 / GPT-NeoX / Pythia style models.
// (reference: cuDNN layer norm executor thunder/executors/cudnn_layernormex.py:30-382, and the
// decomposition thunder/torch/__init__.py layer_norm)
//
// Forward: one 256-thread workgroup per row, the row cached in registers (16-B vector loads),
// mean and variance by two register passes (no E[x^2]-E[x]^2 cancellation), per-row fp32
// mean / rstd saved for the backward.
// Backward: several rows per workgroup; dW and dB partial sums stay in registers and are
// written as one fp32 partial row per workgroup, then reduced column-wise by a second kernel
// (deterministic, no float atomics).  v2 (16-B rows cached in registers, two rows per block
// reduction, as csrc/rmsnorm.hip's backward) also adds the residual stream's gradient in its
// store pass (the transformer block's dx + dresidual).
#include "common.h"
#include "colreduce.h"

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
                                                                 int rows_per_block, const T* __restrict__ res) {
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
      dx[row * cols + i] = from_f32<T>(rs * (gw - a1 - xh * a2) + (res ? to_f32(res[row * cols + i]) : 0.f));
      if (pw) {
        pw[i] += g * xh;
        pw[cols + i] += g;
      }
    }
  }
}

// v2: requires cols % 8 == 0 (16-B vectors), cols <= 4 * 256 * 8 and 16-B aligned rows.  Partials:
// dW rows [nblocks][cols] then dB rows [nblocks][cols].
template <typename T, int CHUNKS>
__global__ __launch_bounds__(kThreads) void layernorm_bwd_v2_kernel(const T* __restrict__ dy, const T* __restrict__ x,
                                                                    const T* __restrict__ w, const float* __restrict__ mean,
                                                                    const float* __restrict__ rstd, T* __restrict__ dx,
                                                                    float* __restrict__ partial, int64_t rows, int cols,
                                                                    int rows_per_block, const T* __restrict__ res) {
  constexpr int V = Vec16<T>::N;
  __shared__ float smem[4 * kWaves];
  float dw_acc[CHUNKS][V], db_acc[CHUNKS][V];
#pragma unroll
  for (int c = 0; c < CHUNKS; ++c)
#pragma unroll
    for (int j = 0; j < V; ++j) dw_acc[c][j] = db_acc[c][j] = 0.f;
  Vec16<T> wv[CHUNKS];
#pragma unroll
  for (int c = 0; c < CHUNKS; ++c) {
    const int idx = (c * kThreads + threadIdx.x) * V;
    if (idx < cols) {
      if (w != nullptr) {
        wv[c] = load16(w + idx);
      } else {
#pragma unroll
        for (int j = 0; j < V; ++j) wv[c].v[j] = from_f32<T>(1.f);
      }
    }
  }
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
  const int64_t r1 = min(rows, r0 + rows_per_block);
  for (int64_t row = r0; row < r1; row += 2) {
    const bool two = row + 1 < r1;
    const float mua = mean[row], rsa = rstd[row];
    const float mub = two ? mean[row + 1] : 0.f, rsb = two ? rstd[row + 1] : 0.f;
    Vec16<T> xv[2][CHUNKS], gv[2][CHUNKS], rv[2][CHUNKS];
#pragma unroll
    for (int c = 0; c < CHUNKS; ++c) {
      const int idx = (c * kThreads + threadIdx.x) * V;
      if (idx < cols) {
        xv[0][c] = load16(x + row * cols + idx);
        gv[0][c] = load16(dy + row * cols + idx);
        if (two) {
          xv[1][c] = load16(x + (row + 1) * cols + idx);
          gv[1][c] = load16(dy + (row + 1) * cols + idx);
        }
        if (res != nullptr) {  // loaded with the row operands: its latency hides under the reduction
          rv[0][c] = load16(res + row * cols + idx);
          if (two) rv[1][c] = load16(res + (row + 1) * cols + idx);
        }
      }
    }
    float s[4] = {0.f, 0.f, 0.f, 0.f};  // row a: sum(g w), sum(g w xhat); row b: the same
#pragma unroll
    for (int c = 0; c < CHUNKS; ++c) {
      const int idx = (c * kThreads + threadIdx.x) * V;
      if (idx < cols) {
#pragma unroll
        for (int j = 0; j < V; ++j) {
          const float wj = to_f32(wv[c].v[j]);
          const float xa = (to_f32(xv[0][c].v[j]) - mua) * rsa, ga = to_f32(gv[0][c].v[j]);
          s[0] += ga * wj;
          s[1] += ga * wj * xa;
          dw_acc[c][j] += ga * xa;
          db_acc[c][j] += ga;
          if (two) {
            const float xb = (to_f32(xv[1][c].v[j]) - mub) * rsb, gb = to_f32(gv[1][c].v[j]);
            s[2] += gb * wj;
            s[3] += gb * wj * xb;
            dw_acc[c][j] += gb * xb;
            db_acc[c][j] += gb;
          }
        }
      }
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) s[k] = wave_sum(s[k]);
    {
      const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
      __syncthreads();  // the previous iteration's reads of smem are done
      if (lane == 0) {
#pragma unroll
        for (int k = 0; k < 4; ++k) smem[k * kWaves + wid] = s[k];
      }
      __syncthreads();
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        float t = 0.f;
#pragma unroll
        for (int i = 0; i < kWaves; ++i) t += smem[k * kWaves + i];
        s[k] = t / (float)cols;
      }
    }
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
      if (hh == 1 && !two) break;
      const int64_t rr = row + hh;
      const float mu = hh ? mub : mua, rs = hh ? rsb : rsa, a1 = s[2 * hh], a2 = s[2 * hh + 1];
#pragma unroll
      for (int c = 0; c < CHUNKS; ++c) {
        const int idx = (c * kThreads + threadIdx.x) * V;
        if (idx < cols) {
          Vec16<T> o;
#pragma unroll
          for (int j = 0; j < V; ++j) {
            const float xh = (to_f32(xv[hh][c].v[j]) - mu) * rs;
            const float gw = to_f32(gv[hh][c].v[j]) * to_f32(wv[c].v[j]);
            const float add = res != nullptr ? to_f32(rv[hh][c].v[j]) : 0.f;
            o.v[j] = from_f32<T>(rs * (gw - a1 - xh * a2) + add);
          }
          store16(dx + rr * cols + idx, o);
        }
      }
    }
  }
  if (partial != nullptr) {
#pragma unroll
    for (int c = 0; c < CHUNKS; ++c) {
      const int idx = (c * kThreads + threadIdx.x) * V;
      if (idx < cols) {
        float* pw = partial + (int64_t)blockIdx.x * cols + idx;
        float* pb = partial + ((int64_t)gridDim.x + blockIdx.x) * cols + idx;
#pragma unroll
        for (int j = 0; j < V; j += 4) {
          *reinterpret_cast<float4*>(pw + j) = make_float4(dw_acc[c][j], dw_acc[c][j + 1], dw_acc[c][j + 2], dw_acc[c][j + 3]);
          *reinterpret_cast<float4*>(pb + j) = make_float4(db_acc[c][j], db_acc[c][j + 1], db_acc[c][j + 2], db_acc[c][j + 3]);
        }
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
               void* db, void* ws, int64_t rows, int cols, int nblocks, const void* res, hipStream_t s) {
  const int rpb = (int)((rows + nblocks - 1) / nblocks);
  float* P = (dw || db) ? (float*)ws : nullptr;
  constexpr int V = Vec16<T>::N;
  const int chunks = (cols + kThreads * V - 1) / (kThreads * V);
  const bool aligned = !((uintptr_t)x % 16) && !((uintptr_t)dy % 16) && !((uintptr_t)dx % 16) &&
                       !(w && (uintptr_t)w % 16) && !(res && (uintptr_t)res % 16);
  if (cols % V == 0 && cols % 4 == 0 && chunks <= 4 && aligned) {
    switch (chunks) {
#define LTA_CASE(C)                                                                                                  \
  case C:                                                                                                            \
    hipLaunchKernelGGL((layernorm_bwd_v2_kernel<T, C>), dim3((unsigned)nblocks), dim3(kThreads), 0, s, (const T*)dy, \
                       (const T*)x, (const T*)w, (const float*)mean, (const float*)rstd, (T*)dx, P, rows, cols, rpb,  \
                       (const T*)res);                                                                               \
    break;
      LTA_CASE(1) LTA_CASE(2) LTA_CASE(3) LTA_CASE(4)
#undef LTA_CASE
    }
    const dim3 g((unsigned)((cols + 31) / 32));
    if (dw) hipLaunchKernelGGL((column_reduce_v4_kernel<T>), g, dim3(kThreads), 0, s, P, (T*)dw, nblocks, cols);
    if (db)
      hipLaunchKernelGGL((column_reduce_v4_kernel<T>), g, dim3(kThreads), 0, s, P + (int64_t)nblocks * cols, (T*)db,
                         nblocks, cols);
    return (int)hipGetLastError();
  }
  hipLaunchKernelGGL((layernorm_bwd_kernel<T>), dim3((unsigned)nblocks), dim3(kThreads), 0, s, (const T*)dy,
                     (const T*)x, (const T*)w, (const float*)mean, (const float*)rstd, (T*)dx, P, rows, cols, rpb,
                     (const T*)res);
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

// res (optional, same shape as dx): added to dx in the same pass (the residual stream's gradient).
// workspace: fp32 [nblocks][2][cols].
LTA_EXPORT int lta_layernorm_bwd_res(int dtype, const void* dy, const void* x, const void* w, const void* mean,
                                     const void* rstd, void* dx, void* dw, void* db, void* workspace, int64_t rows,
                                     int64_t cols, int nblocks, const void* res, hipStream_t stream) {
  switch (dtype) {
    case kBF16: return launch_bwd<__hip_bfloat16>(dy, x, w, mean, rstd, dx, dw, db, workspace, rows, (int)cols, nblocks, res, stream);
    case kF16: return launch_bwd<__half>(dy, x, w, mean, rstd, dx, dw, db, workspace, rows, (int)cols, nblocks, res, stream);
    case kF32: return launch_bwd<float>(dy, x, w, mean, rstd, dx, dw, db, workspace, rows, (int)cols, nblocks, res, stream);
  }
  return -1;
}

LTA_EXPORT int lta_layernorm_bwd(int dtype, const void* dy, const void* x, const void* w, const void* mean,
                                 const void* rstd, void* dx, void* dw, void* db, void* workspace, int64_t rows,
                                 int64_t cols, int nblocks, hipStream_t stream) {
  return lta_layernorm_bwd_res(dtype, dy, x, w, mean, rstd, dx, dw, db, workspace, rows, cols, nblocks, nullptr,
                               stream);
}
