// K4: RMSNorm forward/backward for CDNA4 (gfx950).
// y = x * rsqrt(mean(x^2) + eps) * w, fp32 accumulation (reference decomposition:
// thunder/torch/__init__.py:4450-4477; apex fused RMSNorm / nvFuser in the reference).
//
// Memory-bound: one 256-thread workgroup (4 waves) per row in the forward, each lane
// moving 16 B per access (8 bf16) and caching its slice of the row in registers so the
// row is read from HBM once.  The backward processes several rows per workgroup and keeps
// the per-column dW partial sums in registers, writing one fp32 partial row per workgroup;
// a second kernel reduces the partials (no float atomics: deterministic).
#include <algorithm>

#include "common.h"
#include "colreduce.h"
#include "fp8_cvt.h"

using namespace lta;

namespace {

constexpr int kThreads = 256;
constexpr int kWaves = kThreads / 64;

template <typename T, int CHUNKS>
__global__ __launch_bounds__(kThreads) void rmsnorm_fwd_kernel(const T* __restrict__ x, const T* __restrict__ w,
                                                               T* __restrict__ y, float* __restrict__ rstd_out,
                                                               int64_t rows, int cols, float eps) {
  constexpr int V = Vec16<T>::N;
  __shared__ float smem[kWaves];
  const int64_t row = blockIdx.x;
  const T* xr = x + row * cols;
  T* yr = y + row * cols;
  Vec16<T> xv[CHUNKS];
  float ss = 0.f;
#pragma unroll
  for (int c = 0; c < CHUNKS; ++c) {
    const int idx = (c * kThreads + threadIdx.x) * V;
    if (idx < cols) {
      xv[c] = load16(xr + idx);
#pragma unroll
      for (int j = 0; j < V; ++j) {
        const float f = to_f32(xv[c].v[j]);
        ss += f * f;
      }
    }
  }
  const float total = block_sum<kWaves>(ss, smem);
  const float r = rsqrtf(total / (float)cols + eps);
  if (threadIdx.x == 0 && rstd_out != nullptr) rstd_out[row] = r;
#pragma unroll
  for (int c = 0; c < CHUNKS; ++c) {
    const int idx = (c * kThreads + threadIdx.x) * V;
    if (idx < cols) {
      Vec16<T> o;
      if (w != nullptr) {
        const Vec16<T> wv = load16(w + idx);
#pragma unroll
        for (int j = 0; j < V; ++j) o.v[j] = from_f32<T>(to_f32(xv[c].v[j]) * r * to_f32(wv.v[j]));
      } else {
#pragma unroll
        for (int j = 0; j < V; ++j) o.v[j] = from_f32<T>(to_f32(xv[c].v[j]) * r);
      }
      store16(yr + idx, o);
    }
  }
}

// FP8-linear producer (delayed scaling): the normalised row leaves as e4m3 (q = fp8(bf16(y) s),
// s = fmax / amax_in) instead of bf16 -- the input cast of the following fp8 linears fused into the
// norm (one pass less over the activation); max |bf16(y)| of the whole tensor into amax_out.  A
// capped grid strides over the rows (one amax atomic per workgroup).
template <typename T, int CHUNKS>
__global__ __launch_bounds__(kThreads) void rmsnorm_fwd_fp8_kernel(const T* __restrict__ x, const T* __restrict__ w,
                                                                   uint8_t* __restrict__ q, float* __restrict__ rstd_out,
                                                                   int64_t rows, int cols, float eps,
                                                                   const float* __restrict__ amax_in, float fmax,
                                                                   float* __restrict__ scale_out,
                                                                   float* __restrict__ amax_out) {
  constexpr int V = Vec16<T>::N;
  static_assert(V == 8, "16-bit inputs");
  __shared__ float smem[kWaves];
  __shared__ float red[kWaves];
  const float s = fp8_scale(amax_in, fmax, scale_out);
  float m = 0.f;
  for (int64_t row = blockIdx.x; row < rows; row += gridDim.x) {
    const T* xr = x + row * cols;
    Vec16<T> xv[CHUNKS];
    float ss = 0.f;
#pragma unroll
    for (int c = 0; c < CHUNKS; ++c) {
      const int idx = (c * kThreads + threadIdx.x) * V;
      if (idx < cols) {
        xv[c] = load16(xr + idx);
#pragma unroll
        for (int j = 0; j < V; ++j) {
          const float f = to_f32(xv[c].v[j]);
          ss += f * f;
        }
      }
    }
    const float total = block_sum<kWaves>(ss, smem);
    const float r = rsqrtf(total / (float)cols + eps);
    if (threadIdx.x == 0 && rstd_out != nullptr) rstd_out[row] = r;
#pragma unroll
    for (int c = 0; c < CHUNKS; ++c) {
      const int idx = (c * kThreads + threadIdx.x) * V;
      if (idx < cols) {
        float yv[V];
        const Vec16<T> wv = load16(w + idx);
#pragma unroll
        for (int j = 0; j < V; ++j) {
          yv[j] = to_f32(from_f32<T>(to_f32(xv[c].v[j]) * r * to_f32(wv.v[j])));  // the unfused bf16 y
          m = fmaxf(m, fabsf(yv[j]));
        }
        const uint32_t lo = cvt4<false>(yv[0] * s, yv[1] * s, yv[2] * s, yv[3] * s);
        const uint32_t hi = cvt4<false>(yv[4] * s, yv[5] * s, yv[6] * s, yv[7] * s);
        *reinterpret_cast<uint2*>(q + row * cols + idx) = make_uint2(lo, hi);
      }
    }
    __syncthreads();  // smem is reused by the next row's block_sum
  }
  if (amax_out != nullptr) fp8_amax_out<kWaves>(m, amax_out, red);
}

// Generic (any cols) fallback: strided scalar loops, two passes over the row.
template <typename T>
__global__ __launch_bounds__(kThreads) void rmsnorm_fwd_generic(const T* __restrict__ x, const T* __restrict__ w,
                                                                T* __restrict__ y, float* __restrict__ rstd_out,
                                                                int64_t rows, int cols, float eps) {
  __shared__ float smem[kWaves];
  const int64_t row = blockIdx.x;
  const T* xr = x + row * cols;
  float ss = 0.f;
  for (int i = threadIdx.x; i < cols; i += kThreads) {
    const float f = to_f32(xr[i]);
    ss += f * f;
  }
  const float r = rsqrtf(block_sum<kWaves>(ss, smem) / (float)cols + eps);
  if (threadIdx.x == 0 && rstd_out != nullptr) rstd_out[row] = r;
  for (int i = threadIdx.x; i < cols; i += kThreads) {
    const float wv = w ? to_f32(w[i]) : 1.f;
    y[row * cols + i] = from_f32<T>(to_f32(xr[i]) * r * wv);
  }
}

// FP8-linear consumer of the backward (delayed scaling, Q8): dx also leaves as e5m2 (q = fp8(bf16(dx) s),
// s = fmax / amax_in) for the preceding linear's dgrad / wgrad GEMMs -- the gradient cast fused into the
// norm backward; max |bf16(dx)| of the whole tensor into amax_out.
struct Q8Args {
  uint8_t* q;
  const float* amax_in;
  float fmax;
  float* scale_out;
  float* amax_out;
};

template <typename T, int CHUNKS, bool Q8 = false>
__global__ __launch_bounds__(kThreads) void rmsnorm_bwd_kernel(const T* __restrict__ dy, const T* __restrict__ x,
                                                               const T* __restrict__ w, const float* __restrict__ rstd,
                                                               T* __restrict__ dx, float* __restrict__ dw_partial,
                                                               int64_t rows, int cols, int rows_per_block,
                                                               const T* __restrict__ res, Q8Args q8 = {}) {
  constexpr int V = Vec16<T>::N;
  static_assert(!Q8 || V == 8, "fp8 output: 16-bit gradients");
  __shared__ float smem[2 * kWaves];
  [[maybe_unused]] float qs = 0.f, qm = 0.f;
  if constexpr (Q8) qs = fp8_scale(q8.amax_in, q8.fmax, q8.scale_out);
  float dw_acc[CHUNKS][V];
#pragma unroll
  for (int c = 0; c < CHUNKS; ++c)
#pragma unroll
    for (int j = 0; j < V; ++j) dw_acc[c][j] = 0.f;
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
  // two rows per iteration: both rows' loads are in flight together and their dot products share
  // one block reduction (one barrier pair per two rows); the kernel is latency-bound otherwise
  for (int64_t row = r0; row < r1; row += 2) {
    const bool two = row + 1 < r1;
    const float ra = rstd[row], rb = two ? rstd[row + 1] : 0.f;
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
        // the residual-stream gradient is only added at the store, but is loaded here with the row
        // operands so its latency hides under the block reduction instead of following it
        if (res != nullptr) {
          rv[0][c] = load16(res + row * cols + idx);
          if (two) rv[1][c] = load16(res + (row + 1) * cols + idx);
        }
      }
    }
    float dota = 0.f, dotb = 0.f;
#pragma unroll
    for (int c = 0; c < CHUNKS; ++c) {
      const int idx = (c * kThreads + threadIdx.x) * V;
      if (idx < cols) {
#pragma unroll
        for (int j = 0; j < V; ++j) {
          const float wj = to_f32(wv[c].v[j]);
          const float xa = to_f32(xv[0][c].v[j]) * ra, ga = to_f32(gv[0][c].v[j]);
          dota += ga * wj * xa;
          dw_acc[c][j] += ga * xa;
          if (two) {
            const float xb = to_f32(xv[1][c].v[j]) * rb, gb = to_f32(gv[1][c].v[j]);
            dotb += gb * wj * xb;
            dw_acc[c][j] += gb * xb;
          }
        }
      }
    }
    dota = wave_sum(dota);
    dotb = wave_sum(dotb);
    {
      const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
      __syncthreads();  // the previous iteration's reads of smem are done
      if (lane == 0) {
        smem[wid] = dota;
        smem[kWaves + wid] = dotb;
      }
      __syncthreads();
      dota = 0.f;
      dotb = 0.f;
#pragma unroll
      for (int i = 0; i < kWaves; ++i) {
        dota += smem[i];
        dotb += smem[kWaves + i];
      }
      dota /= (float)cols;
      dotb /= (float)cols;
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      if (h == 1 && !two) break;
      const int64_t rr = row + h;
      const float r = h ? rb : ra, dot = h ? dotb : dota;
#pragma unroll
      for (int c = 0; c < CHUNKS; ++c) {
        const int idx = (c * kThreads + threadIdx.x) * V;
        if (idx < cols) {
          Vec16<T> o;
#pragma unroll
          for (int j = 0; j < V; ++j) {
            const float xh = to_f32(xv[h][c].v[j]) * r;
            const float gw = to_f32(gv[h][c].v[j]) * to_f32(wv[c].v[j]);
            const float add = res != nullptr ? to_f32(rv[h][c].v[j]) : 0.f;  // gradient through the residual
            // explicit fmas: the same rounding in every instantiation (the Q8 variant's e5m2 copy is
            // of exactly the dx the plain kernel stores)
            o.v[j] = from_f32<T>(__builtin_fmaf(r, __builtin_fmaf(-xh, dot, gw), add));
          }
          store16(dx + rr * cols + idx, o);
          if constexpr (Q8) {
            float ov[V];
#pragma unroll
            for (int j = 0; j < V; ++j) {
              ov[j] = to_f32(o.v[j]);  // the unfused bf16 dx
              qm = fmaxf(qm, fabsf(ov[j]));
            }
            const uint32_t lo = cvt4<true>(ov[0] * qs, ov[1] * qs, ov[2] * qs, ov[3] * qs);
            const uint32_t hi = cvt4<true>(ov[4] * qs, ov[5] * qs, ov[6] * qs, ov[7] * qs);
            *reinterpret_cast<uint2*>(q8.q + rr * cols + idx) = make_uint2(lo, hi);
          }
        }
      }
    }
  }
  if (dw_partial != nullptr) {
#pragma unroll
    for (int c = 0; c < CHUNKS; ++c) {
      const int idx = (c * kThreads + threadIdx.x) * V;
      if (idx < cols) {
        float* p = dw_partial + (int64_t)blockIdx.x * cols + idx;
#pragma unroll
        for (int j = 0; j < V; j += 4) *reinterpret_cast<float4*>(p + j) = make_float4(dw_acc[c][j], dw_acc[c][j + 1], dw_acc[c][j + 2], dw_acc[c][j + 3]);
      }
    }
  }
  if constexpr (Q8) {
    __shared__ float red[kWaves];  // not smem: a slower wave may still be reading the last row's dot products
    if (q8.amax_out != nullptr) fp8_amax_out<kWaves>(qm, q8.amax_out, red);
  }
}

template <typename T>
__global__ __launch_bounds__(kThreads) void rmsnorm_bwd_generic(const T* __restrict__ dy, const T* __restrict__ x,
                                                                const T* __restrict__ w, const float* __restrict__ rstd,
                                                                T* __restrict__ dx, float* __restrict__ dw_partial,
                                                                int64_t rows, int cols, int rows_per_block,
                                                                const T* __restrict__ res) {
  __shared__ float smem[kWaves];
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
  const int64_t r1 = min(rows, r0 + rows_per_block);
  for (int i = threadIdx.x; i < cols; i += kThreads) {
    if (dw_partial) dw_partial[(int64_t)blockIdx.x * cols + i] = 0.f;
  }
  for (int64_t row = r0; row < r1; ++row) {
    const float r = rstd[row];
    float dot = 0.f;
    for (int i = threadIdx.x; i < cols; i += kThreads) {
      const float wv = w ? to_f32(w[i]) : 1.f;
      dot += to_f32(dy[row * cols + i]) * wv * to_f32(x[row * cols + i]) * r;
    }
    dot = block_sum<kWaves>(dot, smem) / (float)cols;
    for (int i = threadIdx.x; i < cols; i += kThreads) {
      const float wv = w ? to_f32(w[i]) : 1.f;
      const float xh = to_f32(x[row * cols + i]) * r;
      const float g = to_f32(dy[row * cols + i]);
      const float add = res != nullptr ? to_f32(res[row * cols + i]) : 0.f;
      dx[row * cols + i] = from_f32<T>(r * (g * wv - xh * dot) + add);
      if (dw_partial) dw_partial[(int64_t)blockIdx.x * cols + i] += g * xh;
    }
  }
}

// Column reduction of the fp32 partials: dw[c] = sum_b partial[b, c]
template <typename T>
__global__ __launch_bounds__(kThreads) void column_reduce_kernel(const float* __restrict__ partial, T* __restrict__ out,
                                                                 int nblocks, int cols) {
  // each 256-thread block handles 64 columns with 4 waves splitting the rows
  __shared__ float sm[kWaves][64];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int col = blockIdx.x * 64 + lane;
  float acc = 0.f;
  if (col < cols) {
    for (int b = wid; b < nblocks; b += kWaves) acc += partial[(int64_t)b * cols + col];
  }
  sm[wid][lane] = acc;
  __syncthreads();
  if (wid == 0 && col < cols) {
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < kWaves; ++i) t += sm[i][lane];
    out[col] = from_f32<T>(t);
  }
}

template <typename T>
int launch_fwd(const void* x, const void* w, void* y, void* rstd, int64_t rows, int cols, float eps, hipStream_t s) {
  constexpr int V = Vec16<T>::N;
  const int per_pass = kThreads * V;
  const int chunks = (cols + per_pass - 1) / per_pass;
  const T* X = (const T*)x;
  const T* W = (const T*)w;
  T* Y = (T*)y;
  float* R = (float*)rstd;
  dim3 grid((unsigned)rows), block(kThreads);
  if (cols % V != 0 || chunks > 8 || ((uintptr_t)x % 16) || ((uintptr_t)y % 16) || (w && ((uintptr_t)w % 16))) {
    hipLaunchKernelGGL((rmsnorm_fwd_generic<T>), grid, block, 0, s, X, W, Y, R, rows, cols, eps);
  } else {
    switch (chunks) {
#define LTA_CASE(C) \
  case C: hipLaunchKernelGGL((rmsnorm_fwd_kernel<T, C>), grid, block, 0, s, X, W, Y, R, rows, cols, eps); break;
      LTA_CASE(1) LTA_CASE(2) LTA_CASE(3) LTA_CASE(4) LTA_CASE(5) LTA_CASE(6) LTA_CASE(7) LTA_CASE(8)
#undef LTA_CASE
    }
  }
  return (int)hipGetLastError();
}

template <typename T>
int launch_bwd(const void* dy, const void* x, const void* w, const void* rstd, void* dx, void* dw, void* workspace,
               int64_t rows, int cols, int nblocks, const void* res, hipStream_t s, const Q8Args* q8 = nullptr) {
  constexpr int V = Vec16<T>::N;
  const int per_pass = kThreads * V;
  const int chunks = (cols + per_pass - 1) / per_pass;
  const int rpb = (int)((rows + nblocks - 1) / nblocks);
  float* P = (float*)workspace;
  dim3 grid((unsigned)nblocks), block(kThreads);
  const T* DY = (const T*)dy;
  const T* X = (const T*)x;
  const T* W = (const T*)w;
  const float* R = (const float*)rstd;
  T* DX = (T*)dx;
  float* Pp = dw ? P : nullptr;
  const T* RES = (const T*)res;
  const bool vec_ok = !(cols % V != 0 || chunks > 4 || ((uintptr_t)x % 16) || ((uintptr_t)dy % 16) ||
                        ((uintptr_t)dx % 16) || (w && ((uintptr_t)w % 16)) || ((uintptr_t)res % 16));
  if (q8 != nullptr) {  // fp8 output: the vectorised kernel only (-1: the caller casts separately)
    if constexpr (Vec16<T>::N != 8) {
      return -1;
    } else {
      if (!vec_ok || ((uintptr_t)q8->q % 8)) return -1;
      switch (chunks) {
#define LTA_CASE(C)                                                                                          \
  case C:                                                                                                    \
    hipLaunchKernelGGL((rmsnorm_bwd_kernel<T, C, true>), grid, block, 0, s, DY, X, W, R, DX, Pp, rows, cols, \
                       rpb, RES, *q8);                                                                       \
    break;
        LTA_CASE(1) LTA_CASE(2) LTA_CASE(3) LTA_CASE(4)
#undef LTA_CASE
      }
    }
  } else if (!vec_ok) {
    hipLaunchKernelGGL((rmsnorm_bwd_generic<T>), grid, block, 0, s, DY, X, W, R, DX, Pp, rows, cols, rpb, RES);
  } else {
    switch (chunks) {
#define LTA_CASE(C) \
  case C: hipLaunchKernelGGL((rmsnorm_bwd_kernel<T, C>), grid, block, 0, s, DY, X, W, R, DX, Pp, rows, cols, rpb, RES); break;
      LTA_CASE(1) LTA_CASE(2) LTA_CASE(3) LTA_CASE(4)
#undef LTA_CASE
    }
  }
  if (dw) {
    if (cols % 4 == 0) {
      hipLaunchKernelGGL((column_reduce_v4_kernel<T>), dim3((unsigned)((cols + 31) / 32)), block, 0, s, P, (T*)dw,
                         nblocks, cols);
    } else {
      dim3 g2((unsigned)((cols + 63) / 64));
      hipLaunchKernelGGL((column_reduce_kernel<T>), g2, block, 0, s, P, (T*)dw, nblocks, cols);
    }
  }
  return (int)hipGetLastError();
}

}  // namespace

LTA_EXPORT int lta_rmsnorm_fwd(int dtype, const void* x, const void* w, void* y, void* rstd, int64_t rows, int64_t cols,
                               float eps, hipStream_t stream) {
  switch (dtype) {
    case kBF16: return launch_fwd<__hip_bfloat16>(x, w, y, rstd, rows, (int)cols, eps, stream);
    case kF16: return launch_fwd<__half>(x, w, y, rstd, rows, (int)cols, eps, stream);
    case kF32: return launch_fwd<float>(x, w, y, rstd, rows, (int)cols, eps, stream);
  }
  return -1;
}

// RMSNorm forward with an e4m3 output (rmsnorm_fwd_fp8_kernel): q [rows, cols] uint8, rstd fp32; the
// delayed-scaling scale fmax / *amax_in goes to scale_out, max |y| into amax_out.  16-bit x / w,
// cols % 8 == 0, cols <= 16384, 16-B aligned.  -1 when unsupported.
LTA_EXPORT int lta_rmsnorm_fwd_fp8(int dtype, const void* x, const void* w, void* q, void* rstd, int64_t rows,
                                   int64_t cols, float eps, const void* amax_in, float fmax, void* scale_out,
                                   void* amax_out, hipStream_t stream) {
  const int per_pass = kThreads * 8, chunks = (int)((cols + per_pass - 1) / per_pass);
  if (!w || cols % 8 || chunks > 8 || ((uintptr_t)x % 16) || ((uintptr_t)w % 16) || ((uintptr_t)q % 8)) return -1;
  dim3 grid((unsigned)std::min<int64_t>(rows, 1024)), block(kThreads);
#define LTA_Q8(T, C)                                                                                              \
  hipLaunchKernelGGL((rmsnorm_fwd_fp8_kernel<T, C>), grid, block, 0, stream, (const T*)x, (const T*)w, (uint8_t*)q, \
                     (float*)rstd, rows, (int)cols, eps, (const float*)amax_in, fmax, (float*)scale_out,          \
                     (float*)amax_out)
#define LTA_Q8_T(T)                                                                                               \
  switch (chunks) {                                                                                               \
    case 1: LTA_Q8(T, 1); break;                                                                                  \
    case 2: LTA_Q8(T, 2); break;                                                                                  \
    case 3: LTA_Q8(T, 3); break;                                                                                  \
    case 4: LTA_Q8(T, 4); break;                                                                                  \
    default: LTA_Q8(T, 8); break;                                                                                 \
  }
  if (dtype == kBF16) { LTA_Q8_T(__hip_bfloat16) }
  else if (dtype == kF16) { LTA_Q8_T(__half) }
  else return -1;
#undef LTA_Q8_T
#undef LTA_Q8
  return (int)hipGetLastError();
}

// res (optional, same shape as dx): added to dx in the same pass (the residual stream's gradient)
LTA_EXPORT int lta_rmsnorm_bwd_res(int dtype, const void* dy, const void* x, const void* w, const void* rstd, void* dx,
                                   void* dw, void* workspace, int64_t rows, int64_t cols, int nblocks, const void* res,
                                   hipStream_t stream) {
  switch (dtype) {
    case kBF16: return launch_bwd<__hip_bfloat16>(dy, x, w, rstd, dx, dw, workspace, rows, (int)cols, nblocks, res, stream);
    case kF16: return launch_bwd<__half>(dy, x, w, rstd, dx, dw, workspace, rows, (int)cols, nblocks, res, stream);
    case kF32: return launch_bwd<float>(dy, x, w, rstd, dx, dw, workspace, rows, (int)cols, nblocks, res, stream);
  }
  return -1;
}

// lta_rmsnorm_bwd_res plus an e5m2 copy of dx (Q8Args semantics above): q [rows, cols] uint8, the delayed
// scale fmax / *amax_in to scale_out, max |dx| into amax_out.  16-bit dtypes, the vectorised shapes
// (cols % 8 == 0, cols <= 8192, 16-B aligned rows); -1 when unsupported (nothing launched).
LTA_EXPORT int lta_rmsnorm_bwd_fp8(int dtype, const void* dy, const void* x, const void* w, const void* rstd, void* dx,
                                   void* dw, void* workspace, int64_t rows, int64_t cols, int nblocks, const void* res,
                                   void* q, const void* amax_in, float fmax, void* scale_out, void* amax_out,
                                   hipStream_t stream) {
  const Q8Args q8{(uint8_t*)q, (const float*)amax_in, fmax, (float*)scale_out, (float*)amax_out};
  switch (dtype) {
    case kBF16: return launch_bwd<__hip_bfloat16>(dy, x, w, rstd, dx, dw, workspace, rows, (int)cols, nblocks, res, stream, &q8);
    case kF16: return launch_bwd<__half>(dy, x, w, rstd, dx, dw, workspace, rows, (int)cols, nblocks, res, stream, &q8);
  }
  return -1;
}

LTA_EXPORT int lta_rmsnorm_bwd(int dtype, const void* dy, const void* x, const void* w, const void* rstd, void* dx,
                               void* dw, void* workspace, int64_t rows, int64_t cols, int nblocks, hipStream_t stream) {
  return lta_rmsnorm_bwd_res(dtype, dy, x, w, rstd, dx, dw, workspace, rows, cols, nblocks, nullptr, stream);
}
