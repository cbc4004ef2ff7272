// SwiGLU (silu(a) * b) forward/backward and K7 softmax cross-entropy forward/backward for CDNA4.
//
// SwiGLU is the LLaMA MLP gate ([tokens, 11008] x 2 for Llama-2-7B); forward reads a, b and
// writes y; backward reads g, a, b and writes da, db — one pass each, 16-B vectors.
//
// Cross entropy replaces the reference's in-repo Triton kernels
// (thunder/executors/triton_crossentropy_impl.py:49-540): forward is one online
// max/sum-exp pass per row (logits read once), saving the row's log-sum-exp; backward
// writes (softmax - onehot) * dloss / n_valid in one pass.  Rows are [tokens, vocab]
// with vocab = 32000 for Llama-2 (64 KB of bf16 per row).
#include <algorithm>

#include "common.h"
#include "fp8_cvt.h"

using namespace lta;

namespace {

__device__ __forceinline__ float sigmoidf_(float x) { return 1.f / (1.f + __expf(-x)); }

template <typename T>
__global__ __launch_bounds__(256) void swiglu_fwd_kernel(const T* __restrict__ a, const T* __restrict__ b,
                                                         T* __restrict__ y, int64_t n) {
  constexpr int V = Vec16<T>::N;
  const int64_t nv = n / V;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nv; i += (int64_t)gridDim.x * blockDim.x) {
    const Vec16<T> av = load16(a + i * V), bv = load16(b + i * V);
    Vec16<T> o;
#pragma unroll
    for (int j = 0; j < V; ++j) {
      const float x = to_f32(av.v[j]);
      o.v[j] = from_f32<T>(x * sigmoidf_(x) * to_f32(bv.v[j]));
    }
    store16(y + i * V, o);
  }
  // tail
  for (int64_t i = nv * V + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const float x = to_f32(a[i]);
    y[i] = from_f32<T>(x * sigmoidf_(x) * to_f32(b[i]));
  }
}

// FP8-linear producer (delayed scaling): y = silu(a) b leaves as e4m3 (q = fp8(bf16(y) s), s = fmax /
// amax_in) -- the down projection's input cast fused into the SwiGLU pass; max |bf16(y)| into
// amax_out, one atomic per workgroup of a capped grid.
template <typename T>
__global__ __launch_bounds__(256) void swiglu_fwd_fp8_kernel(const T* __restrict__ a, const T* __restrict__ b,
                                                             uint8_t* __restrict__ q, int64_t n,
                                                             const float* __restrict__ amax_in, float fmax,
                                                             float* __restrict__ scale_out,
                                                             float* __restrict__ amax_out) {
  static_assert(Vec16<T>::N == 8, "16-bit inputs");
  __shared__ float red[4];
  const float s = fp8_scale(amax_in, fmax, scale_out);
  float m = 0.f;
  const int64_t nv = n / 8;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nv; i += (int64_t)gridDim.x * blockDim.x) {
    const Vec16<T> av = load16(a + i * 8), bv = load16(b + i * 8);
    float y[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float x = to_f32(av.v[j]);
      y[j] = to_f32(from_f32<T>(x * sigmoidf_(x) * to_f32(bv.v[j])));  // the unfused bf16 y
      m = fmaxf(m, fabsf(y[j]));
    }
    const uint32_t lo = cvt4<false>(y[0] * s, y[1] * s, y[2] * s, y[3] * s);
    const uint32_t hi = cvt4<false>(y[4] * s, y[5] * s, y[6] * s, y[7] * s);
    *reinterpret_cast<uint2*>(q + i * 8) = make_uint2(lo, hi);
  }
  if (amax_out != nullptr) fp8_amax_out<4>(m, amax_out, red);
}

// FP8-linear producer, backward (delayed scaling): da / db leave as e5m2 (the fc_1 / fc_2 output
// gradients the fp8 dgrad / wgrad GEMMs read), each with its own scale (fmax / amax_in_x) and amax;
// the values are the unfused kernel's bf16 da / db.
template <typename T>
__global__ __launch_bounds__(256) void swiglu_bwd_fp8_kernel(const T* __restrict__ g, const T* __restrict__ a,
                                                             const T* __restrict__ b, uint8_t* __restrict__ qa,
                                                             uint8_t* __restrict__ qb, int64_t n,
                                                             const float* __restrict__ amax_in_a,
                                                             const float* __restrict__ amax_in_b, float fmax,
                                                             float* __restrict__ scale_a, float* __restrict__ scale_b,
                                                             float* __restrict__ amax_a, float* __restrict__ amax_b) {
  static_assert(Vec16<T>::N == 8, "16-bit inputs");
  __shared__ float red[4];
  const float sa = fp8_scale(amax_in_a, fmax, scale_a), sb = fp8_scale(amax_in_b, fmax, scale_b);
  float ma = 0.f, mb = 0.f;
  const int64_t nv = n / 8;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nv; i += (int64_t)gridDim.x * blockDim.x) {
    const Vec16<T> gv = load16(g + i * 8), av = load16(a + i * 8), bv = load16(b + i * 8);
    float ya[8], yb[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float x = to_f32(av.v[j]), gg = to_f32(gv.v[j]), bb = to_f32(bv.v[j]);
      const float s = sigmoidf_(x);
      const float silu = x * s;
      ya[j] = to_f32(from_f32<T>(gg * bb * (s * (1.f + x * (1.f - s)))));
      yb[j] = to_f32(from_f32<T>(gg * silu));
      ma = fmaxf(ma, fabsf(ya[j]));
      mb = fmaxf(mb, fabsf(yb[j]));
    }
    *reinterpret_cast<uint2*>(qa + i * 8) = make_uint2(cvt4<true>(ya[0] * sa, ya[1] * sa, ya[2] * sa, ya[3] * sa),
                                                       cvt4<true>(ya[4] * sa, ya[5] * sa, ya[6] * sa, ya[7] * sa));
    *reinterpret_cast<uint2*>(qb + i * 8) = make_uint2(cvt4<true>(yb[0] * sb, yb[1] * sb, yb[2] * sb, yb[3] * sb),
                                                       cvt4<true>(yb[4] * sb, yb[5] * sb, yb[6] * sb, yb[7] * sb));
  }
  if (amax_a != nullptr) fp8_amax_out<4>(ma, amax_a, red);
  __syncthreads();
  if (amax_b != nullptr) fp8_amax_out<4>(mb, amax_b, red);
}

template <typename T>
__global__ __launch_bounds__(256) void swiglu_bwd_kernel(const T* __restrict__ g, const T* __restrict__ a,
                                                         const T* __restrict__ b, T* __restrict__ da,
                                                         T* __restrict__ db, int64_t n) {
  constexpr int V = Vec16<T>::N;
  const int64_t nv = n / V;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nv; i += (int64_t)gridDim.x * blockDim.x) {
    const Vec16<T> gv = load16(g + i * V), av = load16(a + i * V), bv = load16(b + i * V);
    Vec16<T> oa, ob;
#pragma unroll
    for (int j = 0; j < V; ++j) {
      const float x = to_f32(av.v[j]), gg = to_f32(gv.v[j]), bb = to_f32(bv.v[j]);
      const float s = sigmoidf_(x);
      const float silu = x * s;
      oa.v[j] = from_f32<T>(gg * bb * (s * (1.f + x * (1.f - s))));
      ob.v[j] = from_f32<T>(gg * silu);
    }
    store16(da + i * V, oa);
    store16(db + i * V, ob);
  }
  for (int64_t i = nv * V + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const float x = to_f32(a[i]), gg = to_f32(g[i]), bb = to_f32(b[i]);
    const float s = sigmoidf_(x);
    da[i] = from_f32<T>(gg * bb * (s * (1.f + x * (1.f - s))));
    db[i] = from_f32<T>(gg * x * s);
  }
}

int ew_grid(int64_t n_items) {
  int64_t g = (n_items + 255) / 256;
  if (g > 256 * 16) g = 256 * 16;
  return (int)(g < 1 ? 1 : g);
}

// ---------------------------------------------------------------------------------------------
// Cross entropy.  One 256-thread workgroup per row.
// ---------------------------------------------------------------------------------------------
constexpr int kCeThreads = 256;
constexpr int kCeWaves = kCeThreads / 64;

// Class weights w (optional, fp32 [V]) follow torch: row loss (1-eps) w_t (lse - x_t)
// + eps/V * sum_c w_c (lse - x_c), and 'mean' divides by sum of w_t over the kept rows.
template <typename T>
__global__ __launch_bounds__(kCeThreads) void ce_fwd_kernel(const T* __restrict__ logits, const int64_t* __restrict__ target,
                                                            const float* __restrict__ weight,
                                                            float* __restrict__ loss, float* __restrict__ lse_out,
                                                            int64_t rows, int V, int64_t ignore_index,
                                                            float label_smoothing) {
  constexpr int VEC = Vec16<T>::N;
  __shared__ float sm[kCeWaves];
  const int64_t row = blockIdx.x;
  const T* x = logits + row * (int64_t)V;
  float m = -INFINITY, s = 0.f, sum_x = 0.f, sum_w = 0.f;
  const bool vec = (V % VEC == 0) && (((uintptr_t)logits) % 16 == 0);
  const bool wsm = weight != nullptr && label_smoothing != 0.f;
  if (vec) {
    for (int i = threadIdx.x * VEC; i < V; i += kCeThreads * VEC) {
      const Vec16<T> xv = load16(x + i);
      float lm = -INFINITY;
#pragma unroll
      for (int j = 0; j < VEC; ++j) lm = fmaxf(lm, to_f32(xv.v[j]));
      const float nm = fmaxf(m, lm);
      float acc = s * __expf(m - nm);
#pragma unroll
      for (int j = 0; j < VEC; ++j) {
        const float f = to_f32(xv.v[j]);
        acc += __expf(f - nm);
        if (wsm) {
          sum_x += weight[i + j] * f;
          sum_w += weight[i + j];
        } else {
          sum_x += f;
        }
      }
      s = acc;
      m = nm;
    }
  } else {
    for (int i = threadIdx.x; i < V; i += kCeThreads) {
      const float f = to_f32(x[i]);
      const float nm = fmaxf(m, f);
      s = s * __expf(m - nm) + __expf(f - nm);
      m = nm;
      if (wsm) {
        sum_x += weight[i] * f;
        sum_w += weight[i];
      } else {
        sum_x += f;
      }
    }
  }
  // combine (m, s) across the block
  const float gm = block_max<kCeWaves>(m, sm);
  const float scaled = (m == -INFINITY) ? 0.f : s * __expf(m - gm);
  __syncthreads();
  const float gs = block_sum<kCeWaves>(scaled, sm);
  __syncthreads();
  const float gsum_x = (label_smoothing != 0.f) ? block_sum<kCeWaves>(sum_x, sm) : 0.f;
  __syncthreads();
  const float gsum_w = wsm ? block_sum<kCeWaves>(sum_w, sm) : (float)V;
  if (threadIdx.x == 0) {
    const float lse = gm + __logf(gs);
    lse_out[row] = lse;
    const int64_t t = target[row];
    if (t == ignore_index) {
      loss[row] = 0.f;
    } else {
      const float xt = to_f32(x[t]);
      const float wt = weight ? weight[t] : 1.f;
      float l = wt * (lse - xt);
      if (label_smoothing != 0.f)
        l = (1.f - label_smoothing) * l + label_smoothing * (lse * gsum_w - gsum_x) / (float)V;
      loss[row] = l;
    }
  }
}

// reduction: out[0] = sum(loss)/max(count,1) (mean) or sum; out[1] = count of valid rows
// (weighted: the count is the sum of the kept rows' target weights)
__global__ __launch_bounds__(256) void ce_reduce_kernel(const float* __restrict__ loss, const int64_t* __restrict__ target,
                                                        const float* __restrict__ weight, float* __restrict__ out,
                                                        int64_t rows, int64_t ignore_index, int mean) {
  __shared__ float sm[4];
  float s = 0.f, c = 0.f;
  for (int64_t i = threadIdx.x; i < rows; i += 256) {
    s += loss[i];
    const int64_t t = target[i];
    c += (t != ignore_index) ? (weight ? weight[t] : 1.f) : 0.f;
  }
  const float ts = block_sum<4>(s, sm);
  __syncthreads();
  const float tc = block_sum<4>(c, sm);
  if (threadIdx.x == 0) {
    out[0] = mean ? (weight ? ts / tc : ts / fmaxf(tc, 1.f)) : ts;
    out[1] = tc;
  }
}

template <typename T>
__global__ __launch_bounds__(kCeThreads) void ce_bwd_kernel(const T* __restrict__ logits, const int64_t* __restrict__ target,
                                                            const float* __restrict__ weight,
                                                            const float* __restrict__ lse, const float* __restrict__ gscale,
                                                            const float* __restrict__ stats, T* __restrict__ dlogits,
                                                            int64_t rows, int V, int64_t ignore_index, int mean,
                                                            int per_row_grad, float label_smoothing) {
  constexpr int VEC = Vec16<T>::N;
  const int64_t row = blockIdx.x;
  const int64_t t = target[row];
  const T* x = logits + row * (int64_t)V;
  T* dx = dlogits + row * (int64_t)V;
  float g;
  if (per_row_grad) {
    g = gscale[row];
  } else {
    g = gscale[0];
    if (mean) g = weight ? g / stats[1] : g / fmaxf(stats[1], 1.f);
  }
  if (t == ignore_index) g = 0.f;
  const float l = lse[row];
  const float smooth = label_smoothing / (float)V;
  const float on = 1.f - label_smoothing;
  // d/dx_j = p_j * pc - on * w_t [j == t] - smooth * w_j, pc = on * w_t + smooth * sum_c w_c
  float wt = 1.f, pc = 1.f;
  if (weight) {
    __shared__ float sm[kCeWaves];
    float sw = 0.f;
    if (label_smoothing != 0.f)
      for (int i = threadIdx.x; i < V; i += kCeThreads) sw += weight[i];
    sw = label_smoothing != 0.f ? block_sum<kCeWaves>(sw, sm) : 0.f;
    wt = (t == ignore_index) ? 0.f : weight[t];
    pc = on * wt + smooth * sw;
  }
  const bool vec = (V % VEC == 0) && (((uintptr_t)logits) % 16 == 0) && (((uintptr_t)dlogits) % 16 == 0);
  if (vec) {
    for (int i = threadIdx.x * VEC; i < V; i += kCeThreads * VEC) {
      const Vec16<T> xv = load16(x + i);
      Vec16<T> o;
#pragma unroll
      for (int j = 0; j < VEC; ++j) {
        const float p = __expf(to_f32(xv.v[j]) - l);
        const float oh = (i + j == t) ? on * wt : 0.f;
        const float sj = weight ? smooth * weight[i + j] : smooth;
        o.v[j] = from_f32<T>(g * (p * pc - oh - sj));
      }
      store16(dx + i, o);
    }
  } else {
    for (int i = threadIdx.x; i < V; i += kCeThreads) {
      const float p = __expf(to_f32(x[i]) - l);
      const float oh = (i == t) ? on * wt : 0.f;
      const float sj = weight ? smooth * weight[i] : smooth;
      dx[i] = from_f32<T>(g * (p * pc - oh - sj));
    }
  }
}

}  // namespace

#define LTA_DISPATCH_T(dtype, ...)                                     \
  do {                                                                \
    if (dtype == kBF16) { using T = __hip_bfloat16; __VA_ARGS__; }      \
    else if (dtype == kF16) { using T = __half; __VA_ARGS__; }          \
    else if (dtype == kF32) { using T = float; __VA_ARGS__; }           \
    else { return -1; }                                               \
  } while (0)

LTA_EXPORT int lta_swiglu_fwd(int dtype, const void* a, const void* b, void* y, int64_t n, hipStream_t stream) {
  LTA_DISPATCH_T(dtype, hipLaunchKernelGGL((swiglu_fwd_kernel<T>), dim3(ew_grid(n / Vec16<T>::N + 1)), dim3(256), 0,
                                           stream, (const T*)a, (const T*)b, (T*)y, n));
  return (int)hipGetLastError();
}

// SwiGLU forward with an e4m3 output (swiglu_fwd_fp8_kernel); n % 8 == 0, 16-bit a / b.
LTA_EXPORT int lta_swiglu_fwd_fp8(int dtype, const void* a, const void* b, void* q, int64_t n, const void* amax_in,
                                  float fmax, void* scale_out, void* amax_out, hipStream_t stream) {
  if (n % 8 || ((uintptr_t)a % 16) || ((uintptr_t)b % 16) || ((uintptr_t)q % 8)) return -1;
  const dim3 grid((unsigned)std::min<int64_t>((n / 8 + 255) / 256, 1024)), block(256);
  if (dtype == kBF16)
    hipLaunchKernelGGL((swiglu_fwd_fp8_kernel<__hip_bfloat16>), grid, block, 0, stream, (const __hip_bfloat16*)a,
                       (const __hip_bfloat16*)b, (uint8_t*)q, n, (const float*)amax_in, fmax, (float*)scale_out,
                       (float*)amax_out);
  else if (dtype == kF16)
    hipLaunchKernelGGL((swiglu_fwd_fp8_kernel<__half>), grid, block, 0, stream, (const __half*)a, (const __half*)b,
                       (uint8_t*)q, n, (const float*)amax_in, fmax, (float*)scale_out, (float*)amax_out);
  else
    return -1;
  return (int)hipGetLastError();
}

// SwiGLU backward with e5m2 outputs (swiglu_bwd_fp8_kernel); n % 8 == 0, 16-bit g / a / b.
LTA_EXPORT int lta_swiglu_bwd_fp8(int dtype, const void* g, const void* a, const void* b, void* qa, void* qb,
                                  int64_t n, const void* amax_in_a, const void* amax_in_b, float fmax, void* scale_a,
                                  void* scale_b, void* amax_a, void* amax_b, hipStream_t stream) {
  if (n % 8 || ((uintptr_t)g % 16) || ((uintptr_t)a % 16) || ((uintptr_t)b % 16) || ((uintptr_t)qa % 8) ||
      ((uintptr_t)qb % 8))
    return -1;
  const dim3 grid((unsigned)std::min<int64_t>((n / 8 + 255) / 256, 1024)), block(256);
#define LTA_SB8(T)                                                                                                 \
  hipLaunchKernelGGL((swiglu_bwd_fp8_kernel<T>), grid, block, 0, stream, (const T*)g, (const T*)a, (const T*)b,     \
                     (uint8_t*)qa, (uint8_t*)qb, n, (const float*)amax_in_a, (const float*)amax_in_b, fmax,         \
                     (float*)scale_a, (float*)scale_b, (float*)amax_a, (float*)amax_b)
  if (dtype == kBF16) LTA_SB8(__hip_bfloat16);
  else if (dtype == kF16) LTA_SB8(__half);
  else return -1;
#undef LTA_SB8
  return (int)hipGetLastError();
}

LTA_EXPORT int lta_swiglu_bwd(int dtype, const void* g, const void* a, const void* b, void* da, void* db, int64_t n,
                              hipStream_t stream) {
  LTA_DISPATCH_T(dtype, hipLaunchKernelGGL((swiglu_bwd_kernel<T>), dim3(ew_grid(n / Vec16<T>::N + 1)), dim3(256), 0,
                                           stream, (const T*)g, (const T*)a, (const T*)b, (T*)da, (T*)db, n));
  return (int)hipGetLastError();
}

// reduction: 0 = none (per-row losses returned), 1 = mean, 2 = sum
// weight: optional fp32 [V] class weights (null = unweighted)
LTA_EXPORT int lta_ce_fwd_w(int dtype, const void* logits, const int64_t* target, const void* weight, void* loss_rows,
                            void* lse, void* out, int64_t rows, int64_t V, int64_t ignore_index, int reduction,
                            float label_smoothing, hipStream_t stream) {
  LTA_DISPATCH_T(dtype, hipLaunchKernelGGL((ce_fwd_kernel<T>), dim3((unsigned)rows), dim3(kCeThreads), 0, stream,
                                           (const T*)logits, target, (const float*)weight, (float*)loss_rows,
                                           (float*)lse, rows, (int)V, ignore_index, label_smoothing));
  if (reduction != 0) {
    hipLaunchKernelGGL(ce_reduce_kernel, dim3(1), dim3(256), 0, stream, (const float*)loss_rows, target,
                       (const float*)weight, (float*)out, rows, ignore_index, reduction == 1 ? 1 : 0);
  }
  return (int)hipGetLastError();
}

LTA_EXPORT int lta_ce_fwd(int dtype, const void* logits, const int64_t* target, void* loss_rows, void* lse, void* out,
                          int64_t rows, int64_t V, int64_t ignore_index, int reduction, float label_smoothing,
                          hipStream_t stream) {
  return lta_ce_fwd_w(dtype, logits, target, nullptr, loss_rows, lse, out, rows, V, ignore_index, reduction,
                      label_smoothing, stream);
}

LTA_EXPORT int lta_ce_bwd_w(int dtype, const void* logits, const int64_t* target, const void* weight, const void* lse,
                            const void* gscale, const void* stats, void* dlogits, int64_t rows, int64_t V,
                            int64_t ignore_index, int reduction, float label_smoothing, hipStream_t stream) {
  LTA_DISPATCH_T(dtype, hipLaunchKernelGGL((ce_bwd_kernel<T>), dim3((unsigned)rows), dim3(kCeThreads), 0, stream,
                                           (const T*)logits, target, (const float*)weight, (const float*)lse,
                                           (const float*)gscale,
                                           (const float*)stats, (T*)dlogits, rows, (int)V, ignore_index,
                                           reduction == 1 ? 1 : 0, reduction == 0 ? 1 : 0, label_smoothing));
  return (int)hipGetLastError();
}

LTA_EXPORT int lta_ce_bwd(int dtype, const void* logits, const int64_t* target, const void* lse, const void* gscale,
                          const void* stats, void* dlogits, int64_t rows, int64_t V, int64_t ignore_index,
                          int reduction, float label_smoothing, hipStream_t stream) {
  return lta_ce_bwd_w(dtype, logits, target, nullptr, lse, gscale, stats, dlogits, rows, V, ignore_index, reduction,
                      label_smoothing, stream);
}
