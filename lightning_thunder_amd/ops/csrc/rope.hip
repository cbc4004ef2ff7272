// K6: fused qkv split + RoPE (forward and backward) for CDNA4.
//
// Forward: qkv [B, T, (nh + 2*ng) * hs] (output of the fused QKV projection) ->
//   q [B, nh, T, hs], k [B, ng, T, hs] with LitGPT's rotate-half RoPE on the first `rope_n`
//   elements of every head, v [B, ng, T, hs] (pure layout change).
// Backward: (dq, dk, dv) -> dqkv with the inverse rotation.
// Replaces the reference's torch.compile(Inductor) "torchcompile_cat" RoPE fusion
// (thunder/executors/torch_compile.py:205-234; benchmark LlamaQKVSplitRopeBenchmark).
//
// Each work item moves one 16-byte chunk (8 elements) of a head row and, for rotated chunks,
// also its partner chunk half a rope width away, so every HBM access is a 16-B vector.
#include "common.h"

using namespace lta;

namespace {

// k / v rows go to k + b*ks[0] + g*ks[1] + s*ks[2] with s = pos ? pos[t] : t: with `pos` they are
// written straight into a static KV cache at the decode positions (no separate index_copy launch).
struct KVDst {
  int64_t ksb, ksg, kss, vsb, vsg, vss;
};

template <typename T, typename C>
__global__ __launch_bounds__(256) void qkv_rope_fwd_kernel(const T* __restrict__ qkv, const C* __restrict__ cos_,
                                                           const C* __restrict__ sin_, T* __restrict__ q,
                                                           T* __restrict__ k, T* __restrict__ v,
                                                           const int64_t* __restrict__ pos, KVDst st, int B, int Tn,
                                                           int nh, int ng, int hs, int rope_n) {
  constexpr int VW = Vec16<T>::N;
  const int chunks = hs / VW;
  const int heads = nh + 2 * ng;
  const int64_t total = (int64_t)B * Tn * heads * chunks;
  const int half = rope_n / 2;
  for (int64_t it = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; it < total; it += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)(it % chunks);
    int64_t rest = it / chunks;
    const int h = (int)(rest % heads);
    rest /= heads;
    const int t = (int)(rest % Tn);
    const int b = (int)(rest / Tn);
    const int d0 = c * VW;
    const T* src = qkv + (((int64_t)b * Tn + t) * heads + h) * hs;
    T* dst;
    bool rotate;
    if (h < nh) {
      dst = q + (((int64_t)b * nh + h) * Tn + t) * hs;
      rotate = true;
    } else if (h < nh + ng) {
      const int64_t s = pos ? pos[t] : t;
      dst = k + b * st.ksb + (h - nh) * st.ksg + s * st.kss;
      rotate = true;
    } else {
      const int64_t s = pos ? pos[t] : t;
      dst = v + b * st.vsb + (h - nh - ng) * st.vsg + s * st.vss;
      rotate = false;
    }
    if (!rotate || d0 >= rope_n) {
      store16(dst + d0, load16(src + d0));
      continue;
    }
    if (d0 >= half) continue;  // handled together with its partner chunk
    const Vec16<T> x1 = load16(src + d0);
    const Vec16<T> x2 = load16(src + d0 + half);
    const C* cr = cos_ + (int64_t)t * rope_n;
    const C* sr = sin_ + (int64_t)t * rope_n;
    Vec16<T> o1, o2;
#pragma unroll
    for (int j = 0; j < VW; ++j) {
      const float a = to_f32(x1.v[j]), bb = to_f32(x2.v[j]);
      const float c1 = to_f32(cr[d0 + j]), s1 = to_f32(sr[d0 + j]);
      const float c2 = to_f32(cr[d0 + half + j]), s2 = to_f32(sr[d0 + half + j]);
      o1.v[j] = from_f32<T>(a * c1 - bb * s1);
      o2.v[j] = from_f32<T>(bb * c2 + a * s2);
    }
    store16(dst + d0, o1);
    store16(dst + d0 + half, o2);
  }
}

template <typename T, typename C>
__global__ __launch_bounds__(256) void qkv_rope_bwd_kernel(const T* __restrict__ dq, const T* __restrict__ dk,
                                                           const T* __restrict__ dv, const C* __restrict__ cos_,
                                                           const C* __restrict__ sin_, T* __restrict__ dqkv, int B,
                                                           int Tn, int nh, int ng, int hs, int rope_n) {
  constexpr int VW = Vec16<T>::N;
  const int chunks = hs / VW;
  const int heads = nh + 2 * ng;
  const int64_t total = (int64_t)B * Tn * heads * chunks;
  const int half = rope_n / 2;
  for (int64_t it = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; it < total; it += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)(it % chunks);
    int64_t rest = it / chunks;
    const int h = (int)(rest % heads);
    rest /= heads;
    const int t = (int)(rest % Tn);
    const int b = (int)(rest / Tn);
    const int d0 = c * VW;
    T* dst = dqkv + (((int64_t)b * Tn + t) * heads + h) * hs;
    const T* src;
    bool rotate;
    if (h < nh) {
      src = dq + (((int64_t)b * nh + h) * Tn + t) * hs;
      rotate = true;
    } else if (h < nh + ng) {
      src = dk + (((int64_t)b * ng + (h - nh)) * Tn + t) * hs;
      rotate = true;
    } else {
      src = dv + (((int64_t)b * ng + (h - nh - ng)) * Tn + t) * hs;
      rotate = false;
    }
    if (!rotate || d0 >= rope_n) {
      store16(dst + d0, load16(src + d0));
      continue;
    }
    if (d0 >= half) continue;
    const Vec16<T> g1 = load16(src + d0);
    const Vec16<T> g2 = load16(src + d0 + half);
    const C* cr = cos_ + (int64_t)t * rope_n;
    const C* sr = sin_ + (int64_t)t * rope_n;
    Vec16<T> o1, o2;
#pragma unroll
    for (int j = 0; j < VW; ++j) {
      const float a = to_f32(g1.v[j]), bb = to_f32(g2.v[j]);
      const float c1 = to_f32(cr[d0 + j]), s1 = to_f32(sr[d0 + j]);
      const float c2 = to_f32(cr[d0 + half + j]), s2 = to_f32(sr[d0 + half + j]);
      // y1 = x1*c1 - x2*s1 ; y2 = x2*c2 + x1*s2
      o1.v[j] = from_f32<T>(a * c1 + bb * s2);
      o2.v[j] = from_f32<T>(bb * c2 - a * s1);
    }
    store16(dst + d0, o1);
    store16(dst + d0 + half, o2);
  }
}

// Full-width RoPE (rope_n == hs, the Llama case), one token row per workgroup: each work item owns a
// chunk and its rotation partner half a head away, so no lane idles, and the item -> (head, chunk)
// split is a shift (no 64-bit division); cos / sin rows are read as 16-B vectors.
template <typename C>
__device__ __forceinline__ void load_cs8(const C* p, float (&o)[8]) {
  if constexpr (sizeof(C) == 4) {
    const float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
    o[0] = a.x; o[1] = a.y; o[2] = a.z; o[3] = a.w; o[4] = b.x; o[5] = b.y; o[6] = b.z; o[7] = b.w;
  } else {
    const Vec16<C> v = load16(p);
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = to_f32(v.v[j]);
  }
}

template <typename T, typename C, bool BWD>
__global__ __launch_bounds__(256) void qkv_rope_row_kernel(const T* __restrict__ in0, const T* __restrict__ in1,
                                                           const T* __restrict__ in2, const C* __restrict__ cos_,
                                                           const C* __restrict__ sin_, T* __restrict__ out0,
                                                           T* __restrict__ out1, T* __restrict__ out2,
                                                           const int64_t* __restrict__ pos, KVDst st, int Tn, int nh,
                                                           int ng, int hs, int pair_shift) {
  // fwd: in0 = qkv, out0/1/2 = q/k/v (k/v through st); bwd: in0/1/2 = dq/dk/dv, out0 = dqkv
  constexpr int VW = 8;
  const int row = blockIdx.x;  // b * Tn + t
  const int t = row % Tn, b = row / Tn;
  const int heads = nh + 2 * ng, half = hs / 2;
  const int items = heads << pair_shift;
  const C* cr = cos_ + (int64_t)t * hs;
  const C* sr = sin_ + (int64_t)t * hs;
  for (int it = threadIdx.x; it < items; it += blockDim.x) {
    const int h = it >> pair_shift, d0 = (it & ((1 << pair_shift) - 1)) * VW;
    const T* src;
    T* dst;
    if constexpr (!BWD) {
      src = in0 + ((int64_t)row * heads + h) * hs;
      if (h < nh) {
        dst = out0 + (((int64_t)b * nh + h) * Tn + t) * hs;
      } else {
        const int64_t s = pos ? pos[t] : t;
        dst = h < nh + ng ? out1 + b * st.ksb + (h - nh) * st.ksg + s * st.kss
                          : out2 + b * st.vsb + (h - nh - ng) * st.vsg + s * st.vss;
      }
    } else {
      dst = out0 + ((int64_t)row * heads + h) * hs;
      src = h < nh ? in0 + (((int64_t)b * nh + h) * Tn + t) * hs
                   : (h < nh + ng ? in1 + (((int64_t)b * ng + (h - nh)) * Tn + t) * hs
                                  : in2 + (((int64_t)b * ng + (h - nh - ng)) * Tn + t) * hs);
    }
    const Vec16<T> x1 = load16(src + d0), x2 = load16(src + d0 + half);
    if (h >= nh + ng) {  // v: layout change only
      store16(dst + d0, x1);
      store16(dst + d0 + half, x2);
      continue;
    }
    float c1[8], s1[8], c2[8], s2[8];
    load_cs8(cr + d0, c1);
    load_cs8(sr + d0, s1);
    load_cs8(cr + d0 + half, c2);
    load_cs8(sr + d0 + half, s2);
    Vec16<T> o1, o2;
#pragma unroll
    for (int j = 0; j < VW; ++j) {
      const float a = to_f32(x1.v[j]), bb = to_f32(x2.v[j]);
      if constexpr (!BWD) {
        o1.v[j] = from_f32<T>(a * c1[j] - bb * s1[j]);
        o2.v[j] = from_f32<T>(bb * c2[j] + a * s2[j]);
      } else {  // transpose of the rotation
        o1.v[j] = from_f32<T>(a * c1[j] + bb * s2[j]);
        o2.v[j] = from_f32<T>(bb * c2[j] - a * s1[j]);
      }
    }
    store16(dst + d0, o1);
    store16(dst + d0 + half, o2);
  }
}

// shift with (1 << shift) == hs / 16 (chunk pairs per head), or -1 when the row kernel does not apply
int row_pair_shift(int dtype, int hs, int rope_n) {
  if (dtype == kF32 || rope_n != hs || hs % 16) return -1;
  const int pairs = hs / 16;
  if (pairs & (pairs - 1)) return -1;
  int sh = 0;
  while ((1 << sh) < pairs) ++sh;
  return sh;
}

int grid_for(int64_t total) {
  int64_t g = (total + 255) / 256;
  if (g > 256 * 16) g = 256 * 16;
  return (int)(g < 1 ? 1 : g);
}

}  // namespace

#define LTA_DISPATCH_TC(dtype, cdtype, ...)                       \
  do {                                                           \
    if (dtype == kBF16 && cdtype == kF32) {                      \
      using T = __hip_bfloat16; using C = float; __VA_ARGS__;     \
    } else if (dtype == kBF16 && cdtype == kBF16) {              \
      using T = __hip_bfloat16; using C = __hip_bfloat16; __VA_ARGS__; \
    } else if (dtype == kF16 && cdtype == kF32) {                \
      using T = __half; using C = float; __VA_ARGS__;             \
    } else if (dtype == kF16 && cdtype == kF16) {                \
      using T = __half; using C = __half; __VA_ARGS__;            \
    } else if (dtype == kF32 && cdtype == kF32) {                \
      using T = float; using C = float; __VA_ARGS__;              \
    } else {                                                     \
      return -1;                                                 \
    }                                                            \
  } while (0)

static int qkv_rope_fwd_launch(int dtype, int cdtype, const void* qkv, const void* cos_, const void* sin_, void* q,
                               void* k, void* v, const int64_t* pos, KVDst st, int B, int Tn, int nh, int ng, int hs,
                               int rope_n, hipStream_t stream) {
  if (hs % 8 || rope_n % 16 || rope_n > hs) return -2;
  const int sh = row_pair_shift(dtype, hs, rope_n);
  if (sh >= 0) {
    LTA_DISPATCH_TC(dtype, cdtype,
                    hipLaunchKernelGGL((qkv_rope_row_kernel<T, C, false>), dim3(B * Tn), dim3(256), 0, stream,
                                       (const T*)qkv, (const T*)nullptr, (const T*)nullptr, (const C*)cos_,
                                       (const C*)sin_, (T*)q, (T*)k, (T*)v, pos, st, Tn, nh, ng, hs, sh));
    return (int)hipGetLastError();
  }
  const int64_t total = (int64_t)B * Tn * (nh + 2 * ng) * (hs / (dtype == kF32 ? 4 : 8));
  LTA_DISPATCH_TC(dtype, cdtype,
                  hipLaunchKernelGGL((qkv_rope_fwd_kernel<T, C>), dim3(grid_for(total)), dim3(256), 0, stream,
                                     (const T*)qkv, (const C*)cos_, (const C*)sin_, (T*)q, (T*)k, (T*)v, pos, st, B, Tn,
                                     nh, ng, hs, rope_n));
  return (int)hipGetLastError();
}

LTA_EXPORT int lta_qkv_rope_fwd(int dtype, int cdtype, const void* qkv, const void* cos_, const void* sin_, void* q,
                                void* k, void* v, int B, int Tn, int nh, int ng, int hs, int rope_n,
                                hipStream_t stream) {
  const int64_t sg = (int64_t)Tn * hs, sb = ng * sg;
  return qkv_rope_fwd_launch(dtype, cdtype, qkv, cos_, sin_, q, k, v, nullptr, KVDst{sb, sg, hs, sb, sg, hs}, B, Tn,
                             nh, ng, hs, rope_n, stream);
}

// k/v written in place into caches kc/vc [B, ng, S, hs] (strides in elements, head dim contiguous and
// 16-byte aligned) at rows pos[0..Tn) (int64, one per query position).
LTA_EXPORT int lta_qkv_rope_cache_fwd(int dtype, int cdtype, const void* qkv, const void* cos_, const void* sin_,
                                      void* q, void* kc, void* vc, const void* pos, const int64_t* strides, int B,
                                      int Tn, int nh, int ng, int hs, int rope_n, hipStream_t stream) {
  if ((strides[0] | strides[1] | strides[2] | strides[3] | strides[4] | strides[5]) % 8) return -2;
  const KVDst st{strides[0], strides[1], strides[2], strides[3], strides[4], strides[5]};
  return qkv_rope_fwd_launch(dtype, cdtype, qkv, cos_, sin_, q, kc, vc, (const int64_t*)pos, st, B, Tn, nh, ng, hs,
                             rope_n, stream);
}

LTA_EXPORT int lta_qkv_rope_bwd(int dtype, int cdtype, const void* dq, const void* dk, const void* dv, const void* cos_,
                                const void* sin_, void* dqkv, int B, int Tn, int nh, int ng, int hs, int rope_n,
                                hipStream_t stream) {
  if (hs % 8 || rope_n % 16 || rope_n > hs) return -2;
  const int sh = row_pair_shift(dtype, hs, rope_n);
  if (sh >= 0) {
    LTA_DISPATCH_TC(dtype, cdtype,
                    hipLaunchKernelGGL((qkv_rope_row_kernel<T, C, true>), dim3(B * Tn), dim3(256), 0, stream,
                                       (const T*)dq, (const T*)dk, (const T*)dv, (const C*)cos_, (const C*)sin_,
                                       (T*)dqkv, (T*)nullptr, (T*)nullptr, (const int64_t*)nullptr, KVDst{0, 0, 0, 0, 0, 0},
                                       Tn, nh, ng, hs, sh));
    return (int)hipGetLastError();
  }
  const int64_t total = (int64_t)B * Tn * (nh + 2 * ng) * (hs / (dtype == kF32 ? 4 : 8));
  LTA_DISPATCH_TC(dtype, cdtype,
                  hipLaunchKernelGGL((qkv_rope_bwd_kernel<T, C>), dim3(grid_for(total)), dim3(256), 0, stream,
                                     (const T*)dq, (const T*)dk, (const T*)dv, (const C*)cos_, (const C*)sin_, (T*)dqkv,
                                     B, Tn, nh, ng, hs, rope_n));
  return (int)hipGetLastError();
}
