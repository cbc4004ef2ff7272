// K15: multi-tensor fused AdamW for CDNA4 (one launch for every parameter of the model).
// (reference: the benchmark's torch.optim.AdamW(fused=True), thunder/benchmarks/benchmark_litgpt.py:275-283)
//
// Pure HBM streaming: per element read p, g, m, v and write p, m, v (14 B/elem for bf16
// params with bf16 state; fp32 state is supported too).  Work is cut into fixed-size chunks
// described by a device table {tensor index, element offset}; every lane moves 16-byte
// vectors.  Math in fp32.
#include "common.h"
#include "fp8_cvt.h"
#include <cstdlib>

using namespace lta;

namespace {

struct TensorMeta {
  void* p;
  const void* g;
  void* m;
  void* v;
  int64_t n;
  // fp8 weight shadow (bf16 params of FP8 linears, ops/fp8.py weight shadows; q == nullptr: none): the
  // updated weight leaves the kernel also as e4m3 q = sat(p * fmax / *amax_in) -- bitwise the forward's
  // cast of it -- with the scale used in *scale_out and max |p| folded into *sink (the amax history)
  uint8_t* q;
  const float* amax_in;
  float* scale_out;
  float* sink;
  float fmax;
  int pad_;
};

constexpr int kChunk = 16384;  // elements per workgroup-chunk

template <typename TP, typename TS>
__device__ __forceinline__ void adamw_elem(float& p, float g, float& m, float& v, float lr, float b1, float b2,
                                           float eps, float wd, float bc1, float bc2_sqrt) {
  // explicit FMAs and no compiler contraction: every instantiation (plain, non-temporal, lean) rounds
  // identically, so updates issued from different kernels are bitwise interchangeable
#pragma clang fp contract(off)
  p = p * (1.f - lr * wd);
  m = __builtin_fmaf(b1, m, (1.f - b1) * g);
  v = __builtin_fmaf(b2, v, ((1.f - b2) * g) * g);
  const float denom = sqrtf(v) / bc2_sqrt + eps;
  p = __builtin_fmaf(-(lr / bc1), m / denom, p);
}

// U = 16-byte vectors per lane in flight per operand.  The default (U = 4) streams at full HBM
// rate on an idle GPU.  The lean variant (U = 1, <= 80 VGPRs, 6 waves/SIMD) is for the update
// issued on a side stream during the backward: its waves fit next to a 4-wave gemm4 workgroup
// (168 VGPR + 256 AGPR per wave), so the optimizer streams HBM while the GEMM keeps the MFMAs busy.
template <typename TP, typename TS, int U, bool NT = false, bool SHADOW = false>
__device__ __forceinline__ void adamw_body(const TensorMeta* __restrict__ metas, const int2* __restrict__ chunks,
                                           float lr, float b1, float b2, float eps, float wd, float bc1,
                                           float bc2_sqrt, float grad_scale) {
  const int2 ck = chunks[blockIdx.x];
  const TensorMeta mt = metas[ck.x];
  const int64_t start = (int64_t)ck.y * kChunk;
  const int64_t end = min(mt.n, start + kChunk);
  TP* P = (TP*)mt.p;
  const TP* G = (const TP*)mt.g;
  TS* M = (TS*)mt.m;
  TS* V = (TS*)mt.v;
  constexpr int VP = Vec16<TP>::N;
  [[maybe_unused]] uint8_t* const Q = SHADOW ? mt.q : nullptr;
  [[maybe_unused]] float qs = 0.f, wmax = 0.f;
  if constexpr (SHADOW) {
    if (Q != nullptr) {
      qs = mt.fmax / fmaxf(*mt.amax_in, 1e-12f);
      if (ck.y == 0 && threadIdx.x == 0) *mt.scale_out = qs;
    }
  }
  const bool vec = ((end - start) % VP == 0) && ((uintptr_t)(P + start) % 16 == 0) && ((uintptr_t)(G + start) % 16 == 0) &&
                   (sizeof(TS) == sizeof(TP)) && ((uintptr_t)(M + start) % 16 == 0) && ((uintptr_t)(V + start) % 16 == 0) &&
                   (!SHADOW || Q == nullptr || (VP == 8 && (uintptr_t)(Q + start) % 8 == 0));
  if (vec) {
    // U vectors per lane per trip, all loads issued before any math: 4U 16-B loads in flight per lane
    for (int64_t i0 = start + (int64_t)threadIdx.x * VP; i0 < end; i0 += 256 * VP * U) {
      Vec16<TP> pv[U], gv[U];
      Vec16<TS> mv[U], vv[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t i = i0 + (int64_t)u * 256 * VP;
        if (i < end) {
          if constexpr (NT) {
            pv[u] = load16_nt(P + i);
            gv[u] = load16_nt(G + i);
            mv[u] = load16_nt(M + i);
            vv[u] = load16_nt(V + i);
          } else {
            pv[u] = load16(P + i);
            gv[u] = load16(G + i);
            mv[u] = load16(M + i);
            vv[u] = load16(V + i);
          }
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t i = i0 + (int64_t)u * 256 * VP;
        if (i < end) {
#pragma unroll
          for (int j = 0; j < VP; ++j) {
            float p = to_f32(pv[u].v[j]), m = to_f32(mv[u].v[j]), v = to_f32(vv[u].v[j]);
            adamw_elem<TP, TS>(p, to_f32(gv[u].v[j]) * grad_scale, m, v, lr, b1, b2, eps, wd, bc1, bc2_sqrt);
            pv[u].v[j] = from_f32<TP>(p);
            mv[u].v[j] = from_f32<TS>(m);
            vv[u].v[j] = from_f32<TS>(v);
          }
          if constexpr (SHADOW) {
            if (Q != nullptr) {
              float w[8];
#pragma unroll
              for (int j = 0; j < 8; ++j) {
                w[j] = to_f32(pv[u].v[j]);
                wmax = fmaxf(wmax, fabsf(w[j]));
              }
              const uint32_t lo = cvt4<false>(w[0] * qs, w[1] * qs, w[2] * qs, w[3] * qs);
              const uint32_t hi = cvt4<false>(w[4] * qs, w[5] * qs, w[6] * qs, w[7] * qs);
              *reinterpret_cast<uint2*>(Q + i) = make_uint2(lo, hi);
            }
          }
          if constexpr (NT) {
            store16_nt(P + i, pv[u]);
            store16_nt(M + i, mv[u]);
            store16_nt(V + i, vv[u]);
          } else {
            store16(P + i, pv[u]);
            store16(M + i, mv[u]);
            store16(V + i, vv[u]);
          }
        }
      }
    }
  } else {
    for (int64_t i = start + threadIdx.x; i < end; i += 256) {
      float p = to_f32(P[i]), m = to_f32(M[i]), v = to_f32(V[i]);
      adamw_elem<TP, TS>(p, to_f32(G[i]) * grad_scale, m, v, lr, b1, b2, eps, wd, bc1, bc2_sqrt);
      P[i] = from_f32<TP>(p);
      M[i] = from_f32<TS>(m);
      V[i] = from_f32<TS>(v);
      if constexpr (SHADOW) {
        if (Q != nullptr) {
          const float w = to_f32(P[i]);
          wmax = fmaxf(wmax, fabsf(w));
          Q[i] = (uint8_t)(cvt4<false>(w * qs, 0.f, 0.f, 0.f) & 0xffu);
        }
      }
    }
  }
  if constexpr (SHADOW) {
    if (Q != nullptr) {  // uniform over the workgroup (one tensor per chunk)
      __shared__ float red[4];
      fp8_amax_out<4>(wmax, mt.sink, red);
    }
  }
}

template <typename TP, typename TS, bool NT = false, bool SHADOW = false>
__global__ __launch_bounds__(256) void adamw_kernel(const TensorMeta* __restrict__ metas, const int2* __restrict__ chunks,
                                                    float lr, float b1, float b2, float eps, float wd, float bc1,
                                                    float bc2_sqrt, float grad_scale) {
  adamw_body<TP, TS, 4, NT, SHADOW>(metas, chunks, lr, b1, b2, eps, wd, bc1, bc2_sqrt, grad_scale);
}

// non-temporal loads / stores in the post-backward kernel (LTA_ADAMW_NT=0 turns them off): 5.99 vs
// 5.73 TB/s (scripts/adamw_nt_ab.py).  Before adamw_elem pinned its rounding, the compiler contracted
// this variant differently and it was not bitwise equal to the lean kernel (profiles/adamw_nt_ab.txt)
int g_adamw_nt = [] {
  const char* e = getenv("LTA_ADAMW_NT");
  return (e && e[0] == '0') ? 0 : 1;
}();

template <typename TP, typename TS, bool SHADOW = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(6))) void adamw_lean_kernel(
    const TensorMeta* __restrict__ metas, const int2* __restrict__ chunks, float lr, float b1, float b2, float eps,
    float wd, float bc1, float bc2_sqrt, float grad_scale) {
  adamw_body<TP, TS, 1, false, SHADOW>(metas, chunks, lr, b1, b2, eps, wd, bc1, bc2_sqrt, grad_scale);
}

}  // namespace

LTA_EXPORT int lta_adamw_chunk_size() { return kChunk; }

// A/B switch for the post-backward kernel's non-temporal streaming; returns the previous setting
LTA_EXPORT int lta_adamw_set_nt(int nt) {
  const int old = g_adamw_nt;
  g_adamw_nt = nt ? 1 : 0;
  return old;
}

// metas: device array of TensorMeta; chunks: device int2 array {tensor, chunk index}
// lean = 1: the register-capped variant (see adamw_body) for updates overlapped with compute
// shadow = 1: some tensors carry an fp8 weight shadow (TensorMeta.q; bf16 params only)
LTA_EXPORT int lta_adamw_ex2(int pdtype, int sdtype, const void* metas, const void* chunks, int n_chunks, float lr,
                             float b1, float b2, float eps, float wd, float bc1, float bc2_sqrt, float grad_scale,
                             int lean, int shadow, hipStream_t stream) {
  dim3 grid(n_chunks), block(256);
#define LTA_L(TPt, TSt, SH)                                                                                          \
  do {                                                                                                               \
    if (lean)                                                                                                        \
      hipLaunchKernelGGL((adamw_lean_kernel<TPt, TSt, SH>), grid, block, 0, stream, (const TensorMeta*)metas,        \
                         (const int2*)chunks, lr, b1, b2, eps, wd, bc1, bc2_sqrt, grad_scale);                       \
    else if (g_adamw_nt)                                                                                             \
      hipLaunchKernelGGL((adamw_kernel<TPt, TSt, true, SH>), grid, block, 0, stream, (const TensorMeta*)metas,       \
                         (const int2*)chunks, lr, b1, b2, eps, wd, bc1, bc2_sqrt, grad_scale);                       \
    else                                                                                                             \
      hipLaunchKernelGGL((adamw_kernel<TPt, TSt, false, SH>), grid, block, 0, stream, (const TensorMeta*)metas,      \
                         (const int2*)chunks, lr, b1, b2, eps, wd, bc1, bc2_sqrt, grad_scale);                       \
  } while (0)
  if (shadow) {
    if (pdtype == kBF16 && sdtype == kBF16) LTA_L(__hip_bfloat16, __hip_bfloat16, true);
    else if (pdtype == kBF16 && sdtype == kF32) LTA_L(__hip_bfloat16, float, true);
    else return -1;
  } else if (pdtype == kBF16 && sdtype == kBF16) LTA_L(__hip_bfloat16, __hip_bfloat16, false);
  else if (pdtype == kBF16 && sdtype == kF32) LTA_L(__hip_bfloat16, float, false);
  else if (pdtype == kF16 && sdtype == kF16) LTA_L(__half, __half, false);
  else if (pdtype == kF16 && sdtype == kF32) LTA_L(__half, float, false);
  else if (pdtype == kF32 && sdtype == kF32) LTA_L(float, float, false);
  else return -1;
#undef LTA_L
  return (int)hipGetLastError();
}

LTA_EXPORT int lta_adamw_ex(int pdtype, int sdtype, const void* metas, const void* chunks, int n_chunks, float lr,
                            float b1, float b2, float eps, float wd, float bc1, float bc2_sqrt, float grad_scale, int lean,
                            hipStream_t stream) {
  return lta_adamw_ex2(pdtype, sdtype, metas, chunks, n_chunks, lr, b1, b2, eps, wd, bc1, bc2_sqrt, grad_scale, lean, 0,
                       stream);
}

LTA_EXPORT int lta_adamw(int pdtype, int sdtype, const void* metas, const void* chunks, int n_chunks, float lr, float b1,
                         float b2, float eps, float wd, float bc1, float bc2_sqrt, float grad_scale, hipStream_t stream) {
  return lta_adamw_ex(pdtype, sdtype, metas, chunks, n_chunks, lr, b1, b2, eps, wd, bc1, bc2_sqrt, grad_scale, 0,
                      stream);
}

// bytes of one TensorMeta (the host packs the table)
LTA_EXPORT int lta_adamw_meta_bytes() { return (int)sizeof(TensorMeta); }
