// K9: NF4 (4-bit NormalFloat, block-wise absmax) weight dequantisation for CDNA4.
// (reference: bitsandbytes dequantize_4bit behind thunder/transforms/quantization.py:19-44)
//
// Packed layout (bitsandbytes-compatible): byte i holds element 2i in its high nibble and
// element 2i+1 in its low nibble; absmax[b] scales block b of `blocksize` elements.
// One lane turns 8 packed bytes (16 weights) into two 16-byte bf16/fp16 stores; the 16-entry
// code book lives in registers (LDS would serialise the lookups on bank conflicts).
#include "common.h"

using namespace lta;

namespace {

template <typename T>
__global__ __launch_bounds__(256) void nf4_dequant_kernel(const uint8_t* __restrict__ q, const float* __restrict__ absmax,
                                                         const float* __restrict__ code, T* __restrict__ out, int64_t n,
                                                         int blocksize) {
  float cb[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) cb[i] = code[i];
  const int64_t nchunks = n / 16;
  for (int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; c < nchunks; c += (int64_t)gridDim.x * blockDim.x) {
    const uint2 p = *reinterpret_cast<const uint2*>(q + c * 8);
    const float s = absmax[(c * 16) / blocksize];
    Vec16<T> o0, o1;
    const uint32_t w[2] = {p.x, p.y};
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      const uint32_t byte = (w[b >> 2] >> (8 * (b & 3))) & 0xffu;
      const float hi = cb[byte >> 4] * s, lo = cb[byte & 15u] * s;
      T* dst = (b < 4) ? o0.v : o1.v;
      const int j = (b & 3) * 2;
      dst[j] = from_f32<T>(hi);
      dst[j + 1] = from_f32<T>(lo);
    }
    store16(out + c * 16, o0);
    store16(out + c * 16 + 8, o1);
  }
}

// ---------------------------------------------------------------------------------------------
// Fused NF4 weight-only GEMV (decode, M <= 8 rows): y = x . dequant(W)^T (+ bias), the 4-bit
// weight streamed once and decoded in registers, never materialised in bf16.
//
// The code book lookup is the cost centre (no hardware NF4 format): a 16-entry fp32 table in LDS,
// replicated twice so that the two 16-lane halves of each 32-lane bank group read disjoint banks
// (ds_read_b32 banks are (a/4) mod 32: a lane's copy is lane & 1, the same entry broadcasts,
// different entries hit different banks -> conflict-free).  Each lane owns 32-element chunks of a
// row (16 packed bytes = one 16-B load); the chunk's codes are looked up once and reused by all
// M activation rows, and the absmax scale is applied once per chunk (blocksize % 32 == 0).  A
// wave computes NPW output columns; lanes stride the row's chunks (coalesced 1 KiB per wave
// instruction) and a butterfly reduces the 64 partial sums.
template <typename T, int M, int NPW>
__global__ __launch_bounds__(256) void gemv_nf4_kernel(const T* __restrict__ x, const uint8_t* __restrict__ q,
                                                       const float* __restrict__ absmax,
                                                       const float* __restrict__ code, const T* __restrict__ bias,
                                                       T* __restrict__ y, int N, int K, int ldx, int ldy, int bs) {
  __shared__ float tab[32];
  if (threadIdx.x < 32) tab[threadIdx.x] = code[threadIdx.x & 15];
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int n0 = (blockIdx.x * 4 + wave) * NPW;
  if (n0 >= N) return;  // whole waves; no barrier below
  const float* tb = tab + (lane & 1) * 16;
  const int nchunk = K / 32;
  float acc[M][NPW];
#pragma unroll
  for (int m = 0; m < M; ++m)
#pragma unroll
    for (int j = 0; j < NPW; ++j) acc[m][j] = 0.f;
  for (int c = lane; c < nchunk; c += 64) {
    uint4 wq[NPW];
    float sc[NPW];
#pragma unroll
    for (int j = 0; j < NPW; ++j) {
      const int n = min(n0 + j, N - 1);
      const int64_t e0 = (int64_t)n * K + (int64_t)c * 32;
      wq[j] = *reinterpret_cast<const uint4*>(q + e0 / 2);
      sc[j] = absmax[e0 / bs];
    }
    float cw[NPW][32];
#pragma unroll
    for (int j = 0; j < NPW; ++j) {
      const uint32_t d[4] = {wq[j].x, wq[j].y, wq[j].z, wq[j].w};
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const uint32_t byte = (d[i >> 2] >> (8 * (i & 3))) & 0xffu;
        cw[j][2 * i] = tb[byte >> 4];
        cw[j][2 * i + 1] = tb[byte & 15u];
      }
    }
#pragma unroll
    for (int m = 0; m < M; ++m) {
      const T* xr = x + (int64_t)m * ldx + c * 32;
      float xf[32];
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const Vec16<T> xv = load16(xr + v * 8);
#pragma unroll
        for (int e = 0; e < 8; ++e) xf[v * 8 + e] = to_f32(xv.v[e]);
      }
#pragma unroll
      for (int j = 0; j < NPW; ++j) {
        float p = 0.f;
#pragma unroll
        for (int e = 0; e < 32; ++e) p = fmaf(xf[e], cw[j][e], p);
        acc[m][j] = fmaf(p, sc[j], acc[m][j]);
      }
    }
  }
#pragma unroll
  for (int m = 0; m < M; ++m) {
#pragma unroll
    for (int j = 0; j < NPW; ++j) {
      const float v = wave_sum(acc[m][j]);
      if (lane == 0 && n0 + j < N) {
        const float bv = bias != nullptr ? to_f32(bias[n0 + j]) : 0.f;
        y[(int64_t)m * ldy + n0 + j] = from_f32<T>(v + bv);
      }
    }
  }
}

template <typename T>
int launch_gemv_nf4(const void* x, const void* q, const void* absmax, const void* code, const void* bias, void* y,
                    int M, int N, int K, int ldx, int ldy, int bs, hipStream_t stream) {
  constexpr int NPW = 2;
  dim3 grid((N + 4 * NPW - 1) / (4 * NPW)), block(256);
#define LTA_GN(MM)                                                                                           \
  case MM:                                                                                                   \
    hipLaunchKernelGGL((gemv_nf4_kernel<T, MM, NPW>), grid, block, 0, stream, (const T*)x, (const uint8_t*)q, \
                       (const float*)absmax, (const float*)code, (const T*)bias, (T*)y, N, K, ldx, ldy, bs);  \
    break;
  switch (M) {
    LTA_GN(1) LTA_GN(2) LTA_GN(3) LTA_GN(4) LTA_GN(5) LTA_GN(6) LTA_GN(7) LTA_GN(8)
    default: return -2;
  }
#undef LTA_GN
  return (int)hipGetLastError();
}

}  // namespace

// x [M, K] (row stride ldx, 16-B aligned rows), packed NF4 W [N, K] (bitsandbytes order: high
// nibble = even element), absmax per `bs` elements (bs % 32 == 0), code [16] fp32 -> y [M, N].
LTA_EXPORT int lta_gemv_nf4(int dtype, const void* x, const void* q, const void* absmax, const void* code,
                            const void* bias, void* y, int M, int N, int K, int ldx, int ldy, int bs,
                            hipStream_t stream) {
  if (M < 1 || M > 8 || K % 32 || bs % 32 || ldx % 8 || reinterpret_cast<uintptr_t>(x) % 16) return -2;
  if (dtype == kBF16)
    return launch_gemv_nf4<__hip_bfloat16>(x, q, absmax, code, bias, y, M, N, K, ldx, ldy, bs, stream);
  if (dtype == kF16) return launch_gemv_nf4<__half>(x, q, absmax, code, bias, y, M, N, K, ldx, ldy, bs, stream);
  return -1;
}

LTA_EXPORT int lta_nf4_dequant(int dtype, const void* q, const void* absmax, const void* code, void* out, int64_t n,
                               int blocksize, hipStream_t stream) {
  if (n % 16 != 0 || blocksize % 16 != 0) return -2;
  const int64_t chunks = n / 16;
  const unsigned grid = (unsigned)std::min<int64_t>((chunks + 255) / 256, 8192);
  if (dtype == kBF16)
    hipLaunchKernelGGL(nf4_dequant_kernel<__hip_bfloat16>, dim3(grid), dim3(256), 0, stream, (const uint8_t*)q,
                       (const float*)absmax, (const float*)code, (__hip_bfloat16*)out, n, blocksize);
  else if (dtype == kF16)
    hipLaunchKernelGGL(nf4_dequant_kernel<__half>, dim3(grid), dim3(256), 0, stream, (const uint8_t*)q,
                       (const float*)absmax, (const float*)code, (__half*)out, n, blocksize);
  else
    return -1;
  return (int)hipGetLastError();
}
