// Common device helpers for the CDNA4 (gfx950) kernels of lightning_thunder_amd.
// Wave64 everywhere: reductions use 64-lane butterflies, block sizes are multiples of 64.
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <hip/hip_fp16.h>
#include <stdint.h>

#define LTA_EXPORT extern "C" __attribute__((visibility("default")))

namespace lta {

constexpr int kWave = 64;

// dtype codes shared with the python side (ops/_lib.py)
enum DType : int { kF32 = 0, kF16 = 1, kBF16 = 2, kF64 = 3 };

template <typename T> __device__ __forceinline__ float to_f32(T v);
template <> __device__ __forceinline__ float to_f32<float>(float v) { return v; }
template <> __device__ __forceinline__ float to_f32<__half>(__half v) { return __half2float(v); }
template <> __device__ __forceinline__ float to_f32<__hip_bfloat16>(__hip_bfloat16 v) { return __bfloat162float(v); }

template <typename T> __device__ __forceinline__ T from_f32(float v);
template <> __device__ __forceinline__ float from_f32<float>(float v) { return v; }
template <> __device__ __forceinline__ __half from_f32<__half>(float v) { return __float2half(v); }
template <> __device__ __forceinline__ __hip_bfloat16 from_f32<__hip_bfloat16>(float v) { return __float2bfloat16(v); }

// 16-byte vector of T (8 x 16-bit or 4 x 32-bit) for coalesced 1 KiB-per-wave accesses
template <typename T> struct Vec16 {
  static constexpr int N = 16 / sizeof(T);
  union {
    uint4 raw;
    T v[N];
  };
};

template <typename T>
__device__ __forceinline__ Vec16<T> load16(const T* p) {
  Vec16<T> r;
  r.raw = *reinterpret_cast<const uint4*>(p);
  return r;
}

template <typename T>
__device__ __forceinline__ void store16(T* p, const Vec16<T>& r) {
  *reinterpret_cast<uint4*>(p) = r.raw;
}

// non-temporal forms for pure streams (read once / written once): no L2 / MALL residency
typedef unsigned u32x4v __attribute__((ext_vector_type(4)));

template <typename T>
__device__ __forceinline__ Vec16<T> load16_nt(const T* p) {
  Vec16<T> r;
  r.raw = __builtin_bit_cast(uint4, __builtin_nontemporal_load(reinterpret_cast<const u32x4v*>(p)));
  return r;
}

template <typename T>
__device__ __forceinline__ void store16_nt(T* p, const Vec16<T>& r) {
  __builtin_nontemporal_store(__builtin_bit_cast(u32x4v, r.raw), reinterpret_cast<u32x4v*>(p));
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Block-wide sum for blockDim.x = NWAVES*64; `smem` needs NWAVES floats.
template <int NWAVES>
__device__ __forceinline__ float block_sum(float v, float* smem) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (NWAVES == 1) return v;
  __syncthreads();
  if (lane == 0) smem[wid] = v;
  __syncthreads();
  float t = 0.f;
#pragma unroll
  for (int i = 0; i < NWAVES; ++i) t += smem[i];
  return t;
}

template <int NWAVES>
__device__ __forceinline__ float block_max(float v, float* smem) {
  v = wave_max(v);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (NWAVES == 1) return v;
  __syncthreads();
  if (lane == 0) smem[wid] = v;
  __syncthreads();
  float t = -INFINITY;
#pragma unroll
  for (int i = 0; i < NWAVES; ++i) t = fmaxf(t, smem[i]);
  return t;
}

// XCD-aware bijective remap of a 1-D workgroup id (cdna_hip_programming.md §5 T1): consecutive
// logical tiles land on the same XCD (shared L2). Speed only, never correctness.
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  const int nxcd = 8;
  if (nwg < nxcd) return orig;
  const int q = nwg / nxcd, r = nwg % nxcd;
  const int xcd = orig % nxcd;
  const int base = (xcd < r) ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + orig / nxcd;
}

}  // namespace lta
