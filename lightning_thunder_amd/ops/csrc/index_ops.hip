// Index / routing kernels (SURVEY K11 embedding backward, K12 topk / sort / argsort / cumsum /
// index_add).  The reference gets these from nvFuser / ATen (thunder/executors/nvfuserex_impl.py
// embedding, index_put, scatter, topk, argsort, cumsum); here they are small, deterministic CDNA4
// kernels:
//
//  * sort_rows: one 1024-thread workgroup per row sorts up to 16384 64-bit keys in LDS (128 KiB of
//    the 160 KiB) with a bitonic network.  Key = (order-preserving 32-bit image of the value) << 32
//    | position, so the sort is STABLE and ties resolve to the lower index on every run.
//  * topk_wave: MoE routing shape (rows of <= 2048 expert scores, small k): one wave per row, every
//    lane holds 64-bit keys in registers, k rounds of a 64-lane min-reduction.
//  * cumsum_rows: chunked workgroup scan (8 values per lane, 64-lane shuffle scan, per-wave
//    carries in LDS) with fp32 (float inputs) or int64 (integer inputs) accumulation.
//  * index_rows_sum: out[v] = base[v] + alpha * sum_{i: idx[i] == v} src[i] with the contributions of
//    each v summed in ascending i (the positions come from the stably sorted (idx, i) keys), so the
//    result is bitwise reproducible — no float atomics.  One workgroup per output row writes the
//    whole row (zeros where nothing lands), so no separate memset.  Embedding backward is this with
//    base = 0, padding_idx rows zeroed and optional 1/count scaling (scale_grad_by_freq).
#include "common.h"

namespace lta {
namespace {

enum : int { kI32 = 4, kI64 = 5 };
constexpr int kSortThreads = 1024;
constexpr int kSortMax = 16384;

// Order-preserving unsigned image of a value: a < b  <=>  okey(a) < okey(b).  -0 == +0 and every NaN
// is the canonical positive NaN, ordered above +inf (torch.sort / topk put NaN last / first).
__device__ __forceinline__ uint32_t okey_f(float v) {
  uint32_t b = __float_as_uint(v);
  if (v != v) b = 0x7fc00000u;
  if (v == 0.f) b = 0u;
  return b ^ ((b >> 31) ? 0xFFFFFFFFu : 0x80000000u);
}

template <typename T>
__device__ __forceinline__ uint32_t okey(const T* row, int i) {
  if constexpr (std::is_same<T, int32_t>::value)
    return (uint32_t)row[i] ^ 0x80000000u;
  else if constexpr (std::is_same<T, int64_t>::value)
    return (uint32_t)(int32_t)row[i] ^ 0x80000000u;  // host guarantees |v| < 2^31
  else
    return okey_f(to_f32(row[i]));
}

// bitonic sort of P (power of two) keys in LDS, ascending
__device__ __forceinline__ void bitonic_lds(uint64_t* keys, int P) {
  const int tid = threadIdx.x;
  for (int size = 2; size <= P; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int t = tid; t < (P >> 1); t += kSortThreads) {
        const int lo = 2 * t - (t & (stride - 1));
        const int hi = lo + stride;
        const bool up = (lo & size) == 0;
        const uint64_t a = keys[lo], b = keys[hi];
        if ((a > b) == up) {
          keys[lo] = b;
          keys[hi] = a;
        }
      }
      __syncthreads();
    }
  }
}

template <typename T, bool DESC>
__global__ __launch_bounds__(kSortThreads) void sort_rows_kernel(const T* __restrict__ x, int64_t ldx,
                                                                 T* __restrict__ vals, int64_t* __restrict__ idx,
                                                                 int N, int P, int k_out) {
  extern __shared__ uint64_t keys[];
  const T* row = x + (int64_t)blockIdx.x * ldx;
  for (int i = threadIdx.x; i < P; i += kSortThreads) {
    uint64_t key = ~0ull;  // padding sorts last
    if (i < N) {
      uint32_t o = okey(row, i);
      if (DESC) o = ~o;
      key = ((uint64_t)o << 32) | (uint32_t)i;
    }
    keys[i] = key;
  }
  __syncthreads();
  bitonic_lds(keys, P);
  for (int i = threadIdx.x; i < k_out; i += kSortThreads) {
    const int j = (int)(uint32_t)keys[i];
    if (vals) vals[(int64_t)blockIdx.x * k_out + i] = row[j];
    idx[(int64_t)blockIdx.x * k_out + i] = j;
  }
}

// int64 values: a 64-bit order key plus a separate 32-bit position (12 B per element, N <= 8192)
__global__ __launch_bounds__(kSortThreads) void sort_rows_i64_kernel(const int64_t* __restrict__ x, int64_t ldx,
                                                                     int64_t* __restrict__ vals,
                                                                     int64_t* __restrict__ idx, int N, int P, int k_out,
                                                                     int desc) {
  extern __shared__ uint64_t keys[];
  uint32_t* pos = reinterpret_cast<uint32_t*>(keys + P);
  const int64_t* row = x + (int64_t)blockIdx.x * ldx;
  for (int i = threadIdx.x; i < P; i += kSortThreads) {
    uint64_t k = ~0ull;
    if (i < N) {
      k = (uint64_t)row[i] ^ 0x8000000000000000ull;
      if (desc) k = ~k;
    }
    keys[i] = k;
    pos[i] = i < N ? (uint32_t)i : 0xFFFFFFFFu;
  }
  __syncthreads();
  const int tid = threadIdx.x;
  for (int size = 2; size <= P; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int t = tid; t < (P >> 1); t += kSortThreads) {
        const int lo = 2 * t - (t & (stride - 1));
        const int hi = lo + stride;
        const bool up = (lo & size) == 0;
        const uint64_t a = keys[lo], b = keys[hi];
        const uint32_t ia = pos[lo], ib = pos[hi];
        const bool gt = a > b || (a == b && ia > ib);
        if (gt == up) {
          keys[lo] = b;
          keys[hi] = a;
          pos[lo] = ib;
          pos[hi] = ia;
        }
      }
      __syncthreads();
    }
  }
  for (int i = threadIdx.x; i < k_out; i += kSortThreads) {
    const int j = (int)pos[i];
    if (vals) vals[(int64_t)blockIdx.x * k_out + i] = row[j];
    idx[(int64_t)blockIdx.x * k_out + i] = j;
  }
}

// keys_out[i] = (idx[i] << 32 | i) sorted ascending: the (row, position) order of an index_add
__global__ __launch_bounds__(kSortThreads) void sort_index_keys_kernel(const int64_t* __restrict__ index, int n,
                                                                       int P, uint64_t* __restrict__ keys_out) {
  extern __shared__ uint64_t keys[];
  for (int i = threadIdx.x; i < P; i += kSortThreads)
    keys[i] = i < n ? (((uint64_t)(uint32_t)index[i] << 32) | (uint32_t)i) : ~0ull;
  __syncthreads();
  bitonic_lds(keys, P);
  for (int i = threadIdx.x; i < n; i += kSortThreads) keys_out[i] = keys[i];
}

template <typename T, int NV, bool LARGEST>
__global__ __launch_bounds__(256) void topk_wave_kernel(const T* __restrict__ x, int64_t ldx, T* __restrict__ vals,
                                                        int64_t* __restrict__ idx, int R, int N, int k) {
  const int lane = threadIdx.x & 63;
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= R) return;  // whole waves exit together
  const T* row = x + (int64_t)r * ldx;
  uint64_t key[NV];
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    const int i = lane + 64 * j;
    uint64_t kk = ~0ull;
    if (i < N) {
      uint32_t o = okey(row, i);
      if (LARGEST) o = ~o;
      kk = ((uint64_t)o << 32) | (uint32_t)i;
    }
    key[j] = kk;
  }
  for (int s = 0; s < k; ++s) {
    uint64_t best = key[0];
#pragma unroll
    for (int j = 1; j < NV; ++j) best = key[j] < best ? key[j] : best;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const uint64_t other = __shfl_xor(best, o, 64);
      best = other < best ? other : best;
    }
    const int win = (int)(uint32_t)best;
    // static-index select keeps key[] in VGPRs (a dynamic key[win >> 6] would go to scratch)
#pragma unroll
    for (int j = 0; j < NV; ++j)
      if (j == (win >> 6) && (win & 63) == lane) key[j] = ~0ull;
    if (lane == 0) {
      vals[(int64_t)r * k + s] = row[win];
      idx[(int64_t)r * k + s] = win;
    }
  }
}

template <typename T, typename ACC, typename OUT>
__global__ __launch_bounds__(256) void cumsum_rows_kernel(const T* __restrict__ x, int64_t ldx, OUT* __restrict__ y,
                                                          int64_t N) {
  __shared__ ACC wsum[4];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const T* row = x + (int64_t)blockIdx.x * ldx;
  OUT* out = y + (int64_t)blockIdx.x * N;
  ACC carry = 0;
  for (int64_t base = 0; base < N; base += 256 * 8) {
    ACC v[8];
    const int64_t i0 = base + tid * 8;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      ACC a = 0;
      if (i0 + e < N) {
        if constexpr (std::is_same<ACC, float>::value)
          a = to_f32(row[i0 + e]);
        else
          a = (ACC)row[i0 + e];
      }
      v[e] = e ? v[e - 1] + a : a;
    }
    const ACC tot = v[7];
    ACC s = tot;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const ACC t = __shfl_up(s, o, 64);
      if (lane >= o) s += t;
    }
    if (lane == 63) wsum[wid] = s;
    __syncthreads();
    ACC woff = 0, all = 0;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      if (w < wid) woff += wsum[w];
      all += wsum[w];
    }
    const ACC excl = carry + woff + (s - tot);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      if (i0 + e < N) {
        if constexpr (std::is_same<ACC, float>::value)
          out[i0 + e] = from_f32<OUT>(v[e] + excl);
        else
          out[i0 + e] = (OUT)(v[e] + excl);
      }
    }
    carry += all;
    __syncthreads();
  }
}

template <typename T>
__global__ __launch_bounds__(256) void index_rows_sum_kernel(const T* __restrict__ src, int64_t lds,
                                                             const uint64_t* __restrict__ keys, int n,
                                                             const T* __restrict__ base, int64_t ldb,
                                                             T* __restrict__ out, int64_t ldo, int64_t V, int64_t D,
                                                             int64_t padding_idx, int scale_by_freq, float alpha) {
  constexpr int VEC = Vec16<T>::N;
  const int64_t v = (int64_t)blockIdx.y * gridDim.x + blockIdx.x;
  if (v >= V) return;
  // first sorted key of row v
  int lo = 0, hi = n;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if ((int64_t)(keys[mid] >> 32) < v)
      lo = mid + 1;
    else
      hi = mid;
  }
  int end = lo;
  while (end < n && (int64_t)(keys[end] >> 32) == v) ++end;
  const bool skip = v == padding_idx;
  const float sc = alpha * ((scale_by_freq && end > lo) ? 1.f / (float)(end - lo) : 1.f);
  for (int64_t d0 = (int64_t)threadIdx.x * VEC; d0 < D; d0 += 256 * VEC) {
    float acc[VEC];
#pragma unroll
    for (int e = 0; e < VEC; ++e) acc[e] = 0.f;
    if (!skip) {
      for (int j = lo; j < end; ++j) {
        const int64_t pos = (uint32_t)keys[j];
        const Vec16<T> g = load16(src + pos * lds + d0);
#pragma unroll
        for (int e = 0; e < VEC; ++e) acc[e] += to_f32(g.v[e]);
      }
    }
    Vec16<T> o;
    if (base) {
      const Vec16<T> b = load16(base + v * ldb + d0);
#pragma unroll
      for (int e = 0; e < VEC; ++e) o.v[e] = from_f32<T>(to_f32(b.v[e]) + sc * acc[e]);
    } else {
#pragma unroll
      for (int e = 0; e < VEC; ++e) o.v[e] = from_f32<T>(sc * acc[e]);
    }
    store16(out + v * ldo + d0, o);
  }
}

int pow2_at_least(int n) {
  int p = 1;
  while (p < n) p <<= 1;
  return p;
}

template <typename T, bool DESC>
int launch_sort(const void* x, int64_t ldx, void* vals, void* idx, int R, int N, int k_out, hipStream_t s) {
  const int P = pow2_at_least(N < 2 ? 2 : N);
  const size_t lds = (size_t)P * sizeof(uint64_t);
  auto* fn = sort_rows_kernel<T, DESC>;
  hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL(fn, dim3(R), dim3(kSortThreads), lds, s, (const T*)x, ldx, (T*)vals, (int64_t*)idx, N, P, k_out);
  return (int)hipGetLastError();
}

template <typename T>
int dispatch_sort(const void* x, int64_t ldx, void* vals, void* idx, int R, int N, int k_out, int desc,
                  hipStream_t s) {
  return desc ? launch_sort<T, true>(x, ldx, vals, idx, R, N, k_out, s)
              : launch_sort<T, false>(x, ldx, vals, idx, R, N, k_out, s);
}

template <typename T, bool L>
int launch_topk(const void* x, int64_t ldx, void* vals, void* idx, int R, int N, int k, hipStream_t s) {
  const dim3 grid((R + 3) / 4), block(256);
#define LTA_TOPK(NV)                                                                                       \
  hipLaunchKernelGGL((topk_wave_kernel<T, NV, L>), grid, block, 0, s, (const T*)x, ldx, (T*)vals, (int64_t*)idx, \
                     R, N, k)
  if (N <= 64)
    LTA_TOPK(1);
  else if (N <= 128)
    LTA_TOPK(2);
  else if (N <= 256)
    LTA_TOPK(4);
  else if (N <= 512)
    LTA_TOPK(8);
  else if (N <= 1024)
    LTA_TOPK(16);
  else
    LTA_TOPK(32);
#undef LTA_TOPK
  return (int)hipGetLastError();
}

template <typename T>
int dispatch_topk(const void* x, int64_t ldx, void* vals, void* idx, int R, int N, int k, int largest, hipStream_t s) {
  return largest ? launch_topk<T, true>(x, ldx, vals, idx, R, N, k, s)
                 : launch_topk<T, false>(x, ldx, vals, idx, R, N, k, s);
}

}  // namespace
}  // namespace lta

using namespace lta;

LTA_EXPORT int lta_sort_max() { return kSortMax; }

// Stable sort of R rows of N (<= 16384; int64: <= 8192) values (row stride ldx elements); writes the first k_out
// sorted values (vals may be null) and their int64 positions, [R, k_out] contiguous.
LTA_EXPORT int lta_sort_rows(int dtype, const void* x, int64_t ldx, void* vals, void* idx, int R, int N, int k_out,
                             int desc, hipStream_t s) {
  if (R < 1 || N < 1 || N > kSortMax || k_out < 1 || k_out > N) return (int)hipErrorInvalidValue;
  switch (dtype) {
    case kF32: return dispatch_sort<float>(x, ldx, vals, idx, R, N, k_out, desc, s);
    case kF16: return dispatch_sort<__half>(x, ldx, vals, idx, R, N, k_out, desc, s);
    case kBF16: return dispatch_sort<__hip_bfloat16>(x, ldx, vals, idx, R, N, k_out, desc, s);
    case kI32: return dispatch_sort<int32_t>(x, ldx, vals, idx, R, N, k_out, desc, s);
    case kI64: {
      if (N > kSortMax / 2) return (int)hipErrorInvalidValue;
      const int P = pow2_at_least(N < 2 ? 2 : N);
      const size_t lds = (size_t)P * (sizeof(uint64_t) + sizeof(uint32_t));
      hipFuncSetAttribute((const void*)sort_rows_i64_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      hipLaunchKernelGGL(sort_rows_i64_kernel, dim3(R), dim3(kSortThreads), lds, s, (const int64_t*)x, ldx,
                         (int64_t*)vals, (int64_t*)idx, N, P, k_out, desc);
      return (int)hipGetLastError();
    }
    default: return (int)hipErrorInvalidValue;
  }
}

// Top-k of R rows of N <= 2048 values, k <= N: vals [R, k] (input dtype), idx [R, k] int64, sorted.
LTA_EXPORT int lta_topk_rows(int dtype, const void* x, int64_t ldx, void* vals, void* idx, int R, int N, int k,
                             int largest, hipStream_t s) {
  if (R < 1 || N < 1 || N > 2048 || k < 1 || k > N) return (int)hipErrorInvalidValue;
  switch (dtype) {
    case kF32: return dispatch_topk<float>(x, ldx, vals, idx, R, N, k, largest, s);
    case kF16: return dispatch_topk<__half>(x, ldx, vals, idx, R, N, k, largest, s);
    case kBF16: return dispatch_topk<__hip_bfloat16>(x, ldx, vals, idx, R, N, k, largest, s);
    case kI32: return dispatch_topk<int32_t>(x, ldx, vals, idx, R, N, k, largest, s);
    default: return (int)hipErrorInvalidValue;
  }
}

// Inclusive scan of R rows of N values (row stride ldx) into y [R, N] contiguous.  Float inputs
// accumulate in fp32 and keep their dtype; int32 / int64 inputs accumulate in int64 and store
// int64, or int32 when out_i32 (torch.cumsum(..., dtype=torch.int32), MoE routing offsets).
LTA_EXPORT int lta_cumsum_rows(int dtype, const void* x, int64_t ldx, void* y, int R, int64_t N, int out_i32,
                               hipStream_t s) {
  if (R < 1 || N < 1) return (int)hipErrorInvalidValue;
  const dim3 grid(R), block(256);
  if (out_i32) {
    if (dtype == kI32)
      hipLaunchKernelGGL((cumsum_rows_kernel<int32_t, int64_t, int32_t>), grid, block, 0, s, (const int32_t*)x, ldx,
                         (int32_t*)y, N);
    else if (dtype == kI64)
      hipLaunchKernelGGL((cumsum_rows_kernel<int64_t, int64_t, int32_t>), grid, block, 0, s, (const int64_t*)x, ldx,
                         (int32_t*)y, N);
    else
      return (int)hipErrorInvalidValue;
    return (int)hipGetLastError();
  }
  switch (dtype) {
    case kF32:
      hipLaunchKernelGGL((cumsum_rows_kernel<float, float, float>), grid, block, 0, s, (const float*)x, ldx, (float*)y, N);
      break;
    case kF16:
      hipLaunchKernelGGL((cumsum_rows_kernel<__half, float, __half>), grid, block, 0, s, (const __half*)x, ldx,
                         (__half*)y, N);
      break;
    case kBF16:
      hipLaunchKernelGGL((cumsum_rows_kernel<__hip_bfloat16, float, __hip_bfloat16>), grid, block, 0, s,
                         (const __hip_bfloat16*)x, ldx, (__hip_bfloat16*)y, N);
      break;
    case kI32:
      hipLaunchKernelGGL((cumsum_rows_kernel<int32_t, int64_t, int64_t>), grid, block, 0, s, (const int32_t*)x, ldx,
                         (int64_t*)y, N);
      break;
    case kI64:
      hipLaunchKernelGGL((cumsum_rows_kernel<int64_t, int64_t, int64_t>), grid, block, 0, s, (const int64_t*)x, ldx,
                         (int64_t*)y, N);
      break;
    default: return (int)hipErrorInvalidValue;
  }
  return (int)hipGetLastError();
}

// keys [n] = sort_ascending(index[i] << 32 | i) for 0 <= index < 2^31, n <= 16384.
LTA_EXPORT int lta_sort_index_keys(const void* index, int n, void* keys, hipStream_t s) {
  if (n < 1 || n > kSortMax) return (int)hipErrorInvalidValue;
  const int P = pow2_at_least(n < 2 ? 2 : n);
  const size_t lds = (size_t)P * sizeof(uint64_t);
  hipFuncSetAttribute((const void*)sort_index_keys_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL(sort_index_keys_kernel, dim3(1), dim3(kSortThreads), lds, s, (const int64_t*)index, n, P,
                     (uint64_t*)keys);
  return (int)hipGetLastError();
}

// out[v, :] = base[v, :] (or 0) + alpha * sum over sorted keys of row v of src[pos, :]   (v < V)
// rows of D elements, D % (16 / sizeof(T)) == 0, 16-byte aligned rows; padding_idx row (if >= 0)
// gets no contributions; scale_by_freq divides a row's sum by its count.
LTA_EXPORT int lta_index_rows_sum(int dtype, const void* src, int64_t lds, const void* keys, int n, const void* base,
                                  int64_t ldb, void* out, int64_t ldo, int64_t V, int64_t D, int64_t padding_idx,
                                  int scale_by_freq, float alpha, hipStream_t s) {
  if (V < 1 || D < 1 || n < 0) return (int)hipErrorInvalidValue;
  const int64_t gx = V < 65536 ? V : 65536;
  const dim3 grid((unsigned)gx, (unsigned)((V + gx - 1) / gx)), block(256);
#define LTA_IRS(T)                                                                                              \
  hipLaunchKernelGGL(index_rows_sum_kernel<T>, grid, block, 0, s, (const T*)src, lds, (const uint64_t*)keys, n, \
                     (const T*)base, ldb, (T*)out, ldo, V, D, padding_idx, scale_by_freq, alpha)
  switch (dtype) {
    case kF32:
      if (D % 4) return (int)hipErrorInvalidValue;
      LTA_IRS(float);
      break;
    case kF16:
      if (D % 8) return (int)hipErrorInvalidValue;
      LTA_IRS(__half);
      break;
    case kBF16:
      if (D % 8) return (int)hipErrorInvalidValue;
      LTA_IRS(__hip_bfloat16);
      break;
    default: return (int)hipErrorInvalidValue;
  }
#undef LTA_IRS
  return (int)hipGetLastError();
}

// Graph-safe RNG (core/rng.py): the two int64 words [seed, Philox base] a captured region's kernels read,
// written stream-ordered right before the graph's replay (lane 0 stores from vector registers).
namespace {
__global__ __launch_bounds__(64) void store_i64x2_kernel(long long* __restrict__ p, long long a, long long b) {
  if (threadIdx.x == 0) {
    const longlong2 v = make_longlong2(a, b);
    *reinterpret_cast<longlong2*>(p) = v;
  }
}
}  // namespace

LTA_EXPORT int lta_store_i64x2(void* p, long long a, long long b, hipStream_t s) {
  if (!p || ((uintptr_t)p & 15)) return -2;
  hipLaunchKernelGGL(store_i64x2_kernel, dim3(1), dim3(64), 0, s, (long long*)p, a, b);
  return (int)hipGetLastError();
}
