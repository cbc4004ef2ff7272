// Decode attention for small query counts (K3d): softmax(q k^T * scale + mask) v for T <= 16 query
// rows against a long key/value cache (incremental decoding with a static KV cache, HF/LitGPT
// "mask from a cache of masks" style), GQA, bool or no mask, optional top-left causal.
//
// Why not the flash kernel: with T = 1 an MFMA tile would be 97% padding; decode is bound by
// reading K/V once.  Layout of the work (wave64, CDNA4):
//   * one wave owns one query row (b, hq, t); a 256-thread block holds 4 rows with consecutive
//     hq, i.e. heads of the same KV group (GQA) -> the 4 waves stream the same K/V rows (L1/L2 hits);
//   * lane l owns key j0+l of each 64-key block for both products: QK^T reads its K row with
//     16-byte loads against q broadcast from LDS, PV accumulates p * V-row into a per-lane
//     acc[D] (no serial per-key loop); a block whose mask is all-false is skipped before any
//     K/V byte is read;
//   * online softmax with wave max/sum butterflies once per 64 keys;
//   * the per-lane partial outputs are combined once per row by a recursive-halving
//     reduce-scatter of shuffles (D/2 + D/4 + ... + D/64 of them), leaving each lane D/64
//     contiguous output dims;
//   * split-K over the cache (grid.y) when the cache is long: partial (m, l, acc) go to an fp32
//     workspace and a combine kernel merges them (flash-decoding).
#include "common.h"

namespace lta {
namespace {

constexpr int kRowsPerBlock = 4;

// WSPLIT (few rows, e.g. batch-1 decode: 32 rows would occupy 8 CUs): one row per block, the 4
// waves take interleaved 64-key blocks of the row's range and merge their (m, l, acc) through LDS,
// so a row's serial key loop is 4x shorter without a second launch.
template <typename T, int D, bool WSPLIT>
__global__ __launch_bounds__(256) void decode_attn_kernel(
    const T* __restrict__ q, const T* __restrict__ k, const T* __restrict__ v, const uint8_t* __restrict__ mask,
    T* __restrict__ o, float* __restrict__ ws_acc, float* __restrict__ ws_ml, int B, int Hq, int Hkv, int Tq, int S,
    int64_t qsb, int64_t qsh, int64_t qst, int64_t ksb, int64_t ksh, int64_t kss, int64_t vsb, int64_t vsh,
    int64_t vss, int64_t msb, int64_t msh, int64_t mst, int64_t mss, int chunk, int causal, float scale) {
  constexpr int DPL = D / 64;          // output dims per lane after the final reduce-scatter
  constexpr int NV = Vec16<T>::N;      // elements per 16-byte load
  __shared__ float q_lds[kRowsPerBlock][D];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int rows = B * Tq * Hq;
  const int row = WSPLIT ? blockIdx.x : blockIdx.x * kRowsPerBlock + w;
  if (!WSPLIT && row >= rows) return;  // whole wave exits together (no block-level sync below)
  const int hq = row % Hq;
  const int t = (row / Hq) % Tq;
  const int b = row / (Hq * Tq);
  const int hk = hq / (Hq / Hkv);
  const int split = blockIdx.y;
  const int j_begin = split * chunk;
  int j_end = min(S, j_begin + chunk);
  if (causal) j_end = min(j_end, t + 1);

  // scaled q row -> wave-private LDS (read back as broadcasts)
  const T* qrow = q + b * qsb + hq * qsh + t * qst;
  for (int d = lane; d < D; d += 64) q_lds[w][d] = to_f32(qrow[d]) * scale;
  __builtin_amdgcn_wave_barrier();
  const T* kbase = k + b * ksb + hk * ksh;
  const T* vbase = v + b * vsb + hk * vsh;
  const uint8_t* mrow = mask ? mask + b * msb + hq * msh + t * mst : nullptr;

  // every lane owns one key per 64-key block: QK and PV are both lane-parallel; the per-lane
  // partial outputs acc[D] are reduce-scattered across the wave once at the end.
  float m = -INFINITY, l = 0.f;
  float acc[D];
#pragma unroll
  for (int i = 0; i < D; ++i) acc[i] = 0.f;

  for (int j0 = j_begin + (WSPLIT ? w * 64 : 0); j0 < j_end; j0 += (WSPLIT ? kRowsPerBlock * 64 : 64)) {
    const int j = j0 + lane;
    bool valid = j < j_end;
    if (valid && mrow) valid = mrow[(int64_t)j * mss] != 0;
    if (!__any(valid)) continue;  // fully masked block: no K/V traffic
    float s = -INFINITY;
    if (valid) {
      const T* krow = kbase + (int64_t)j * kss;
      float dot = 0.f;
#pragma unroll
      for (int d = 0; d < D; d += NV) {
        Vec16<T> x = load16(krow + d);
#pragma unroll
        for (int e = 0; e < NV; ++e) dot = fmaf(q_lds[w][d + e], to_f32(x.v[e]), dot);
      }
      s = dot;
    }
    const float m_new = fmaxf(m, wave_max(s));
    const float p = valid ? __expf(s - m_new) : 0.f;
    const float corr = __expf(m - m_new);  // m = -inf on the first block -> 0
    l = l * corr + wave_sum(p);
    m = m_new;
    if (valid) {
      const T* vrow = vbase + (int64_t)j * vss;
#pragma unroll
      for (int d = 0; d < D; d += NV) {
        Vec16<T> x = load16(vrow + d);
#pragma unroll
        for (int e = 0; e < NV; ++e) acc[d + e] = fmaf(p, to_f32(x.v[e]), acc[d + e] * corr);
      }
    } else {
#pragma unroll
      for (int i = 0; i < D; ++i) acc[i] *= corr;
    }
  }

  // recursive-halving reduce-scatter over the 64 lanes: lane ends with dims [lane*DPL, lane*DPL+DPL)
#pragma unroll
  for (int off = 32, n = D; off >= 1; off >>= 1, n >>= 1) {
    const bool upper = (lane & off) != 0;
    const int half = n >> 1;
#pragma unroll
    for (int i = 0; i < half; ++i) {
      const float give = upper ? acc[i] : acc[half + i];
      const float keep = upper ? acc[half + i] : acc[i];
      acc[i] = keep + __shfl_xor(give, off, 64);
    }
  }

  if constexpr (WSPLIT) {
    __shared__ float c_acc[kRowsPerBlock][D];
    __shared__ float c_ml[kRowsPerBlock][2];
#pragma unroll
    for (int i = 0; i < DPL; ++i) c_acc[w][lane * DPL + i] = acc[i];
    if (lane == 0) {
      c_ml[w][0] = m;
      c_ml[w][1] = l;
    }
    __syncthreads();
    if (w != 0) return;
    float M = -INFINITY;
#pragma unroll
    for (int u = 0; u < kRowsPerBlock; ++u) M = fmaxf(M, c_ml[u][0]);
    float L = 0.f;
#pragma unroll
    for (int i = 0; i < DPL; ++i) acc[i] = 0.f;
#pragma unroll
    for (int u = 0; u < kRowsPerBlock; ++u) {
      const float c = c_ml[u][0] == -INFINITY ? 0.f : __expf(c_ml[u][0] - M);
      L = fmaf(c, c_ml[u][1], L);
#pragma unroll
      for (int i = 0; i < DPL; ++i) acc[i] = fmaf(c, c_acc[u][lane * DPL + i], acc[i]);
    }
    m = M;
    l = L;
  }

  if (gridDim.y == 1) {
    const float inv = 1.f / l;  // fully masked row -> 0 * inf = nan, like PyTorch SDPA
    T* orow = o + (((int64_t)b * Hq + hq) * Tq + t) * D + lane * DPL;  // o is [B, Hq, Tq, D]
#pragma unroll
    for (int i = 0; i < DPL; ++i) orow[i] = from_f32<T>(acc[i] * inv);
  } else {
    float* wa = ws_acc + ((int64_t)split * rows + row) * D + lane * DPL;
#pragma unroll
    for (int i = 0; i < DPL; ++i) wa[i] = acc[i];
    if (lane == 0) {
      ws_ml[((int64_t)split * rows + row) * 2 + 0] = m;
      ws_ml[((int64_t)split * rows + row) * 2 + 1] = l;
    }
  }
}

template <typename T, int D>
__global__ __launch_bounds__(64) void decode_attn_combine_kernel(const float* __restrict__ ws_acc,
                                                                 const float* __restrict__ ws_ml, T* __restrict__ o,
                                                                 int rows, int nsplit, int Hq, int Tq) {
  constexpr int DPL = D / 64;
  const int row = blockIdx.x, lane = threadIdx.x;
  const int hq = row % Hq, t = (row / Hq) % Tq, b = row / (Hq * Tq);
  float M = -INFINITY;
  for (int s = 0; s < nsplit; ++s) M = fmaxf(M, ws_ml[((int64_t)s * rows + row) * 2]);
  float L = 0.f, acc[DPL];
#pragma unroll
  for (int i = 0; i < DPL; ++i) acc[i] = 0.f;
  for (int s = 0; s < nsplit; ++s) {
    const float ms = ws_ml[((int64_t)s * rows + row) * 2];
    if (ms == -INFINITY) continue;
    const float c = __expf(ms - M);
    L += c * ws_ml[((int64_t)s * rows + row) * 2 + 1];
    const float* wa = ws_acc + ((int64_t)s * rows + row) * D + lane * DPL;
#pragma unroll
    for (int i = 0; i < DPL; ++i) acc[i] = fmaf(c, wa[i], acc[i]);
  }
  const float inv = 1.f / L;
  T* orow = o + (((int64_t)b * Hq + hq) * Tq + t) * D + lane * DPL;
#pragma unroll
  for (int i = 0; i < DPL; ++i) orow[i] = from_f32<T>(acc[i] * inv);
}

template <typename T, int D>
int launch(const void* q, const void* k, const void* v, const void* mask, void* o, void* ws_acc, void* ws_ml, int B,
           int Hq, int Hkv, int Tq, int S, const int64_t* st, int chunk, int nsplit, int causal, float scale,
           int wsplit, hipStream_t stream) {
  const int rows = B * Tq * Hq;
  if (wsplit) {
    hipLaunchKernelGGL((decode_attn_kernel<T, D, true>), dim3(rows, nsplit), dim3(256), 0, stream, (const T*)q,
                       (const T*)k, (const T*)v, (const uint8_t*)mask, (T*)o, (float*)ws_acc, (float*)ws_ml, B, Hq, Hkv,
                       Tq, S, st[0], st[1], st[2], st[3], st[4], st[5], st[6], st[7], st[8], st[9], st[10], st[11],
                       st[12], chunk, causal, scale);
  } else {
    dim3 grid((rows + kRowsPerBlock - 1) / kRowsPerBlock, nsplit);
    hipLaunchKernelGGL((decode_attn_kernel<T, D, false>), grid, dim3(256), 0, stream, (const T*)q, (const T*)k,
                       (const T*)v, (const uint8_t*)mask, (T*)o, (float*)ws_acc, (float*)ws_ml, B, Hq, Hkv, Tq, S,
                       st[0], st[1], st[2], st[3], st[4], st[5], st[6], st[7], st[8], st[9], st[10], st[11], st[12],
                       chunk, causal, scale);
  }
  if (nsplit > 1)
    hipLaunchKernelGGL((decode_attn_combine_kernel<T, D>), dim3(rows), dim3(64), 0, stream, (const float*)ws_acc,
                       (const float*)ws_ml, (T*)o, rows, nsplit, Hq, Tq);
  return (int)hipGetLastError();
}

}  // namespace
}  // namespace lta

// strides (elements): q b,h,t | k b,h,s | v b,h,s | mask b,h,t,s (0 for broadcast dims); head dim contiguous.
LTA_EXPORT int lta_decode_attn(int dtype, const void* q, const void* k, const void* v, const void* mask, void* o,
                               void* ws_acc, void* ws_ml, int B, int Hq, int Hkv, int Tq, int S, int D,
                               const int64_t* strides, int chunk, int nsplit, int causal, float scale, int wsplit,
                               void* stream) {
  using namespace lta;
  hipStream_t s = (hipStream_t)stream;
  if (Hkv <= 0 || Hq % Hkv != 0 || chunk <= 0 || nsplit <= 0) return (int)hipErrorInvalidValue;
  if (dtype == kBF16) {
    if (D == 64) return launch<__hip_bfloat16, 64>(q, k, v, mask, o, ws_acc, ws_ml, B, Hq, Hkv, Tq, S, strides, chunk, nsplit, causal, scale, wsplit, s);
    if (D == 128) return launch<__hip_bfloat16, 128>(q, k, v, mask, o, ws_acc, ws_ml, B, Hq, Hkv, Tq, S, strides, chunk, nsplit, causal, scale, wsplit, s);
  } else if (dtype == kF16) {
    if (D == 64) return launch<__half, 64>(q, k, v, mask, o, ws_acc, ws_ml, B, Hq, Hkv, Tq, S, strides, chunk, nsplit, causal, scale, wsplit, s);
    if (D == 128) return launch<__half, 128>(q, k, v, mask, o, ws_acc, ws_ml, B, Hq, Hkv, Tq, S, strides, chunk, nsplit, causal, scale, wsplit, s);
  }
  return (int)hipErrorInvalidValue;
}
