// Decode attention for small query counts (K3d): softmax(q k^T * scale + mask) v for T <= 16 query
// rows against a long key/value cache (incremental decoding with a static KV cache, HF/LitGPT
// "mask from a cache of masks" style), GQA, bool or no mask, optional top-left causal.
//
// Why not the flash kernel: with T = 1 an MFMA tile would be 97% padding; decode is bound by
// reading K/V once.  Layout of the work (wave64, CDNA4):
//   * one wave owns one query row (b, hq, t); a 256-thread block holds 4 rows with consecutive
//     hq, i.e. heads of the same KV group (GQA) -> the 4 waves stream the same K/V rows (L1/L2 hits);
//   * QK^T: lane l scores key j0+l (its K row read with 16-byte loads, q held in VGPRs as fp32);
//     a 64-key block whose mask is all-false is skipped before any K/V byte is read;
//   * online softmax with wave max/sum butterflies once per 64 keys;
//   * PV: lane l owns head dims {l} (D=64) or {2l, 2l+1} (D=128) -> every V row is one coalesced
//     128/256-byte wave load; p is broadcast from wave-private LDS;
//   * split-K over the cache (grid.y) when the cache is long: partial (m, l, acc) go to an fp32
//     workspace and a combine kernel merges them (flash-decoding).
#include "common.h"

namespace lta {
namespace {

constexpr int kRowsPerBlock = 4;

template <typename T, int D>
__global__ __launch_bounds__(256) void decode_attn_kernel(
    const T* __restrict__ q, const T* __restrict__ k, const T* __restrict__ v, const uint8_t* __restrict__ mask,
    T* __restrict__ o, float* __restrict__ ws_acc, float* __restrict__ ws_ml, int B, int Hq, int Hkv, int Tq, int S,
    int64_t qsb, int64_t qsh, int64_t qst, int64_t ksb, int64_t ksh, int64_t kss, int64_t vsb, int64_t vsh,
    int64_t vss, int64_t msb, int64_t msh, int64_t mst, int64_t mss, int chunk, int causal, float scale) {
  constexpr int DPL = D / 64;  // output dims per lane
  __shared__ float p_lds[kRowsPerBlock][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int rows = B * Tq * Hq;
  const int row = blockIdx.x * kRowsPerBlock + w;
  if (row >= rows) return;  // whole wave exits together (no block-level sync below)
  const int hq = row % Hq;
  const int t = (row / Hq) % Tq;
  const int b = row / (Hq * Tq);
  const int hk = hq / (Hq / Hkv);
  const int split = blockIdx.y;
  const int j_begin = split * chunk;
  int j_end = min(S, j_begin + chunk);
  if (causal) j_end = min(j_end, t + 1);

  // q row in fp32 registers (same address for all lanes: broadcast loads)
  float qf[D];
  const T* qrow = q + b * qsb + hq * qsh + t * qst;
#pragma unroll
  for (int d = 0; d < D; d += Vec16<T>::N) {
    Vec16<T> x = load16(qrow + d);
#pragma unroll
    for (int e = 0; e < Vec16<T>::N; ++e) qf[d + e] = to_f32(x.v[e]) * scale;
  }
  const T* kbase = k + b * ksb + hk * ksh;
  const T* vbase = v + b * vsb + hk * vsh;
  const uint8_t* mrow = mask ? mask + b * msb + hq * msh + t * mst : nullptr;

  float m = -INFINITY, l = 0.f;
  float acc[DPL];
#pragma unroll
  for (int i = 0; i < DPL; ++i) acc[i] = 0.f;

  for (int j0 = j_begin; j0 < j_end; j0 += 64) {
    const int j = j0 + lane;
    bool valid = j < j_end;
    if (valid && mrow) valid = mrow[(int64_t)j * mss] != 0;
    if (!__any(valid)) continue;
    float s = -INFINITY;
    if (valid) {
      const T* krow = kbase + (int64_t)j * kss;
      float dot = 0.f;
#pragma unroll
      for (int d = 0; d < D; d += Vec16<T>::N) {
        Vec16<T> x = load16(krow + d);
#pragma unroll
        for (int e = 0; e < Vec16<T>::N; ++e) dot = fmaf(qf[d + e], to_f32(x.v[e]), dot);
      }
      s = dot;
    }
    const float bm = wave_max(s);
    const float m_new = fmaxf(m, bm);
    const float p = valid ? __expf(s - m_new) : 0.f;
    const float corr = __expf(m - m_new);  // m = -inf on the first block -> 0
    l = l * corr + wave_sum(p);
#pragma unroll
    for (int i = 0; i < DPL; ++i) acc[i] *= corr;
    m = m_new;
    p_lds[w][lane] = p;
    __builtin_amdgcn_wave_barrier();
    const int nk = min(64, j_end - j0);
    for (int kk = 0; kk < nk; ++kk) {
      const float pk = p_lds[w][kk];
      if (pk == 0.f) continue;  // masked key (uniform across the wave)
      const T* vrow = vbase + (int64_t)(j0 + kk) * vss + lane * DPL;
      if (DPL == 2) {
        const uint32_t raw = *reinterpret_cast<const uint32_t*>(vrow);
        const T* pair = reinterpret_cast<const T*>(&raw);
        acc[0] = fmaf(pk, to_f32(pair[0]), acc[0]);
        acc[DPL - 1] = fmaf(pk, to_f32(pair[1]), acc[DPL - 1]);
      } else {
        acc[0] = fmaf(pk, to_f32(vrow[0]), acc[0]);
      }
    }
    __builtin_amdgcn_wave_barrier();
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
           hipStream_t stream) {
  const int rows = B * Tq * Hq;
  dim3 grid((rows + kRowsPerBlock - 1) / kRowsPerBlock, nsplit);
  hipLaunchKernelGGL((decode_attn_kernel<T, D>), grid, dim3(256), 0, stream, (const T*)q, (const T*)k, (const T*)v,
                     (const uint8_t*)mask, (T*)o, (float*)ws_acc, (float*)ws_ml, B, Hq, Hkv, Tq, S, st[0], st[1],
                     st[2], st[3], st[4], st[5], st[6], st[7], st[8], st[9], st[10], st[11], st[12], chunk, causal,
                     scale);
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
                               const int64_t* strides, int chunk, int nsplit, int causal, float scale, void* stream) {
  using namespace lta;
  hipStream_t s = (hipStream_t)stream;
  if (Hkv <= 0 || Hq % Hkv != 0 || chunk <= 0 || nsplit <= 0) return (int)hipErrorInvalidValue;
  if (dtype == kBF16) {
    if (D == 64) return launch<__hip_bfloat16, 64>(q, k, v, mask, o, ws_acc, ws_ml, B, Hq, Hkv, Tq, S, strides, chunk, nsplit, causal, scale, s);
    if (D == 128) return launch<__hip_bfloat16, 128>(q, k, v, mask, o, ws_acc, ws_ml, B, Hq, Hkv, Tq, S, strides, chunk, nsplit, causal, scale, s);
  } else if (dtype == kF16) {
    if (D == 64) return launch<__half, 64>(q, k, v, mask, o, ws_acc, ws_ml, B, Hq, Hkv, Tq, S, strides, chunk, nsplit, causal, scale, s);
    if (D == 128) return launch<__half, 128>(q, k, v, mask, o, ws_acc, ws_ml, B, Hq, Hkv, Tq, S, strides, chunk, nsplit, causal, scale, s);
  }
  return (int)hipErrorInvalidValue;
}
