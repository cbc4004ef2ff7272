// Skinny GEMM for decode (K2b): y[M, N] = act(x[M, K] @ w[N, K]^T + bias) + residual for M <= 8
// activation rows (batch-1..8 incremental decoding, LM head on the last position).
//
// Why not the MFMA GEMM / hipBLASLt: at M = 1 the problem is a weight stream (Llama-3.2-1B:
// 8-67 MB per projection) and a library tile of 16 x 16 leaves most of the chip idle or
// serialises K.  Layout (cdna_hip_programming.md §5 "GEMV / M <= 16": straight to VGPRs, deep
// unroll, late vmcnt):
//   * a 256-thread block owns kRows = 8 consecutive output columns (rows of w); its 4 waves split
//     K, lane l reading the 16-byte piece [k0 + 8 l, k0 + 8 l + 8) of all 8 weight rows at once
//     (8 x 1 KiB fully coalesced row segments per wave step; up to 4 steps' rows requested before
//     the first FMA -> up to 32 loads in flight per lane);
//   * x (<= 8 rows, L2-resident, shared by every block) is read with the same 16-byte pieces;
//   * the M x 8 per-lane partial dots are combined by a recursive-halving reduce-scatter of
//     shuffles (V/2 + V/4 + ... shuffles for V values instead of 6 V for V butterflies), then
//     across the 4 waves through 1 KiB of LDS; bias / activation / residual are applied by the
//     V threads that write the outputs.
// Grid = ceil(N / 8) blocks (N / 4 gated): >= 256 for every projection of a 1B+ model (N >= 2048).
#include "common.h"

namespace lta {
namespace {

constexpr int kRows = 8;
constexpr int kWaves = 4;
constexpr int kStep = 64 * 8;  // K elements per wave step (8 x 16-bit per lane)

__device__ __forceinline__ float gemv_act(float v, int act) {
  switch (act) {
    case 1: {  // gelu (tanh approximation)
      const float u = 0.7978845608028654f * (v + 0.044715f * v * v * v);
      return 0.5f * v * (1.f + tanhf(u));
    }
    case 2:
      return 0.5f * v * (1.f + erff(v * 0.7071067811865476f));
    case 3:
      return v / (1.f + __expf(-v));
    case 4:
      return fmaxf(v, 0.f);
    default:
      return v;
  }
}

template <int V>
struct Log2 {
  static constexpr int value = 1 + Log2<V / 2>::value;
};
template <>
struct Log2<1> {
  static constexpr int value = 0;
};

// NORM: x is replaced by rmsnorm(x) * g (the row's rstd computed per wave from the L2-resident x
//   rows, so no block barrier sits in front of the weight loads); normalized values are rounded to
//   T exactly as the stand-alone rmsnorm kernel would store them.
// GATED: the block streams 4 rows of w and the same 4 rows of w2 and writes act(x w^T) * (x w2^T)
//   (SwiGLU / GeGLU: the two up-projections and the gate in one launch); both products are
//   rounded to T first, as the unfused linear -> swiglu chain stores them.
// GROUP: up to 3 projections of the same x (e.g. attention q / k / v, each with its own weight and
// output) in one launch; blocks [0, b0) compute segment 0, [b0, b0 + b1) segment 1, the rest 2.
struct GemvGroup {
  const void* w[3];
  void* y[3];
  int n[3];
  int blocks[2];
  int64_t ldw[3], ldy[3];
};

template <typename T, int MM, bool NORM, bool GATED, int U, int KR, bool GROUP = false>
__global__ __launch_bounds__(256) void gemv_kernel(const T* __restrict__ x, const T* __restrict__ w_,
                                                   const T* __restrict__ w2, const T* __restrict__ g, float eps,
                                                   const T* __restrict__ bias, const T* __restrict__ res,
                                                   T* __restrict__ y_, int M, int N_, int K, int64_t ldx, int64_t ldw_,
                                                   int64_t ldy_, int64_t ldr, int act, GemvGroup grp = GemvGroup{}) {
  constexpr int V = MM * KR;  // partial sums per lane (power of two, <= 64)
  constexpr int LOGV = Log2<V>::value;
  constexpr int NV = Vec16<T>::N;
  constexpr int COLS = GATED ? KR / 2 : KR;  // output columns per block
  static_assert(V <= 64 && (V & (V - 1)) == 0, "V must be a power of two <= 64");
  __shared__ float part[kWaves][V];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const T* w = w_;
  T* y = y_;
  int N = N_;
  int64_t ldw = ldw_, ldy = ldy_;
  int blk = blockIdx.x;
  if constexpr (GROUP) {
    int sg = 0;
    if (blk >= grp.blocks[0]) {
      blk -= grp.blocks[0];
      sg = 1;
      if (blk >= grp.blocks[1]) {
        blk -= grp.blocks[1];
        sg = 2;
      }
    }
    w = (const T*)grp.w[sg];
    y = (T*)grp.y[sg];
    N = grp.n[sg];
    ldw = grp.ldw[sg];
    ldy = grp.ldy[sg];
  }
  const int n0 = blk * COLS;

  const T* wrow[KR];
#pragma unroll
  for (int r = 0; r < KR; ++r) {
    const int c = GATED ? (r % COLS) : r;
    const T* base = (GATED && r >= COLS) ? w2 : w;
    wrow[r] = base + (int64_t)min(n0 + c, N - 1) * ldw;  // clamp: read valid rows, never write them
  }

  // Loads are issued a group of U wave-steps at a time, x pieces first and then every weight row
  // piece of the group (vmcnt retires in order: waiting for x never waits for the weights), so up
  // to U * KR 16-byte weight loads per lane are in flight before the first FMA.  U is chosen
  // per launch from K (a group covers the whole row when it can) within the VGPR budget.
  constexpr int kStride = kWaves * kStep;
  const int kbase = wv * kStep + lane * NV;
  const int steps = (K + kStride - 1) / kStride;
  __shared__ float ss_part[kWaves][MM];

  float rstd[MM];
#pragma unroll
  for (int m = 0; m < MM; ++m) rstd[m] = 1.f;
  // NORM with more steps than one group holds: row statistics up front (K > U * 2048 only)
  if (NORM && steps > U) {
#pragma unroll
    for (int m = 0; m < MM; ++m) {
      float ss = 0.f;
      if (m < M) {
        for (int kk = lane * NV; kk < K; kk += 64 * NV) {
          const Vec16<T> xv = load16(x + (int64_t)m * ldx + kk);
#pragma unroll
          for (int e = 0; e < NV; ++e) {
            const float f = to_f32(xv.v[e]);
            ss = fmaf(f, f, ss);
          }
        }
      }
      rstd[m] = rsqrtf(wave_sum(ss) / (float)K + eps);
    }
  }

  float acc[V];
#pragma unroll
  for (int i = 0; i < V; ++i) acc[i] = 0.f;

  for (int s0 = 0; s0 < steps; s0 += U) {
    Vec16<T> xv[U][MM];
    Vec16<T> wr[U][KR];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int k = kbase + (s0 + u) * kStride;
      if (k < K) {
#pragma unroll
        for (int m = 0; m < MM; ++m)
          if (m < M) xv[u][m] = load16(x + (int64_t)m * ldx + k);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int k = kbase + (s0 + u) * kStride;
      if (k < K) {
#pragma unroll
        for (int r = 0; r < KR; ++r) wr[u][r] = load16(wrow[r] + k);
      }
    }
    if (NORM && steps <= U) {
      // this wave's x pieces cover its share of every row: block-reduce the sums of squares
      // (plain global loads stay in flight across the barrier)
#pragma unroll
      for (int m = 0; m < MM; ++m) {
        float ss = 0.f;
#pragma unroll
        for (int u = 0; u < U; ++u) {
          if (m < M && kbase + (s0 + u) * kStride < K) {
#pragma unroll
            for (int e = 0; e < NV; ++e) {
              const float f = to_f32(xv[u][m].v[e]);
              ss = fmaf(f, f, ss);
            }
          }
        }
        ss = wave_sum(ss);
        if (lane == 0) ss_part[wv][m] = ss;
      }
      __syncthreads();
#pragma unroll
      for (int m = 0; m < MM; ++m)
        rstd[m] = rsqrtf((ss_part[0][m] + ss_part[1][m] + ss_part[2][m] + ss_part[3][m]) / (float)K + eps);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int k = kbase + (s0 + u) * kStride;
      if (k < K) {
        Vec16<T> gv;
        if constexpr (NORM) {
          if (g) gv = load16(g + k);
        }
#pragma unroll
        for (int m = 0; m < MM; ++m) {
          if (m < M) {
#pragma unroll
            for (int e = 0; e < NV; ++e) {
              float xf = to_f32(xv[u][m].v[e]);
              if constexpr (NORM) xf = to_f32(from_f32<T>(xf * rstd[m] * (g ? to_f32(gv.v[e]) : 1.f)));
#pragma unroll
              for (int r = 0; r < KR; ++r)
                acc[m * KR + r] = fmaf(xf, to_f32(wr[u][r].v[e]), acc[m * KR + r]);
            }
          }
        }
      }
    }
  }

  // reduce-scatter: after LOGV halvings the lane holds element (lane >> (6 - LOGV)) summed over the
  // lanes that share those top bits; a butterfly over the remaining low bits completes the sum.
#pragma unroll
  for (int step = 0; step < LOGV; ++step) {
    const int off = 32 >> step;
    const int half = V >> (step + 1);  // compile-time after unrolling: acc stays in VGPRs
    const bool upper = (lane & off) != 0;
#pragma unroll
    for (int i = 0; i < half; ++i) {
      const float give = upper ? acc[i] : acc[half + i];
      const float keep = upper ? acc[half + i] : acc[i];
      acc[i] = keep + __shfl_xor(give, off, 64);
    }
  }
  float s = acc[0];
#pragma unroll
  for (int off = 32 >> LOGV; off >= 1; off >>= 1) s += __shfl_xor(s, off, 64);
  if ((lane & ((64 >> LOGV) - 1)) == 0) part[wv][lane >> (6 - LOGV)] = s;
  __syncthreads();

  if (threadIdx.x < V) {
    const int e = threadIdx.x;
    const int m = e / KR, r = e % KR;
    if (GATED) {
      const int nn = n0 + r;
      if (r < COLS && m < M && nn < N) {
        const float a = to_f32(from_f32<T>(part[0][e] + part[1][e] + part[2][e] + part[3][e]));
        const int e2 = e + COLS;
        const float b = to_f32(from_f32<T>(part[0][e2] + part[1][e2] + part[2][e2] + part[3][e2]));
        y[(int64_t)m * ldy + nn] = from_f32<T>(gemv_act(a, act) * b);
      }
    } else {
      const int nn = n0 + r;
      if (m < M && nn < N) {
        float v = part[0][e] + part[1][e] + part[2][e] + part[3][e];
        if (bias) v += to_f32(bias[nn]);
        v = gemv_act(v, act);
        if (res) v += to_f32(res[(int64_t)m * ldr + nn]);
        y[(int64_t)m * ldy + nn] = from_f32<T>(v);
      }
    }
  }
}

template <typename T, int MM, bool NORM, bool GATED, int KR>
void launch_kr(const T* x, const T* w, const T* w2, const T* g, float eps, const T* bias, const T* res, T* y, int M,
               int N, int K, int64_t ldx, int64_t ldw, int64_t ldy, int64_t ldr, int act, hipStream_t s) {
  constexpr int COLS = GATED ? KR / 2 : KR;
  dim3 grid((N + COLS - 1) / COLS), block(256);
  const int steps = (K + kWaves * kStep - 1) / (kWaves * kStep);
  // weight registers: U * KR * 4 VGPRs; MM <= 2 affords U = 4, MM = 4 U = 2, MM = 8 U = 1
  if (MM <= 2 && steps >= 3)
    hipLaunchKernelGGL((gemv_kernel<T, MM, NORM, GATED, (MM <= 2 ? 4 : 1), KR>), grid, block, 0, s, x, w, w2, g, eps,
                       bias, res, y, M, N, K, ldx, ldw, ldy, ldr, act);
  else if (MM <= 4 && steps >= 2)
    hipLaunchKernelGGL((gemv_kernel<T, MM, NORM, GATED, (MM <= 4 ? 2 : 1), KR>), grid, block, 0, s, x, w, w2, g, eps,
                       bias, res, y, M, N, K, ldx, ldw, ldy, ldr, act);
  else
    hipLaunchKernelGGL((gemv_kernel<T, MM, NORM, GATED, 1, KR>), grid, block, 0, s, x, w, w2, g, eps, bias, res, y, M,
                       N, K, ldx, ldw, ldy, ldr, act);
}

template <typename T, int MM, bool NORM, bool GATED>
void launch_mm(const T* x, const T* w, const T* w2, const T* g, float eps, const T* bias, const T* res, T* y, int M,
               int N, int K, int64_t ldx, int64_t ldw, int64_t ldy, int64_t ldr, int act, hipStream_t s) {
  // narrow outputs (N < 4096: the 2048-wide projections of a 1B model) would leave one workgroup
  // per CU with 8-row tiles: 4-row tiles double the workgroups and the waves streaming per CU
  if (!GATED && MM <= 2 && N < 4096)
    launch_kr<T, MM, NORM, GATED, 4>(x, w, w2, g, eps, bias, res, y, M, N, K, ldx, ldw, ldy, ldr, act, s);
  else
    launch_kr<T, MM, NORM, GATED, kRows>(x, w, w2, g, eps, bias, res, y, M, N, K, ldx, ldw, ldy, ldr, act, s);
}

template <typename T, bool NORM, bool GATED>
void launch_m(const T* x, const T* w, const T* w2, const T* g, float eps, const T* bias, const T* res, T* y, int M,
              int N, int K, int64_t ldx, int64_t ldw, int64_t ldy, int64_t ldr, int act, hipStream_t s) {
  if (M == 1)
    launch_mm<T, 1, NORM, GATED>(x, w, w2, g, eps, bias, res, y, M, N, K, ldx, ldw, ldy, ldr, act, s);
  else if (M == 2)
    launch_mm<T, 2, NORM, GATED>(x, w, w2, g, eps, bias, res, y, M, N, K, ldx, ldw, ldy, ldr, act, s);
  else if (M <= 4)
    launch_mm<T, 4, NORM, GATED>(x, w, w2, g, eps, bias, res, y, M, N, K, ldx, ldw, ldy, ldr, act, s);
  else
    launch_mm<T, 8, NORM, GATED>(x, w, w2, g, eps, bias, res, y, M, N, K, ldx, ldw, ldy, ldr, act, s);
}

template <typename T>
int launch(const void* x, const void* w, const void* w2, const void* g, int norm, float eps, const void* bias,
           const void* res, void* y, int M, int N, int K, int64_t ldx, int64_t ldw, int64_t ldy, int64_t ldr, int act,
           hipStream_t s) {
  const T *xp = (const T*)x, *wp = (const T*)w, *w2p = (const T*)w2, *gp = (const T*)g, *bp = (const T*)bias,
          *rp = (const T*)res;
  T* yp = (T*)y;
  if (norm && w2p) launch_m<T, true, true>(xp, wp, w2p, gp, eps, bp, rp, yp, M, N, K, ldx, ldw, ldy, ldr, act, s);
  else if (norm) launch_m<T, true, false>(xp, wp, w2p, gp, eps, bp, rp, yp, M, N, K, ldx, ldw, ldy, ldr, act, s);
  else if (w2p) launch_m<T, false, true>(xp, wp, w2p, gp, eps, bp, rp, yp, M, N, K, ldx, ldw, ldy, ldr, act, s);
  else launch_m<T, false, false>(xp, wp, w2p, gp, eps, bp, rp, yp, M, N, K, ldx, ldw, ldy, ldr, act, s);
  return (int)hipGetLastError();
}

template <typename T, int MM, bool NORM, int KR>
void launch_group(const T* x, const T* g, float eps, int M, int K, int64_t ldx, GemvGroup grp, int nseg,
                  hipStream_t s) {
  int total = 0;
  for (int i = 0; i < nseg; ++i) {
    const int b = (grp.n[i] + KR - 1) / KR;
    if (i < 2) grp.blocks[i] = b;
    total += b;
  }
  for (int i = nseg; i < 2; ++i) grp.blocks[i] = 1 << 30;
  const int steps = (K + kWaves * kStep - 1) / (kWaves * kStep);
  dim3 grid(total), block(256);
#define LTA_G(UU)                                                                                                  \
  hipLaunchKernelGGL((gemv_kernel<T, MM, NORM, false, UU, KR, true>), grid, block, 0, s, x, (const T*)nullptr,      \
                     (const T*)nullptr, g, eps, (const T*)nullptr, (const T*)nullptr, (T*)nullptr, M, 0, K, ldx,    \
                     (int64_t)0, (int64_t)0, (int64_t)0, 0, grp)
  if (MM <= 2 && steps >= 3) { LTA_G((MM <= 2 ? 4 : 1)); }
  else if (MM <= 4 && steps >= 2) { LTA_G((MM <= 4 ? 2 : 1)); }
  else { LTA_G(1); }
#undef LTA_G
}

template <typename T, bool NORM>
int launch_group_m(const void* x, const void* g, float eps, int M, int K, int64_t ldx, GemvGroup grp, int nseg,
                   hipStream_t s) {
  const T* xp = (const T*)x;
  const T* gp = (const T*)g;
  if (M == 1) launch_group<T, 1, NORM, 4>(xp, gp, eps, M, K, ldx, grp, nseg, s);
  else if (M == 2) launch_group<T, 2, NORM, 4>(xp, gp, eps, M, K, ldx, grp, nseg, s);
  else if (M <= 4) launch_group<T, 4, NORM, kRows>(xp, gp, eps, M, K, ldx, grp, nseg, s);
  else launch_group<T, 8, NORM, kRows>(xp, gp, eps, M, K, ldx, grp, nseg, s);
  return (int)hipGetLastError();
}

}  // namespace
}  // namespace lta

// Grouped decode projections: y_i[M, N_i] = x' w_i^T for i < nseg (<= 3) in one launch, x' = x or
// rmsnorm(x, g, eps) (norm != 0).  w_i [N_i, K] (row stride ldw_i), y_i row stride ldy_i.
LTA_EXPORT int lta_gemv_group(int dtype, const void* x, const void* g, int norm, float eps, int nseg,
                              const void* const* ws, void* const* ys, const int* ns, const int64_t* ldws,
                              const int64_t* ldys, int M, int K, int64_t ldx, void* stream) {
  using namespace lta;
  if (M < 1 || M > 8 || nseg < 1 || nseg > 3 || K < 8 || K % 8 || ldx % 8) return (int)hipErrorInvalidValue;
  GemvGroup grp{};
  for (int i = 0; i < nseg; ++i) {
    if (ldws[i] % 8 || ns[i] < 1) return (int)hipErrorInvalidValue;
    grp.w[i] = ws[i];
    grp.y[i] = ys[i];
    grp.n[i] = ns[i];
    grp.ldw[i] = ldws[i];
    grp.ldy[i] = ldys[i];
  }
  hipStream_t s = (hipStream_t)stream;
  if (dtype == kBF16) return norm ? launch_group_m<__hip_bfloat16, true>(x, g, eps, M, K, ldx, grp, nseg, s)
                                  : launch_group_m<__hip_bfloat16, false>(x, g, eps, M, K, ldx, grp, nseg, s);
  if (dtype == kF16) return norm ? launch_group_m<__half, true>(x, g, eps, M, K, ldx, grp, nseg, s)
                                 : launch_group_m<__half, false>(x, g, eps, M, K, ldx, grp, nseg, s);
  return (int)hipErrorInvalidValue;
}

// x [M, K] (row stride ldx), w (and w2) [N, K] (row stride ldw), y [M, N]; K % 8 == 0, 16-byte aligned
// rows.  norm != 0: x -> rmsnorm(x, g, eps) first; w2 != null: y = act(x w^T) * (x w2^T) (no bias/residual).
LTA_EXPORT int lta_gemv_nt(int dtype, const void* x, const void* w, const void* w2, const void* g, int norm, float eps,
                           const void* bias, const void* res, void* y, int M, int N, int K, int64_t ldx, int64_t ldw,
                           int64_t ldy, int64_t ldr, int act, void* stream) {
  using namespace lta;
  if (M < 1 || M > 8 || N < 1 || K < 8 || K % 8 || ldx % 8 || ldw % 8) return (int)hipErrorInvalidValue;
  if (w2 && (bias || res)) return (int)hipErrorInvalidValue;
  hipStream_t s = (hipStream_t)stream;
  if (dtype == kBF16) return launch<__hip_bfloat16>(x, w, w2, g, norm, eps, bias, res, y, M, N, K, ldx, ldw, ldy, ldr, act, s);
  if (dtype == kF16) return launch<__half>(x, w, w2, g, norm, eps, bias, res, y, M, N, K, ldx, ldw, ldy, ldr, act, s);
  return (int)hipErrorInvalidValue;
}
