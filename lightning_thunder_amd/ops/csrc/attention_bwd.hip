// K3 flash-attention backward for CDNA4 (gfx950): recompute P from Q, K and the forward LSE.
//
// Three launches (FA2-style split; no float atomics, bitwise reproducible):
//  1. preprocess: delta[q] = rowsum(dO[q] * O[q])                                  (fp32)
//  2. dK/dV: one workgroup per 128-key block (32 keys per wave, K and V rows held in registers
//     as MFMA B operands), sweeping 32-query tiles of every query head of the kv group:
//        S = Q K^T (key on the lane), P = exp2(S*c - lse*log2e), dP = dO V^T,
//        dS = P (dP - delta),  dV^T += dO^T P,  dK^T += Q^T dS
//     The S/dP accumulators feed dV^T/dK^T directly as B operands (attention.h), dO^T and Q^T
//     come from transposed LDS reads.
//  3. dQ: one workgroup per 128-query block (as the forward), sweeping 64-key tiles:
//        S^T = K Q^T, P^T, dP^T = V dO^T, dS^T,  dQ^T += K^T dS^T
// Both main kernels skip fully masked tiles under causal masking.
#include "attention.h"

using namespace lta;
using namespace lta::attn;

namespace {

constexpr int kThreads = 256;
typedef __attribute__((address_space(3))) void lds_void;
typedef float f32x4v __attribute__((ext_vector_type(4)));

template <int D> struct BCfg {
  static constexpr int BN = D > 128 ? 32 : 64;  // dQ kernel: keys per tile (D = 256: registers)
  static constexpr int NKT = BN / 32;
  static constexpr int RSTR = D + 8;    // row-read image stride (ds_read_b128 conflict-free)
  static constexpr int TSTR = D + 32;   // transposed-read image stride (ds_read_b64_tr_b16 conflict-free)
  static constexpr int CH = D / 8;
  static constexpr int KS = D / 16;
  static constexpr int DT = D / 32;
};

// ---------------------------------------------------------------------------------------------
// Row strides: dO and O may be any [B,H,T] strided layout with the head dim contiguous (e.g. the
// [B,T,H,D] storage that the output projection reads without a copy); s*[0..2] = batch/head/token.
struct RowStrides {
  int64_t b, h, t;
};

template <typename T, int D>
__global__ __launch_bounds__(256) void attn_bwd_preprocess(const T* __restrict__ dO, const T* __restrict__ O,
                                                           float* __restrict__ delta, int64_t rows, int H, int Tq,
                                                           RowStrides sdo, RowStrides so) {
  // 8 lanes per row (16 B each per step)
  const int64_t row = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / 8;
  const int sub = threadIdx.x & 7;
  float acc = 0.f;
  // row order: heads fastest when dO is stored token-major ([B, T, H, D], the output projection's
  // layout), so a wave's 8 rows are 2 KiB of contiguous memory rather than 8 rows 8 KiB apart
  const bool hfast = sdo.h < sdo.t;
  int64_t t = 0, hh = 0, bb = 0;
  if (hfast) {
    hh = row % H;
    t = (row / H) % Tq;
    bb = row / ((int64_t)H * Tq);
  } else {
    t = row % Tq;
    hh = (row / Tq) % H;
    bb = row / ((int64_t)H * Tq);
  }
  if (row < rows) {
    const T* a = dO + bb * sdo.b + hh * sdo.h + t * sdo.t;
    const T* b = O + bb * so.b + hh * so.h + t * so.t;
#pragma unroll
    for (int c = sub * 8; c < D; c += 64) {
      const Vec16<T> x = load16(a + c), y = load16(b + c);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc += to_f32(x.v[j]) * to_f32(y.v[j]);
    }
  }
  acc += __shfl_xor(acc, 1, 64);
  acc += __shfl_xor(acc, 2, 64);
  acc += __shfl_xor(acc, 4, 64);
  if (row < rows && sub == 0) delta[(bb * H + hh) * Tq + t] = acc;
}

// dK^T / dV^T accumulate in the accumulator (AGPR) file through inline-asm MFMAs: they are only
// ever MFMA C/D operands, and pinning them there leaves the 256 architectural VGPRs to K, the S / dP
// tiles and their softmax (hipcc otherwise parks S / dP in AGPRs and copies them out every tile).
// `s_nop 1` covers the VALU (cvt_pk) write -> MFMA operand read; an accumulate chain needs none.
__device__ __forceinline__ void mfma_acc_agpr(f32x16& acc, const bf16x8& a, const bf16x8& b) {
  asm volatile("s_nop 1\n\tv_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
}
__device__ __forceinline__ void mfma_acc_agpr(f32x16& acc, const f16x8& a, const f16x8& b) {
  asm volatile("s_nop 1\n\tv_mfma_f32_32x32x16_f16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
}

// One lane's 128-wide row of a dQ^T / dK^T / dV^T accumulator set (d-tile dt, element i: d = dt*32 +
// acc_row(i, h)) times `mul` -> the T row at `row` (4 consecutive d per 8-byte store).  With `cs` / `sn`
// (this token's fp32 cos / sin rows) the transpose of the rotate-half RoPE is applied on the fp32
// values first — d and its partner d + 64 are tiles dt and dt + 2 of the same lane:
//   o[d] = x[d] cos[d] + x[d+64] sin[d+64],  o[d+64] = x[d+64] cos[d+64] - x[d] sin[d]
// (the rotation the forward applied to q / k, transposed: csrc/rope.hip's backward, one rounding).
// fp32 variant (the GQA head split's partial rows, summed by attn_bwd_dkdv_reduce): same layout and
// rotation, 4 consecutive d per 16-byte store
template <typename ACC>
__device__ __forceinline__ void store_row_d128_f32(float* row, const ACC& acc, float mul, int h, const float* cs,
                                                   const float* sn) {
  if (cs == nullptr) {
#pragma unroll
    for (int dt = 0; dt < 4; ++dt)
#pragma unroll
      for (int a = 0; a < 4; ++a)
        *reinterpret_cast<float4*>(row + dt * 32 + 8 * a + 4 * h) =
            make_float4(acc[dt][4 * a] * mul, acc[dt][4 * a + 1] * mul, acc[dt][4 * a + 2] * mul, acc[dt][4 * a + 3] * mul);
    return;
  }
#pragma unroll
  for (int dt = 0; dt < 2; ++dt)
#pragma unroll
    for (int a = 0; a < 4; ++a) {
      const int d = dt * 32 + 8 * a + 4 * h;
      const float4 c1 = *reinterpret_cast<const float4*>(cs + d), s1 = *reinterpret_cast<const float4*>(sn + d);
      const float4 c2 = *reinterpret_cast<const float4*>(cs + d + 64), s2 = *reinterpret_cast<const float4*>(sn + d + 64);
      const float cl[4] = {c1.x, c1.y, c1.z, c1.w}, sl[4] = {s1.x, s1.y, s1.z, s1.w};
      const float ch[4] = {c2.x, c2.y, c2.z, c2.w}, sh[4] = {s2.x, s2.y, s2.z, s2.w};
      float lo[4], hi[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float x1 = acc[dt][4 * a + e] * mul, x2 = acc[dt + 2][4 * a + e] * mul;
        lo[e] = x1 * cl[e] + x2 * sh[e];
        hi[e] = x2 * ch[e] - x1 * sl[e];
      }
      *reinterpret_cast<float4*>(row + d) = make_float4(lo[0], lo[1], lo[2], lo[3]);
      *reinterpret_cast<float4*>(row + d + 64) = make_float4(hi[0], hi[1], hi[2], hi[3]);
    }
}

template <typename T, typename ACC>
__device__ __forceinline__ void store_row_d128(T* row, const ACC& acc, float mul, int h, const float* cs,
                                               const float* sn) {
  union P4 {
    T v[4];
    uint2 u;
  };
  if (cs == nullptr) {
#pragma unroll
    for (int dt = 0; dt < 4; ++dt)
#pragma unroll
      for (int a = 0; a < 4; ++a) {
        P4 pk;
#pragma unroll
        for (int e = 0; e < 4; ++e) pk.v[e] = from_f32<T>(acc[dt][4 * a + e] * mul);
        *reinterpret_cast<uint2*>(row + dt * 32 + 8 * a + 4 * h) = pk.u;
      }
    return;
  }
#pragma unroll
  for (int dt = 0; dt < 2; ++dt)
#pragma unroll
    for (int a = 0; a < 4; ++a) {
      const int d = dt * 32 + 8 * a + 4 * h;
      const float4 c1 = *reinterpret_cast<const float4*>(cs + d), s1 = *reinterpret_cast<const float4*>(sn + d);
      const float4 c2 = *reinterpret_cast<const float4*>(cs + d + 64), s2 = *reinterpret_cast<const float4*>(sn + d + 64);
      const float cl[4] = {c1.x, c1.y, c1.z, c1.w}, sl[4] = {s1.x, s1.y, s1.z, s1.w};
      const float ch[4] = {c2.x, c2.y, c2.z, c2.w}, sh[4] = {s2.x, s2.y, s2.z, s2.w};
      P4 lo, hi;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float x1 = acc[dt][4 * a + e] * mul, x2 = acc[dt + 2][4 * a + e] * mul;
        lo.v[e] = from_f32<T>(x1 * cl[e] + x2 * sh[e]);
        hi.v[e] = from_f32<T>(x2 * ch[e] - x1 * sl[e]);
      }
      *reinterpret_cast<uint2*>(row + d) = lo.u;
      *reinterpret_cast<uint2*>(row + d + 64) = hi.u;
    }
}

// ---------------------------------------------------------------------------------------------
// dK / dV
// ---------------------------------------------------------------------------------------------
constexpr int kKB = 128;  // keys per workgroup
constexpr int kQT = 32;   // queries per inner tile

// SPLIT (GQA / MQA head split, as the v4 kernel's): the grid's x holds B Hkv hsplit workgroups, workgroup
// (bh, hs) sweeps query heads hs gsz .. hs gsz + gsz - 1 of its kv group (gsz = group / hsplit) and stores
// fp32 partial dK / dV rows part[hs][bh][key][dK | dV][D] that attn_bwd_dkdv_reduce sums: Gemma-2b's one kv
// head at T = 4096 is 32 workgroups of 128 keys without it (8 query heads each), 256 with it.
template <typename T, int D, bool CAUSAL, int EX = 0, bool SPLIT = false>
__global__ __launch_bounds__(kThreads, 1) void attn_bwd_dkdv_kernel(const T* __restrict__ Q, const T* __restrict__ K,
                                                                    const T* __restrict__ V, const T* __restrict__ dO,
                                                                    const float* __restrict__ LSE,
                                                                    const float* __restrict__ DELTA, T* __restrict__ dK,
                                                                    T* __restrict__ dV, int Hq, int Hkv, int Tq, int Sk,
                                                                    float scale, float scale_log2, RowStrides sdo,
                                                                    AttnExtra ex) {
  constexpr bool MASK = EX & kExMask, DROP = EX & kExDrop, MGRAD = EX & kExMaskGrad;
  using C = BCfg<D>;
  using F = typename Frag<T>::type;
  // Double-buffered Q / dO tiles: the global loads of tile i+1 are issued before the MFMAs of
  // tile i and land in the other buffer afterwards, so HBM/L2 latency hides behind compute and
  // one barrier per tile suffices.
  constexpr int BUF = 2 * kQT * C::RSTR + 2 * kQT * C::TSTR;
  __shared__ __attribute__((aligned(16))) short smem[2 * BUF];
  __shared__ float s_lse[2][kQT], s_delta[2][kQT];
  __shared__ __attribute__((aligned(16))) unsigned s_qterm[2][DROP ? kQT : 4];  // the tile's query terms (dropout)

  const int n_kb = (Sk + kKB - 1) / kKB;
  (void)n_kb;
  // grid = (B*Hkv, key blocks): heaviest (causal) key blocks of every head first, balanced over XCDs
  const int kb = (int)blockIdx.y;
  const int nsplit = SPLIT ? ex.hsplit : 1;
  const int bh = SPLIT ? (int)blockIdx.x / nsplit : (int)blockIdx.x;
  const int hs = SPLIT ? (int)blockIdx.x - bh * nsplit : 0;
  const int b = bh / Hkv, hk = bh % Hkv;
  const int group = Hq / Hkv;
  const int gsz = group / nsplit;              // query heads this workgroup sweeps
  const int hbase = hk * group + hs * gsz;     // the first of them
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 31, h = lane >> 5, g = lane >> 4, l16 = lane & 15;
  const int kw = kb * kKB + wave * 32;  // this wave's first key
  const int key = kw + r;               // this lane's key
  const T* Kb = K + b * ex.sx.kb + hk * ex.sx.kh;
  const T* Vb = V + b * ex.sx.vb + hk * ex.sx.vh;

  F kf[C::KS], vf[C::KS];
  {
    const int krow = min(key, Sk - 1);
#pragma unroll
    for (int s = 0; s < C::KS; ++s) {
      kf[s] = load_frag<F>(Kb + (int64_t)krow * ex.sx.kt + 16 * s + 8 * h);
      vf[s] = load_frag<F>(Vb + (int64_t)krow * ex.sx.vt + 16 * s + 8 * h);
    }
  }
  f32x16 dkacc[C::DT], dvacc[C::DT];
#pragma unroll
  for (int dt = 0; dt < C::DT; ++dt)
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      dkacc[dt][i] = 0.f;
      dvacc[dt][i] = 0.f;
    }

  const int n_qt = (Tq + kQT - 1) / kQT;
  const int qt_begin = CAUSAL ? min((kb * kKB) / kQT, n_qt) : 0;
  const int nq = n_qt - qt_begin;
  const int total = gsz * nq;
  // 16-B chunks per thread per tile, rounded up (D = 96: 384 chunks over 256 threads); the tail is
  // guarded by NCH
  constexpr int NCH = kQT * C::CH, LOADS = (NCH + kThreads - 1) / kThreads;

  uint4 pq[LOADS], po[LOADS];
  float plse = 0.f, pdel = 0.f;
  auto issue = [&](int it) {
    const int hq = hbase + it / nq;
    const int qbase = (qt_begin + it % nq) * kQT;
    const T* Qb = Q + b * ex.sx.qb + hq * ex.sx.qh;
    const T* dOb = dO + b * sdo.b + hq * sdo.h;
#pragma unroll
    for (int c = 0; c < LOADS; ++c) {
      const int id = c * kThreads + tid;
      if (NCH % kThreads != 0 && id >= NCH) break;
      const int row = id / C::CH, ch = id % C::CH;
      const int qc = min(qbase + row, Tq - 1);
      pq[c] = *reinterpret_cast<const uint4*>(Qb + (int64_t)qc * ex.sx.qt + ch * 8);
      po[c] = *reinterpret_cast<const uint4*>(dOb + qc * sdo.t + ch * 8);
    }
    if (tid < kQT) {
      const int qc = min(qbase + tid, Tq - 1);
      plse = LSE[((int64_t)b * Hq + hq) * Tq + qc];
      pdel = DELTA[((int64_t)b * Hq + hq) * Tq + qc];
    }
  };
  auto stash = [&](int it, int buf) {
    const int qbase = (qt_begin + it % nq) * kQT;
    short* Qr = smem + buf * BUF;
    short* dOr = Qr + kQT * C::RSTR;
    short* Qt = dOr + kQT * C::RSTR;
    short* dOt = Qt + kQT * C::TSTR;
#pragma unroll
    for (int c = 0; c < LOADS; ++c) {
      const int id = c * kThreads + tid;
      if (NCH % kThreads != 0 && id >= NCH) break;
      const int row = id / C::CH, ch = id % C::CH;
      uint4 xq = pq[c], xo = po[c];
      if (qbase + row >= Tq) {
        xq = make_uint4(0, 0, 0, 0);
        xo = make_uint4(0, 0, 0, 0);
      }
      *reinterpret_cast<uint4*>(Qr + row * C::RSTR + ch * 8) = xq;
      *reinterpret_cast<uint4*>(dOr + row * C::RSTR + ch * 8) = xo;
      *reinterpret_cast<uint4*>(Qt + row * C::TSTR + ch * 8) = xq;
      *reinterpret_cast<uint4*>(dOt + row * C::TSTR + ch * 8) = xo;
    }
    if (tid < kQT) {
      const bool ok = qbase + tid < Tq;
      s_lse[buf][tid] = ok ? plse * 1.44269504088896340736f : INFINITY;
      s_delta[buf][tid] = ok ? pdel : 0.f;
      if constexpr (DROP) s_qterm[buf][tid] = rng_q(rng_head(ex, b * Hq + hbase + it / nq), qbase + tid);
    }
  };

  if (total > 0) {
    issue(0);
    stash(0, 0);
  }
  __syncthreads();
  for (int it = 0; it < total; ++it) {
    const int buf = it & 1;
    const bool more = it + 1 < total;
    if (more) issue(it + 1);
    const int qbase = (qt_begin + it % nq) * kQT;
    const short* Qr = smem + buf * BUF;
    const short* dOr = Qr + kQT * C::RSTR;
    const __attribute__((address_space(3))) short* Qt3 =
        (const __attribute__((address_space(3))) short*)(dOr + kQT * C::RSTR);
    const __attribute__((address_space(3))) short* dOt3 = Qt3 + kQT * C::TSTR;
    const float* sl = s_lse[buf];
    const float* sd = s_delta[buf];

    // S = Q K^T  (rows: queries of this tile, cols: this wave's keys)
    f32x16 sacc, pacc;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      sacc[i] = 0.f;
      pacc[i] = 0.f;
    }
#pragma unroll
    for (int s = 0; s < C::KS; ++s) {
      const F qa = load_frag<F>(Qr + r * C::RSTR + 16 * s + 8 * h);
      const F oa = load_frag<F>(dOr + r * C::RSTR + 16 * s + 8 * h);
      sacc = mfma(qa, kf[s], sacc);
      pacc = mfma(oa, vf[s], pacc);  // dP = dO V^T
    }
    // P and dS (element i: query qbase + acc_row(i,h), key = this lane's key)
    [[maybe_unused]] const int hq_it = hbase + it / nq;
    [[maybe_unused]] unsigned kterm = 0;
    if constexpr (DROP) kterm = rng_k(key);
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int qr = acc_row(i, h);
      const int qq = qbase + qr;
      float sv = sacc[i] * scale_log2;
      if constexpr (MASK)
        sv += ex.mask[b * ex.mb + hq_it * ex.mh + (int64_t)min(qq, Tq - 1) * ex.mq + min(key, Sk - 1)] *
              1.44269504088896340736f;
      float p = __builtin_amdgcn_exp2f(sv - sl[qr]);
      p = (key >= Sk || qq >= Tq || (CAUSAL && key > qq)) ? 0.f : p;
      float dp = pacc[i];
      float pd = p;
      if constexpr (DROP) {  // dropped P feeds dV; dS = P (dP_dropped * keep / (1-p) - delta)
        const uint4 qv = rng_tab4(s_qterm[buf], i >> 2, h);  // query terms stashed with the tile
        const unsigned qw4[4] = {qv.x, qv.y, qv.z, qv.w};
        const bool keep = rng_keep(ex, qw4[i & 3], kterm);
        pd = keep ? p * ex.keep_scale : 0.f;
        dp = keep ? dp * ex.keep_scale : 0.f;
      }
      sacc[i] = pd;                          // P (after dropout)
      pacc[i] = p * (dp - sd[qr]);           // dS
      if constexpr (MGRAD) {
        if (key < Sk && qq < Tq) ex.dmask[(((int64_t)b * Hq + hq_it) * Tq + qq) * Sk + key] = pacc[i];
      }
    }
    F pf0, pf1, df0, df1;
    pack_frag(pf0, sacc, 0);
    pack_frag(pf1, sacc, 1);
    pack_frag(df0, pacc, 0);
    pack_frag(df1, pacc, 1);
#pragma unroll
    for (int dt = 0; dt < C::DT; ++dt) {
      const int col0 = dt * 32 + 16 * (g & 1);
      const F oa0 = tr_frag<F>(dOt3, 4 * h, col0, C::TSTR, l16);
      const F oa1 = tr_frag<F>(dOt3, 16 + 4 * h, col0, C::TSTR, l16);
      const F qa0 = tr_frag<F>(Qt3, 4 * h, col0, C::TSTR, l16);
      const F qa1 = tr_frag<F>(Qt3, 16 + 4 * h, col0, C::TSTR, l16);
      if constexpr (D > 128) {  // 2 x 128 accumulators: pinned to the AGPR file (K, V fill the VGPRs)
        mfma_acc_agpr(dvacc[dt], oa0, pf0);
        mfma_acc_agpr(dvacc[dt], oa1, pf1);
        mfma_acc_agpr(dkacc[dt], qa0, df0);
        mfma_acc_agpr(dkacc[dt], qa1, df1);
      } else {
        dvacc[dt] = mfma(oa0, pf0, dvacc[dt]);
        dvacc[dt] = mfma(oa1, pf1, dvacc[dt]);
        dkacc[dt] = mfma(qa0, df0, dkacc[dt]);
        dkacc[dt] = mfma(qa1, df1, dkacc[dt]);
      }
    }
    if (more) stash(it + 1, buf ^ 1);
    __syncthreads();
  }

  if constexpr (D > 128) {  // the last asm MFMAs' results must be complete before they are read
#pragma unroll
    for (int dt = 0; dt < C::DT; ++dt) asm volatile("s_nop 15\n\ts_nop 15" : "+a"(dkacc[dt]), "+a"(dvacc[dt]));
  }
  // dK^T / dV^T: element i of tile dt is d = dt*32 + acc_row(i,h), key = this lane's key
  if (SPLIT && key < Sk) {  // fp32 partial rows of this head split (summed by attn_bwd_dkdv_reduce)
    const int nbh = (int)gridDim.x / nsplit;
    float* prow = ex.part + (((int64_t)hs * nbh + bh) * Sk + key) * (2 * D);
#pragma unroll
    for (int dt = 0; dt < C::DT; ++dt)
#pragma unroll
      for (int a = 0; a < 4; ++a) {
        const int d = dt * 32 + 8 * a + 4 * h;
        *reinterpret_cast<float4*>(prow + d) = make_float4(dkacc[dt][4 * a] * scale, dkacc[dt][4 * a + 1] * scale,
                                                           dkacc[dt][4 * a + 2] * scale, dkacc[dt][4 * a + 3] * scale);
        *reinterpret_cast<float4*>(prow + D + d) =
            make_float4(dvacc[dt][4 * a], dvacc[dt][4 * a + 1], dvacc[dt][4 * a + 2], dvacc[dt][4 * a + 3]);
      }
  } else if (key < Sk) {
    T* dkrow = dK + (int64_t)b * ex.sx.dkb + (int64_t)hk * ex.sx.dkh + (int64_t)key * ex.sx.dkt;
    T* dvrow = dV + (int64_t)b * ex.sx.dvb + (int64_t)hk * ex.sx.dvh + (int64_t)key * ex.sx.dvt;
#pragma unroll
    for (int dt = 0; dt < C::DT; ++dt) {
#pragma unroll
      for (int a = 0; a < 4; ++a) {
        const int d = dt * 32 + 8 * a + 4 * h;
        union {
          T v[4];
          uint2 u;
        } pk, pv;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          pk.v[e] = from_f32<T>(dkacc[dt][4 * a + e] * scale);
          pv.v[e] = from_f32<T>(dvacc[dt][4 * a + e]);
        }
        *reinterpret_cast<uint2*>(dkrow + d) = pk.u;
        *reinterpret_cast<uint2*>(dvrow + d) = pv.u;
      }
    }
  }
}

// ---------------------------------------------------------------------------------------------
// dK / dV, D = 128 (v2).  Same decomposition as above; restructured after PMC counters showed the
// v1 loop VALU-bound (355 VALU per wave-iteration against 32 MFMAs, 20 % MFMA busy, 296 VGPRs with
// the S/dP accumulators shuttled through AGPRs):
//  * Q and dO tiles reach LDS by global_load_lds (no VGPR staging, no stash pass) as ONE image per
//    tile that serves both the row reads (ds_read_b128, A operand of S and dP) and the transposed
//    reads (ds_read_b64_tr_b16, A operand of dV^T and dK^T): 8-row x 32-column subtiles of 512 B
//    (cdna_hip_programming.md T10, layout (a)), the swizzle applied to the DMA source address; both
//    read kinds are conflict-free, and every transposed read of a lane is one of two base
//    addresses plus an immediate;
//  * the transposed reads are issued from inline asm: as intrinsics hipcc cannot tell them from
//    the stage the DMA in flight is writing and drains the DMA queue (vmcnt(0)) in front of them;
//  * V lives in LDS (read each tile as the dP B operand), K stays in registers: the loop fits the
//    256 architectural VGPRs;
//  * the causal / bounds mask runs only on the tiles that straddle the diagonal or an edge (a
//    wave-uniform branch); rows past Tq are clamped copies whose P and dS are masked to zero.
// ---------------------------------------------------------------------------------------------
// layout (a): byte offset of 16-B chunk ch (0..15) of row r in a [32][128 x 16-bit] image
__device__ __forceinline__ int du_off(int row, int ch) {
  return 2048 * (row >> 3) + 512 * (ch >> 2) + 64 * (row & 7) + 16 * ((ch & 3) ^ ((row >> 2) & 3));
}

// 16 transposed reads (4 d-tiles x {rows 4h.., 8+4h.., 16+4h.., 24+4h..}) of one image -> the 8 A
// fragments of an X^T . P product (frag 2*dt: query rows 0..15, 2*dt+1: rows 16..31 of the k
// order the P fragment carries), one wait at the end.  ba / bb: the lane's byte address of rows
// 4h+q / 8+4h+q of d-tile 0; d-tile dt adds 512*dt, rows 16.. add 4096.
__device__ __forceinline__ void tr_frags8(bf16x8 (&f)[8], unsigned ba, unsigned bb) {
  typedef short s16x4v __attribute__((ext_vector_type(4)));
  s16x4v x[16];
  asm volatile(
      "ds_read_b64_tr_b16 %0, %16\n\tds_read_b64_tr_b16 %1, %17\n\t"
      "ds_read_b64_tr_b16 %2, %16 offset:4096\n\tds_read_b64_tr_b16 %3, %17 offset:4096\n\t"
      "ds_read_b64_tr_b16 %4, %16 offset:512\n\tds_read_b64_tr_b16 %5, %17 offset:512\n\t"
      "ds_read_b64_tr_b16 %6, %16 offset:4608\n\tds_read_b64_tr_b16 %7, %17 offset:4608\n\t"
      "ds_read_b64_tr_b16 %8, %16 offset:1024\n\tds_read_b64_tr_b16 %9, %17 offset:1024\n\t"
      "ds_read_b64_tr_b16 %10, %16 offset:5120\n\tds_read_b64_tr_b16 %11, %17 offset:5120\n\t"
      "ds_read_b64_tr_b16 %12, %16 offset:1536\n\tds_read_b64_tr_b16 %13, %17 offset:1536\n\t"
      "ds_read_b64_tr_b16 %14, %16 offset:5632\n\tds_read_b64_tr_b16 %15, %17 offset:5632\n\t"
      "s_waitcnt lgkmcnt(0)"
      : "=&v"(x[0]), "=&v"(x[1]), "=&v"(x[2]), "=&v"(x[3]), "=&v"(x[4]), "=&v"(x[5]), "=&v"(x[6]), "=&v"(x[7]),
        "=&v"(x[8]), "=&v"(x[9]), "=&v"(x[10]), "=&v"(x[11]), "=&v"(x[12]), "=&v"(x[13]), "=&v"(x[14]), "=&v"(x[15])
      : "v"(ba), "v"(bb)
      : "memory");
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    union {
      struct { s16x4v a, b; } s;
      bf16x8 f;
    } u;
    u.s.a = x[2 * i];
    u.s.b = x[2 * i + 1];
    f[i] = u.f;
  }
}
__device__ __forceinline__ void tr_frags8(f16x8 (&f)[8], unsigned ba, unsigned bb) {
  bf16x8 t[8];
  tr_frags8(t, ba, bb);
#pragma unroll
  for (int i = 0; i < 8; ++i) f[i] = __builtin_bit_cast(f16x8, t[i]);
}

// tr_frags8 in two halves: issue the 16 transposed reads (no wait) and, later, wait and assemble.
// Between the two, LDS reads the compiler issues are still waited for correctly (LDS returns in
// order, so a compiler lgkmcnt(N) only gets stricter); nothing may read `x` before tr_wait16.
typedef short s16x4t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void tr_issue16(s16x4t (&x)[16], unsigned ba, unsigned bb) {
  asm volatile(
      "ds_read_b64_tr_b16 %0, %16\n\tds_read_b64_tr_b16 %1, %17\n\t"
      "ds_read_b64_tr_b16 %2, %16 offset:4096\n\tds_read_b64_tr_b16 %3, %17 offset:4096\n\t"
      "ds_read_b64_tr_b16 %4, %16 offset:512\n\tds_read_b64_tr_b16 %5, %17 offset:512\n\t"
      "ds_read_b64_tr_b16 %6, %16 offset:4608\n\tds_read_b64_tr_b16 %7, %17 offset:4608\n\t"
      "ds_read_b64_tr_b16 %8, %16 offset:1024\n\tds_read_b64_tr_b16 %9, %17 offset:1024\n\t"
      "ds_read_b64_tr_b16 %10, %16 offset:5120\n\tds_read_b64_tr_b16 %11, %17 offset:5120\n\t"
      "ds_read_b64_tr_b16 %12, %16 offset:1536\n\tds_read_b64_tr_b16 %13, %17 offset:1536\n\t"
      "ds_read_b64_tr_b16 %14, %16 offset:5632\n\tds_read_b64_tr_b16 %15, %17 offset:5632"
      : "=&v"(x[0]), "=&v"(x[1]), "=&v"(x[2]), "=&v"(x[3]), "=&v"(x[4]), "=&v"(x[5]), "=&v"(x[6]), "=&v"(x[7]),
        "=&v"(x[8]), "=&v"(x[9]), "=&v"(x[10]), "=&v"(x[11]), "=&v"(x[12]), "=&v"(x[13]), "=&v"(x[14]), "=&v"(x[15])
      : "v"(ba), "v"(bb)
      : "memory");
}
template <typename F>
__device__ __forceinline__ void tr_wait16(F (&f)[8], s16x4t (&x)[16]) {
  asm volatile("s_waitcnt lgkmcnt(0)"
               : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7]),
                 "+v"(x[8]), "+v"(x[9]), "+v"(x[10]), "+v"(x[11]), "+v"(x[12]), "+v"(x[13]), "+v"(x[14]), "+v"(x[15])
               :
               : "memory");
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    union {
      struct { s16x4t a, b; } s;
      F f;
    } u;
    u.s.a = x[2 * i];
    u.s.b = x[2 * i + 1];
    f[i] = u.f;
  }
}

typedef int dsi32x4 __attribute__((ext_vector_type(4)));

// ---------------------------------------------------------------------------------------------
// dK / dV, D = 128: one workgroup per 256 keys, 64 per wave in two 32-key halves.  Every Q / dO
// image read (row reads for S and dP, transposed reads for dV^T and dK^T) feeds both halves' MFMAs;
// K of the wave's 64 keys stays in registers (B operand of S), V lives in LDS, the dK^T / dV^T
// accumulators fill the 256 AGPRs (cdna_hip_programming.md, Appendix B 'Attention backward').
// (The retired v2 / v3 dK/dV kernels: profiles/attn_bwd_v1_v2_ab.txt, profiles/attn_bwd_dkdv_v4_ab.txt.)
// ---------------------------------------------------------------------------------------------
constexpr int kKB3 = 256;

// ---------------------------------------------------------------------------------------------
// dK / dV, D = 128 (v4): v3's data flow with the tile's VALU work moved into the MFMA shadows.
// v3 runs S -> exp -> dP -> dS -> dV -> dK as dependent blocks, so at one wave per SIMD the
// exponentials and dS (about 200 VALU per lane and tile) serialise against the MFMA pipe.  Here
// the tile is four phases, each an MFMA chain with independent VALU interleaved (pinned with
// sched_barrier, since hipcc otherwise gathers the VALU in front of or behind the chain):
//   A: S = Q K^T (16 MFMA)      B: dP = dO V^T (16) | P = exp2(S c - LSE)
//   C: dV^T += dO^T P (16) | dS = P (dP - delta), pack    D: dK^T += Q^T dS (16)
// ---------------------------------------------------------------------------------------------
// STAMP (diagnostic builds only, -DLTA_ATTN_DIAG): s_memtime at the phase boundaries of workgroup (0, 0)'s
// first 64 query tiles, kept in LDS and copied to `dbg` at the end ([4 waves][64 tiles][8] u64)
// WDS: also store dS^T to `dSt` (the dQ-from-dS path); a template flag so the default build keeps
// its register allocation
template <typename T, bool CAUSAL, int STAMP = 0, bool WDS = false, bool SPLIT = false>
__global__ __launch_bounds__(kThreads, 1) void attn_bwd_dkdv_v4_kernel(const T* __restrict__ Q, const T* __restrict__ K,
                                                                       const T* __restrict__ V, const T* __restrict__ dO,
                                                                       const float* __restrict__ LSE,
                                                                       const float* __restrict__ DELTA, T* __restrict__ dK,
                                                                       T* __restrict__ dV, int Hq, int Hkv, int Tq, int Sk,
                                                                       float scale, float scale_log2, RowStrides sdo, QKVStrides sx,
                                                                       int qrev = 0, uint64_t* dbg = nullptr,
                                                                       T* __restrict__ dSt = nullptr, int hsplit = 1,
                                                                       float* __restrict__ part = nullptr) {
  constexpr int D = 128;
  using C = BCfg<D>;
  using F = typename Frag<T>::type;
  constexpr int NST = 3;
  constexpr int IMG = kQT * 256;
  constexpr int STAGE = 2 * IMG + 256;
  constexpr int VOFF = NST * STAGE;
  constexpr int SBASE = VOFF + kKB3 * C::RSTR * 2;
  __shared__ __attribute__((aligned(1024))) char smem[SBASE + (STAMP ? 4 * 64 * 8 * 8 : 0)];
  short* Vs = reinterpret_cast<short*>(smem + VOFF);

  const int kb = (int)blockIdx.y;
  // GQA head split (hsplit > 1): workgroup x = (b, kv head, split) and the split owns group / hsplit of
  // the kv group's query heads, storing fp32 partial dK / dV rows to `part` ([hsplit][B Hkv Sk][2][128],
  // summed by attn_bwd_dkdv_reduce): B Hkv key blocks alone do not fill 256 CUs when Hkv is small
  // SPLIT is a template flag so the unsplit build keeps its scalar-register allocation (no spills)
  const int nsplit = SPLIT ? hsplit : 1;
  const int bh = SPLIT ? (int)blockIdx.x / nsplit : (int)blockIdx.x, hs = SPLIT ? (int)blockIdx.x % nsplit : 0;
  const int b = bh / Hkv, hk = bh % Hkv;
  const int group = Hq / Hkv;
  const int gsz = group / nsplit, hbase = hk * group + hs * gsz;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 31, h = lane >> 5;
  const int kw = kb * kKB3 + wave * 64;  // this wave's first key; half j: keys kw + 32 j + r
  const T* Kb = K + b * sx.kb + hk * sx.kh;
  const T* Vb = V + b * sx.vb + hk * sx.vh;

  // V rows of the workgroup's 256 keys -> LDS; K rows of this wave's 64 keys -> registers
#pragma unroll
  for (int c = 0; c < kKB3 * C::CH / kThreads; ++c) {
    const int id = c * kThreads + tid;
    const int row = id / C::CH, ch = id % C::CH;
    const int vr = min(kb * kKB3 + row, Sk - 1);
    *reinterpret_cast<uint4*>(Vs + row * C::RSTR + ch * 8) = *reinterpret_cast<const uint4*>(Vb + (int64_t)vr * sx.vt + ch * 8);
  }
  F kf[2][C::KS];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int kr = min(kw + 32 * j + r, Sk - 1);
#pragma unroll
    for (int s = 0; s < C::KS; ++s) kf[j][s] = load_frag<F>(Kb + (int64_t)kr * sx.kt + 16 * s + 8 * h);
  }

  f32x16 dkacc[2][C::DT], dvacc[2][C::DT];
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int dt = 0; dt < C::DT; ++dt)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        dkacc[j][dt][i] = 0.f;
        dvacc[j][dt][i] = 0.f;
      }

  const int n_qt = (Tq + kQT - 1) / kQT;
  const int qt_begin = CAUSAL ? min((kb * kKB3) / kQT, n_qt) : 0;
  const int nq = n_qt - qt_begin;
  const int total = gsz * nq;

  float plse = 0.f, pdel = 0.f;
  auto stash_stats = [&](int st) {
    if (wave == 0 && lane < kQT) {
      float* sp = reinterpret_cast<float*>(smem + st * STAGE + 2 * IMG);
      sp[lane] = -plse * 1.44269504088896340736f;  // stored as -LSE log2 e: exp2(S c + this) = P
      sp[kQT + lane] = pdel;
    }
  };
  auto issue = [&](int hi, int ti, int st) {
    const int hq = hbase + hi;
    // qrev: every key block sweeps the query tiles from the last one down, so the workgroups of one
    // head (one XCD: grid x = head) read the same Q / dO tile at about the same time (L2 reuse)
    const int qbase = (qt_begin + (qrev ? nq - 1 - ti : ti)) * kQT;
    const T* Qb = Q + b * sx.qb + hq * sx.qh;
    const T* dOb = dO + b * sdo.b + hq * sdo.h;
    char* qimg = smem + st * STAGE;
    if (wave == 0) {
      const int64_t srow = ((int64_t)b * Hq + hq) * Tq + min(qbase + (lane & 31), Tq - 1);
      asm volatile("global_load_dword %0, %2, off\n\tglobal_load_dword %1, %3, off"
                   : "=&v"(plse), "=&v"(pdel)
                   : "v"(LSE + srow), "v"(DELTA + srow)
                   : "memory");
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int k = wave * 2 + i;
      const int u = 64 * k + lane;
      const int row = ((u >> 7) << 3) | ((u >> 2) & 7);
      const int ch = (((u >> 5) & 3) << 2) | ((u & 3) ^ ((row >> 2) & 3));
      const int qc = min(qbase + row, Tq - 1);
      __builtin_amdgcn_global_load_lds((const void*)(Qb + (int64_t)qc * sx.qt + ch * 8),
                                       (lds_void*)(qimg + k * 1024), 16, 0, 0);
      __builtin_amdgcn_global_load_lds((const void*)(dOb + qc * sdo.t + ch * 8),
                                       (lds_void*)(qimg + IMG + k * 1024), 16, 0, 0);
    }
  };
  // everything but the newest tile's 4 DMA pieces (and, WDS, the 4 dS stores issued after them:
  // vmcnt counts stores too, and the plain count would drain the prefetch of tile + 2 every tile)
  auto wait_all_but_newest = [&](bool after_stores) {
    if (WDS && after_stores)
      asm volatile("s_waitcnt vmcnt(8)" : "+v"(plse), "+v"(pdel)::"memory");
    else
      asm volatile("s_waitcnt vmcnt(4)" : "+v"(plse), "+v"(pdel)::"memory");
  };

  int nhi = 0, nti = 0;
  auto advance = [&]() {
    if (++nti == nq) {
      nti = 0;
      ++nhi;
    }
  };
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // K / V staging loads
  if (total > 0) {
    issue(nhi, nti, 0);
    advance();
    asm volatile("s_waitcnt vmcnt(0)" : "+v"(plse), "+v"(pdel)::"memory");
    stash_stats(0);
  }
  if (total > 1) {
    issue(nhi, nti, 1);
    advance();
    wait_all_but_newest(false);
    stash_stats(1);
  }
  __syncthreads();

  unsigned tr_a, tr_b;
  {
    const int l16 = lane & 15, g = lane >> 4;
    const int q = l16 >> 2, p = l16 & 3, cl = 2 * (g & 1) + (p >> 1);
    const unsigned base = (unsigned)(uintptr_t)(__attribute__((address_space(3))) char*)smem;
    tr_a = base + 64 * (4 * h + q) + 16 * (cl ^ h) + 8 * (p & 1);
    tr_b = base + 2048 + 64 * (4 * h + q) + 16 * (cl ^ (2 + h)) + 8 * (p & 1);
  }
  constexpr float kLog2e = 1.44269504088896340736f;
  int ti = 0, st = 0;
  auto stamp = [&](int it, int k) {
    if constexpr (STAMP != 0) {
      if (blockIdx.x == 0 && blockIdx.y == 0 && it < 64) {
        __builtin_amdgcn_sched_barrier(0);
        const uint64_t ts = __builtin_amdgcn_s_memtime();
        if (lane == 0) *reinterpret_cast<uint64_t*>(smem + SBASE + ((wave * 64 + it) * 8 + k) * 8) = ts;
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  };
  for (int it = 0; it < total; ++it) {
    stamp(it, 0);
    const bool issue_next = it + 2 < total;
    const int st2 = st >= 1 ? st - 1 : 2;
    if (issue_next) issue(nhi, nti, st2);
    const int qt_abs = qt_begin + (qrev ? nq - 1 - ti : ti);
    const int qbase = qt_abs * kQT;
    {
      const char* qimg = smem + st * STAGE;
      const char* oimg = qimg + IMG;
      const float* sl = reinterpret_cast<const float*>(qimg + 2 * IMG);
      // row statistics of this query tile: LSE now (phase B), delta after phase B (phase C), so the
      // two are never live together; plain LDS loads, waited on at first use
      f32x4v L[4], Dl[4];
#pragma unroll
      for (int a = 0; a < 4; ++a) L[a] = *reinterpret_cast<const f32x4v*>(sl + 4 * h + 8 * a);
      f32x16 sacc[2], pacc[2];
      F pf[2][2], df[2][2];
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          sacc[j][i] = 0.f;
          pacc[j][i] = 0.f;
        }
      // phase A: S = Q K^T for both halves (nothing of this tile is ready to overlap yet); all 8 Q
      // fragments are read up front so the MFMA chain never waits on one LDS read at a time
      {
        F qa[C::KS];
#pragma unroll
        for (int s = 0; s < C::KS; ++s) qa[s] = load_frag<F>(qimg + du_off(r, 2 * s + h));
#pragma unroll
        for (int s = 0; s < C::KS; ++s)
#pragma unroll
          for (int j = 0; j < 2; ++j) sacc[j] = mfma(qa[s], kf[j][s], sacc[j]);
      }
      __builtin_amdgcn_sched_barrier(0);
      stamp(it, 1);
      // phase B: dP = dO V^T, with P = exp2(S c - LSE log2 e) in the MFMAs' shadow: slice s of the
      // exponentials (4 of the 32 per lane) follows the two MFMAs of k-step s, whose operands were
      // read one slice earlier
      {
        F oa = load_frag<F>(oimg + du_off(r, h));
        F va0 = load_frag<F>(Vs + (wave * 64 + r) * C::RSTR + 8 * h);
        F va1 = load_frag<F>(Vs + (wave * 64 + 32 + r) * C::RSTR + 8 * h);
#pragma unroll
        for (int s = 0; s < C::KS; ++s) {
          F ob = oa, vb0 = va0, vb1 = va1;
          if (s + 1 < C::KS) {
            ob = load_frag<F>(oimg + du_off(r, 2 * (s + 1) + h));
            vb0 = load_frag<F>(Vs + (wave * 64 + r) * C::RSTR + 16 * (s + 1) + 8 * h);
            vb1 = load_frag<F>(Vs + (wave * 64 + 32 + r) * C::RSTR + 16 * (s + 1) + 8 * h);
          }
          pacc[0] = mfma(oa, va0, pacc[0]);
          pacc[1] = mfma(oa, va1, pacc[1]);
          const int j = s >> 2, i0 = 4 * (s & 3);
#pragma unroll
          for (int i = i0; i < i0 + 4; ++i)
            sacc[j][i] = __builtin_amdgcn_exp2f(__builtin_fmaf(sacc[j][i], scale_log2, L[i >> 2][i & 3]));
          if (s == 4 || s == 5) pack_frag(pf[0][s - 4], sacc[0], s - 4);  // half 0 is complete (unmasked form)
          __builtin_amdgcn_sched_barrier(0);
          oa = ob;
          va0 = vb0;
          va1 = vb1;
        }
      }
      stamp(it, 2);
#pragma unroll
      for (int a = 0; a < 4; ++a) Dl[a] = *reinterpret_cast<const f32x4v*>(sl + kQT + 4 * h + 8 * a);
      s16x4t xr[16];
      tr_issue16(xr, tr_a + (unsigned)(st * STAGE + IMG), tr_b + (unsigned)(st * STAGE + IMG));  // dO^T, waited below
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int key = kw + 32 * j + r;
        const bool masked = (CAUSAL && kw + 32 * j + 31 > qbase) || kw + 32 * j + 32 > Sk || qbase + kQT > Tq;
        if (masked) {
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            const int qq = qbase + acc_row(i, h);
            if (key >= Sk || qq >= Tq || (CAUSAL && key > qq)) sacc[j][i] = 0.f;
          }
          if (j == 0) {  // re-pack the masked half 0
            pack_frag(pf[0][0], sacc[0], 0);
            pack_frag(pf[0][1], sacc[0], 1);
          }
        }
      }
      pack_frag(pf[1][0], sacc[1], 0);
      pack_frag(pf[1][1], sacc[1], 1);
      stamp(it, 3);
      {
        F xt[8];
        tr_wait16(xt, xr);
        // phase C: dV^T += dO^T P, with dS = P (dP - delta) and its packing in the MFMAs' shadow
#pragma unroll
        for (int dt = 0; dt < C::DT; ++dt) {
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            mfma_acc_agpr(dvacc[j][dt], xt[2 * dt], pf[j][0]);
            mfma_acc_agpr(dvacc[j][dt], xt[2 * dt + 1], pf[j][1]);
            const int jj = dt >> 1, i0 = 8 * (dt & 1) + 4 * j;
#pragma unroll
            for (int i = i0; i < i0 + 4; ++i) pacc[jj][i] = sacc[jj][i] * (pacc[jj][i] - Dl[i >> 2][i & 3]);
            // sched_barrier does not hold IR-level sinking: pin the slice here, not at the pack below
            asm volatile("" : "+v"(pacc[jj]));
            __builtin_amdgcn_sched_barrier(0);
          }
          if (dt & 1) {  // half dt>>1 of dS complete: pack it
            pack_frag(df[dt >> 1][0], pacc[dt >> 1], 0);
            pack_frag(df[dt >> 1][1], pacc[dt >> 1], 1);
            // half 0's S / dP registers are free now: Q^T's transposed reads (phase D) go out here
            if (dt == 1) tr_issue16(xr, tr_a + (unsigned)(st * STAGE), tr_b + (unsigned)(st * STAGE));
            __builtin_amdgcn_sched_barrier(0);
          }
        }
        stamp(it, 4);
        tr_wait16(xt, xr);  // Q^T
        // phase D: dK^T += Q^T dS
#pragma unroll
        for (int dt = 0; dt < C::DT; ++dt)
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            mfma_acc_agpr(dkacc[j][dt], xt[2 * dt], df[j][0]);
            mfma_acc_agpr(dkacc[j][dt], xt[2 * dt + 1], df[j][1]);
          }
        if constexpr (WDS) {
          // dS^T for the dQ pass (attn_bwd_dq_ds_kernel): [b, hq][query block of 256][key][256] bf16,
          // so the reader's 64-key tiles are contiguous 32 KiB; this lane's 8 packed values of each
          // fragment as one 16-B store at q offset 16 s + 8 h of the 32-query tile (the fragment's own
          // order: query acc_row(8 s + e, h) at offset e; the reader un-permutes).  Streaming stores:
          // the next kernel reads them, nothing in this one does.  Buffer stores: the wave's 64 key rows as one resource whose size drops the rows past Sk,
          // the half j as a scalar offset, so the loop spends one VGPR on the address (every term is
          // wave-uniform; readfirstlane says so, or the resource would be waterfalled)
          const int hq_cur = hbase + it / nq;
          const int nqb = (Tq + 255) >> 8;
          const uint64_t wa = (uint64_t)(uintptr_t)(dSt + ((((int64_t)(b * Hq + hq_cur) * nqb + (qbase >> 8)) * Sk + kw) * 256 +
                                                           (qbase & 255)));
          const uint64_t wu = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(wa >> 32)) << 32) |
                              (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)wa);
          const int wbytes = __builtin_amdgcn_readfirstlane(max(0, min(64, Sk - kw)) * 512);
          const __amdgpu_buffer_rsrc_t rs =
              __builtin_amdgcn_make_buffer_rsrc((void*)(uintptr_t)wu, (short)0, wbytes, 0x00020000);
          const int loff = (r * 256 + 8 * h) * 2;
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(dsi32x4, df[j][0]), rs, loff, j * 16384, 2);
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(dsi32x4, df[j][1]), rs, loff, j * 16384 + 32, 2);
          }
        }
      }
    }
    stamp(it, 5);
    if (issue_next) {
      advance();
      wait_all_but_newest(true);
      stash_stats(st2);
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    stamp(it, 6);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    stamp(it, 7);
    ti = ti + 1 == nq ? 0 : ti + 1;
    st = st == 2 ? 0 : st + 1;
  }
  if constexpr (STAMP != 0) {
    if (blockIdx.x == 0 && blockIdx.y == 0 && dbg != nullptr) {
      __syncthreads();
      for (int i = tid; i < 4 * 64 * 8; i += kThreads) dbg[i] = *reinterpret_cast<const uint64_t*>(smem + SBASE + i * 8);
    }
  }
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int dt = 0; dt < C::DT; ++dt) asm volatile("s_nop 15\n\ts_nop 15" : "+a"(dkacc[j][dt]), "+a"(dvacc[j][dt]));

  if constexpr (SPLIT) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int key = kw + 32 * j + r;
      if (key < Sk) {
        const int64_t nbh = gridDim.x / nsplit;
        float* prow = part + (((int64_t)hs * nbh + bh) * Sk + key) * 256;
        const bool rope = sx.rope_cos != nullptr;
        store_row_d128_f32(prow, dkacc[j], scale, h, rope ? sx.rope_cos + (int64_t)key * 128 : nullptr,
                           rope ? sx.rope_sin + (int64_t)key * 128 : nullptr);
        store_row_d128_f32(prow + 128, dvacc[j], 1.f, h, nullptr, nullptr);
      }
    }
    return;
  }
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int key = kw + 32 * j + r;
    if (key < Sk) {
      T* dkrow = dK + (int64_t)b * sx.dkb + (int64_t)hk * sx.dkh + (int64_t)key * sx.dkt;
      T* dvrow = dV + (int64_t)b * sx.dvb + (int64_t)hk * sx.dvh + (int64_t)key * sx.dvt;
      const bool rope = sx.rope_cos != nullptr;
      store_row_d128(dkrow, dkacc[j], scale, h, rope ? sx.rope_cos + (int64_t)key * 128 : nullptr,
                     rope ? sx.rope_sin + (int64_t)key * 128 : nullptr);
      store_row_d128(dvrow, dvacc[j], 1.f, h, nullptr, nullptr);
    }
  }
}

// ---------------------------------------------------------------------------------------------
// dQ
// ---------------------------------------------------------------------------------------------
constexpr int kBM = 128;
constexpr int kBN = 64;

template <typename T, int D, bool CAUSAL, int EX = 0>
__global__ __launch_bounds__(kThreads, (EX || D > 128) ? 1 : 2) void attn_bwd_dq_kernel(const T* __restrict__ Q, const T* __restrict__ K,
                                                                  const T* __restrict__ V, const T* __restrict__ dO,
                                                                  const float* __restrict__ LSE,
                                                                  const float* __restrict__ DELTA, T* __restrict__ dQ,
                                                                  int Hq, int Hkv, int Tq, int Sk, float scale,
                                                                  float scale_log2, RowStrides sdo, AttnExtra ex) {
  constexpr bool MASK = EX & kExMask, DROP = EX & kExDrop;
  using C = BCfg<D>;
  using F = typename Frag<T>::type;
  __shared__ __attribute__((aligned(16))) short smem[2 * C::BN * C::RSTR + C::BN * C::TSTR];
  __shared__ __attribute__((aligned(16))) unsigned ktab[DROP ? 4 * C::BN : 4];  // per-wave key terms (dropout)
  short* Kr = smem;                    // [64][RSTR]  K rows (A operand of S^T)
  short* Vr = Kr + C::BN * C::RSTR;      // [64][RSTR]  V rows (A operand of dP^T)
  short* Kt = Vr + C::BN * C::RSTR;      // [64][TSTR]  K image for transposed reads (A of dQ^T)
  const __attribute__((address_space(3))) short* Kt3 = (const __attribute__((address_space(3))) short*)Kt;

  const int n_qt = (Tq + kBM - 1) / kBM;
  const int qt = n_qt - 1 - (int)blockIdx.y;
  const int bh = blockIdx.x;
  const int b = bh / Hq, hq = bh % Hq;
  const int hk = hq / (Hq / Hkv);
  const T* Qb = Q + b * ex.sx.qb + hq * ex.sx.qh;
  const T* dOb = dO + b * sdo.b + hq * sdo.h;
  const T* Kb = K + b * ex.sx.kb + hk * ex.sx.kh;
  const T* Vb = V + b * ex.sx.vb + hk * ex.sx.vh;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 31, h = lane >> 5, g = lane >> 4, l16 = lane & 15;
  const int q0 = qt * kBM + wave * 32;
  const int qi = q0 + r;
  const int qrow = min(qi, Tq - 1);

  F qf[C::KS], of[C::KS];
#pragma unroll
  for (int s = 0; s < C::KS; ++s) {
    qf[s] = load_frag<F>(Qb + (int64_t)qrow * ex.sx.qt + 16 * s + 8 * h);
    of[s] = load_frag<F>(dOb + qrow * sdo.t + 16 * s + 8 * h);
  }
  const float lse2 = LSE[((int64_t)b * Hq + hq) * Tq + qrow] * 1.44269504088896340736f;
  const float dlt = DELTA[((int64_t)b * Hq + hq) * Tq + qrow];
  const float* mrow = nullptr;
  if constexpr (MASK) mrow = ex.mask + b * ex.mb + hq * ex.mh + (int64_t)qrow * ex.mq;
  unsigned qterm = 0;
  if constexpr (DROP) qterm = rng_q(rng_head(ex, bh), qi);

  f32x16 dqacc[C::DT];
#pragma unroll
  for (int dt = 0; dt < C::DT; ++dt)
#pragma unroll
    for (int i = 0; i < 16; ++i) dqacc[dt][i] = 0.f;

  int n_tiles = (Sk + C::BN - 1) / C::BN;
  if (CAUSAL) n_tiles = min(n_tiles, (min(qt * kBM + kBM, Tq) + C::BN - 1) / C::BN);
  constexpr int LOADS = C::BN * C::CH / kThreads;
  static_assert(C::BN * C::CH % kThreads == 0, "K/V staging must cover the tile");

  // K/V tiles are prefetched into registers one tile ahead (latency hides behind the MFMAs).
  uint4 pk[LOADS], pv[LOADS];
  auto issue = [&](int t) {
#pragma unroll
    for (int c = 0; c < LOADS; ++c) {
      const int id = c * kThreads + tid;
      const int row = id / C::CH, ch = id % C::CH;
      const int kc = min(t * C::BN + row, Sk - 1);
      pk[c] = *reinterpret_cast<const uint4*>(Kb + (int64_t)kc * ex.sx.kt + ch * 8);
      pv[c] = *reinterpret_cast<const uint4*>(Vb + (int64_t)kc * ex.sx.vt + ch * 8);
    }
  };
  if (n_tiles > 0) issue(0);
  for (int t = 0; t < n_tiles; ++t) {
    __syncthreads();
#pragma unroll
    for (int c = 0; c < LOADS; ++c) {
      const int id = c * kThreads + tid;
      const int row = id / C::CH, ch = id % C::CH;
      uint4 xk = pk[c], xv = pv[c];
      if (t * C::BN + row >= Sk) {
        xk = make_uint4(0, 0, 0, 0);
        xv = make_uint4(0, 0, 0, 0);
      }
      *reinterpret_cast<uint4*>(Kr + row * C::RSTR + ch * 8) = xk;
      *reinterpret_cast<uint4*>(Vr + row * C::RSTR + ch * 8) = xv;
      *reinterpret_cast<uint4*>(Kt + row * C::TSTR + ch * 8) = xk;
    }
    __syncthreads();
    if (t + 1 < n_tiles) issue(t + 1);

    f32x16 sacc[C::NKT], pacc[C::NKT];
#pragma unroll
    for (int kt = 0; kt < C::NKT; ++kt)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        sacc[kt][i] = 0.f;
        pacc[kt][i] = 0.f;
      }
#pragma unroll
    for (int s = 0; s < C::KS; ++s) {
#pragma unroll
      for (int kt = 0; kt < C::NKT; ++kt) {
        const F ka = load_frag<F>(Kr + (kt * 32 + r) * C::RSTR + 16 * s + 8 * h);
        const F va = load_frag<F>(Vr + (kt * 32 + r) * C::RSTR + 16 * s + 8 * h);
        sacc[kt] = mfma(ka, qf[s], sacc[kt]);  // S^T = K Q^T
        pacc[kt] = mfma(va, of[s], pacc[kt]);  // dP^T = V dO^T
      }
    }
    const int kbase = t * C::BN;
    [[maybe_unused]] unsigned* krow = ktab + wave * C::BN;
    if constexpr (DROP)
      if (lane < C::BN) krow[lane] = rng_k(kbase + lane);
    if constexpr (MASK) {
#pragma unroll
      for (int kt = 0; kt < C::NKT; ++kt)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float4 mv = *reinterpret_cast<const float4*>(mrow + kbase + kt * 32 + 8 * j + 4 * h);
          sacc[kt][4 * j + 0] = sacc[kt][4 * j + 0] * scale_log2 + mv.x * 1.44269504088896340736f;
          sacc[kt][4 * j + 1] = sacc[kt][4 * j + 1] * scale_log2 + mv.y * 1.44269504088896340736f;
          sacc[kt][4 * j + 2] = sacc[kt][4 * j + 2] * scale_log2 + mv.z * 1.44269504088896340736f;
          sacc[kt][4 * j + 3] = sacc[kt][4 * j + 3] * scale_log2 + mv.w * 1.44269504088896340736f;
        }
    }
#pragma unroll
    for (int kt = 0; kt < C::NKT; ++kt) {
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int kk = kbase + kt * 32 + acc_row(i, h);
        float p = __builtin_amdgcn_exp2f((MASK ? sacc[kt][i] : sacc[kt][i] * scale_log2) - lse2);
        p = (kk >= Sk || (CAUSAL && kk > qi)) ? 0.f : p;
        float dp = pacc[kt][i];
        if constexpr (DROP) {
          const uint4 kv = rng_tab4(krow + kt * 32, i >> 2, h);
          const unsigned kw4[4] = {kv.x, kv.y, kv.z, kv.w};
          const bool keep = rng_keep(ex, qterm, kw4[i & 3]);
          dp = keep ? dp * ex.keep_scale : 0.f;
        }
        pacc[kt][i] = p * (dp - dlt);  // dS^T
      }
    }
    F df[C::NKT][2];
#pragma unroll
    for (int kt = 0; kt < C::NKT; ++kt) {
      pack_frag(df[kt][0], pacc[kt], 0);
      pack_frag(df[kt][1], pacc[kt], 1);
    }
#pragma unroll
    for (int dt = 0; dt < C::DT; ++dt) {
      const int col0 = dt * 32 + 16 * (g & 1);
#pragma unroll
      for (int kt = 0; kt < C::NKT; ++kt) {
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          const F ka = tr_frag<F>(Kt3, kt * 32 + 16 * s + 4 * h, col0, C::TSTR, l16);
          dqacc[dt] = mfma(ka, df[kt][s], dqacc[dt]);  // dQ^T += K^T dS^T
        }
      }
    }
  }

  if (qi < Tq) {
    T* drow = dQ + (int64_t)b * ex.sx.dqb + (int64_t)hq * ex.sx.dqh + (int64_t)qi * ex.sx.dqt;
#pragma unroll
    for (int dt = 0; dt < C::DT; ++dt) {
#pragma unroll
      for (int a = 0; a < 4; ++a) {
        const int d = dt * 32 + 8 * a + 4 * h;
        union {
          T v[4];
          uint2 u;
        } pk;
#pragma unroll
        for (int e = 0; e < 4; ++e) pk.v[e] = from_f32<T>(dqacc[dt][4 * a + e] * scale);
        *reinterpret_cast<uint2*>(drow + d) = pk.u;
      }
    }
  }
}

// ---------------------------------------------------------------------------------------------
// dQ, D = 128: one workgroup per 256 queries, 64 per wave in two 32-row halves: Q rows in registers
// (B operand of S^T = K Q^T), the workgroup's dO rows in LDS (B operand of dP^T = V dO^T), 32-key
// K / V tiles streamed by global_load_lds into a 3-stage ring of images that serve the row reads
// of S^T / dP^T and the transposed reads of dQ^T += K^T dS^T; dQ^T accumulates in the AGPR file.
// (The retired v2 / v3 dQ kernels: profiles/attn_dq_v3_ab.txt.)
// ---------------------------------------------------------------------------------------------
constexpr int kQB3 = 256;  // queries per workgroup
constexpr int kKT3 = 32;   // keys per streamed tile

// dQ v4: v3's data flow with the VALU work of a tile in the MFMA shadows (as dK/dV v4):
//   A: S^T half 0 (8 MFMA), S^T half 1 (8) | P half 0      B0: dP^T half 0 (8) | P half 1
//   B1: dP^T half 1 (8) | dS^T half 0, pack                 C0: dQ^T half 0 (8) | dS^T half 1, pack
//   C1: dQ^T half 1 (8)
// The dP^T chains start at -delta (row constant as the initial accumulator), so dS^T = P * acc.
template <typename T, bool CAUSAL>
__global__ __launch_bounds__(kThreads, 1) void attn_bwd_dq_v4_kernel(const T* __restrict__ Q, const T* __restrict__ K,
                                                                     const T* __restrict__ V, const T* __restrict__ dO,
                                                                     const float* __restrict__ LSE,
                                                                     const float* __restrict__ DELTA, T* __restrict__ dQ,
                                                                     int Hq, int Hkv, int Tq, int Sk, float scale,
                                                                     float scale_log2, RowStrides sdo, QKVStrides sx,
                                                                     const T* __restrict__ O = nullptr, RowStrides so = {}) {
  constexpr int D = 128;
  using C = BCfg<D>;
  using F = typename Frag<T>::type;
  constexpr int NST = 3;
  constexpr int IMG = kKT3 * 256;  // 32 rows x 128 x 16-bit
  constexpr int STAGE = 2 * IMG;   // K image, V image
  constexpr int OOFF = NST * STAGE;
  __shared__ __attribute__((aligned(1024))) char smem[OOFF + kQB3 * C::RSTR * 2];
  short* Os = reinterpret_cast<short*>(smem + OOFF);

  const int n_qb = (Tq + kQB3 - 1) / kQB3;
  const int qb = n_qb - 1 - (int)blockIdx.y;  // heaviest causal blocks first
  const int bh = blockIdx.x;
  const int b = bh / Hq, hq = bh % Hq;
  const int hk = hq / (Hq / Hkv);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 31, h = lane >> 5;
  const int qw = qb * kQB3 + wave * 64;  // this wave's first query; half j: queries qw + 32 j + r
  const T* Qb = Q + b * sx.qb + hq * sx.qh;
  const T* dOb = dO + b * sdo.b + hq * sdo.h;
  const T* Kb = K + b * sx.kb + hk * sx.kh;
  const T* Vb = V + b * sx.vb + hk * sx.vh;

  // dO rows of the workgroup's 256 queries -> LDS; Q rows and row statistics of this wave's 64
  // queries -> registers (rows past Tq are clamped copies; their dQ is not stored)
#pragma unroll
  for (int c = 0; c < kQB3 * C::CH / kThreads; ++c) {
    const int id = c * kThreads + tid;
    const int row = id / C::CH, ch = id % C::CH;
    const int orow = min(qb * kQB3 + row, Tq - 1);
    *reinterpret_cast<uint4*>(Os + row * C::RSTR + ch * 8) = *reinterpret_cast<const uint4*>(dOb + (int64_t)orow * sdo.t + ch * 8);
  }
  constexpr float kLog2e = 1.44269504088896340736f;
  F qf[2][C::KS];
  float nl2[2], dl[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int qr = min(qw + 32 * j + r, Tq - 1);
#pragma unroll
    for (int s = 0; s < C::KS; ++s) qf[j][s] = load_frag<F>(Qb + (int64_t)qr * sx.qt + 16 * s + 8 * h);
    nl2[j] = -LSE[((int64_t)b * Hq + hq) * Tq + qr] * kLog2e;
    if (O != nullptr) {  // delta = rowsum(dO * O) here (no preprocess launch; dK/dV runs after this kernel)
      const T* Orow = O + (int64_t)b * so.b + (int64_t)hq * so.h + (int64_t)qr * so.t;
      const T* Drow = dOb + (int64_t)qr * sdo.t;
      float acc = 0.f;
#pragma unroll
      for (int s = 0; s < C::KS; ++s) {
        const F ov = load_frag<F>(Orow + 16 * s + 8 * h), dv = load_frag<F>(Drow + 16 * s + 8 * h);
#pragma unroll
        for (int e = 0; e < 8; ++e) acc += (float)dv[e] * (float)ov[e];
      }
      dl[j] = acc + __shfl_xor(acc, 32, 64);
      if (h == 0 && qw + 32 * j + r < Tq) const_cast<float*>(DELTA)[((int64_t)b * Hq + hq) * Tq + qw + 32 * j + r] = dl[j];
    } else {
      dl[j] = DELTA[((int64_t)b * Hq + hq) * Tq + qr];
    }
  }

  f32x16 dqacc[2][C::DT];
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int dt = 0; dt < C::DT; ++dt)
#pragma unroll
      for (int i = 0; i < 16; ++i) dqacc[j][dt][i] = 0.f;

  int n_kt = (Sk + kKT3 - 1) / kKT3;
  if (CAUSAL) n_kt = min(n_kt, (min(qb * kQB3 + kQB3, Tq) + kKT3 - 1) / kKT3);

  // one 32-key tile: 8 x 1 KiB of K and of V per workgroup, lane-linear DMA into layout (a)
  // (the swizzle is applied to the source row / chunk; see dK/dV v3)
  auto issue = [&](int t, int st) {
    char* kimg = smem + st * STAGE;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int k = wave * 2 + i;
      const int u = 64 * k + lane;
      const int row = ((u >> 7) << 3) | ((u >> 2) & 7);
      const int ch = (((u >> 5) & 3) << 2) | ((u & 3) ^ ((row >> 2) & 3));
      const int kc = min(t * kKT3 + row, Sk - 1);
      __builtin_amdgcn_global_load_lds((const void*)(Kb + (int64_t)kc * sx.kt + ch * 8), (lds_void*)(kimg + k * 1024), 16,
                                       0, 0);
      __builtin_amdgcn_global_load_lds((const void*)(Vb + (int64_t)kc * sx.vt + ch * 8),
                                       (lds_void*)(kimg + IMG + k * 1024), 16, 0, 0);
    }
  };
  if (n_kt > 0) issue(0, 0);
  if (n_kt > 1) {
    issue(1, 1);
    asm volatile("s_waitcnt vmcnt(4)" ::: "memory");  // tile 0 landed (tile 1 may be in flight)
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();

  unsigned tr_a, tr_b;
  {
    const int l16 = lane & 15, g = lane >> 4;
    const int q = l16 >> 2, p = l16 & 3, cl = 2 * (g & 1) + (p >> 1);
    const unsigned base = (unsigned)(uintptr_t)(__attribute__((address_space(3))) char*)smem;
    tr_a = base + 64 * (4 * h + q) + 16 * (cl ^ h) + 8 * (p & 1);
    tr_b = base + 2048 + 64 * (4 * h + q) + 16 * (cl ^ (2 + h)) + 8 * (p & 1);
  }
  int st = 0;
  for (int t = 0; t < n_kt; ++t) {
    const bool issue_next = t + 2 < n_kt;
    const int st2 = st >= 1 ? st - 1 : 2;
    if (issue_next) issue(t + 2, st2);
    const char* kimg = smem + st * STAGE;
    const char* vimg = kimg + IMG;
    const short* o0 = Os + (wave * 64 + r) * C::RSTR + 8 * h;  // dO rows of half 0 (half 1: + 32 rows)
    const int kbase = t * kKT3;
    f32x16 sacc[2], pacc[2];
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        sacc[j][i] = 0.f;
        pacc[j][i] = -dl[j];  // the dP^T chain starts at -delta: it ends as dP - delta
      }
    auto exp_slice = [&](int j, int i0, int n) {
#pragma unroll
      for (int i = i0; i < i0 + n; ++i)
        sacc[j][i] = __builtin_amdgcn_exp2f(__builtin_fmaf(sacc[j][i], scale_log2, nl2[j]));
    };
    auto mask_half = [&](int j) {  // wave-uniform: only tiles on the diagonal or the key edge
      const int qi = qw + 32 * j + r;
      if (kbase + kKT3 > Sk || (CAUSAL && kbase + kKT3 - 1 > qw + 32 * j)) {
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int key = kbase + acc_row(i, h);
          if (key >= Sk || (CAUSAL && key > qi)) sacc[j][i] = 0.f;
        }
      }
    };
    // phase A: S^T = K Q^T, half 0 then half 1; P of half 0 in the second chain's shadow
    F fa[C::KS];
#pragma unroll
    for (int s = 0; s < C::KS; ++s) fa[s] = load_frag<F>(kimg + du_off(r, 2 * s + h));
#pragma unroll
    for (int s = 0; s < C::KS; ++s) sacc[0] = mfma(fa[s], qf[0][s], sacc[0]);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int s = 0; s < C::KS; ++s) {
      sacc[1] = mfma(fa[s], qf[1][s], sacc[1]);
      exp_slice(0, 2 * s, 2);
      __builtin_amdgcn_sched_barrier(0);
    }
    mask_half(0);
    // V fragments (A operand of both dP^T chains) replace the K fragments
#pragma unroll
    for (int s = 0; s < C::KS; ++s) fa[s] = load_frag<F>(vimg + du_off(r, 2 * s + h));
    // phase B0: dP^T of half 0 | P of half 1
    {
      F oa = load_frag<F>(o0);
#pragma unroll
      for (int s = 0; s < C::KS; ++s) {
        F ob = oa;
        if (s + 1 < C::KS) ob = load_frag<F>(o0 + 16 * (s + 1));
        pacc[0] = mfma(fa[s], oa, pacc[0]);
        exp_slice(1, 2 * s, 2);
        __builtin_amdgcn_sched_barrier(0);
        oa = ob;
      }
    }
    mask_half(1);
    // K^T transposed reads for the dQ chains go out now (waited before phase C)
    s16x4t xr[16];
    tr_issue16(xr, tr_a + (unsigned)(st * STAGE), tr_b + (unsigned)(st * STAGE));
    // phase B1: dP^T of half 1 | dS^T = P (dP - delta) of half 0 (its chain is complete), packed
    F df[2][2];
    {
      F oa = load_frag<F>(o0 + 32 * C::RSTR);
#pragma unroll
      for (int s = 0; s < C::KS; ++s) {
        F ob = oa;
        if (s + 1 < C::KS) ob = load_frag<F>(o0 + 32 * C::RSTR + 16 * (s + 1));
        pacc[1] = mfma(fa[s], oa, pacc[1]);
#pragma unroll
        for (int i = 2 * s; i < 2 * s + 2; ++i) pacc[0][i] *= sacc[0][i];
        asm volatile("" : "+v"(pacc[0]));  // keep the slice here (sched_barrier does not stop IR sinking)
        if (s == 7) {
          pack_frag(df[0][0], pacc[0], 0);
          pack_frag(df[0][1], pacc[0], 1);
        }
        __builtin_amdgcn_sched_barrier(0);
        oa = ob;
      }
    }
    {
      F xt[8];
      tr_wait16(xt, xr);
      // phase C0: dQ^T += K^T dS^T of half 0 | dS^T of half 1, packed
#pragma unroll
      for (int dt = 0; dt < C::DT; ++dt) {
        mfma_acc_agpr(dqacc[0][dt], xt[2 * dt], df[0][0]);
        mfma_acc_agpr(dqacc[0][dt], xt[2 * dt + 1], df[0][1]);
#pragma unroll
        for (int i = 4 * dt; i < 4 * dt + 4; ++i) pacc[1][i] *= sacc[1][i];
        asm volatile("" : "+v"(pacc[1]));
        __builtin_amdgcn_sched_barrier(0);
      }
      pack_frag(df[1][0], pacc[1], 0);
      pack_frag(df[1][1], pacc[1], 1);
      // phase C1: dQ^T of half 1
#pragma unroll
      for (int dt = 0; dt < C::DT; ++dt) {
        mfma_acc_agpr(dqacc[1][dt], xt[2 * dt], df[1][0]);
        mfma_acc_agpr(dqacc[1][dt], xt[2 * dt + 1], df[1][1]);
      }
    }
    if (issue_next)
      asm volatile("s_waitcnt vmcnt(4)" ::: "memory");  // tile t+1 landed; t+2 may be in flight
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    st = st == 2 ? 0 : st + 1;
  }
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int dt = 0; dt < C::DT; ++dt) asm volatile("s_nop 15\n\ts_nop 15" : "+a"(dqacc[j][dt]));

#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int qi = qw + 32 * j + r;
    if (qi < Tq) {
      T* drow = dQ + (int64_t)b * sx.dqb + (int64_t)hq * sx.dqh + (int64_t)qi * sx.dqt;
      const bool rope = sx.rope_cos != nullptr;
      store_row_d128(drow, dqacc[j], scale, h, rope ? sx.rope_cos + (int64_t)qi * 128 : nullptr,
                     rope ? sx.rope_sin + (int64_t)qi * 128 : nullptr);
    }
  }
}

// ---------------------------------------------------------------------------------------------
// dQ from the stored dS (LTA_ATTN_DQ_FROM_DS, D = 128): the dK/dV kernel already forms dS = P (dP -
// delta) for every (key, query) pair and writes it (bf16, [b, hq][query block][key][256 queries],
// 0.5 GB per causal Llama-2-7B layer); dQ = scale dS K is then one streaming product per head instead of a second pass that
// recomputes S, P and dP (two of the dQ v4 kernel's three MFMA chains).  Workgroup: 256 queries x all
// 128 d, 4 waves of 64 queries; 64-key tiles of K ([key][d], 16 KiB) and dS^T ([key][query], 32 KiB)
// stream through a 3-stage LDS-DMA ring; dQ^T[d][q] = K^T dS^T on 32x32x16 MFMAs with both operands
// read by ds_read_b64_tr_b16 (chunk c of row R at slot c ^ ((R & 3) << 2): conflict-free), so each
// lane ends up owning one query row of dQ (the dK epilogue's store, RoPE transpose included).
// Host: Tq == Sk, Sk % 64 == 0, Tq % 32 == 0.
// one 16-key step of the dQ-from-dS product: the transposed fragments of 4 K^T blocks (256-B rows)
// and 2 dS^T blocks (512-B rows), rows 16 S + {0..3} and + 8.  Inline asm: the compiler's LDS-DMA
// alias tracking would put a vmcnt(0) in front of builtin LDS reads (a full memory round trip per
// tile); the ring's own vmcnt + barrier order them
template <int S>
__device__ __forceinline__ void dqds_issue(s16x4t (&x)[12], const uint32_t (&ka)[4], const uint32_t (&sa)[2]) {
  asm volatile(
      "ds_read_b64_tr_b16 %0, %12 offset:%18\n\tds_read_b64_tr_b16 %1, %12 offset:%19\n\t"
      "ds_read_b64_tr_b16 %2, %13 offset:%18\n\tds_read_b64_tr_b16 %3, %13 offset:%19\n\t"
      "ds_read_b64_tr_b16 %4, %14 offset:%18\n\tds_read_b64_tr_b16 %5, %14 offset:%19\n\t"
      "ds_read_b64_tr_b16 %6, %15 offset:%18\n\tds_read_b64_tr_b16 %7, %15 offset:%19\n\t"
      "ds_read_b64_tr_b16 %8, %16 offset:%20\n\tds_read_b64_tr_b16 %9, %16 offset:%21\n\t"
      "ds_read_b64_tr_b16 %10, %17 offset:%20\n\tds_read_b64_tr_b16 %11, %17 offset:%21"
      : "=&v"(x[0]), "=&v"(x[1]), "=&v"(x[2]), "=&v"(x[3]), "=&v"(x[4]), "=&v"(x[5]), "=&v"(x[6]), "=&v"(x[7]),
        "=&v"(x[8]), "=&v"(x[9]), "=&v"(x[10]), "=&v"(x[11])
      : "v"(ka[0]), "v"(ka[1]), "v"(ka[2]), "v"(ka[3]), "v"(sa[0]), "v"(sa[1]), "i"(S * 4096), "i"(S * 4096 + 2048),
        "i"(S * 8192), "i"(S * 8192 + 4096)
      : "memory");
}

template <int S, int NSS, typename F>
__device__ __forceinline__ void dqds_steps(f32x16 (&acc)[2][4], s16x4t (&cur)[12], s16x4t (&nxt)[12],
                                           const uint32_t (&ka)[4], const uint32_t (&sa)[2]) {
  asm volatile("s_waitcnt lgkmcnt(0)"
               : "+v"(cur[0]), "+v"(cur[1]), "+v"(cur[2]), "+v"(cur[3]), "+v"(cur[4]), "+v"(cur[5]), "+v"(cur[6]),
                 "+v"(cur[7]), "+v"(cur[8]), "+v"(cur[9]), "+v"(cur[10]), "+v"(cur[11])
               :
               : "memory");
  if constexpr (S + 1 < NSS) dqds_issue<S + 1>(nxt, ka, sa);
  F f[6];
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    union {
      struct {
        s16x4t a, b;
      } s;
      F f;
    } u;
    u.s.a = cur[2 * i];
    u.s.b = cur[2 * i + 1];
    f[i] = u.f;
  }
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) mfma_acc_agpr(acc[x][dt], f[dt], f[4 + x]);
  if constexpr (S + 1 < NSS) dqds_steps<S + 1, NSS, F>(acc, nxt, cur, ka, sa);
}

template <typename T, bool CAUSAL>
__global__ __launch_bounds__(kThreads, 1) void attn_bwd_dq_ds_kernel(const T* __restrict__ K, const T* __restrict__ dSt,
                                                                     T* __restrict__ dQ, int Hq, int Hkv, int Tq, int Sk,
                                                                     float scale, QKVStrides sx) {
  using F = typename Frag<T>::type;
  // KT-key tiles, NST-stage ring, NST - 1 tiles in flight (64 x 3 measured best of 64 x 3, 32 x 6,
  // 16 x 10 and two-workgroups-per-CU 32 x 3 / 16 x 6: profiles/attn_dq_from_ds.txt)
  constexpr int KT = 64, NST = 3;
  constexpr int KIMG = KT * 256, SIMG = KT * 512, STG = KIMG + SIMG;
  constexpr int NK = KT / 16, NS = KT / 8;  // LDS-DMA instructions per wave per tile: K, dS^T
  static_assert(KT % 16 == 0 && NST * STG <= 160 * 1024, "dq_ds tiling");
  __shared__ __attribute__((aligned(1024))) char smem[NST * STG];
  const int n_qb = (Tq + 255) / 256;
  const int qb = CAUSAL ? n_qb - 1 - (int)blockIdx.y : (int)blockIdx.y;  // causal: heavy blocks first
  const int bh = blockIdx.x, b = bh / Hq, hq = bh % Hq, hk = hq / (Hq / Hkv);
  const int q0 = qb * 256;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int hh = lane >> 5, g = lane >> 4, l16 = lane & 15, vq = l16 >> 2, vp = l16 & 3;
  const T* Kb = K + b * sx.kb + hk * sx.kh;
  const T* Sb = dSt + ((int64_t)bh * n_qb + qb) * Sk * 256;
  const int kend = CAUSAL ? min(Sk, q0 + 256) : Sk;
  const int nt = (kend + KT - 1) / KT;
  const uint32_t lds0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)smem;

  // LDS-DMA of key tile t into stage st: wave w fills K rows KT/4 w .. (NK pieces of 4 rows) and
  // dS^T rows KT/4 w .. (NS pieces of 2 rows of 512 B); the swizzle is applied to the source chunk
  auto issue = [&](int t, int st) {
    char* kimg = smem + st * STG;
    char* simg = kimg + KIMG;
#pragma unroll
    for (int i = 0; i < NK; ++i) {
      const int R = (KT / 4) * wave + 4 * i + (lane >> 4), slot = lane & 15, c = slot ^ ((R & 3) << 2);
      __builtin_amdgcn_global_load_lds((const void*)(Kb + (int64_t)(t * KT + R) * sx.kt + c * 8),
                                       (lds_void*)(kimg + (NK * wave + i) * 1024), 16, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < NS; ++i) {
      const int R = (KT / 4) * wave + 2 * i + (lane >> 5), slot = lane & 31, c = slot ^ ((R & 3) << 2);
      // columns past Tq of a partial last block were never written: they only reach unstored dQ rows
      // dS is read exactly once: nontemporal (aux nt), so it streams past the L2 that keeps K
      __builtin_amdgcn_global_load_lds((const void*)(Sb + (int64_t)(t * KT + R) * 256 + c * 8),
                                       (lds_void*)(simg + (NS * wave + i) * 1024), 16, 0, 2);
    }
  };
  // transposed fragments (keys 16 s + 4 hh + {0..3, 8..11} of 32-column block `blk`) of the
  // [key][column] images: this lane's byte offsets for s = 0
  uint32_t koff[4], soff[2];
#pragma unroll
  for (int blk = 0; blk < 4; ++blk)
    koff[blk] = (4 * hh + vq) * 256 + ((4 * (blk ^ vq) + 2 * (g & 1) + (vp >> 1)) << 4) + 8 * (vp & 1);
#pragma unroll
  for (int x = 0; x < 2; ++x)
    soff[x] = (4 * hh + vq) * 512 + ((4 * ((2 * wave + x) ^ vq) + 2 * (g & 1) + (vp >> 1)) << 4) + 8 * (vp & 1);

  f32x16 acc[2][4];
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int dt = 0; dt < 4; ++dt)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[x][dt][i] = 0.f;

#pragma unroll
  for (int p = 0; p < NST - 1; ++p)
    if (p < nt) issue(p, p);
  for (int t = 0; t < nt; ++t) {
    // tile t landed: tile t + 1 (NK + NS pieces per wave) may still be in flight
    static_assert(NST == 3, "one tile in flight behind the one waited for");
    if (t + 1 < nt)
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NK + NS) : "memory");
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // ... for every wave; stage (t + NST - 1) % NST (tile t - 1) is free
    if (t + NST - 1 < nt) issue(t + NST - 1, (t + NST - 1) % NST);
    const uint32_t kimg = lds0 + (t % NST) * STG, simg = kimg + KIMG;
    const uint32_t ka[4] = {kimg + koff[0], kimg + koff[1], kimg + koff[2], kimg + koff[3]};
    const uint32_t sa[2] = {simg + soff[0], simg + soff[1]};
    s16x4t xa[12], xb[12];
    dqds_issue<0>(xa, ka, sa);
    dqds_steps<0, KT / 16, F>(acc, xa, xb, ka, sa);
  }
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) asm volatile("s_nop 15\n\ts_nop 15" : "+a"(acc[x][dt]));
  // lane column n of block 2 wave + x holds stored query offset n: query acc_row(8 s + e, h) of the
  // 32-query tile for n = 16 s + 8 h + e (the dK/dV kernel's fragment order)
  const bool rope = sx.rope_cos != nullptr;
#pragma unroll
  for (int x = 0; x < 2; ++x) {
    const int n = lane & 31, e = n & 7;
    const int q = q0 + 32 * (2 * wave + x) + (e & 3) + 8 * (e >> 2) + 4 * ((n >> 3) & 1) + 16 * (n >> 4);
    if (q < Tq) {
      T* qrow = dQ + (int64_t)b * sx.dqb + (int64_t)hq * sx.dqh + (int64_t)q * sx.dqt;
      store_row_d128(qrow, acc[x], scale, hh, rope ? sx.rope_cos + (int64_t)q * 128 : nullptr,
                     rope ? sx.rope_sin + (int64_t)q * 128 : nullptr);
    }
  }
}


template <typename T, int D, int EX>
void launch_masked(const void* dO, const void* Q, const void* K, const void* V, const void* LSE, void* DELTA, void* dQ,
                   void* dK, void* dV, int B, int Hq, int Hkv, int Tq, int Sk, float scale, float sl2, int causal,
                   RowStrides sdo, const AttnExtra& ex, hipStream_t s) {
  dim3 g1(B * Hkv, (Sk + kKB - 1) / kKB), g2(B * Hq, (Tq + kBM - 1) / kBM), blk(kThreads);
  constexpr int EXQ = EX & (kExMask | kExDrop);
#define LTA_DKDV(CA)                                                                                               \
  hipLaunchKernelGGL((attn_bwd_dkdv_kernel<T, D, CA, EX>), g1, blk, 0, s, (const T*)Q, (const T*)K, (const T*)V,   \
                     (const T*)dO, (const float*)LSE, (const float*)DELTA, (T*)dK, (T*)dV, Hq, Hkv, Tq, Sk, scale, sl2, \
                     sdo, ex)
#define LTA_DQ(CA)                                                                                                 \
  hipLaunchKernelGGL((attn_bwd_dq_kernel<T, D, CA, EXQ>), g2, blk, 0, s, (const T*)Q, (const T*)K, (const T*)V,    \
                     (const T*)dO, (const float*)LSE, (const float*)DELTA, (T*)dQ, Hq, Hkv, Tq, Sk, scale, sl2, sdo, ex)
  if (causal) {
    LTA_DKDV(true);
    LTA_DQ(true);
  } else {
    LTA_DKDV(false);
    LTA_DQ(false);
  }
#undef LTA_DKDV
#undef LTA_DQ
}

#ifdef LTA_ATTN_DIAG
uint64_t* g_dkdv_stamps = nullptr;  // diagnostic builds: dK/dV phase stamps (lta_attn_bwd_set_stamps)
#endif
// dK/dV sweep order of the D = 128 kernel: query tiles last-to-first (A/B: LTA_DKDV_QREV=0)
int g_dkdv_qrev = [] {
  const char* e = getenv("LTA_DKDV_QREV");
  return (e && e[0] == '0') ? 0 : 1;
}();

#ifdef LTA_ATTN_DIAG
#define LTA_DKDV_LAUNCH(CA)                                                                                          \
  if (g_dkdv_stamps)                                                                                                 \
    hipLaunchKernelGGL((attn_bwd_dkdv_v4_kernel<T, CA, 1>), gk, blk, 0, s, (const T*)Q, (const T*)K, (const T*)V,   \
                       (const T*)dO, (const float*)LSE, (const float*)DELTA, (T*)dK, (T*)dV, Hq, Hkv, Tq, Sk, scale, \
                       sl2, sdo, ex.sx, g_dkdv_qrev, g_dkdv_stamps);                                                  \
  else                                                                                                               \
    hipLaunchKernelGGL((attn_bwd_dkdv_v4_kernel<T, CA>), gk, blk, 0, s, (const T*)Q, (const T*)K, (const T*)V,       \
                       (const T*)dO, (const float*)LSE, (const float*)DELTA, (T*)dK, (T*)dV, Hq, Hkv, Tq, Sk, scale, \
                       sl2, sdo, ex.sx, g_dkdv_qrev, nullptr)
#else
#define LTA_DKDV_LAUNCH(CA)                                                                                          \
  {                                                                                                                  \
    const int hsplit = (ex.part && ex.hsplit > 1) ? ex.hsplit : 1;                                                   \
    dim3 gks(gk.x * hsplit, gk.y);                                                                                   \
    if (hsplit > 1) {                                                                                                \
      hipLaunchKernelGGL((attn_bwd_dkdv_v4_kernel<T, CA, 0, false, true>), gks, blk, 0, s, (const T*)Q, (const T*)K, \
                         (const T*)V, (const T*)dO, (const float*)LSE, (const float*)DELTA, (T*)dK, (T*)dV, Hq, Hkv,   \
                         Tq, Sk, scale, sl2, sdo, ex.sx, g_dkdv_qrev, nullptr, nullptr, hsplit, ex.part);            \
      launch_dkdv_reduce<T>(dK, dV, B, Hkv, Sk, ex, s);                                                              \
    } else {                                                                                                         \
      hipLaunchKernelGGL((attn_bwd_dkdv_v4_kernel<T, CA>), gk, blk, 0, s, (const T*)Q, (const T*)K, (const T*)V,     \
                         (const T*)dO, (const float*)LSE, (const float*)DELTA, (T*)dK, (T*)dV, Hq, Hkv, Tq, Sk,       \
                         scale, sl2, sdo, ex.sx, g_dkdv_qrev, nullptr);                                              \
    }                                                                                                                \
  }
#endif

// Sum of the GQA head split's fp32 partial dK / dV rows -> the gradients' dtype at their strides.
// One thread per 8 consecutive d of one (kv head, key, dK|dV) row.
template <typename T, int D = 128>
__global__ __launch_bounds__(256) void attn_bwd_dkdv_reduce(const float* __restrict__ part, T* __restrict__ dK,
                                                            T* __restrict__ dV, int nbh, int Hkv, int Sk, int hsplit,
                                                            QKVStrides sx) {
  constexpr int CH = D / 8;  // 8-float chunks per row
  const int64_t id = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (id >= (int64_t)nbh * Sk * 2 * CH) return;
  const int c = (int)(id % CH);
  const int64_t row = id / CH;  // (bh * Sk + key) * 2 + which
  const int which = (int)(row & 1);
  const int64_t bk = row >> 1;
  const int key = (int)(bk % Sk), bh = (int)(bk / Sk);
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (int s = 0; s < hsplit; ++s) {
    const float4* src = reinterpret_cast<const float4*>(part + (((int64_t)s * nbh + bh) * Sk + key) * (2 * D) + which * D + c * 8);
    const float4 a = src[0], b = src[1];
    acc[0] += a.x; acc[1] += a.y; acc[2] += a.z; acc[3] += a.w;
    acc[4] += b.x; acc[5] += b.y; acc[6] += b.z; acc[7] += b.w;
  }
  const int b = bh / Hkv, hk = bh % Hkv;
  T* dst = which ? dV + (int64_t)b * sx.dvb + (int64_t)hk * sx.dvh + (int64_t)key * sx.dvt
                 : dK + (int64_t)b * sx.dkb + (int64_t)hk * sx.dkh + (int64_t)key * sx.dkt;
  union {
    T v[8];
    uint4 u;
  } pk;
#pragma unroll
  for (int e = 0; e < 8; ++e) pk.v[e] = from_f32<T>(acc[e]);
  *reinterpret_cast<uint4*>(dst + c * 8) = pk.u;
}

template <typename T, int D = 128>
void launch_dkdv_reduce(void* dK, void* dV, int B, int Hkv, int Sk, const AttnExtra& ex, hipStream_t s) {
  const int64_t n = (int64_t)B * Hkv * Sk * 2 * (D / 8);
  hipLaunchKernelGGL((attn_bwd_dkdv_reduce<T, D>), dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s,
                     (const float*)ex.part, (T*)dK, (T*)dV, B * Hkv, Hkv, Sk, ex.hsplit, ex.sx);
}

// dQ from the stored dS (attn_bwd_dq_ds_kernel): delta by the preprocess kernel, dK / dV (+ dS^T
// into ds_ws), then the dQ product.  D = 128, Tq == Sk, Sk % 64 == 0, Tq % 32 == 0.
template <typename T>
int launch_bwd_ds(const void* dO, const void* Q, const void* K, const void* V, const void* O, const void* LSE,
                  void* DELTA, void* dQ, void* dK, void* dV, void* dS, int B, int Hq, int Hkv, int Tq, int Sk,
                  float scale, int causal, RowStrides sdo, RowStrides so, const AttnExtra& ex, hipStream_t s) {
  const float sl2 = scale * 1.44269504088896340736f;
  const int64_t rows = (int64_t)B * Hq * Tq;
  dim3 blk(kThreads);
  hipLaunchKernelGGL((attn_bwd_preprocess<T, 128>), dim3((unsigned)((rows * 8 + 255) / 256)), dim3(256), 0, s,
                     (const T*)dO, (const T*)O, (float*)DELTA, rows, Hq, Tq, sdo, so);
  const int hsplit = (ex.part && ex.hsplit > 1) ? ex.hsplit : 1;
  dim3 gk(B * Hkv * hsplit, (Sk + kKB3 - 1) / kKB3), gq(B * Hq, (Tq + 255) / 256);
#define LTA_DS(CA)                                                                                                   \
  if (hsplit > 1) {                                                                                                  \
    hipLaunchKernelGGL((attn_bwd_dkdv_v4_kernel<T, CA, 0, true, true>), gk, blk, 0, s, (const T*)Q, (const T*)K,   \
                       (const T*)V, (const T*)dO, (const float*)LSE, (const float*)DELTA, (T*)dK, (T*)dV, Hq, Hkv, Tq,  \
                       Sk, scale, sl2, sdo, ex.sx, g_dkdv_qrev, nullptr, (T*)dS, hsplit, ex.part);                   \
    launch_dkdv_reduce<T>(dK, dV, B, Hkv, Sk, ex, s);                                                                \
  } else {                                                                                                           \
    hipLaunchKernelGGL((attn_bwd_dkdv_v4_kernel<T, CA, 0, true>), gk, blk, 0, s, (const T*)Q, (const T*)K,          \
                       (const T*)V, (const T*)dO, (const float*)LSE, (const float*)DELTA, (T*)dK, (T*)dV, Hq, Hkv, Tq,  \
                       Sk, scale, sl2, sdo, ex.sx, g_dkdv_qrev, nullptr, (T*)dS);                                    \
  }                                                                                                                  \
  hipLaunchKernelGGL((attn_bwd_dq_ds_kernel<T, CA>), gq, blk, 0, s, (const T*)K, (const T*)dS, (T*)dQ, Hq, Hkv, Tq,   \
                     Sk, scale, ex.sx)
  if (causal) { LTA_DS(true); }
  else { LTA_DS(false); }
#undef LTA_DS
  return (int)hipGetLastError();
}

template <typename T, int D>
int launch_bwd(const void* dO, const void* Q, const void* K, const void* V, const void* O, const void* LSE, void* DELTA,
               void* dQ, void* dK, void* dV, int B, int Hq, int Hkv, int Tq, int Sk, float scale, int causal,
               RowStrides sdo, RowStrides so, int fast, const AttnExtra& ex, int exf, hipStream_t s) {
  const float sl2 = scale * 1.44269504088896340736f;
  const int64_t rows = (int64_t)B * Hq * Tq;
  dim3 blk(kThreads);
  if (exf == 0 && D == 128 && fast && Tq > 0 && Sk > 0) {
    // production path: the dQ kernel computes delta = rowsum(dO O) itself and runs first (the dK/dV
    // kernel reads it), so there is no preprocess launch
    dim3 gq(B * Hq, (Tq + kQB3 - 1) / kQB3), gk(B * Hkv, (Sk + kKB3 - 1) / kKB3);
#define LTA_FAST(CA)                                                                                                 \
  hipLaunchKernelGGL((attn_bwd_dq_v4_kernel<T, CA>), gq, blk, 0, s, (const T*)Q, (const T*)K, (const T*)V,            \
                     (const T*)dO, (const float*)LSE, (const float*)DELTA, (T*)dQ, Hq, Hkv, Tq, Sk, scale, sl2, sdo,   \
                     ex.sx, (const T*)O, so);                                                                          \
  LTA_DKDV_LAUNCH(CA)
    if (causal) { LTA_FAST(true); }
    else { LTA_FAST(false); }
#undef LTA_FAST
    return (int)hipGetLastError();
  }
  hipLaunchKernelGGL((attn_bwd_preprocess<T, D>), dim3((unsigned)((rows * 8 + 255) / 256)), dim3(256), 0, s,
                     (const T*)dO, (const T*)O, (float*)DELTA, rows, Hq, Tq, sdo, so);
  if (exf) {  // masks / dropout: the plain-HIP kernels with the extra terms compiled in
    switch (exf) {
#define LTA_M(F)                                                                                                  \
  case F:                                                                                                         \
    launch_masked<T, D, F>(dO, Q, K, V, LSE, DELTA, dQ, dK, dV, B, Hq, Hkv, Tq, Sk, scale, sl2, causal, sdo, ex, s); \
    break;
      LTA_M(kExMask)
      LTA_M(kExDrop)
      LTA_M(kExMask | kExDrop)
      LTA_M(kExMask | kExMaskGrad)
      LTA_M(kExMask | kExDrop | kExMaskGrad)
#undef LTA_M
      default:
        return -1;
    }
    return (int)hipGetLastError();
  }
  const int hsplit = (ex.part && ex.hsplit > 1) ? ex.hsplit : 1;
  dim3 g1(B * Hkv * hsplit, (Sk + kKB - 1) / kKB), g2(B * Hq, (Tq + kBM - 1) / kBM);
#define LTA_V1(CA)                                                                                                   \
  if (hsplit > 1) {                                                                                                  \
    hipLaunchKernelGGL((attn_bwd_dkdv_kernel<T, D, CA, 0, true>), g1, blk, 0, s, (const T*)Q, (const T*)K,           \
                       (const T*)V, (const T*)dO, (const float*)LSE, (const float*)DELTA, (T*)dK, (T*)dV, Hq, Hkv, Tq, \
                       Sk, scale, sl2, sdo, ex);                                                                       \
    launch_dkdv_reduce<T, D>(dK, dV, B, Hkv, Sk, ex, s);                                                               \
  } else {                                                                                                           \
    hipLaunchKernelGGL((attn_bwd_dkdv_kernel<T, D, CA>), g1, blk, 0, s, (const T*)Q, (const T*)K, (const T*)V,        \
                       (const T*)dO, (const float*)LSE, (const float*)DELTA, (T*)dK, (T*)dV, Hq, Hkv, Tq, Sk, scale,   \
                       sl2, sdo, ex);                                                                                  \
  }                                                                                                                  \
  hipLaunchKernelGGL((attn_bwd_dq_kernel<T, D, CA>), g2, blk, 0, s, (const T*)Q, (const T*)K, (const T*)V,            \
                     (const T*)dO, (const float*)LSE, (const float*)DELTA, (T*)dQ, Hq, Hkv, Tq, Sk, scale, sl2, sdo, ex)
  if (causal) { LTA_V1(true); }
  else { LTA_V1(false); }
#undef LTA_V1
  return (int)hipGetLastError();
}

}  // namespace

// LTA_ATTN_BWD_V1=1: the plain-HIP (v1) kernels for D = 128 too (A/B and bisection switch)
static int fast_enabled() {
  static const int fast = [] {
    const char* e = getenv("LTA_ATTN_BWD_V1");
    return (e && e[0] == '1') ? 0 : 1;
  }();
  return fast;
}

// GQA head split of the dK/dV pass (hsplit > 1 with an fp32 workspace of hsplit B Hkv Sk 256 floats):
// validates it and records it in `ex`.  hsplit <= 1 or no workspace: no split.
static bool gqa_split_ok(AttnExtra& ex, void* part_ws, int64_t part_bytes, int hsplit, int B, int Hq, int Hkv, int Sk,
                         int D = 128) {
  if (hsplit <= 1 || part_ws == nullptr) return true;
  const int group = Hq / Hkv;
  if (group % hsplit != 0 || part_bytes < (int64_t)hsplit * B * Hkv * Sk * 2 * D * 4 || (uintptr_t)part_ws % 16) return false;
  ex.part = static_cast<float*>(part_ws);
  ex.hsplit = hsplit;
  return true;
}

// Attention backward with the RoPE backward fused into the dQ / dK epilogues (self-attention,
// D = 128, no mask / dropout, dK/dV v4 + dQ v2..v4): rope_cos / rope_sin are fp32 [Tq][128] (the
// forward rotated q and k with them), dQ / dK / dV may point into one [B, T, (Hq + 2 Hkv) * 128]
// buffer through grad_strides, so the attention input projection's gradient is written in place.
// Returns -1 when the configuration is not covered (the caller runs the two passes instead).
LTA_EXPORT int lta_attn_bwd_rope(int dtype, const void* dO, const void* Q, const void* K, const void* V, const void* O,
                                 const void* LSE, void* DELTA, void* dQ, void* dK, void* dV, int B, int Hq, int Hkv,
                                 int Tq, int Sk, int D, float scale, int causal, const int64_t* strides,
                                 const int64_t* qkv_strides, const int64_t* grad_strides, const float* rope_cos,
                                 const float* rope_sin, void* part_ws, int64_t part_bytes, int hsplit,
                                 hipStream_t stream) {
  if (D != 128 || Tq != Sk || Tq <= 0 || Hq % Hkv != 0 || !rope_cos || !rope_sin || !fast_enabled())
    return -1;
  const RowStrides dflt{(int64_t)Hq * Tq * D, (int64_t)Tq * D, D};
  const RowStrides sdo = strides ? RowStrides{strides[0], strides[1], strides[2]} : dflt;
  const RowStrides so = strides ? RowStrides{strides[3], strides[4], strides[5]} : dflt;
  AttnExtra ex{};
  ex.sx = QKVStrides::from(qkv_strides, Hq, Hkv, Tq, Sk, D);
  ex.sx.set_grad(grad_strides);
  ex.sx.rope_cos = rope_cos;
  ex.sx.rope_sin = rope_sin;
  if (!gqa_split_ok(ex, part_ws, part_bytes, hsplit, B, Hq, Hkv, Sk)) return -2;
  if (dtype == kBF16)
    return launch_bwd<__hip_bfloat16, 128>(dO, Q, K, V, O, LSE, DELTA, dQ, dK, dV, B, Hq, Hkv, Tq, Sk, scale, causal, sdo,
                                           so, 1, ex, 0, stream);
  if (dtype == kF16)
    return launch_bwd<__half, 128>(dO, Q, K, V, O, LSE, DELTA, dQ, dK, dV, B, Hq, Hkv, Tq, Sk, scale, causal, sdo, so, 1,
                                   ex, 0, stream);
  return -1;
}

// strides: optional int64[6] = dO (batch, head, token), O (batch, head, token) element strides
// (head dim contiguous); null = contiguous [B,H,T,D] for both.  mask / dropout as lta_attn_fwd_ex;
// dmask (optional, needs mask): fp32 [B][Hq][Tq][Sk] receives dS, the additive mask's gradient
// before the reduction over its broadcast dims.
// qkv_strides: optional int64[9] = (batch, head, token) strides of Q, K, V (as lta_attn_fwd_ex2)
// grad_strides: optional int64[9] = dQ, dK, dV (batch, head, token) element strides (head dim
// contiguous, rows 16-byte aligned); null = dense [B, H, T, D] gradients.
// lta_attn_bwd_rope with dQ computed from the stored dS (launch_bwd_ds); ds_ws: >= B Hq Sk
// ceil(Tq / 256) 256 elements of the input dtype.  -1 when the shape does not qualify (the caller then takes lta_attn_bwd_rope).
LTA_EXPORT int lta_attn_bwd_rope_ds(int dtype, const void* dO, const void* Q, const void* K, const void* V,
                                    const void* O, const void* LSE, void* DELTA, void* dQ, void* dK, void* dV, int B,
                                    int Hq, int Hkv, int Tq, int Sk, int D, float scale, int causal,
                                    const int64_t* strides, const int64_t* qkv_strides, const int64_t* grad_strides,
                                    const float* rope_cos, const float* rope_sin, void* ds_ws, int64_t ds_bytes,
                                    void* part_ws, int64_t part_bytes, int hsplit, hipStream_t stream) {
  if (D != 128 || Tq != Sk || Tq <= 0 || Tq % 32 || Sk % 64 || Hq % Hkv != 0 || !rope_cos || !rope_sin || !ds_ws ||
      ds_bytes < (int64_t)B * Hq * ((Tq + 255) / 256) * 256 * Sk * 2)
    return -1;
  const RowStrides dflt{(int64_t)Hq * Tq * D, (int64_t)Tq * D, D};
  const RowStrides sdo = strides ? RowStrides{strides[0], strides[1], strides[2]} : dflt;
  const RowStrides so = strides ? RowStrides{strides[3], strides[4], strides[5]} : dflt;
  AttnExtra ex{};
  ex.sx = QKVStrides::from(qkv_strides, Hq, Hkv, Tq, Sk, D);
  ex.sx.set_grad(grad_strides);
  ex.sx.rope_cos = rope_cos;
  ex.sx.rope_sin = rope_sin;
  if (!gqa_split_ok(ex, part_ws, part_bytes, hsplit, B, Hq, Hkv, Sk)) return -2;
  if (dtype == kBF16)
    return launch_bwd_ds<__hip_bfloat16>(dO, Q, K, V, O, LSE, DELTA, dQ, dK, dV, ds_ws, B, Hq, Hkv, Tq, Sk, scale,
                                         causal, sdo, so, ex, stream);
  if (dtype == kF16)
    return launch_bwd_ds<__half>(dO, Q, K, V, O, LSE, DELTA, dQ, dK, dV, ds_ws, B, Hq, Hkv, Tq, Sk, scale, causal, sdo,
                                 so, ex, stream);
  return -1;
}

// GQA / MQA head split of the next lta_attn_bwd_ex3 call of this host thread (fp32 workspace of hsplit B Hkv
// Sk 2 D floats; taken and cleared by that call)
struct GqaWs {
  void* part = nullptr;
  int64_t bytes = 0;
  int hsplit = 1;
};
inline thread_local GqaWs g_gqa_ws;
LTA_EXPORT void lta_attn_set_gqa_workspace(void* part, int64_t bytes, int hsplit) { g_gqa_ws = GqaWs{part, bytes, hsplit}; }

LTA_EXPORT int lta_attn_bwd_ex3(int dtype, const void* dO, const void* Q, const void* K, const void* V, const void* O,
                                const void* LSE, void* DELTA, void* dQ, void* dK, void* dV, int B, int Hq, int Hkv,
                                int Tq, int Sk, int D, float scale, int causal, const int64_t* strides, const void* mask,
                                int mask_b, int mask_h, void* dmask, float dropout_p, uint64_t seed, uint64_t offset,
                                const int64_t* qkv_strides, const int64_t* grad_strides, hipStream_t stream) {
  const long long* rng = take_attn_rng();
  const GqaWs gws = g_gqa_ws;
  g_gqa_ws = GqaWs{};
  if (Hq % Hkv != 0 || dropout_p < 0.f || dropout_p >= 1.f || (dmask && !mask)) return -2;
  const RowStrides dflt{(int64_t)Hq * Tq * D, (int64_t)Tq * D, D};
  const RowStrides sdo = strides ? RowStrides{strides[0], strides[1], strides[2]} : dflt;
  const RowStrides so = strides ? RowStrides{strides[3], strides[4], strides[5]} : dflt;
  const int v2 = fast_enabled();
  AttnExtra ex{};
  ex.sx = QKVStrides::from(qkv_strides, Hq, Hkv, Tq, Sk, D);
  ex.sx.set_grad(grad_strides);
  if (!mask && dropout_p == 0.f && !gqa_split_ok(ex, gws.part, gws.bytes, gws.hsplit, B, Hq, Hkv, Sk, D)) return -2;
  int exf = 0;
  if (mask) {
    const int64_t skp = (int64_t)(Sk + 63) / 64 * 64;
    ex.mask = (const float*)mask;
    ex.mq = skp;
    ex.mh = mask_h ? (int64_t)Tq * skp : 0;
    ex.mb = mask_b ? (int64_t)(mask_h ? Hq : 1) * Tq * skp : 0;
    exf |= kExMask;
    if (dmask) {
      ex.dmask = (float*)dmask;
      exf |= kExMaskGrad;
    }
  }
  if (dropout_p > 0.f) {
    ex.keep_scale = 1.f / (1.f - dropout_p);
    ex.keep_thresh = (unsigned)fmin((double)dropout_p * 4294967296.0, 4294967295.0);
    ex.seed_lo = (unsigned)seed;
    ex.seed_hi = (unsigned)(seed >> 32);
    ex.offset = (unsigned)offset;
    ex.rng = rng;
    exf |= kExDrop;
  }
#define LTA_B(TT, DD)                                                                                             \
  return launch_bwd<TT, DD>(dO, Q, K, V, O, LSE, DELTA, dQ, dK, dV, B, Hq, Hkv, Tq, Sk, scale, causal, sdo, so, v2, ex, \
                            exf, stream)
  if (dtype == kBF16) {
    if (D == 128) LTA_B(__hip_bfloat16, 128);
    if (D == 64) LTA_B(__hip_bfloat16, 64);
    if (D == 96) LTA_B(__hip_bfloat16, 96);
    if (D == 256) LTA_B(__hip_bfloat16, 256);
  } else if (dtype == kF16) {
    if (D == 128) LTA_B(__half, 128);
    if (D == 64) LTA_B(__half, 64);
    if (D == 96) LTA_B(__half, 96);
    if (D == 256) LTA_B(__half, 256);
  }
#undef LTA_B
  return -1;
}

LTA_EXPORT int lta_attn_bwd_ex2(int dtype, const void* dO, const void* Q, const void* K, const void* V, const void* O,
                                const void* LSE, void* DELTA, void* dQ, void* dK, void* dV, int B, int Hq, int Hkv,
                                int Tq, int Sk, int D, float scale, int causal, const int64_t* strides, const void* mask,
                                int mask_b, int mask_h, void* dmask, float dropout_p, uint64_t seed, uint64_t offset,
                                const int64_t* qkv_strides, hipStream_t stream) {
  return lta_attn_bwd_ex3(dtype, dO, Q, K, V, O, LSE, DELTA, dQ, dK, dV, B, Hq, Hkv, Tq, Sk, D, scale, causal, strides,
                          mask, mask_b, mask_h, dmask, dropout_p, seed, offset, qkv_strides, nullptr, stream);
}

LTA_EXPORT int lta_attn_bwd_ex(int dtype, const void* dO, const void* Q, const void* K, const void* V, const void* O,
                               const void* LSE, void* DELTA, void* dQ, void* dK, void* dV, int B, int Hq, int Hkv,
                               int Tq, int Sk, int D, float scale, int causal, const int64_t* strides, const void* mask,
                               int mask_b, int mask_h, void* dmask, float dropout_p, uint64_t seed, uint64_t offset,
                               hipStream_t stream) {
  return lta_attn_bwd_ex2(dtype, dO, Q, K, V, O, LSE, DELTA, dQ, dK, dV, B, Hq, Hkv, Tq, Sk, D, scale, causal, strides,
                          mask, mask_b, mask_h, dmask, dropout_p, seed, offset, nullptr, stream);
}

LTA_EXPORT int lta_attn_bwd_s(int dtype, const void* dO, const void* Q, const void* K, const void* V, const void* O,
                              const void* LSE, void* DELTA, void* dQ, void* dK, void* dV, void* workspace, int B, int Hq,
                              int Hkv, int Tq, int Sk, int D, float scale, int causal, const int64_t* strides,
                              hipStream_t stream) {
  return lta_attn_bwd_ex(dtype, dO, Q, K, V, O, LSE, DELTA, dQ, dK, dV, B, Hq, Hkv, Tq, Sk, D, scale, causal, strides,
                         nullptr, 0, 0, nullptr, 0.f, 0, 0, stream);
}

LTA_EXPORT int lta_attn_bwd(int dtype, const void* dO, const void* Q, const void* K, const void* V, const void* O,
                            const void* LSE, void* DELTA, void* dQ, void* dK, void* dV, void* workspace, int B, int Hq,
                            int Hkv, int Tq, int Sk, int D, float scale, int causal, hipStream_t stream) {
  return lta_attn_bwd_s(dtype, dO, Q, K, V, O, LSE, DELTA, dQ, dK, dV, workspace, B, Hq, Hkv, Tq, Sk, D, scale, causal,
                        nullptr, stream);
}

#ifdef LTA_ATTN_DIAG
// diagnostic builds: route the dK/dV kernel to its phase-stamp build, stamps into `dbg` (null: off)
LTA_EXPORT int lta_attn_bwd_set_stamps(void* dbg) {
  g_dkdv_stamps = (uint64_t*)dbg;
  return 0;
}
#endif
// dK/dV query-tile order of the D = 128 kernel (A/B measurement hook): 1 = last tile first, 0 = first
// tile first; returns the previous choice
LTA_EXPORT int lta_attn_bwd_set_dkdv_qrev(int rev) {
  const int old = g_dkdv_qrev;
  g_dkdv_qrev = rev ? 1 : 0;
  return old;
}
