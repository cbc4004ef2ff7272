// Shared MFMA / LDS helpers for the CDNA4 flash-attention kernels (K3).
//
// MFMA: v_mfma_f32_32x32x16_bf16 (one wave computes a 32x32 fp32 tile, K = 16).
// Operand lane maps (cdna_hip_programming.md §3), lane l, r = l & 31, h = l >> 5:
//   A[row r][k = 8h + j]          (j = 0..7 of the 8-element fragment)
//   B[k = 8h + j][col r]
//   C/D reg i: row = (i & 3) + 8 * (i >> 2) + 4h, col = r
// An fp32 accumulator X reused as the B operand (sum over X's rows) takes registers 8s..8s+7
// for k-step s; element j then carries row 16s + 8(j>>2) + 4h + (j&3) of X, so the A operand
// must supply those k's: with A held row-major in LDS that is exactly what a
// ds_read_b64_tr_b16 of 4 consecutive rows delivers (T10 transposed read).
#pragma once
#include "common.h"

namespace lta {
namespace attn {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

template <typename T> struct Frag;
template <> struct Frag<__hip_bfloat16> { typedef bf16x8 type; };
template <> struct Frag<__half> { typedef f16x8 type; };

__device__ __forceinline__ f32x16 mfma(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x16 mfma(f16x8 a, f16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
}

template <typename F>
__device__ __forceinline__ F load_frag(const void* p) {
  return *reinterpret_cast<const F*>(p);
}

// Two transposed 4x16 LDS reads (rows row0..row0+3 and row0+8..row0+11 of a row-major 16-bit
// tile) assembled into one 8-element A fragment; `lds_base` points at the first row,
// `stride` is the row stride in elements, `col0` the first column of this 16-lane group.
template <typename F>
__device__ __forceinline__ F tr_frag(const __attribute__((address_space(3))) short* base, int row0, int col0, int stride,
                                     int lane16) {
  const int q = lane16 >> 2, p = lane16 & 3;
  const __attribute__((address_space(3))) short* p0 = base + (row0 + q) * stride + col0 + 4 * p;
  const __attribute__((address_space(3))) short* p1 = p0 + 8 * stride;
  s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)p0);
  s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)p1);
  union {
    struct { s16x4 a, b; } s;
    F f;
  } u;
  u.s.a = lo;
  u.s.b = hi;
  return u.f;
}

__device__ __forceinline__ void pack_frag(bf16x8& f, const f32x16& x, int s) {
#pragma unroll
  for (int j = 0; j < 8; ++j) f[j] = (__bf16)x[8 * s + j];
}
__device__ __forceinline__ void pack_frag(f16x8& f, const f32x16& x, int s) {
#pragma unroll
  for (int j = 0; j < 8; ++j) f[j] = (_Float16)x[8 * s + j];
}

__device__ __forceinline__ int acc_row(int i, int h) { return (i & 3) + 8 * (i >> 2) + 4 * h; }

// ---------------------------------------------------------------------------------------------
// Attention masks and dropout (reference: cuDNN SDPA additive / boolean masks + dropout seed and
// offset, thunder/executors/cudnn_sdpa.py; aten flash dropout, sdpaex.py:274-336).
// EX bit flags of a kernel instantiation (compile-time: the plain causal path carries no cost):
enum : int { kExMask = 1, kExDrop = 2, kExMaskGrad = 4 };

// Element strides (batch, head, token) of Q, K and V (head dim contiguous, rows 16-byte aligned):
// views into a fused qkv projection are read in place.  contiguous(): dense [B, H, T, D].
struct QKVStrides {
  int64_t qb, qh, qt, kb, kh, kt, vb, vh, vt;
  // backward only: dQ / dK / dV (batch, head, token) strides; the host lays the gradients out like
  // their operands (e.g. [B, T, H, D] for heads split from a fused projection), so the usual
  // transpose + reshape back to [B, T, H*D] that follows is a view instead of a copy
  int64_t dqb, dqh, dqt, dkb, dkh, dkt, dvb, dvh, dvt;
  // backward only, optional: fp32 [T][D] cos / sin of a rotate-half RoPE applied to q and k in the
  // forward; dQ and dK are then stored with the rotation's transpose applied (the RoPE backward
  // fused into the attention backward's epilogue)
  const float* rope_cos;
  const float* rope_sin;
  static QKVStrides contiguous(int Hq, int Hkv, int Tq, int Sk, int D) {
    const int64_t q[3] = {(int64_t)Hq * Tq * D, (int64_t)Tq * D, D}, k[3] = {(int64_t)Hkv * Sk * D, (int64_t)Sk * D, D};
    return {q[0], q[1], q[2], k[0], k[1], k[2], k[0], k[1], k[2], q[0], q[1], q[2], k[0], k[1], k[2], k[0], k[1], k[2],
            nullptr, nullptr};
  }
  static QKVStrides from(const int64_t* s, int Hq, int Hkv, int Tq, int Sk, int D) {
    QKVStrides r = contiguous(Hq, Hkv, Tq, Sk, D);
    if (s) r = QKVStrides{s[0], s[1], s[2], s[3], s[4], s[5], s[6], s[7], s[8], r.dqb, r.dqh, r.dqt,
                          r.dkb, r.dkh, r.dkt, r.dvb, r.dvh, r.dvt, nullptr, nullptr};
    return r;
  }
  void set_grad(const int64_t* g) {  // optional int64[9]: dQ, dK, dV (batch, head, token) strides
    if (!g) return;
    dqb = g[0], dqh = g[1], dqt = g[2], dkb = g[3], dkh = g[4], dkt = g[5], dvb = g[6], dvh = g[7], dvt = g[8];
  }
  bool is_contiguous(int Hq, int Hkv, int Tq, int Sk, int D) const {
    const QKVStrides c = contiguous(Hq, Hkv, Tq, Sk, D);
    return qb == c.qb && qh == c.qh && qt == c.qt && kb == c.kb && kh == c.kh && kt == c.kt && vb == c.vb &&
           vh == c.vh && vt == c.vt;
  }
};

struct AttnExtra {
  QKVStrides sx;          // Q / K / V strides (every kernel reads its operands through them)
  const float* mask;      // additive mask (natural-log domain), fp32 [Bm][Hm][Tq][Skp], key dim padded to 64
  int64_t mb, mh, mq;     // element strides (0 for a broadcast batch / head)
  float* dmask;           // kExMaskGrad: dS written as fp32 [B][Hq][Tq][Sk] (reduced over broadcast dims by the host)
  float keep_scale;       // 1 / (1 - p)
  unsigned keep_thresh;   // keep iff hash >= p * 2^32
  unsigned seed_lo, seed_hi, offset;
  float* part;            // GQA head split of the dK/dV pass: fp32 partial rows [hsplit][B Hkv Sk][2][128]
  int hsplit;             // > 1: query heads of a kv group split over that many workgroups (attn_bwd_dkdv_reduce sums)
  const long long* rng;   // graph-safe dropout (core/rng.py GraphRngInt): int64 [seed, base] on the device,
                          // `offset` then relative to base; null: seed / offset are the values above
};

// the device RNG state for the NEXT attention launch of this host thread (lta_attn_set_rng_state): the
// entry points take it (and clear it) when they build their AttnExtra
inline thread_local const long long* g_attn_rng = nullptr;
inline const long long* take_attn_rng() {
  const long long* r = g_attn_rng;
  g_attn_rng = nullptr;
  return r;
}

// e4m3 side output of the D = 128 v4 forward (the FP8 output projection's input, delayed scaling):
// q8 holds fp8(bf16(O) s) in O's element layout (1 byte per element), s = fmax / *amax_in goes to
// scale_out, max |bf16(O)| into amax_out.  Requested for the NEXT lta_attn_fwd_ex2 call of this host
// thread (lta_attn_set_fp8_out); lta_attn_fp8_out_used() says whether the launched kernel wrote it.
struct AttnQ8 {
  uint8_t* q;
  const float* amax_in;
  float fmax;
  float* scale_out;
  float* amax_out;
};
inline thread_local AttnQ8 g_attn_q8{};
inline thread_local int g_attn_q8_used = 0;
inline AttnQ8 take_attn_q8() {
  const AttnQ8 r = g_attn_q8;
  g_attn_q8 = AttnQ8{};
  return r;
}
// v4 forward with an optional e4m3 side output (attention_fwd4.hip); -1 when unsupported
int attn_fwd_v4_q8(int dtype, const void* q, const void* k, const void* v, void* o, void* lse, int B, int Hq, int Hkv,
                   int Tq, int Sk, int D, float scale, int causal, const int64_t* o_strides,
                   const int64_t* qkv_strides, int defer, const AttnQ8* q8, hipStream_t stream);

// Counter-based dropout mask: a pure function of (seed, offset, query head, query, key), so the
// forward and both backward kernels regenerate the same keep bit in any iteration order.
__device__ __forceinline__ unsigned fmix32(unsigned h) {
  h ^= h >> 16;
  h *= 0x85ebca6bu;
  h ^= h >> 13;
  h *= 0xc2b2ae35u;
  h ^= h >> 16;
  return h;
}
__device__ __forceinline__ unsigned rng_head(const AttnExtra& e, int bh) {
  unsigned slo = e.seed_lo, shi = e.seed_hi, off = e.offset;
  if (e.rng != nullptr) {  // graph-safe: seed and Philox base written before each graph replay
    const unsigned long long sd = (unsigned long long)e.rng[0];
    slo = (unsigned)sd;
    shi = (unsigned)(sd >> 32);
    off = (unsigned)((unsigned long long)e.rng[1] + (unsigned long long)e.offset);
  }
  return fmix32((unsigned)bh * 0x9e3779b9u ^ fmix32(slo ^ (off * 0x27d4eb2fu)) ^ shi);
}
__device__ __forceinline__ unsigned rng_q(unsigned head, int q) { return fmix32((unsigned)q * 0x61c88647u + head); }
__device__ __forceinline__ unsigned rng_k(int k) { return fmix32((unsigned)k * 0x7feb352du + 0x3c6ef372u); }
__device__ __forceinline__ bool rng_keep(const AttnExtra& e, unsigned qterm, unsigned kterm) {
  return fmix32(qterm ^ kterm) >= e.keep_thresh;
}
// A tile's key (or query) terms through a wave-private LDS row: lane l writes the term of index
// base + l, and the 4 indices 8 a + 4 h + {0..3} a lane's accumulator elements 4 a .. 4 a + 3 carry
// (acc_row) come back as one 16-B read, instead of one hash per element (a wave's LDS write -> read
// needs no barrier: its LDS operations complete in order).
__device__ __forceinline__ uint4 rng_tab4(const unsigned* row, int a, int h) {
  return *reinterpret_cast<const uint4*>(row + 8 * a + 4 * h);
}

}  // namespace attn
}  // namespace lta
