// K8 (v2): FP8 (OCP e4m3 / e5m2) NT GEMM, C[M,N] bf16 = (A . B^T) / (sa * sb) (+ bias), one 256x256
// output tile per 4-wave workgroup on v_mfma_f32_16x16x128_f8f6f4 (2x the bf16 MFMA rate).
// (reference: TransformerEngine's cuBLASLt FP8 GEMMs, thunder/executors/transformer_engineex_impl.py)
//
// Same skeleton as csrc/gemm4.hip (one wave per SIMD, 128x128 per wave in 256 AGPR accumulators,
// LDS-DMA staging through buffer resources issued as inline asm, XCD-aware bijective tile map),
// re-timed for the fp8 MFMA, whose K of 128 makes one K-tile (128-B rows, the bf16 kernel's LDS
// image byte for byte) a single k-step:
//
//   top of tile t:  vmcnt(0) lgkmcnt(0), s_barrier   (tile t+1 landed; every wave holds tile t's
//                                                      fragments, so tile t's buffer is free)
//   rows 0..7 of 8 MFMAs (32 cycles each) on the fragments of tile t (registers):
//     rows 0..3: the 16 LDS-DMA pieces of tile t+2 into tile t's buffer, one per 2 MFMAs
//     row m >= 1: read tile t+1's A fragment m-1 (its register's last use was row m-1)
//     row 7: after MFMA (7, n) read tile t+1's B fragment n, after (7, 7) A fragment 7
//
// so the DMA of a tile has a whole tile (2048 MFMA cycles) to land and every LDS read overlaps
// MFMAs.  A fragment of the 16x16x128 operand is 32 B per lane: 16-B chunks g and 4 + g of its
// 128-B row (g = lane >> 4); A and B use the same k assignment, so the sum over k is exact.
#include <type_traits>

#include "common.h"

using namespace lta;

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int v8i __attribute__((ext_vector_type(8)));

constexpr int BM = 256, BN = 256, BKB = 128, NTHR = 256;
constexpr int OP_BYTES = BM * BKB;    // 32 KiB per operand per stage
constexpr int STAGE = 2 * OP_BYTES;   // 64 KiB

__device__ __forceinline__ int xcd_tile(int orig, int nwg) {
  const int xcd = orig & 7, q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
}

__device__ __forceinline__ i32x4 make_rsrc(const void* base, int bytes) {
  const uint64_t a = (uint64_t)(uintptr_t)base;
  return i32x4{(int)(uint32_t)a, (int)((uint32_t)(a >> 32) & 0xffffu), bytes, 0x00020000};
}

// K-major operand rows of 128 B per K-tile: instruction i (0..7) of wave w fills LDS bytes
// [(4i + w) KiB, +1 KiB) = rows 8(4i + w) .. +7; lane -> row + (lane >> 3), stored chunk lane & 7
// holding logical chunk (lane & 7) ^ (row & 7).
struct StagerB {
  i32x4 rsrc;
  int voff, istride;
  __device__ __forceinline__ void init(const char* X, int ld, int r0, int K, int wave, int lane) {
    const char* base = X + (int64_t)r0 * ld;
    rsrc = make_rsrc(base, (BM - 1) * ld + K);
    const int r = lane >> 3, c = (lane & 7) ^ r;
    voff = (wave * 8 + r) * ld + c * 16;
    istride = 32 * ld;
  }
  __device__ __forceinline__ void issue(int i, int kt, char* img, int wave) const {
    const uint32_t dst = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)(img + (i * 4 + wave) * 1024);
    asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %3 offen lds"
                 :
                 : "s"(dst), "v"(voff), "s"(rsrc), "s"(i * istride + kt * BKB)
                 : "memory", "m0");
  }
};

// MN-major operand (stored [K][M or N], the backward's dY / X / W read in place, no transposed copy):
// the K-tile's image is 128 k-rows of 256 B (the tile's 256 M or N bytes), 16-B chunk c of k-row R at
// slot c ^ swz(R), swz(R) = (R & 7) | ((R >> 4) & 1) << 3, so the transposed fragment reads below are
// bank-conflict free.  Instruction i (0..7) of wave w fills k-rows 16 i + 4 w .. +3 (LDS bytes
// [(4i + w) KiB, +1 KiB), lane-linear); bit 4 of the row is i & 1, so even and odd instructions use
// two lane offsets.
struct StagerT {
  i32x4 rsrc;
  int voff[2], ld;
  __device__ __forceinline__ void init(const char* X, int ld_, int c0, int K, int wave, int lane) {
    ld = ld_;
    rsrc = make_rsrc(X + c0, K * ld);
    const int ro = lane >> 4, slot = lane & 15, r = 4 * wave + ro;
    voff[0] = r * ld + ((slot ^ (r & 7)) << 4);
    voff[1] = (16 + r) * ld + ((slot ^ ((r & 7) | 8)) << 4);
  }
  __device__ __forceinline__ void issue(int i, int kt, char* img, int wave) const {
    const uint32_t dst = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)(img + (i * 4 + wave) * 1024);
    asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %3 offen lds"
                 :
                 : "s"(dst), "v"(voff[i & 1]), "s"(rsrc), "s"((kt * BKB + 32 * (i >> 1)) * ld)
                 : "memory", "m0");
  }
};

typedef int v2i __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) v2i lds_v2i;

// Lane base of the transposed fragment reads of an MN-major image (LDS byte address; XOR-ed with the
// fragment's (stage, 16-column block) constant, see read_frag_t).  ds_read_b64_tr_b8 (probed:
// scripts/exp/tr8_probe.py): per 16-lane group a block of 8 k-rows x 16 bytes, lane 2q + p giving the
// address of row q, bytes 8p .. 8p + 7, lane i receiving column i of the 8 rows.  Lane (column fr,
// group g) reads k-rows 16g + q (+8, +64, +72): the k order of the K-major fragment (chunks g, 4 + g).
__device__ __forceinline__ uint32_t tr_base(uint32_t img, int wblock, int lane) {
  const int g = lane >> 4, q = (lane & 15) >> 1, p = lane & 1;
  return img + (uint32_t)((16 * g + q) * 256 + 8 * p + ((((wblock ^ (g & 1)) << 3) | q) << 4));
}
// fragment of the 16-column block `blk` (0..7 within the wave's 128 columns) from the image whose
// stage / operand offset `xo` is XOR-ed into the lane base (bits 4..6 select the chunk, 15..16 the
// image); four 8-byte transposed reads at k-row offsets 0, 8, 64, 72
__device__ __forceinline__ v8i read_frag_t(uint32_t base, uint32_t xo) {
  const uint32_t a = base ^ xo;
  auto rd = [&](uint32_t off) {
    return __builtin_amdgcn_ds_read_tr8_b64_v2i32((lds_v2i*)(uintptr_t)(a + off));
  };
  const v2i r0 = rd(0), r1 = rd(8 * 256), r2 = rd(64 * 256), r3 = rd(72 * 256);
  return v8i{r0.x, r0.y, r1.x, r1.y, r2.x, r2.y, r3.x, r3.y};
}

__device__ __forceinline__ v8i read_frag8(const char* img, int row, int g) {
  const uint4 lo = *reinterpret_cast<const uint4*>(img + row * 128 + ((g ^ (row & 7)) << 4));
  const uint4 hi = *reinterpret_cast<const uint4*>(img + row * 128 + (((4 + g) ^ (row & 7)) << 4));
  return v8i{(int)lo.x, (int)lo.y, (int)lo.z, (int)lo.w, (int)hi.x, (int)hi.y, (int)hi.z, (int)hi.w};
}

template <int FA, int FB>
__device__ __forceinline__ void mfma8(f32x4& acc, const v8i& a, const v8i& b) {
  if constexpr (FA == 0 && FB == 0)
    asm volatile("v_mfma_f32_16x16x128_f8f6f4 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
  else if constexpr (FA == 1 && FB == 0)
    asm volatile("v_mfma_f32_16x16x128_f8f6f4 %0, %1, %2, %0 cbsz:1" : "+a"(acc) : "v"(a), "v"(b));
  else
    asm volatile("v_mfma_f32_16x16x128_f8f6f4 %0, %1, %2, %0 blgp:1" : "+a"(acc) : "v"(a), "v"(b));
}

#define LTA_FENCE() __builtin_amdgcn_sched_barrier(0)

typedef float f32x2_t __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
// two f32 -> one packed bf16 pair on ONE v_cvt_pk_bf16_f32 (round to nearest even, as __float2bfloat16)
__device__ __forceinline__ uint32_t pack_bf16x2(float lo, float hi) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2_t{lo, hi}, bf16x2_t));
}

// RES: C = bf16(bf16(A.B^T / (sa sb) + bias) + R) — the residual add of the unfused pair, with the
// same two rounding points (the FP8 transformer block's residual stream and the dgrad sum of the
// gate / up projections never take a separate elementwise pass).
// AT / BT: operand A / B stored MN-major ([K][M] / [K][N], pitches lda / ldb in bytes), read through
// transposed LDS reads; else K-major ([M][K] / [N][K]).
// QKV: the attention input projection's epilogue of csrc/gemm4.hip (EPI 3) on the fp8 product: the
// [q heads | k heads | v heads] x 128 columns go straight to q [B, nh, T, 128] (C), k / v
// [B, ng, T, 128] (qk.k, qk.v) with the rotate-half RoPE on q and k, applied to the bf16-rounded
// dequantised projection as csrc/rope.hip does (the qkv tensor is never written).
struct QkvArgs {
  __hip_bfloat16* k;
  __hip_bfloat16* v;
  const float* cos_;
  const float* sin_;
  int T, nh, ng;
};

template <int FA, int FB, bool BIAS, bool RES = false, bool AT = false, bool BT = false, bool QKV = false>
__global__ __launch_bounds__(NTHR, 1) void gemm4_fp8_kernel(const char* __restrict__ A, const char* __restrict__ B,
                                                           __hip_bfloat16* __restrict__ C,
                                                           const __hip_bfloat16* __restrict__ bias, int M, int N,
                                                           int K, int lda, int ldb, int ldc,
                                                           const float* __restrict__ sa,
                                                           const float* __restrict__ sb,
                                                           const __hip_bfloat16* __restrict__ R = nullptr,
                                                           int ldr = 0, QkvArgs qk = {}) {
  static_assert(!QKV || (!BIAS && !RES && !AT && !BT), "qkv rope: forward layout, no other epilogue");
  __shared__ __attribute__((aligned(1024))) char smem[2 * STAGE];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int fr = lane & 15, fg = lane >> 4;

  const int nTm = M / BM, nTn = N / BN, nwg = nTm * nTn;
  const int wg = xcd_tile((int)blockIdx.x, nwg);
  constexpr int G = 8;
  const int per_group = G * nTn;
  const int group = wg / per_group;
  const int first_m = group * G;
  const int gm = min(nTm - first_m, G);
  const int in_group = wg % per_group;
  const int tm = first_m + in_group % gm, tn = in_group / gm;
  const int m0 = tm * BM, n0 = tn * BN;

  std::conditional_t<AT, StagerT, StagerB> st_a;
  std::conditional_t<BT, StagerT, StagerB> st_b;
  st_a.init(A, lda, m0, K, wave, lane);
  st_b.init(B, ldb, n0, K, wave, lane);
  const uint32_t lds0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)smem;
  [[maybe_unused]] const uint32_t tra = tr_base(lds0, wm, lane), trb = tr_base(lds0 + OP_BYTES, wn, lane);
  // fragment m of A / n of B from stage S (0 / 1)
  auto frag_a = [&](int S, int m) -> v8i {
    if constexpr (AT)
      return read_frag_t(tra, (uint32_t)(S * STAGE) | (uint32_t)(m << 4));
    else
      return read_frag8(smem + S * STAGE, wm * 128 + fr + m * 16, fg);
  };
  auto frag_b = [&](int S, int n) -> v8i {
    if constexpr (BT)
      return read_frag_t(trb, (uint32_t)(S * STAGE) | (uint32_t)(n << 4));
    else
      return read_frag8(smem + S * STAGE + OP_BYTES, wn * 128 + fr + n * 16, fg);
  };
  auto glds = [&](int j, int kt, char* stage) {
    if (j < 8)
      st_a.issue(j, kt, stage, wave);
    else
      st_b.issue(j - 8, kt, stage + OP_BYTES, wave);
  };

  f32x4 acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  v8i fa[8], fb[8];

  const int nk = K / BKB;
  // ---- prologue: tiles 0 and 1 in flight, tile 0's fragments into registers ----
#pragma unroll
  for (int j = 0; j < 16; ++j) glds(j, 0, smem);
#pragma unroll
  for (int j = 0; j < 16; ++j) glds(j, 1, smem + STAGE);
  asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  __builtin_amdgcn_s_barrier();
#pragma unroll
  for (int m = 0; m < 8; ++m) fa[m] = frag_a(0, m);
#pragma unroll
  for (int n = 0; n < 8; ++n) fb[n] = frag_b(0, n);

  auto body = [&](int t, auto cur_c) {
    constexpr int CUR = decltype(cur_c)::value;
    char* const bc = smem + CUR * STAGE;
    const int t2 = min(t + 2, nk - 1);
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    LTA_FENCE();
#pragma unroll
    for (int i = 0; i < 64; ++i) {
      const int m = i >> 3, n = i & 7;
      // operands swapped (the B fragment and its format first): the accumulator holds the transposed
      // 16 x 16 block, 4 consecutive C columns of one row per lane (register epilogue below)
      mfma8<FB, FA>(acc[m][n], fb[n], fa[m]);
      if (i < 32 && (i & 1) == 0) glds(i >> 1, t2, bc);
      if (m >= 1 && n == 0) fa[m - 1] = frag_a(CUR ^ 1, m - 1);
      if (m == 7) fb[n] = frag_b(CUR ^ 1, n);
      if (i == 63) fa[7] = frag_a(CUR ^ 1, 7);
      LTA_FENCE();
    }
  };
  // nk is even (K % 256 == 0, checked by the host)
  for (int t = 0; t < nk; t += 2) {
    body(t, std::integral_constant<int, 0>{});
    body(t + 1, std::integral_constant<int, 1>{});
  }

#pragma unroll
  for (int m = 0; m < 8; ++m)
#pragma unroll
    for (int n = 0; n < 8; ++n) asm volatile("" : "+a"(acc[m][n]));
  asm volatile("s_nop 15\n\ts_nop 15" ::: "memory");
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();

  // ---- register epilogue (as csrc/gemm4.hip): alpha = 1 / (sa * sb), + bias, bf16; blocks n, n + 1
  // through v_permlane16_swap -> 16 B of one row per lane -> (+ residual) -> store.  No LDS image.
  const float alpha = 1.f / (*sa * *sb);
  const int rsel = fg & 1, csel = fg >> 1;
  if constexpr (QKV) {
    // this wave's 128 columns are one head (see csrc/gemm4.hip EPI 3); a dimension d < 64 (block n < 4)
    // and its rotate-half partner d + 64 (block n + 4) sit in the same lane and register
    const int cb = (n0 + wn * 128) >> 7;
    const bool is_q = cb < qk.nh, is_k = !is_q && cb < qk.nh + qk.ng;
    __hip_bfloat16* const dst = is_q ? C : (is_k ? qk.k : qk.v);
    const int hh = is_q ? cb : (is_k ? cb - qk.nh : cb - qk.nh - qk.ng);
    const int nheads = is_q ? qk.nh : qk.ng;
    const bool rope = is_q || is_k;
    // cos / sin of row block m + 1 are loaded while block m is rotated and stored (one row block per
    // sched region: loading them inside it exposed an L2 round trip per block, +26 us per GEMM)
    float4 cc[4], sc[4];
    auto load_cs = [&](int m, float4 (&c)[4], float4 (&sn)[4]) {
      const int t = (m0 + wm * 128 + m * 16 + fr) % qk.T;
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        c[n] = *reinterpret_cast<const float4*>(qk.cos_ + (int64_t)t * 128 + n * 16 + fg * 4);
        sn[n] = *reinterpret_cast<const float4*>(qk.sin_ + (int64_t)t * 128 + n * 16 + fg * 4);
      }
    };
    if (rope) load_cs(0, cc, sc);
#pragma unroll
    for (int m = 0; m < 8; ++m) {
      float4 cn[4], snx[4];
      if (rope && m < 7) load_cs(m + 1, cn, snx);
      const int grow = m0 + wm * 128 + m * 16 + fr;  // M % 256 == 0: every row is in range
      const int bi = grow / qk.T, t = grow - bi * qk.T;
      __hip_bfloat16* const orow = dst + (((int64_t)bi * nheads + hh) * qk.T + t) * 128;
      uint32_t lo[4][2], hi[4][2];
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        float x1[4], x2[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          x1[j] = __bfloat162float(__float2bfloat16(acc[m][n][j] * alpha));
          x2[j] = __bfloat162float(__float2bfloat16(acc[m][n + 4][j] * alpha));
        }
        if (rope) {
          const float cs[4] = {cc[n].x, cc[n].y, cc[n].z, cc[n].w}, ss[4] = {sc[n].x, sc[n].y, sc[n].z, sc[n].w};
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const float a = x1[j], b = x2[j];
            x1[j] = a * cs[j] - b * ss[j];
            x2[j] = b * cs[j] + a * ss[j];
          }
        }
        lo[n][0] = pack_bf16x2(x1[0], x1[1]);
        lo[n][1] = pack_bf16x2(x1[2], x1[3]);
        hi[n][0] = pack_bf16x2(x2[0], x2[1]);
        hi[n][1] = pack_bf16x2(x2[2], x2[3]);
      }
#pragma unroll
      for (int np = 0; np < 2; ++np) {
        const int n = 2 * np;
        const auto a0 = __builtin_amdgcn_permlane16_swap(lo[n][0], lo[n + 1][0], false, false);
        const auto a1 = __builtin_amdgcn_permlane16_swap(lo[n][1], lo[n + 1][1], false, false);
        const auto b0 = __builtin_amdgcn_permlane16_swap(hi[n][0], hi[n + 1][0], false, false);
        const auto b1 = __builtin_amdgcn_permlane16_swap(hi[n][1], hi[n + 1][1], false, false);
        const int col = (n + rsel) * 16 + csel * 8;
        *reinterpret_cast<uint4*>(orow + col) = make_uint4(a0[0], a1[0], a0[1], a1[1]);
        *reinterpret_cast<uint4*>(orow + col + 64) = make_uint4(b0[0], b1[0], b0[1], b1[1]);
      }
      if (rope && m < 7) {
#pragma unroll
        for (int n = 0; n < 4; ++n) {
          cc[n] = cn[n];
          sc[n] = snx[n];
        }
      }
      __builtin_amdgcn_sched_barrier(0);  // one row block at a time: bounded VGPR use
    }
    return;
  }
  float bv[8][4];
#pragma unroll
  for (int n = 0; n < 8; ++n) {
#pragma unroll
    for (int j = 0; j < 4; ++j) bv[n][j] = 0.f;
    if constexpr (BIAS) {
      const uint2 u = *reinterpret_cast<const uint2*>(bias + n0 + wn * 128 + n * 16 + fg * 4);
      const __hip_bfloat16* h = reinterpret_cast<const __hip_bfloat16*>(&u);
#pragma unroll
      for (int j = 0; j < 4; ++j) bv[n][j] = to_f32(h[j]);
    }
  }
#pragma unroll
  for (int m = 0; m < 8; ++m) {
    const int64_t grow = m0 + wm * 128 + m * 16 + fr;
#pragma unroll
    for (int np = 0; np < 4; ++np) {
      const int n = 2 * np;
      float v[2][4];
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int j = 0; j < 4; ++j) v[h][j] = acc[m][n + h][j] * alpha + bv[n + h][j];
      const auto s0 = __builtin_amdgcn_permlane16_swap(pack_bf16x2(v[0][0], v[0][1]), pack_bf16x2(v[1][0], v[1][1]),
                                                       false, false);
      const auto s1 = __builtin_amdgcn_permlane16_swap(pack_bf16x2(v[0][2], v[0][3]), pack_bf16x2(v[1][2], v[1][3]),
                                                       false, false);
      uint4 val = make_uint4(s0[0], s1[0], s0[1], s1[1]);
      const int gcol = n0 + wn * 128 + (n + rsel) * 16 + csel * 8;
      if constexpr (RES) {
        const uint4 rv = *reinterpret_cast<const uint4*>(R + grow * ldr + gcol);
        const __hip_bfloat16* a = reinterpret_cast<const __hip_bfloat16*>(&val);
        const __hip_bfloat16* b = reinterpret_cast<const __hip_bfloat16*>(&rv);
        union {
          uint4 u;
          __hip_bfloat16 h[8];
        } o;
#pragma unroll
        for (int e = 0; e < 8; ++e) o.h[e] = __float2bfloat16(__bfloat162float(a[e]) + __bfloat162float(b[e]));
        val = o.u;
      }
      *reinterpret_cast<uint4*>(C + grow * ldc + gcol) = val;
      __builtin_amdgcn_sched_barrier(0);  // one block pair at a time: bounded VGPR use
    }
  }
}

#undef LTA_FENCE

}  // namespace

// C[M,N] bf16 = (A . B^T) / (*sa * *sb) (+ bias); A [M,K], B [N,K] fp8 as bytes (row pitches lda /
// ldb in bytes), fmt 0 = e4m3fn, 1 = e5m2 (e5m2 on one operand at most).  M, N % 256 == 0,
// K % 256 == 0, 16-B aligned rows, operands under 2 GiB.
LTA_EXPORT int lta_gemm4_fp8(const void* A, const void* B, void* C, const void* bias, int M, int N, int K, int lda,
                             int ldb, int ldc, int fmt_a, int fmt_b, const void* sa, const void* sb,
                             hipStream_t stream) {
  if (M % BM || N % BN || K % (2 * BKB) || M <= 0 || N <= 0 || lda % 16 || ldb % 16 || ldc % 8) return -2;
  if ((int64_t)M * lda >= (1ll << 31) || (int64_t)N * ldb >= (1ll << 31)) return -2;
  dim3 grid((M / BM) * (N / BN)), block(NTHR);
#define LTA_G8(FA, FB, BI)                                                                                       \
  hipLaunchKernelGGL((gemm4_fp8_kernel<FA, FB, BI>), grid, block, 0, stream, (const char*)A, (const char*)B,      \
                     (__hip_bfloat16*)C, (const __hip_bfloat16*)bias, M, N, K, lda, ldb, ldc, (const float*)sa, \
                     (const float*)sb)
  const bool bi = bias != nullptr;
  if (fmt_a == 0 && fmt_b == 0) { if (bi) LTA_G8(0, 0, true); else LTA_G8(0, 0, false); }
  else if (fmt_a == 1 && fmt_b == 0) { if (bi) LTA_G8(1, 0, true); else LTA_G8(1, 0, false); }
  else if (fmt_a == 0 && fmt_b == 1) { if (bi) LTA_G8(0, 1, true); else LTA_G8(0, 1, false); }
  else return -1;
#undef LTA_G8
  return (int)hipGetLastError();
}

// Backward layouts without transposed fp8 copies: at = 1 reads A stored [K][M] (e.g. dY for the wgrad
// dW = dY^T X), bt = 1 reads B stored [K][N] (W for the dgrad dX = dY W, X for the wgrad), both through
// ds_read_b64_tr_b8.  C = (opA . opB) / (sa sb) (+ R, bt-only layout); (at, bt) in {(0,1), (1,1)};
// formats as lta_gemm4_fp8 (0 e4m3, 1 e5m2; e5m2 on A only).  Pitches in bytes, multiples of 16.
LTA_EXPORT int lta_gemm4_fp8_layout(const void* A, const void* B, void* C, const void* R, int M, int N, int K, int lda,
                                    int ldb, int ldc, int ldr, int fmt_a, int fmt_b, int at, int bt, const void* sa,
                                    const void* sb, hipStream_t stream) {
  if (M % BM || N % BN || K % (2 * BKB) || M <= 0 || N <= 0 || lda % 16 || ldb % 16 || ldc % 8 || ldr % 8) return -2;
  if (!bt || (at && R) || fmt_b != 0 || (fmt_a != 0 && fmt_a != 1)) return -1;
  const int64_t ea = at ? (int64_t)K * lda : (int64_t)M * lda, eb = (int64_t)K * ldb;
  if (ea >= (1ll << 31) || eb >= (1ll << 31) || (at && lda < M) || ldb < N) return -2;
  dim3 grid((M / BM) * (N / BN)), block(NTHR);
#define LTA_G8L(FA, RE, AT_)                                                                                       \
  hipLaunchKernelGGL((gemm4_fp8_kernel<FA, 0, false, RE, AT_, true>), grid, block, 0, stream, (const char*)A,      \
                     (const char*)B, (__hip_bfloat16*)C, nullptr, M, N, K, lda, ldb, ldc, (const float*)sa,         \
                     (const float*)sb, (const __hip_bfloat16*)R, ldr)
  if (at) {
    if (fmt_a == 0) LTA_G8L(0, false, true); else LTA_G8L(1, false, true);
  } else if (R) {
    if (fmt_a == 0) LTA_G8L(0, true, false); else LTA_G8L(1, true, false);
  } else {
    if (fmt_a == 0) LTA_G8L(0, false, false); else LTA_G8L(1, false, false);
  }
#undef LTA_G8L
  return (int)hipGetLastError();
}

// q, k, v = rope split of (A . B^T) / (sa sb) for a [q heads | k heads | v heads] x 128 projection
// (the fp8 counterpart of lta_gemm4_qkv_rope): A [M, K] fp8 rows of M = B_ * T tokens, B [N, K] with
// N = (nh + 2 ng) * 128; cos / sin [T][128] fp32 with equal halves (rotate-half caches).
LTA_EXPORT int lta_gemm4_fp8_qkv_rope(const void* A, const void* B, const void* sa, const void* sb, const float* cos_,
                                      const float* sin_, void* q, void* k, void* v, int M, int K, int lda, int ldb,
                                      int T, int nh, int ng, int fmt_a, int fmt_b, hipStream_t stream) {
  const int N = (nh + 2 * ng) * 128;
  if (M % BM || N % BN || K % (2 * BKB) || M <= 0 || T <= 0 || M % T || nh <= 0 || ng <= 0 || lda % 16 || ldb % 16)
    return -2;
  if ((int64_t)M * lda >= (1ll << 31) || (int64_t)N * ldb >= (1ll << 31) || !q || !k || !v || !cos_ || !sin_) return -2;
  dim3 grid((M / BM) * (N / BN)), block(NTHR);
  const QkvArgs qa{(__hip_bfloat16*)k, (__hip_bfloat16*)v, cos_, sin_, T, nh, ng};
#define LTA_G8Q(FA, FB)                                                                                             \
  hipLaunchKernelGGL((gemm4_fp8_kernel<FA, FB, false, false, false, false, true>), grid, block, 0, stream,         \
                     (const char*)A, (const char*)B, (__hip_bfloat16*)q, nullptr, M, N, K, lda, ldb, 0,             \
                     (const float*)sa, (const float*)sb, nullptr, 0, qa)
  if (fmt_a == 0 && fmt_b == 0) LTA_G8Q(0, 0);
  else return -1;
#undef LTA_G8Q
  return (int)hipGetLastError();
}

// lta_gemm4_fp8 + residual: C = bf16(bf16((A . B^T) / (sa sb) (+ bias)) + R), R [M, N] bf16 (pitch ldr).
LTA_EXPORT int lta_gemm4_fp8_res(const void* A, const void* B, void* C, const void* bias, const void* R, int M, int N,
                                 int K, int lda, int ldb, int ldc, int ldr, int fmt_a, int fmt_b, const void* sa,
                                 const void* sb, hipStream_t stream) {
  if (!R) return lta_gemm4_fp8(A, B, C, bias, M, N, K, lda, ldb, ldc, fmt_a, fmt_b, sa, sb, stream);
  if (M % BM || N % BN || K % (2 * BKB) || M <= 0 || N <= 0 || lda % 16 || ldb % 16 || ldc % 8 || ldr % 8) return -2;
  if ((int64_t)M * lda >= (1ll << 31) || (int64_t)N * ldb >= (1ll << 31)) return -2;
  dim3 grid((M / BM) * (N / BN)), block(NTHR);
#define LTA_G8R(FA, FB, BI)                                                                                      \
  hipLaunchKernelGGL((gemm4_fp8_kernel<FA, FB, BI, true>), grid, block, 0, stream, (const char*)A, (const char*)B, \
                     (__hip_bfloat16*)C, (const __hip_bfloat16*)bias, M, N, K, lda, ldb, ldc, (const float*)sa,  \
                     (const float*)sb, (const __hip_bfloat16*)R, ldr)
  const bool bi = bias != nullptr;
  if (fmt_a == 0 && fmt_b == 0) { if (bi) LTA_G8R(0, 0, true); else LTA_G8R(0, 0, false); }
  else if (fmt_a == 1 && fmt_b == 0) { if (bi) LTA_G8R(1, 0, true); else LTA_G8R(1, 0, false); }
  else if (fmt_a == 0 && fmt_b == 1) { if (bi) LTA_G8R(0, 1, true); else LTA_G8R(0, 1, false); }
  else return -1;
#undef LTA_G8R
  return (int)hipGetLastError();
}
