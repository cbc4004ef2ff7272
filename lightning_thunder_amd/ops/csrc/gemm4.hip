// K2 (v2): bf16 GEMM on CDNA4 MFMA, one 256x256 output tile per 4-wave workgroup.
//
//   C[M,N] = act(alpha * A . B + bias[col]) (+ R)        (reference: cuBLAS(Lt) behind ATen linear /
//                                                          matmul, thunder/executors/torchex.py; nvFuser
//                                                          linear/matmul, nvfuserex_impl.py:2437-2488)
// A is [M][K] (K-major, AT = 0) or stored [K][M] (MN-major, AT = 1); B is [N][K] (the nn.Linear
// weight, BT = 0) or stored [K][N] (BT = 1).  The three layouts of a training linear are
//   forward  Y  = X  . W^T : AT 0, BT 0      dgrad dX = dY . W : AT 0, BT 1      wgrad dW = dY^T . X : AT 1, BT 1
// so no operand is ever transposed in memory.
//
// Why this shape (cdna_hip_programming.md §5; MI355X_MICROARCH.md §LDS, §Two waves per SIMD):
//   * 4 waves (one per SIMD), each owning a 128x128 quadrant = 8x8 v_mfma_f32_16x16x32_bf16 tiles
//     (256 fp32 accumulators per lane).  Per 32-deep k-step a wave issues 64 MFMAs (1024 cycles) for
//     16 fragment reads: half the LDS read bytes per FLOP of a 2x4-wave 128x64 split, and the
//     16x16x32 shape holds a higher clock than 32x32x16 on random data (DVFS give-back item 7).
//   * Operands are staged HBM/L2 -> LDS with global_load_lds_dwordx4 (no VGPR round trip) into
//     two 64 KiB stages (BK = 64).  K-major images are 128-B rows with the 16-B chunk c of row r at
//     c ^ (r & 7) (conflict-free ds_read_b128); MN-major images are 512-B k-rows read with
//     ds_read_b64_tr_b16 (T10) under the tr_swz XOR (conflict-free transposed reads).  glds writes
//     lane-linearly, so both swizzles are applied to the per-lane SOURCE address (rule 21).
//   * ONE barrier per 64-deep K-tile, placed in the middle of the second k-step's MFMA stream: the
//     MFMAs before it use fragments already in registers, the ones after it hide the next tile's
//     first fragment reads and the prefetch of the tile after that.  So the only exposed cost per
//     K-tile is the barrier skew, not a read-after-barrier latency:
//        phase A  (k-step 0): 64 MFMA  | ds_read k-step-1 fragments of tile t
//        phase B1 (k-step 1): 32 MFMA  | -
//        vmcnt(0) lgkmcnt(0) s_barrier          (tile t+1 landed everywhere; tile t fully read)
//        phase B2 (k-step 1): 32 MFMA  | ds_read k-step-0 fragments of tile t+1, glds of tile t+2
//     The glds of tile t+2 go into the buffer of tile t (free after that barrier) and must land by
//     the next barrier, ~96 MFMAs (1500+ cycles) later.  VAR selects how the 16 glds per wave and
//     tile are split between phase B2 and the first half of the next phase A.
//   * Instruction order inside each phase is pinned with sched_barrier(0) after every MFMA group.
//   * blockIdx -> tile: bijective XCD remap, then groups of 8 tile-rows (L2 reuse of A and B panels).
//   * Epilogue: fp32 alpha / bias / activation in registers -> bf16 in a per-wave swizzled LDS image
//     -> 16-B row-contiguous stores (+ residual, same rounding points as ATen's linear then add).
//   * SwiGLU epilogues (EPI, lta_gemm4_swiglu): the LLaMA MLP's gate/up pair and its backward never
//     round-trip through HBM between the GEMM and the gating:
//       EPI 1 (forward, "gate-up"): every 256-column output tile is 128 columns of W1 and the same 128
//         columns of W2 (B staged from two weight tensors: LDS-DMA instructions 0-3 read W1 rows, 4-7 W2
//         rows), so one workgroup holds a = x W1^T and b = x W2^T for the same 128 columns in its two
//         wave columns; after the images meet in LDS it stores a, b (saved for the backward) and
//         y = silu(a) * b — the separate swiglu pass (read a, b; write y) disappears.
//       EPI 2 (backward, dgrad layout): g = dY . W_proj never leaves the chip; the store pass reads a, b
//         and writes da = g b silu'(a), db = g silu(a) (the swiglu backward pass and g's round trip
//         disappear).  Both round exactly where the unfused ops round (a, b, g in bf16).
//   * EPI 3 (attention input projection, lta_gemm4_qkv_rope): the [q heads | k heads | v heads] x 128
//     output columns are stored straight into q [B, nh, T, 128], k / v [B, ng, T, 128] with the
//     rotate-half RoPE applied to q and k from the bf16 image (a dimension's partner d +- 64 is the
//     chunk ch ^ 8 of the same image row): the qkv tensor is never written, the split/RoPE pass
//     (read qkv, write q, k, v) disappears; same rounding points as csrc/rope.hip.
#include "common.h"

using namespace lta;

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

constexpr int BM = 256, BN = 256, BK = 64, NTHR = 256;
constexpr int OP_BYTES = BM * BK * 2;  // 32 KiB per operand per stage
constexpr int STAGE = 2 * OP_BYTES;    // 64 KiB

enum Act : int { kNone = 0, kGeluTanh = 1, kGeluErf = 2, kSilu = 3, kRelu = 4 };

template <int ACT>
__device__ __forceinline__ float act_fn(float x) {
  if constexpr (ACT == kGeluTanh) {
    const float u = 0.7978845608028654f * (x + 0.044715f * x * x * x);
    return 0.5f * x * (1.f + tanhf(u));
  } else if constexpr (ACT == kGeluErf) {
    return 0.5f * x * (1.f + erff(x * 0.7071067811865476f));
  } else if constexpr (ACT == kSilu) {
    return x / (1.f + __expf(-x));
  } else if constexpr (ACT == kRelu) {
    return x > 0.f ? x : 0.f;
  } else {
    return x;
  }
}

__device__ __forceinline__ int xcd_tile(int orig, int nwg) {
  const int xcd = orig & 7, q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
}

// MN-major image swizzle: the 16-B chunk c of k-row k sits at chunk c ^ tr_swz(k).  A 32-lane half
// of a transposed fragment read touches rows {k0+q, k0+4+q} (q < 4) at chunks {c0, c0+1}; tr_swz
// maps those rows to distinct even chunk offsets of the 256-B bank row.
__device__ __forceinline__ int tr_swz(int k) { return ((k & 3) | (((k >> 3) & 1) << 2)) << 1; }

// Per-lane LDS-DMA source of one operand (buffer_load ... lds through a buffer resource, so the
// per-lane part is ONE 32-bit VGPR offset and the per-instruction / per-K-tile parts are scalar
// soffsets).  Instruction i (0..7) of wave w fills LDS bytes [(4i + w) KiB, +1 KiB) of the image.
// Issued as inline asm: hipcc cannot prove that the transposed fragment reads (ds_read_b64_tr_b16)
// miss the DMA's destination and puts an s_waitcnt vmcnt(0) in front of EVERY one of them,
// draining the prefetch (measured: MN-major layouts at 1/3 of the K-major rate).  Completion of
// the DMA is therefore tracked only by the explicit vmcnt waits of the main loop and epilogue.
__device__ __forceinline__ i32x4 make_rsrc(const void* base, int bytes) {
  const uint64_t a = (uint64_t)(uintptr_t)base;
  return i32x4{(int)(uint32_t)a, (int)((uint32_t)(a >> 32) & 0xffffu), bytes, 0x00020000};
}

template <bool MN, bool DUAL = false, bool KEDGE = false>
struct Stager {
  i32x4 rsrc, rsrc2;     // DUAL (K-major only): tile rows alternate in 64-row groups between rsrc and rsrc2
                         // (rows 0-63: rsrc 0-63, 64-127: rsrc2 0-63, 128-191: rsrc 64-127, 192-255: rsrc2 64-127)
  // KEDGE (MN-major, grouped wgrad): the reduction length `kred` need not divide the K-tile.  Every
  // K-tile gets its own buffer resource ending at the last valid k-row, and the k-row offsets live
  // in the per-lane voffset (the range check covers voffset, not soffset), so k-rows past the end
  // arrive in LDS as zeros (verified: tests/test_hip_kernels.py::test_lds_dma_out_of_range_lanes_write_zero)
  const char* kbase;
  int kred, ldb2;
  int voff[8];           // K-major: per instruction i (edge rows clamped); MN-major: [0] even, [1] odd i
  int istride, kstride;  // bytes between consecutive i (MN-major, DUAL) / consecutive K-tiles
  // X + r0 (rows / columns of this tile); ld = row pitch in elements; K = reduction length;
  // valid = rows (K-major) / columns (MN-major) of the tile inside the operand (< BM on an edge
  // tile: the sources of the rest are clamped to the last valid one, whose copies only feed
  // output rows / columns that are never stored — no out-of-bounds read, no reliance on the
  // buffer range check)
  __device__ __forceinline__ void init(const __hip_bfloat16* X, int ld, int r0, int K, int wave, int lane,
                                       const __hip_bfloat16* X2 = nullptr, int valid = BM) {
    if constexpr (DUAL) {
      // r0 = the row of BOTH sources this tile starts at; each source contributes 128 rows
      rsrc = make_rsrc(X + (int64_t)r0 * ld, (BM / 2 - 1) * ld * 2 + K * 2);
      rsrc2 = make_rsrc(X2 + (int64_t)r0 * ld, (BM / 2 - 1) * ld * 2 + K * 2);
      const int r = lane >> 3, c = (lane & 7) ^ r;
      voff[0] = ((wave * 8 + r) * ld + c * 8) * 2;
      istride = 32 * ld * 2;
      kstride = BK * 2;
    } else if constexpr (!MN) {
      // 8 rows of 128 B per instruction: lane -> row 8(4i + w) + (lane >> 3), stored chunk lane & 7,
      // which holds logical chunk (lane & 7) ^ row & 7
      const __hip_bfloat16* base = X + (int64_t)r0 * ld;
      rsrc = make_rsrc(base, (BM - 1) * ld * 2 + K * 2);
      const int r = lane >> 3, c = (lane & 7) ^ r;
#pragma unroll
      for (int i = 0; i < 8; ++i) voff[i] = (min(32 * i + wave * 8 + r, valid - 1) * ld + c * 8) * 2;
      istride = 0;
      kstride = BK * 2;
    } else {
      // 2 k-rows of 512 B per instruction: lane -> k-row 2(4i + w) + (lane >> 5), stored chunk
      // lane & 31 holding logical chunk (lane & 31) ^ tr_swz(k-row); tr_swz flips bit 3 with i & 1
      const __hip_bfloat16* base = X + r0;
      rsrc = make_rsrc(base, (K - 1) * ld * 2 + BM * 2);
      const int half = lane >> 5, slot = lane & 31;
      const int kr = 2 * wave + half;  // k-row for i = 0
      const int c0 = slot ^ tr_swz(kr), cmax = (valid >> 3) - 1;  // valid % 8 == 0 (16-B rows)
      if constexpr (KEDGE) {
#pragma unroll
        for (int i = 0; i < 8; ++i) voff[i] = ((8 * i + kr) * ld + min((i & 1) ? c0 ^ 8 : c0, cmax) * 8) * 2;
        kbase = reinterpret_cast<const char*>(base);
        kred = K;
        ldb2 = ld * 2;
      } else {
        voff[0] = (kr * ld + min(c0, cmax) * 8) * 2;
        voff[1] = (kr * ld + min(c0 ^ 8, cmax) * 8) * 2;
      }
      istride = 8 * ld * 2;
      kstride = BK * ld * 2;
    }
  }
  __device__ __forceinline__ void issue(int i, int kt, char* img, int wave) const {
    const uint32_t dst = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)(img + (i * 4 + wave) * 1024);
    if constexpr (KEDGE) {
      // the group bounds come from device memory: readfirstlane makes the (uniform) descriptor provably
      // scalar (cdna_hip_programming.md T20)
      const int rows = max(0, min(BK, kred - kt * BK));
      const uint64_t a = (uint64_t)(uintptr_t)(kbase + (int64_t)kt * BK * ldb2);
      const i32x4 rk = i32x4{__builtin_amdgcn_readfirstlane((int)(uint32_t)a),
                             __builtin_amdgcn_readfirstlane((int)((uint32_t)(a >> 32) & 0xffffu)),
                             __builtin_amdgcn_readfirstlane(rows * ldb2), 0x00020000};
      asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds"
                   :
                   : "s"(dst), "v"(voff[i]), "s"(rk)
                   : "memory", "m0");
      return;
    }
    // DUAL: instruction i fills tile rows 32 i .. 32 i + 31 = source rows 64 (i >> 2) + 32 (i & 1) + .. of
    // W1 (i & 2 == 0) or W2, so each wave's 128 columns are 64 of a = x W1^T and the same 64 of b = x W2^T
    const bool second = DUAL && ((i >> 1) & 1);
    const int vo = DUAL ? voff[0] : (MN ? voff[i & 1] : voff[i]);
    const int so = DUAL ? (2 * (i >> 2) + (i & 1)) * istride + kt * kstride
                        : (MN ? i * istride + kt * kstride : kt * kstride);
    asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %3 offen lds"
                 :
                 : "s"(dst), "v"(vo), "s"(second ? rsrc2 : rsrc), "s"(so)
                 : "memory", "m0");
  }
};

// 8-element fragment (k = 32 kk + 8 fq .. +7 of row/column `rc + fr`) of a staged operand image.
template <bool MN>
__device__ __forceinline__ bf16x8 read_frag(const char* img, int rc, int kk, int fr, int fq) {
  if constexpr (!MN) {
    const int row = rc + fr;
    return *reinterpret_cast<const bf16x8*>(img + row * 128 + (((kk * 4 + fq) ^ (fr & 7)) << 4));
  } else {
    // lane 4q+p of the 16-lane group addresses k-row k0 + q, columns rc + 4p .. +3
    const int q = fr >> 2, p = fr & 3;
    const int k = kk * 32 + fq * 8 + q;
    const int c = (rc >> 3) + (p >> 1);
    const char* a0 = img + k * 512 + ((c ^ tr_swz(k)) << 4) + 8 * (p & 1);
    const char* a1 = img + (k + 4) * 512 + ((c ^ tr_swz(k + 4)) << 4) + 8 * (p & 1);
    const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(__attribute__((address_space(3))) char*)a0);
    const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(__attribute__((address_space(3))) char*)a1);
    union {
      struct {
        s16x4 a, b;
      } s;
      bf16x8 f;
    } u;
    u.s.a = lo;
    u.s.b = hi;
    return u.f;
  }
}

#define LTA_FENCE() __builtin_amdgcn_sched_barrier(0)

// The 256 accumulators live in the AGPR file through inline-asm MFMAs ("+a"): as intrinsics hipcc
// splits them between the VGPR and AGPR files and spills.  Fragments come straight from ds_read
// (waited by hipcc's lgkmcnt), so no VALU->MFMA operand hazard needs padding; the AGPR results are
// read only after the explicit s_nop drain before the epilogue.
__device__ __forceinline__ void mfma16(f32x4& acc, const bf16x8& a, const bf16x8& b) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
}

__device__ __forceinline__ float sigmoid_f(float x) { return 1.f / (1.f + __expf(-x)); }

__device__ __forceinline__ float bf16_round(float x) { return __bfloat162float(__float2bfloat16(x)); }

typedef float f32x2_t __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
// two f32 -> one packed bf16 pair on ONE v_cvt_pk_bf16_f32 (round to nearest even, as __float2bfloat16)
__device__ __forceinline__ uint32_t pack_bf16x2(float lo, float hi) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2_t{lo, hi}, bf16x2_t));
}

// Register epilogue of the swapped layout (see the kernel): lane (fq, fr) holds 4 consecutive columns
// 4 fq .. 4 fq + 3 of row fr in every 16 x 16 block.  Blocks n and n + 1 of one row block, packed to
// bf16 (x = block n, y = block n + 1, 2 dwords each), go through v_permlane16_swap: afterwards every
// lane holds 8 consecutive columns (16 B) of ONE row - lanes with fq even block n, fq odd block
// n + 1; fq < 2 columns 0..7, fq >= 2 columns 8..15 of their block (cdna_hip_programming.md T21).
__device__ __forceinline__ uint4 swap_pair(uint32_t x0, uint32_t x1, uint32_t y0, uint32_t y1) {
  const auto s0 = __builtin_amdgcn_permlane16_swap(x0, y0, false, false);
  const auto s1 = __builtin_amdgcn_permlane16_swap(x1, y1, false, false);
  return make_uint4(s0[0], s1[0], s0[1], s1[1]);
}

// Extra operands of the fused epilogues.
struct EpiArgs {
  const __hip_bfloat16* B2;  // EPI 1: W2
  __hip_bfloat16* C2;        // EPI 1: b; EPI 2: db; EPI 3: k
  __hip_bfloat16* C3;        // EPI 1: y; EPI 3: v
  const __hip_bfloat16* R2;  // EPI 2: b
  const float* cos_;         // EPI 3: [T][128] fp32
  const float* sin_;
  int T, nh, ng;             // EPI 3: tokens per sequence, q heads, kv heads
  const int* offs;           // GRP 1 / 2: int32 cumulative group ends (device)
  int G;                     // GRP: number of groups
  int64_t bstride, cstride;  // GRP 1: elements between groups' B; GRP 2: between groups' C
  // GRP 0 K splits (lta_gemm4_bf16_ws / _splitk): this launch covers the linear tiles [tile_base,
  // tile_base + tile_count) (kernel TAIL = 1 and 2); TAIL 2: workgroup b computes K slice b % ksplit of
  // tile tile_base + b / ksplit and stores the fp32 partial [ksplit][tile_count][256][256] (plain products)
  int tile_base, tile_count, ksplit;
  float* partial;
};

// linear tile index -> (tile row, tile column): groups of 8 tile-rows walked column-major (the A and B
// panels of a group stay in L2)
__device__ __forceinline__ void tile_coords(int wg, int nTm, int nTn, int& tm, int& tn) {
  constexpr int G = 8;
  const int per_group = G * nTn;
  const int group = wg / per_group;
  const int first_m = group * G;
  const int gm = min(nTm - first_m, G);
  const int in_group = wg % per_group;
  tm = first_m + in_group % gm;
  tn = in_group / gm;
}

// EPI 0: plain (bias / act / residual); 1: gate-up forward (B2 = W2; C = a, C2 = b, C3 = y, each
// [M][N/2] with pitch ldc; C / C2 may be null); 2: swiglu backward (R = a, R2 = b, C = da, C2 = db,
// all [M][N] with pitch ldc); 3: qkv + RoPE (C = q, C2 = k, C3 = v).  See the header.
// GRP 0: one GEMM.  GRP 1 (MoE forward / dgrad): rows [offs[g-1], offs[g]) of A times group g's B
// (B + g * bstride); a row tile never spans two groups (grid: ceil(M / 256) + G row slots per
// column tile, each workgroup scans the device offsets for its (group, row tile); no host sync).
// GRP 2 (MoE wgrad): C[g] (C + g * cstride) = A_g^T . B_g, A / B stored [rows][.] (AT = BT = 1)
// with group g's rows as the reduction; the reduction tail is zero-filled (Stager KEDGE).
template <int ACT, bool BIAS, bool RES, bool AT, bool BT, int VAR, int EPI = 0, int GRP = 0, int TAIL = 0>
__global__ __launch_bounds__(NTHR, 1) void gemm4_bf16_kernel(const __hip_bfloat16* __restrict__ A,
                                                            const __hip_bfloat16* __restrict__ B,
                                                            __hip_bfloat16* __restrict__ C,
                                                            const __hip_bfloat16* __restrict__ bias,
                                                            const __hip_bfloat16* __restrict__ R, int M, int N, int K,
                                                            int lda, int ldb, int ldc, int ldr, float alpha,
                                                            EpiArgs ep = {}) {
  const __hip_bfloat16* const B2 = ep.B2;
  __hip_bfloat16* const C2 = ep.C2;
  __hip_bfloat16* const C3 = ep.C3;
  const __hip_bfloat16* const R2 = ep.R2;
  static_assert(EPI != 1 || (!AT && !BT && !BIAS && !RES && ACT == 0), "gate-up: forward layout, no other epilogue");
  static_assert(EPI != 3 || (!AT && !BT && !BIAS && !RES && ACT == 0), "qkv rope: forward layout, no other epilogue");
  static_assert(EPI != 2 || (!AT && BT && !BIAS && !RES && ACT == 0), "swiglu backward: dgrad layout only");
  static_assert(GRP == 0 || (EPI == 0 && !BIAS && !RES && ACT == 0), "grouped: plain products");
  static_assert(GRP != 1 || !AT, "grouped rows: A row-major");
  static_assert(GRP != 2 || (AT && BT), "grouped reduction: A and B stored [rows][.]");
  // SW: MFMA operands swapped (D = B-fragment x A-fragment^T, the TRANSPOSED 16 x 16 block), so each
  // lane accumulates 4 consecutive COLUMNS of one C row and the epilogue is register-only (cvt_pk +
  // permlane16_swap -> 16-B row stores), no LDS image: the image's 256 ds_write_b16 per lane cost
  // ~8.4k of a tile's ~12k epilogue cycles (profiles/gemm4_epilogue_anatomy.txt).  Every epilogue runs in
  // registers: for the gate-up GEMM (EPI 1) the B tile interleaves W1 / W2 rows in 64-row groups so a lane
  // holds a (block n) and b (block n + 4) of the same output element.
  constexpr bool SW = true;
  __shared__ __attribute__((aligned(1024))) char smem[2 * STAGE];  // the ONLY LDS object (rule 4a)

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int fr = lane & 15, fq = lane >> 4;

  const int nTm = (M + BM - 1) / BM, nTn = (N + BN - 1) / BN, nwg = nTm * nTn;
  const __hip_bfloat16* Ag = A;
  const __hip_bfloat16* Bg = B;
  __hip_bfloat16* Cg = C;
  int Mlim = M, Kr = K, m0, n0;
  [[maybe_unused]] int wg_lin = 0, kpart = 0;
  if constexpr (GRP == 0) {
    // TAIL 0: every tile (the production instantiations keep exactly this code: a run-time tile
    // range here changed hipcc's schedule of the GELU + bias epilogue into wrong results);
    // 1: tiles [tile_base, tile_base + tile_count); 2: the K-split tail (ksplit == 2, the host's only
    // split: shifts keep the index scalar)
    int wg;
    if constexpr (TAIL == 2) {
      // workgroup b: K slice b % ksplit of tile tile_base + b / ksplit (readfirstlane: the division's
      // VALU sequence must not turn the tile / slice indices into per-lane values)
      const int t = __builtin_amdgcn_readfirstlane((int)blockIdx.x / ep.ksplit);
      kpart = __builtin_amdgcn_readfirstlane((int)blockIdx.x - t * ep.ksplit);
      wg = ep.tile_base + t;
    }
    else if constexpr (TAIL == 1)
      wg = ep.tile_base + xcd_tile((int)blockIdx.x, ep.tile_count);
    else
      wg = xcd_tile((int)blockIdx.x, nwg);
    wg_lin = wg;
    int tm, tn;
    tile_coords(wg, nTm, nTn, tm, tn);
    m0 = tm * BM;
    n0 = tn * BN;
    if constexpr (TAIL == 2) {
      // this workgroup's K slice: the K / 2 BK tile pairs dealt as evenly as possible over the ksplit
      // slices (the first P % ksplit slices take one pair more; K % 2 BK == 0, P >= ksplit: host)
      const int P = K / (2 * BK), q = __builtin_amdgcn_readfirstlane(P / ep.ksplit), r = P - q * ep.ksplit;
      const int k0 = (kpart * q + min(kpart, r)) * (2 * BK);
      Kr = (q + (kpart < r ? 1 : 0)) * (2 * BK);
      Ag = A + (AT ? (int64_t)k0 * lda : (int64_t)k0);
      Bg = B + (BT ? (int64_t)k0 * ldb : (int64_t)k0);
    }
  } else if constexpr (GRP == 1) {
    const int bid = (int)blockIdx.x, tn = bid % nTn;
    int slot = bid / nTn, g = 0, start = 0, end = 0;
    bool found = false;
    for (; g < ep.G; ++g) {
      end = ep.offs[g];
      const int tiles = (end - start + BM - 1) / BM;
      if (slot < tiles) {
        found = true;
        break;
      }
      slot -= tiles;
      start = end;
    }
    if (!found) return;  // uniform over the workgroup (scalar offsets): no barrier is skipped by part of it
    m0 = start + slot * BM;
    n0 = tn * BN;
    Mlim = end;
    Bg = B + (int64_t)g * ep.bstride;
  } else {
    const int g = (int)blockIdx.x / nwg, t = (int)blockIdx.x % nwg;
    const int start = g ? ep.offs[g - 1] : 0, end = ep.offs[g];
    m0 = (t / nTn) * BM;
    n0 = (t % nTn) * BN;
    Ag = A + (int64_t)start * lda;
    Bg = B + (int64_t)start * ldb;
    Cg = C + (int64_t)g * ep.cstride;
    Kr = max(0, end - start);
  }

  Stager<AT, false, GRP == 2> sa;
  Stager<BT, EPI == 1, GRP == 2> sb;
  sa.init(Ag, lda, m0, Kr, wave, lane, nullptr, min(BM, Mlim - m0));
  if constexpr (EPI == 1)
    sb.init(Bg, ldb, n0 / 2, Kr, wave, lane, B2);
  else
    sb.init(Bg, ldb, n0, Kr, wave, lane, nullptr, min(BN, N - n0));
  // glds j (0..15) of a K-tile: j < 8 -> A instruction j, else B instruction j - 8
  auto glds = [&](int j, int kt, char* stage) {
    if (j < 8)
      sa.issue(j, kt, stage, wave);
    else
      sb.issue(j - 8, kt, stage + OP_BYTES, wave);
  };

  f32x4 acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  bf16x8 fa0[8], fb0[8], fa1[8], fb1[8];
  auto mma = [](f32x4& c, const bf16x8& a, const bf16x8& b) {
    if constexpr (SW) mfma16(c, b, a); else mfma16(c, a, b);
  };
  // fragment read r (0..15) of one k-step, in the order the MFMAs consume them: A0, B0..B7, A1..A7
  auto read_one = [&](const char* stage, int kk, int r, bf16x8* fa, bf16x8* fb) {
    if (r == 0)
      fa[0] = read_frag<AT>(stage, wm * 128, kk, fr, fq);
    else if (r <= 8)
      fb[r - 1] = read_frag<BT>(stage + OP_BYTES, wn * 128 + (r - 1) * 16, kk, fr, fq);
    else
      fa[r - 8] = read_frag<AT>(stage, wm * 128 + (r - 8) * 16, kk, fr, fq);
  };

  // glds split: NB2 instructions of tile t+2 in phase B2 of tile t, the rest (16 - NB2) in the first
  // half of phase A of tile t+1.  (Staging through registers + ds_write_b128 instead of LDS-DMA
  // was measured 5-10 % slower for K-major operands and 35-50 % slower for the wgrad layout,
  // where its 64 staging VGPRs spill: profiles/gemm4_microbench.json history, round 3.)
  constexpr int NB2 = VAR == 0 ? 16 : (VAR == 1 ? 8 : 4);
  constexpr int NA = 16 - NB2;

  // GRP 2: ceil to an even K-tile count (the zero-filled tail tiles add nothing)
  const int nk = GRP == 2 ? (Kr + 2 * BK - 1) / (2 * BK) * 2 : Kr / BK;
  // ---- prologue: tile 0 whole, tile 1's phase-B2 share; wait for tile 0 ----
#pragma unroll
  for (int j = 0; j < 16; ++j) glds(j, 0, smem);
#pragma unroll
  for (int j = 0; j < NB2; ++j) glds(j, 1, smem + STAGE);
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NB2) : "memory");
  __builtin_amdgcn_s_barrier();
#pragma unroll
  for (int r = 0; r < 16; ++r) read_one(smem, 0, r, fa0, fb0);

  // one K-tile; CUR = its stage buffer.  No branch inside the pinned instruction stream: past the
  // last K-tile the prefetch re-stages tile nk-1 (an L2 hit into a buffer nobody reads again) and the
  // next-tile fragment reads read a stale buffer whose values are never used.
  auto body = [&](int t, auto cur_c) {
    constexpr int CUR = decltype(cur_c)::value;
    char* const bc = smem + CUR * STAGE;
    char* const bn = smem + (CUR ^ 1) * STAGE;
    const int t1 = min(t + 1, nk - 1), t2 = min(t + 2, nk - 1);
    // phase A: k-step 0 of tile t from (fa0, fb0); read k-step 1; finish tile t+1's staging
#pragma unroll
    for (int i = 0; i < 64; ++i) {
      mma(acc[i >> 3][i & 7], fa0[i >> 3], fb0[i & 7]);
      if ((i & 3) == 0) read_one(bc, 1, i >> 2, fa1, fb1);
      if (NA > 0 && (i & 3) == 2 && (i >> 2) < NA) glds(NB2 + (i >> 2), t1, bn);
      LTA_FENCE();
    }
    // phase B1: rows 0..3 of k-step 1
#pragma unroll
    for (int i = 0; i < 32; ++i) {
      mma(acc[i >> 3][i & 7], fa1[i >> 3], fb1[i & 7]);
      LTA_FENCE();
    }
    // tile t+1 has landed for this wave and tile t is fully read by it; then for everyone
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    LTA_FENCE();
    // phase B2: rows 4..7 of k-step 1; read k-step 0 of tile t+1; stage tile t+2 into this buffer
#pragma unroll
    for (int i = 32; i < 64; ++i) {
      mma(acc[i >> 3][i & 7], fa1[i >> 3], fb1[i & 7]);
      const int s = i - 32;
      if ((s & 1) == 0)
        read_one(bn, 0, s >> 1, fa0, fb0);
      else if (NB2 == 16 || ((s & 3) == 1 && (s >> 2) < NB2))
        glds(NB2 == 16 ? (s >> 1) : (s >> 2), t2, bc);
      LTA_FENCE();
    }
  };
  // nk is even (K % 128 == 0, checked by the host).  An odd-K-tile tail (K % 128 == 64) as a third body
  // instance after this loop changed hipcc's schedule of the plain instantiation into wrong results
  // (tests/test_hip_kernels.py::test_gemm4_edge_tiles, round 6): such K take the other GEMM paths.
  for (int t = 0; t < nk; t += 2) {
    body(t, std::integral_constant<int, 0>{});
    body(t + 1, std::integral_constant<int, 1>{});
  }

  // the last asm MFMAs' results must be complete before the epilogue reads the accumulators
#pragma unroll
  for (int m = 0; m < 8; ++m)
#pragma unroll
    for (int n = 0; n < 8; ++n) asm volatile("" : "+a"(acc[m][n]));
  asm volatile("s_nop 15\n\ts_nop 15" ::: "memory");
  // the last K-tile's (dummy) prefetch of every wave must have landed before any wave overwrites
  // the stage buffers with its output image
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();

  if constexpr (TAIL == 2) {  // K split: the fp32 partial of this K slice (summed by gemm4_tail_fixup)
    static_assert(SW, "tail split: swapped layout");
    float* P = ep.partial + ((int64_t)kpart * ep.tile_count + (wg_lin - ep.tile_base)) * (BM * BN);
#pragma unroll
    for (int m = 0; m < 8; ++m)
#pragma unroll
      for (int n = 0; n < 8; ++n) {
        // 4 consecutive fp32 columns of one row per lane: one 16-B store
        *reinterpret_cast<f32x4*>(P + (wm * 128 + m * 16 + fr) * BN + wn * 128 + n * 16 + fq * 4) = acc[m][n];
        __builtin_amdgcn_sched_barrier(0);  // one accumulator block at a time: bounded VGPR use
      }
    return;
  }
  if constexpr (SW) {
    const int rsel = fq & 1, csel = fq >> 1;
    if constexpr (EPI == 1) {
      // gate-up: blocks 0-3 of this wave are a = x W1^T and blocks 4-7 b = x W2^T for the SAME 64 output
      // columns c0 .. c0 + 63 (c0 = n0 / 2 + 64 wn); y = silu(a) * b from the bf16-rounded a, b (the
      // unfused path's rounding points)
      const int c0 = n0 / 2 + wn * 64;
#pragma unroll
      for (int m = 0; m < 8; ++m) {
        const int64_t grow = m0 + wm * 128 + m * 16 + fr;
        uint32_t pa[4][2], pb[4][2], py[4][2];
#pragma unroll
        for (int n = 0; n < 4; ++n) {
          float a[4], b[4], y[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            a[j] = bf16_round(acc[m][n][j]);
            b[j] = bf16_round(acc[m][n + 4][j]);
            y[j] = a[j] * sigmoid_f(a[j]) * b[j];
          }
          pa[n][0] = pack_bf16x2(a[0], a[1]);
          pa[n][1] = pack_bf16x2(a[2], a[3]);
          pb[n][0] = pack_bf16x2(b[0], b[1]);
          pb[n][1] = pack_bf16x2(b[2], b[3]);
          py[n][0] = pack_bf16x2(y[0], y[1]);
          py[n][1] = pack_bf16x2(y[2], y[3]);
        }
#pragma unroll
        for (int np = 0; np < 2; ++np) {
          const int n = 2 * np;
          const uint4 va = swap_pair(pa[n][0], pa[n][1], pa[n + 1][0], pa[n + 1][1]);
          const uint4 vb = swap_pair(pb[n][0], pb[n][1], pb[n + 1][0], pb[n + 1][1]);
          const uint4 vy = swap_pair(py[n][0], py[n][1], py[n + 1][0], py[n + 1][1]);
          if (grow < M) {
            const int64_t o = grow * ldc + c0 + (n + rsel) * 16 + csel * 8;
            if (C != nullptr) *reinterpret_cast<uint4*>(C + o) = va;
            if (C2 != nullptr) *reinterpret_cast<uint4*>(C2 + o) = vb;
            *reinterpret_cast<uint4*>(C3 + o) = vy;
          }
        }
        __builtin_amdgcn_sched_barrier(0);  // one row block at a time: bounded VGPR use
      }
      return;
    }
    if constexpr (EPI == 2) {
      // swiglu backward in the dgrad epilogue: g (rounded to bf16, as the unfused dgrad stores it) and
      // a, b at the same 8 elements -> da = g b silu'(a), db = g silu(a); g never leaves the chip
#pragma unroll
      for (int m = 0; m < 8; ++m) {
        const int64_t grow = m0 + wm * 128 + m * 16 + fr;
#pragma unroll
        for (int np = 0; np < 4; ++np) {
          const int n = 2 * np;
          const uint4 gv = swap_pair(pack_bf16x2(acc[m][n][0], acc[m][n][1]), pack_bf16x2(acc[m][n][2], acc[m][n][3]),
                                     pack_bf16x2(acc[m][n + 1][0], acc[m][n + 1][1]),
                                     pack_bf16x2(acc[m][n + 1][2], acc[m][n + 1][3]));
          const int gcol = n0 + wn * 128 + (n + rsel) * 16 + csel * 8;
          if (grow < M) {
            const uint4 va = *reinterpret_cast<const uint4*>(R + grow * ldc + gcol);
            const uint4 vb = *reinterpret_cast<const uint4*>(R2 + grow * ldc + gcol);
            const __hip_bfloat16* g = reinterpret_cast<const __hip_bfloat16*>(&gv);
            const __hip_bfloat16* a = reinterpret_cast<const __hip_bfloat16*>(&va);
            const __hip_bfloat16* b = reinterpret_cast<const __hip_bfloat16*>(&vb);
            float da[8], db[8];
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              const float x = __bfloat162float(a[e]), gg = __bfloat162float(g[e]), bb = __bfloat162float(b[e]);
              const float sg = sigmoid_f(x);
              da[e] = gg * bb * (sg * (1.f + x * (1.f - sg)));
              db[e] = gg * (x * sg);
            }
            *reinterpret_cast<uint4*>(C + grow * ldc + gcol) =
                make_uint4(pack_bf16x2(da[0], da[1]), pack_bf16x2(da[2], da[3]), pack_bf16x2(da[4], da[5]),
                           pack_bf16x2(da[6], da[7]));
            *reinterpret_cast<uint4*>(C2 + grow * ldc + gcol) =
                make_uint4(pack_bf16x2(db[0], db[1]), pack_bf16x2(db[2], db[3]), pack_bf16x2(db[4], db[5]),
                           pack_bf16x2(db[6], db[7]));
          }
          __builtin_amdgcn_sched_barrier(0);  // one block pair at a time: bounded VGPR use
        }
      }
      return;
    }
    if constexpr (EPI == 3) {
      // this wave's 128 columns are one head: q head cb, k head cb - nh or v head cb - nh - ng.  A
      // dimension d < 64 (block n < 4) and its rotate-half partner d + 64 (block n + 4) sit in the same
      // lane and register; both use cos / sin of d (rotate-half duplicates them), applied to the
      // bf16-rounded projection as csrc/rope.hip does
      const int cb = (n0 + wn * 128) >> 7;
      const bool is_q = cb < ep.nh, is_k = !is_q && cb < ep.nh + ep.ng;
      __hip_bfloat16* const dst = is_q ? C : (is_k ? C2 : C3);
      const int hh = is_q ? cb : (is_k ? cb - ep.nh : cb - ep.nh - ep.ng);
      const int nheads = is_q ? ep.nh : ep.ng;
      const bool rope = is_q || is_k;
      // cos / sin of row block m + 1 are loaded while block m is rotated and stored (loading them inside
      // its own sched region exposed an L2 round trip per row block)
      float4 cc[4], sc[4];
      auto load_cs = [&](int m, float4 (&c)[4], float4 (&sn)[4]) {
        const int t = min(m0 + wm * 128 + m * 16 + fr, M - 1) % ep.T;
#pragma unroll
        for (int n = 0; n < 4; ++n) {
          c[n] = *reinterpret_cast<const float4*>(ep.cos_ + (int64_t)t * 128 + n * 16 + fq * 4);
          sn[n] = *reinterpret_cast<const float4*>(ep.sin_ + (int64_t)t * 128 + n * 16 + fq * 4);
        }
      };
      if (rope) load_cs(0, cc, sc);
#pragma unroll
      for (int m = 0; m < 8; ++m) {
        float4 cn[4], snx[4];
        if (rope && m < 7) load_cs(m + 1, cn, snx);
        const int grow = m0 + wm * 128 + m * 16 + fr;
        const int gr = min(grow, M - 1);
        const int bi = gr / ep.T, t = gr - bi * ep.T;
        __hip_bfloat16* const orow = dst + (((int64_t)bi * nheads + hh) * ep.T + t) * 128;
        uint32_t lo[4][2], hi[4][2];  // blocks n (dims < 64) and n + 4 (partners), packed
#pragma unroll
        for (int n = 0; n < 4; ++n) {
          float x1[4], x2[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            x1[j] = bf16_round(acc[m][n][j]);
            x2[j] = bf16_round(acc[m][n + 4][j]);
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
          const uint4 vlo = swap_pair(lo[n][0], lo[n][1], lo[n + 1][0], lo[n + 1][1]);
          const uint4 vhi = swap_pair(hi[n][0], hi[n][1], hi[n + 1][0], hi[n + 1][1]);
          if (grow < M) {
            const int col = (n + rsel) * 16 + csel * 8;
            *reinterpret_cast<uint4*>(orow + col) = vlo;
            *reinterpret_cast<uint4*>(orow + col + 64) = vhi;
          }
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
    } else {
      // plain / bias / activation / residual (GRP 0, 1, 2)
      float bv[8][4];
#pragma unroll
      for (int n = 0; n < 8; ++n)
#pragma unroll
        for (int j = 0; j < 4; ++j) bv[n][j] = 0.f;
      if constexpr (BIAS) {
#pragma unroll
        for (int n = 0; n < 8; ++n) {
          const int c0 = n0 + wn * 128 + n * 16 + fq * 4;  // N % 8 == 0: the 4 columns are all in or all out
          if (c0 < N) {
            const uint2 u = *reinterpret_cast<const uint2*>(bias + c0);
            const __hip_bfloat16* h = reinterpret_cast<const __hip_bfloat16*>(&u);
#pragma unroll
            for (int j = 0; j < 4; ++j) bv[n][j] = to_f32(h[j]);
          }
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
            for (int j = 0; j < 4; ++j) {
              float x = acc[m][n + h][j] * alpha;
              if constexpr (BIAS) x += bv[n + h][j];
              v[h][j] = act_fn<ACT>(x);
            }
          uint4 val = swap_pair(pack_bf16x2(v[0][0], v[0][1]), pack_bf16x2(v[0][2], v[0][3]),
                                pack_bf16x2(v[1][0], v[1][1]), pack_bf16x2(v[1][2], v[1][3]));
          const int gcol = n0 + wn * 128 + (n + rsel) * 16 + csel * 8;
          if (grow < Mlim && gcol < N) {  // edge tile (or group end): N % 8 == 0, a chunk is all in or out
            if constexpr (RES) {
              // y (rounded to bf16, as ATen's linear stores it) + r, rounded once more
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
            *reinterpret_cast<uint4*>(Cg + grow * ldc + gcol) = val;
          }
          __builtin_amdgcn_sched_barrier(0);  // one block pair at a time: bounded VGPR use
        }
      }
      return;
    }
  } else {
  // ---- epilogue: every wave has passed the last barrier after its final LDS read, so the stage
  // buffers are free: registers -> swizzled bf16 image (per wave 128 x 128, 256-B rows) -> stores
  char* wbuf = smem + wave * (128 * 256);
#pragma unroll
  for (int n = 0; n < 8; ++n) {
    const int col = n * 16 + fr;
    float bv = 0.f;
    if constexpr (BIAS) bv = (n0 + wn * 128 + col < N) ? to_f32(bias[n0 + wn * 128 + col]) : 0.f;
    const int ch = col >> 3, co = (col & 7) * 2;
#pragma unroll
    for (int m = 0; m < 8; ++m) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int row = m * 16 + fq * 4 + j;
        float v = acc[m][n][j] * alpha + bv;
        v = act_fn<ACT>(v);
        *reinterpret_cast<__hip_bfloat16*>(wbuf + row * 256 + ((ch ^ (row & 15)) << 4) + co) = __float2bfloat16(v);
      }
    }
    __builtin_amdgcn_sched_barrier(0);  // one accumulator column block at a time: bounded VGPR use
  }
  __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's image is complete
  if constexpr (EPI == 1) {
    __syncthreads();  // the partner wave's image (b for a, a for b) is read below
  } else {
    __builtin_amdgcn_wave_barrier();
  }
  if constexpr (EPI == 1) {
    // a (wn = 0) / b (wn = 1) quadrant of this wave -> its own output at column n0/2 + ...
    __hip_bfloat16* const dst = wn ? C2 : C;
    if (dst != nullptr) {
#pragma unroll
      for (int it = 0; it < 32; ++it) {
        const int id = it * 64 + lane;
        const int row = id >> 4, ch = id & 15;
        const uint4 v = *reinterpret_cast<const uint4*>(wbuf + row * 256 + ((ch ^ (row & 15)) << 4));
        if (m0 + wm * 128 + row < M)
          *reinterpret_cast<uint4*>(dst + (int64_t)(m0 + wm * 128 + row) * ldc + n0 / 2 + ch * 8) = v;
      }
    }
    // y = silu(a) * b: wave (wm, wn) takes rows wn*64 .. +63 of the wm row half
    const char* ia = smem + (wm * 2) * (128 * 256);
    const char* ib = smem + (wm * 2 + 1) * (128 * 256);
#pragma unroll 4
    for (int it = 0; it < 16; ++it) {
      const int id = it * 64 + lane;
      const int row = wn * 64 + (id >> 4), ch = id & 15;
      const int off = row * 256 + ((ch ^ (row & 15)) << 4);
      const uint4 va = *reinterpret_cast<const uint4*>(ia + off), vb = *reinterpret_cast<const uint4*>(ib + off);
      const __hip_bfloat16* a = reinterpret_cast<const __hip_bfloat16*>(&va);
      const __hip_bfloat16* b = reinterpret_cast<const __hip_bfloat16*>(&vb);
      union {
        uint4 u;
        __hip_bfloat16 h[8];
      } o;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float x = __bfloat162float(a[e]);
        o.h[e] = __float2bfloat16(x * sigmoid_f(x) * __bfloat162float(b[e]));
      }
      if (m0 + wm * 128 + row < M)
        *reinterpret_cast<uint4*>(C3 + (int64_t)(m0 + wm * 128 + row) * ldc + n0 / 2 + ch * 8) = o.u;
    }
    return;
  }
  if constexpr (EPI == 3) {
    // this wave's 128 columns are one head: q head cb, k head cb - nh or v head cb - nh - ng
    const int cb = (n0 + wn * 128) >> 7;
    const bool is_q = cb < ep.nh, is_k = !is_q && cb < ep.nh + ep.ng;
    __hip_bfloat16* const dst = is_q ? C : (is_k ? C2 : C3);
    const int hh = is_q ? cb : (is_k ? cb - ep.nh : cb - ep.nh - ep.ng);
    const int nheads = is_q ? ep.nh : ep.ng;
    // one lane = one row's chunk pair (ch, ch + 8): a dimension d < 64 and its partner d + 64 share
    // cos / sin (rotate-half duplicates them), so each pair loads them once
#pragma unroll 4
    for (int it = 0; it < 16; ++it) {
      const int id = it * 64 + lane;
      const int row = id >> 3, ch = id & 7;
      uint4 v0 = *reinterpret_cast<const uint4*>(wbuf + row * 256 + ((ch ^ (row & 15)) << 4));
      uint4 v1 = *reinterpret_cast<const uint4*>(wbuf + row * 256 + (((ch + 8) ^ (row & 15)) << 4));
      const int grow = m0 + wm * 128 + row;
      if (grow >= M) continue;  // edge tile (prefill with T*B % 256 != 0)
      const int bi = grow / ep.T, t = grow - bi * ep.T;
      __hip_bfloat16* const o = dst + (((int64_t)bi * nheads + hh) * ep.T + t) * 128 + ch * 8;
      if (is_q || is_k) {
        const float4* cp = reinterpret_cast<const float4*>(ep.cos_ + (int64_t)t * 128 + ch * 8);
        const float4* sp = reinterpret_cast<const float4*>(ep.sin_ + (int64_t)t * 128 + ch * 8);
        const float4 c0 = cp[0], c1 = cp[1], s0 = sp[0], s1 = sp[1];
        const float cs[8] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w};
        const float sn[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
        const __hip_bfloat16* x1 = reinterpret_cast<const __hip_bfloat16*>(&v0);
        const __hip_bfloat16* x2 = reinterpret_cast<const __hip_bfloat16*>(&v1);
        union {
          uint4 u;
          __hip_bfloat16 h[8];
        } o1, o2;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float a = __bfloat162float(x1[e]), bb = __bfloat162float(x2[e]);
          o1.h[e] = __float2bfloat16(a * cs[e] - bb * sn[e]);
          o2.h[e] = __float2bfloat16(bb * cs[e] + a * sn[e]);
        }
        v0 = o1.u;
        v1 = o2.u;
      }
      *reinterpret_cast<uint4*>(o) = v0;
      *reinterpret_cast<uint4*>(o + 64) = v1;
    }
    return;
  }
#pragma unroll
  for (int it = 0; it < 32; ++it) {
    const int id = it * 64 + lane;
    const int row = id >> 4, ch = id & 15;
    uint4 v = *reinterpret_cast<const uint4*>(wbuf + row * 256 + ((ch ^ (row & 15)) << 4));
    const int64_t grow = m0 + wm * 128 + row;
    const int gcol = n0 + wn * 128 + ch * 8;
    if (grow >= Mlim || gcol >= N) continue;  // edge tile (or group end): N % 8 == 0, a chunk is all in or out
    if constexpr (EPI == 2) {
      // v = g (bf16, as the unfused dgrad stores it); a, b at the same element
      const uint4 va = *reinterpret_cast<const uint4*>(R + grow * ldc + gcol);
      const uint4 vb = *reinterpret_cast<const uint4*>(R2 + grow * ldc + gcol);
      const __hip_bfloat16* g = reinterpret_cast<const __hip_bfloat16*>(&v);
      const __hip_bfloat16* a = reinterpret_cast<const __hip_bfloat16*>(&va);
      const __hip_bfloat16* b = reinterpret_cast<const __hip_bfloat16*>(&vb);
      union {
        uint4 u;
        __hip_bfloat16 h[8];
      } oa, ob;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float x = __bfloat162float(a[e]), gg = __bfloat162float(g[e]), bb = __bfloat162float(b[e]);
        const float sg = sigmoid_f(x);
        oa.h[e] = __float2bfloat16(gg * bb * (sg * (1.f + x * (1.f - sg))));
        ob.h[e] = __float2bfloat16(gg * (x * sg));
      }
      *reinterpret_cast<uint4*>(C + grow * ldc + gcol) = oa.u;
      *reinterpret_cast<uint4*>(C2 + grow * ldc + gcol) = ob.u;
      continue;
    }
    if constexpr (RES) {
      const uint4 rv = *reinterpret_cast<const uint4*>(R + grow * ldr + gcol);
      const __hip_bfloat16* a = reinterpret_cast<const __hip_bfloat16*>(&v);
      const __hip_bfloat16* b = reinterpret_cast<const __hip_bfloat16*>(&rv);
      union {
        uint4 u;
        __hip_bfloat16 h[8];
      } o;
#pragma unroll
      for (int e = 0; e < 8; ++e) o.h[e] = __float2bfloat16(__bfloat162float(a[e]) + __bfloat162float(b[e]));
      v = o.u;
    }
    *reinterpret_cast<uint4*>(Cg + grow * ldc + gcol) = v;
  }
  }  // !SW
}

#undef LTA_FENCE

// C tiles of a tail split: sum the K-slice partials (fixed order), scale, round, store (edges masked).
// One thread per 8 consecutive columns of a tile row.
__global__ __launch_bounds__(256) void gemm4_tail_fixup(const float* __restrict__ partial, __hip_bfloat16* __restrict__ C,
                                                        int ksplit, int tile_base, int tile_count, int M, int N,
                                                        int ldc, float alpha,
                                                        const __hip_bfloat16* __restrict__ bias = nullptr) {
  const int64_t id = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int t = (int)(id / (BM * BN / 8));
  if (t >= tile_count) return;
  const int rem = (int)(id % (BM * BN / 8)), row = rem / (BN / 8), ch = rem % (BN / 8);
  int tm, tn;
  tile_coords(tile_base + t, (M + BM - 1) / BM, (N + BN - 1) / BN, tm, tn);
  const int64_t grow = (int64_t)tm * BM + row;
  const int gcol = tn * BN + ch * 8;
  if (grow >= M || gcol >= N) return;
  float a[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (int k = 0; k < ksplit; ++k) {
    const float* p = partial + ((int64_t)k * tile_count + t) * (BM * BN) + row * BN + ch * 8;
    const float4 x = *reinterpret_cast<const float4*>(p), y = *reinterpret_cast<const float4*>(p + 4);
    a[0] += x.x; a[1] += x.y; a[2] += x.z; a[3] += x.w; a[4] += y.x; a[5] += y.y; a[6] += y.z; a[7] += y.w;
  }
  union {
    uint4 u;
    __hip_bfloat16 h[8];
  } o;
  if (bias != nullptr) {  // the unsplit epilogue's alpha * acc + bias, one rounding
    const uint4 bu = *reinterpret_cast<const uint4*>(bias + gcol);
    const __hip_bfloat16* bh = reinterpret_cast<const __hip_bfloat16*>(&bu);
#pragma unroll
    for (int e = 0; e < 8; ++e) o.h[e] = __float2bfloat16(a[e] * alpha + __bfloat162float(bh[e]));
  } else {
#pragma unroll
    for (int e = 0; e < 8; ++e) o.h[e] = __float2bfloat16(a[e] * alpha);
  }
  *reinterpret_cast<uint4*>(C + grow * ldc + gcol) = o.u;
}

// Plain product with a wave-quantisation tail: the last partial wave of tiles (at most half as many
// tiles as CUs) runs as 2 K-slices per tile (so it takes half a tile time instead of a whole one), then a
// fixup sums the two fp32 partials.  Returns -1 when the shape does not qualify.
// Compute units of the current device (one resident workgroup each): the wave size of the tile grid.
int device_cus() {
  int dev = 0, n = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    return 256;
  return n > 0 ? n : 256;
}

template <bool AT, bool BT>
int launch4_tail(const void* A, const void* B, void* C, int M, int N, int K, int lda, int ldb, int ldc, float alpha,
                 void* ws, int64_t ws_bytes, hipStream_t s) {
  const int cus = device_cus();
  const int nwg = ((M + BM - 1) / BM) * ((N + BN - 1) / BN), tail = nwg % cus;
  if (nwg <= cus || tail == 0 || 2 * tail > cus || K % (2 * BK * 2) || !ws || ws_bytes < (int64_t)2 * tail * BM * BN * 4)
    return -1;
  EpiArgs ep{};
  ep.tile_base = 0;
  ep.tile_count = nwg - tail;
  hipLaunchKernelGGL((gemm4_bf16_kernel<kNone, false, false, AT, BT, 1, 0, 0, 1>), dim3(nwg - tail), dim3(NTHR), 0, s,
                     (const __hip_bfloat16*)A, (const __hip_bfloat16*)B, (__hip_bfloat16*)C, nullptr, nullptr, M, N, K,
                     lda, ldb, ldc, 0, alpha, ep);
  ep.tile_base = nwg - tail;
  ep.tile_count = tail;
  ep.ksplit = 2;
  ep.partial = (float*)ws;
  hipLaunchKernelGGL((gemm4_bf16_kernel<kNone, false, false, AT, BT, 1, 0, 0, 2>), dim3(2 * tail), dim3(NTHR), 0, s,
                     (const __hip_bfloat16*)A, (const __hip_bfloat16*)B, (__hip_bfloat16*)C, nullptr, nullptr, M, N, K,
                     lda, ldb, ldc, 0, 1.f, ep);
  hipLaunchKernelGGL(gemm4_tail_fixup, dim3((unsigned)((int64_t)tail * (BM * BN / 8) / 256)), dim3(256), 0, s,
                     (const float*)ws, (__hip_bfloat16*)C, 2, nwg - tail, tail, M, N, ldc, alpha);
  return (int)hipGetLastError();
}

// Plain product whose whole tile grid is at most half a wave (wgrad / dgrad of narrow layers: e.g. the
// 16 - 128 tiles of GPT-2-medium's d = 1024 GEMMs): ksplit K slices per tile fill the CUs, a fixup
// sums the fp32 partials in a fixed order (deterministic).  K % 2 BK == 0; the slices differ by at most
// one 2 BK pair.
template <bool AT, bool BT>
int launch4_splitk(const void* A, const void* B, void* C, const void* bias, int M, int N, int K, int lda, int ldb,
                   int ldc, float alpha, int ksplit, void* ws, int64_t ws_bytes, hipStream_t s) {
  const int nwg = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  if (ksplit < 2 || ksplit > 64 || K % (2 * BK) || K / (2 * BK) < ksplit || !ws ||
      ws_bytes < (int64_t)ksplit * nwg * BM * BN * 4)
    return -2;
  EpiArgs ep{};
  ep.tile_base = 0;
  ep.tile_count = nwg;
  ep.ksplit = ksplit;
  ep.partial = (float*)ws;
  hipLaunchKernelGGL((gemm4_bf16_kernel<kNone, false, false, AT, BT, 1, 0, 0, 2>), dim3(ksplit * nwg), dim3(NTHR), 0,
                     s, (const __hip_bfloat16*)A, (const __hip_bfloat16*)B, (__hip_bfloat16*)C, nullptr, nullptr, M, N,
                     K, lda, ldb, ldc, 0, 1.f, ep);
  hipLaunchKernelGGL(gemm4_tail_fixup, dim3((unsigned)((int64_t)nwg * (BM * BN / 8) / 256)), dim3(256), 0, s,
                     (const float*)ws, (__hip_bfloat16*)C, ksplit, 0, nwg, M, N, ldc, alpha,
                     (const __hip_bfloat16*)bias);
  return (int)hipGetLastError();
}

template <int ACT, bool AT, bool BT, int VAR>
int launch4(const void* A, const void* B, void* C, const void* bias, const void* R, int M, int N, int K, int lda,
            int ldb, int ldc, int ldr, float alpha, hipStream_t s) {
  dim3 grid(((M + BM - 1) / BM) * ((N + BN - 1) / BN)), block(NTHR);
#define LTA_G4(BI, RE)                                                                                            \
  hipLaunchKernelGGL((gemm4_bf16_kernel<ACT, BI, RE, AT, BT, VAR>), grid, block, 0, s, (const __hip_bfloat16*)A,  \
                     (const __hip_bfloat16*)B, (__hip_bfloat16*)C, (const __hip_bfloat16*)bias,                  \
                     (const __hip_bfloat16*)R, M, N, K, lda, ldb, ldc, ldr, alpha)
  if (bias && R) { LTA_G4(true, true); }
  else if (bias) { LTA_G4(true, false); }
  else if (R) { LTA_G4(false, true); }
  else { LTA_G4(false, false); }
#undef LTA_G4
  return (int)hipGetLastError();
}

template <int VAR>
int dispatch_layout(const void* A, const void* B, void* C, const void* bias, const void* R, int M, int N, int K,
                    int lda, int ldb, int ldc, int ldr, float alpha, int act, int at, int bt, hipStream_t s) {
  if (!at && !bt) {
    switch (act) {
      case kNone: return launch4<kNone, false, false, VAR>(A, B, C, bias, R, M, N, K, lda, ldb, ldc, ldr, alpha, s);
      case kGeluTanh: return launch4<kGeluTanh, false, false, VAR>(A, B, C, bias, R, M, N, K, lda, ldb, ldc, ldr, alpha, s);
      case kGeluErf: return launch4<kGeluErf, false, false, VAR>(A, B, C, bias, R, M, N, K, lda, ldb, ldc, ldr, alpha, s);
      case kSilu: return launch4<kSilu, false, false, VAR>(A, B, C, bias, R, M, N, K, lda, ldb, ldc, ldr, alpha, s);
      case kRelu: return launch4<kRelu, false, false, VAR>(A, B, C, bias, R, M, N, K, lda, ldb, ldc, ldr, alpha, s);
      default: return -1;
    }
  }
  if (act != kNone || bias) return -1;  // backward layouts carry no epilogue but the residual
  if (!at && bt) return launch4<kNone, false, true, VAR>(A, B, C, nullptr, R, M, N, K, lda, ldb, ldc, ldr, alpha, s);
  if (at && !bt) return launch4<kNone, true, false, VAR>(A, B, C, nullptr, R, M, N, K, lda, ldb, ldc, ldr, alpha, s);
  return launch4<kNone, true, true, VAR>(A, B, C, nullptr, R, M, N, K, lda, ldb, ldc, ldr, alpha, s);
}

}  // namespace

// C[M,N] = act(alpha * opA . opB + bias) (+ R), bf16 in / fp32 accumulate / bf16 out.
//   at = 0: A [M][K] (lda = row pitch)        at = 1: A stored [K][M] (lda = its row pitch)
//   bt = 0: B [N][K] (nn.Linear weight)       bt = 1: B stored [K][N]
// act/bias only with at = bt = 0.  Any M, N with N % 8 == 0 (edge tiles: clamped operand sources,
// masked stores), K % 128 == 0, 16-B aligned rows, operands under 2 GiB (32-bit buffer offsets).
// variant: glds split; 1 (half of a K-tile's LDS-DMA loads in the barrier phase) is the only one built.
LTA_EXPORT int lta_gemm4_bf16(const void* A, const void* B, void* C, const void* bias, const void* R, int M, int N,
                              int K, int lda, int ldb, int ldc, int ldr, float alpha, int act, int at, int bt,
                              int variant, hipStream_t s) {
  if (N % 8 || K % (2 * BK) || M <= 0 || N <= 0 || K <= 0) return -2;
  if (at && M % 8) return -2;  // MN-major A: 16-B rows
  // buffer-resource byte offsets are 32-bit
  const int64_t ea = at ? (int64_t)K * lda : (int64_t)M * lda, eb = bt ? (int64_t)K * ldb : (int64_t)N * ldb;
  if (ea * 2 >= (1ll << 31) || eb * 2 >= (1ll << 31)) return -2;
  // variant: the LDS-DMA split (1 = 8 of a K-tile's 16 LDS-DMA loads in the previous tile's second
  // half).  The measured alternatives (0: all 16, 2: 4; profiles/gemm4_microbench.json g4v0 / g4v2)
  // are retired from the library; the argument stays in the ABI.
  if (variant != 1) return -1;
  return dispatch_layout<1>(A, B, C, bias, R, M, N, K, lda, ldb, ldc, ldr, alpha, act, at, bt, s);
}

// lta_gemm4_bf16 with a workspace: a plain product (no act / bias / residual, variant 1) whose tile
// grid ends in a partial wave of <= 128 tiles runs that tail split over K (launch4_tail); ws: fp32,
// >= 2 * tail * 256 * 256 elements.  Everything else is lta_gemm4_bf16.
LTA_EXPORT int lta_gemm4_bf16_ws(const void* A, const void* B, void* C, const void* bias, const void* R, int M, int N,
                                 int K, int lda, int ldb, int ldc, int ldr, float alpha, int act, int at, int bt,
                                 int variant, void* ws, int64_t ws_bytes, hipStream_t s) {
  if (ws && variant == 1 && act == kNone && !bias && !R && N % 8 == 0 && M > 0 && N > 0 && K > 0 && !(at && M % 8)) {
    const int64_t ea = at ? (int64_t)K * lda : (int64_t)M * lda, eb = bt ? (int64_t)K * ldb : (int64_t)N * ldb;
    if (ea * 2 < (1ll << 31) && eb * 2 < (1ll << 31)) {
      int rc = -1;
      if (!at && !bt) rc = launch4_tail<false, false>(A, B, C, M, N, K, lda, ldb, ldc, alpha, ws, ws_bytes, s);
      else if (!at && bt) rc = launch4_tail<false, true>(A, B, C, M, N, K, lda, ldb, ldc, alpha, ws, ws_bytes, s);
      else if (at && !bt) rc = launch4_tail<true, false>(A, B, C, M, N, K, lda, ldb, ldc, alpha, ws, ws_bytes, s);
      else rc = launch4_tail<true, true>(A, B, C, M, N, K, lda, ldb, ldc, alpha, ws, ws_bytes, s);
      if (rc != -1) return rc;
    }
  }
  return lta_gemm4_bf16(A, B, C, bias, R, M, N, K, lda, ldb, ldc, ldr, alpha, act, at, bt, variant, s);
}

// C = alpha * opA . opB (+ bias, forward layout) split over K into ksplit slices (launch4_splitk); ws:
// fp32, >= ksplit * tiles * 256 * 256 elements.  Same layouts / limits as lta_gemm4_bf16; -2 on a bad split.
LTA_EXPORT int lta_gemm4_bf16_splitk(const void* A, const void* B, void* C, const void* bias, int M, int N, int K,
                                     int lda, int ldb, int ldc, float alpha, int at, int bt, int ksplit, void* ws,
                                     int64_t ws_bytes, hipStream_t s) {
  if (N % 8 || M <= 0 || N <= 0 || K <= 0 || (at && M % 8) || (bias && (at || bt))) return -2;
  const int64_t ea = at ? (int64_t)K * lda : (int64_t)M * lda, eb = bt ? (int64_t)K * ldb : (int64_t)N * ldb;
  if (ea * 2 >= (1ll << 31) || eb * 2 >= (1ll << 31)) return -2;
  if (!at && !bt) return launch4_splitk<false, false>(A, B, C, bias, M, N, K, lda, ldb, ldc, alpha, ksplit, ws, ws_bytes, s);
  if (!at && bt) return launch4_splitk<false, true>(A, B, C, bias, M, N, K, lda, ldb, ldc, alpha, ksplit, ws, ws_bytes, s);
  if (at && !bt) return launch4_splitk<true, false>(A, B, C, bias, M, N, K, lda, ldb, ldc, alpha, ksplit, ws, ws_bytes, s);
  return launch4_splitk<true, true>(A, B, C, bias, M, N, K, lda, ldb, ldc, alpha, ksplit, ws, ws_bytes, s);
}

// Grouped GEMMs for mixture-of-experts training (K10; reference nvFuser _grouped_mm forward and
// backward, thunder/executors/nvfuserex_impl.py:3226-3252), bf16, variant-1 pipeline.
//   mode 1: C[M][N] rows of group g = A[rows of g][K] . op(B_g), B_g = B + g * bstride:
//           bt = 0: B_g stored [N][K] (the expert weight: MoE forward), bt = 1: stored [K][N] (dgrad:
//           dY . W_g with W_g [N_out = K-of-forward][...]); K % 128 == 0, N % 8 == 0.
//   mode 2: C[g][M][N] (C + g * cstride) = A_g^T . B_g with A stored [rows][M] (lda), B stored
//           [rows][N] (ldb) and group g's rows the reduction (wgrad); any group sizes (zero-filled
//           reduction tails, empty groups give zeros); M, N % 8 == 0.
// offs: int32 [G] cumulative group ends on the device (no host synchronisation).
LTA_EXPORT int lta_gemm4_grouped(int mode, const void* A, const void* B, void* C, const void* offs, int G, int M, int N,
                                 int K, int lda, int ldb, int ldc, int64_t bstride, int64_t cstride, int bt,
                                 hipStream_t s) {
  if (G <= 0 || M <= 0 || N <= 0 || N % 8 || !offs) return -2;
  EpiArgs ep{};
  ep.offs = (const int*)offs;
  ep.G = G;
  ep.bstride = bstride;
  ep.cstride = cstride;
  const int nTn = (N + BN - 1) / BN;
  if (mode == 1) {
    if (K % (2 * BK) || K <= 0) return -2;
    const dim3 grid(((M + BM - 1) / BM + G) * nTn);
    if (bt)
      hipLaunchKernelGGL((gemm4_bf16_kernel<kNone, false, false, false, true, 1, 0, 1>), grid, dim3(NTHR), 0, s,
                         (const __hip_bfloat16*)A, (const __hip_bfloat16*)B, (__hip_bfloat16*)C, nullptr, nullptr, M,
                         N, K, lda, ldb, ldc, 0, 1.f, ep);
    else
      hipLaunchKernelGGL((gemm4_bf16_kernel<kNone, false, false, false, false, 1, 0, 1>), grid, dim3(NTHR), 0, s,
                         (const __hip_bfloat16*)A, (const __hip_bfloat16*)B, (__hip_bfloat16*)C, nullptr, nullptr, M,
                         N, K, lda, ldb, ldc, 0, 1.f, ep);
    return (int)hipGetLastError();
  }
  if (mode == 2) {
    if (M % 8) return -2;
    const dim3 grid(G * ((M + BM - 1) / BM) * nTn);
    hipLaunchKernelGGL((gemm4_bf16_kernel<kNone, false, false, true, true, 1, 0, 2>), grid, dim3(NTHR), 0, s,
                       (const __hip_bfloat16*)A, (const __hip_bfloat16*)B, (__hip_bfloat16*)C, nullptr, nullptr, M, N,
                       K, lda, ldb, ldc, 0, 1.f, ep);
    return (int)hipGetLastError();
  }
  return -1;
}

// Fused SwiGLU GEMMs (see the header), bf16, variant-1 pipeline:
//   mode 1 (gate-up forward): A = x [M][K] (lda), B = W1, B2 = W2, each [Nh][K] (pitch ldb);
//     C = a, C2 = b (either may be null: not needed), C3 = y = silu(a) * b, each [M][Nh] (pitch ldc).
//     Requires Nh % 128 == 0.
//   mode 2 (swiglu backward): A = dY [M][K] (lda), B = W stored [K][Nh] (pitch ldb); R = a, R2 = b,
//     C = da, C2 = db, each [M][Nh] (pitch ldc).  Requires Nh % 256 == 0.
// Any M (edge row tiles), K % 128 == 0, 16-B aligned rows, operands under 2 GiB.
LTA_EXPORT int lta_gemm4_swiglu(const void* A, const void* B, const void* B2, void* C, void* C2, void* C3,
                                const void* R, const void* R2, int M, int Nh, int K, int lda, int ldb, int ldc,
                                int mode, hipStream_t s) {
  if (K % (2 * BK) || M <= 0 || Nh <= 0 || K <= 0) return -2;
  if ((int64_t)M * lda * 2 >= (1ll << 31)) return -2;
  const dim3 block(NTHR);
  const int nTm = (M + BM - 1) / BM;
  if (mode == 1) {
    if (Nh % (BN / 2) || !B2 || !C3 || (int64_t)Nh * ldb * 2 >= (1ll << 31)) return -2;
    const int N = 2 * Nh;
    hipLaunchKernelGGL((gemm4_bf16_kernel<kNone, false, false, false, false, 1, 1>), dim3(nTm * (N / BN)), block,
                       0, s, (const __hip_bfloat16*)A, (const __hip_bfloat16*)B, (__hip_bfloat16*)C, nullptr, nullptr,
                       M, N, K, lda, ldb, ldc, 0, 1.f,
                       EpiArgs{(const __hip_bfloat16*)B2, (__hip_bfloat16*)C2, (__hip_bfloat16*)C3, nullptr, nullptr,
                               nullptr, 0, 0, 0});
    return (int)hipGetLastError();
  }
  if (mode == 2) {
    if (Nh % BN || !R || !R2 || !C || !C2 || (int64_t)K * ldb * 2 >= (1ll << 31)) return -2;
    hipLaunchKernelGGL((gemm4_bf16_kernel<kNone, false, false, false, true, 1, 2>), dim3(nTm * (Nh / BN)), block,
                       0, s, (const __hip_bfloat16*)A, (const __hip_bfloat16*)B, (__hip_bfloat16*)C, nullptr,
                       (const __hip_bfloat16*)R, M, Nh, K, lda, ldb, ldc, ldc, 1.f,
                       EpiArgs{nullptr, (__hip_bfloat16*)C2, nullptr, (const __hip_bfloat16*)R2, nullptr, nullptr, 0, 0,
                               0});
    return (int)hipGetLastError();
  }
  return -1;
}

// q, k, v = RoPE-split(x . W^T) (EPI 3): A = x [M = B*T][K] (lda), B = W [(nh + 2 ng) * 128][K]
// (ldb, rows = q heads, then k heads, then v heads); cos / sin fp32 [T][128] (rotate-half, full
// width); q [B][nh][T][128], k / v [B][ng][T][128] contiguous.  Requires head size 128,
// (nh + 2 ng) even, K % 128 == 0 (any M = B * T: edge row tiles).
LTA_EXPORT int lta_gemm4_qkv_rope(const void* A, const void* B, const float* cos_, const float* sin_, void* q, void* k,
                                  void* v, int M, int K, int lda, int ldb, int T, int nh, int ng, hipStream_t s) {
  const int N = (nh + 2 * ng) * 128;
  if (K % (2 * BK) || N % BN || M <= 0 || K <= 0 || T <= 0 || M % T || nh <= 0 || ng <= 0) return -2;
  if ((int64_t)M * lda * 2 >= (1ll << 31) || (int64_t)N * ldb * 2 >= (1ll << 31)) return -2;
  if (!q || !k || !v || !cos_ || !sin_) return -2;
  hipLaunchKernelGGL((gemm4_bf16_kernel<kNone, false, false, false, false, 1, 3>), dim3(((M + BM - 1) / BM) * (N / BN)),
                     dim3(NTHR), 0, s, (const __hip_bfloat16*)A, (const __hip_bfloat16*)B, (__hip_bfloat16*)q, nullptr,
                     nullptr, M, N, K, lda, ldb, 0, 0, 1.f,
                     EpiArgs{nullptr, (__hip_bfloat16*)k, (__hip_bfloat16*)v, nullptr, cos_, sin_, T, nh, ng});
  return (int)hipGetLastError();
}
