// K2: bf16 GEMM with fused epilogues on CDNA4 MFMA, C[M,N] = act(alpha * A[M,K] . B[N,K]^T + bias) (+ R).
// (reference: cuBLAS(Lt) behind ATen linear, thunder/executors/torchex.py; nvFuser matmul epilogues)
//
// "NT" layout = nn.Linear forward: activations A [M,K] and weights B [N,K] both K-contiguous.
// Geometry (cdna_hip_programming.md §5, 256² template):
//   * 256x256 output tile per workgroup, BK = 64, 512 threads = 8 waves as 2 (M) x 4 (N);
//     each wave owns 128x64 = 8x4 tiles of v_mfma_f32_16x16x32_bf16 (128 fp32 accumulators/lane).
//   * A and B tiles are staged global -> LDS with global_load_lds_dwordx4 (16 B per lane, no VGPR
//     round trip) into two LDS buffers (2 x 64 KiB): the loads of tile t+1 are in flight while
//     tile t is multiplied.
//   * LDS image: 128-B rows (64 bf16 of K); the 16-B chunk c of row r is stored at chunk c ^ (r & 7).
//     glds writes LDS lane-linearly, so the swizzle is applied to each lane's *global* source
//     address; fragment reads (ds_read_b128, 16 rows x 16 B per lane group) then hit 16 distinct
//     16-B slots of the 256-B bank row: conflict-free.
//   * blockIdx -> tile: bijective XCD remap (each XCD gets a contiguous range of tiles), then
//     groups of 8 tile-rows so the 32 CUs of an XCD share A rows and B columns in their L2.
//   * Epilogue: alpha, bias[col], activation in fp32 registers -> bf16 into a swizzled LDS image
//     -> 16-B row-contiguous global stores, with the residual added there (same rounding points
//     as ATen's linear followed by add).
#include "common.h"

using namespace lta;

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void;

constexpr int BM = 256, BN = 256, BK = 64, NTHR = 512;
constexpr int TILE_BYTES = BM * BK * 2;      // 32 KiB per operand per stage
constexpr int STAGE_BYTES = 2 * TILE_BYTES;  // A + B

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

// ---- operand images -------------------------------------------------------------------------
// K-major operand (A [M][K] / B [N][K], the nn.Linear forward): 128-B rows of 64 k, 16-B chunk c of
// row r at chunk c ^ (r & 7); fragments are ds_read_b128 of 8 consecutive k.
// MN-major operand (stored [K][M] / [K][N]: the transposed operands of dgrad and wgrad): 512-B rows
// of 256 m (or n) per k, 16-B chunk c of row k at chunk c ^ tr_swz(k); fragments are two
// ds_read_b64_tr_b16 (cdna_hip_programming.md T10) of rows k..k+3 and k+4..k+7, which deliver the
// 8 consecutive k of column m in natural order.  tr_swz makes every transposed read conflict-free:
// a 32-lane half reads rows {k0+q, k0+8+q} (q < 4) at chunks {c0, c0+1}, and tr_swz maps those 8
// rows to 8 distinct even chunk offsets in the 16-slot bank row.
__device__ __forceinline__ int tr_swz(int k) { return ((k & 3) | (((k >> 3) & 1) << 2)) << 1; }

// one 64 x 256 MN-major tile (64 rows of 512 B) -> LDS at `dst` with global_load_lds: each
// wave-instruction fills two rows (1 KiB, lane-linear), so the swizzle goes on the global source
template <bool MN>
__device__ __forceinline__ void stage_operand(const __hip_bfloat16* __restrict__ X, int ldx, int r0, int k0, char* dst,
                                              int wave, int lane) {
  if constexpr (!MN) {
    const int r = lane >> 3, p = lane & 7;
    const int c = p ^ r;  // swizzled source chunk (row & 7 == r: chunks start at multiples of 8 rows)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int chunk = i * 8 + wave;  // 8 rows per wave-instruction
      const int row = chunk * 8 + r;
      const __hip_bfloat16* g = X + (int64_t)(r0 + row) * ldx + k0 + c * 8;
      __builtin_amdgcn_global_load_lds((const void*)g, (lds_void*)(dst + chunk * 1024), 16, 0, 0);
    }
  } else {
    const int half = lane >> 5, slot = lane & 31;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int chunk = i * 8 + wave;  // rows 2*chunk, 2*chunk + 1
      const int krow = chunk * 2 + half;
      const int c = slot ^ tr_swz(krow);
      const __hip_bfloat16* g = X + (int64_t)(k0 + krow) * ldx + r0 + c * 8;
      __builtin_amdgcn_global_load_lds((const void*)g, (lds_void*)(dst + chunk * 1024), 16, 0, 0);
    }
  }
}

// stage one BMxBK (A) and one BNxBK (B) tile into LDS buffer `sbase`
template <bool AT = false, bool BT = false>
__device__ __forceinline__ void stage_tile(const __hip_bfloat16* __restrict__ A, const __hip_bfloat16* __restrict__ B,
                                           int lda, int ldb, int m0, int n0, int k0, char* sbase, int wave, int lane) {
  stage_operand<AT>(A, lda, m0, k0, sbase, wave, lane);
  stage_operand<BT>(B, ldb, n0, k0, sbase + TILE_BYTES, wave, lane);
}

// 8-element fragment (k = kb + 8*fq .. +7 of row / column `rc`) of a staged operand image
template <bool MN>
__device__ __forceinline__ bf16x8 read_frag(const char* img, int rc, int kk, int fr, int fq) {
  if constexpr (!MN) {
    const int c = kk * 4 + fq;
    return *reinterpret_cast<const bf16x8*>(img + rc * 128 + ((c ^ (rc & 7)) << 4));
  } else {
    // rc = first column of this 16-lane group's block (multiple of 16); lane 4q+p of the group
    // addresses row k0 + q, columns rc + 4p .. +3
    const int q = fr >> 2, p = fr & 3;
    const int k = kk * 32 + fq * 8 + q;
    const int c = (rc >> 3) + (p >> 1);
    typedef short s16x4 __attribute__((ext_vector_type(4)));
    typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
    const char* p0 = img + k * 512 + ((c ^ tr_swz(k)) << 4) + 8 * (p & 1);
    const char* p1 = img + (k + 4) * 512 + ((c ^ tr_swz(k + 4)) << 4) + 8 * (p & 1);
    const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(__attribute__((address_space(3))) char*)p0);
    const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(__attribute__((address_space(3))) char*)p1);
    union {
      struct { s16x4 a, b; } s;
      bf16x8 f;
    } u;
    u.s.a = lo;
    u.s.b = hi;
    return u.f;
  }
}

template <int ACT, bool BIAS, bool RES, bool AT = false, bool BT = false>
__global__ __launch_bounds__(NTHR, 1) void gemm_nt_bf16_kernel(const __hip_bfloat16* __restrict__ A,
                                                              const __hip_bfloat16* __restrict__ B,
                                                              __hip_bfloat16* __restrict__ C,
                                                              const __hip_bfloat16* __restrict__ bias,
                                                              const __hip_bfloat16* __restrict__ R, int M, int N, int K,
                                                              int lda, int ldb, int ldc, int ldr, float alpha) {
  __shared__ __attribute__((aligned(1024))) char smem[2 * STAGE_BYTES];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 2, wn = wave & 3;

  // tile assignment
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

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = K / BK;
  stage_tile<AT, BT>(A, B, lda, ldb, m0, n0, 0, smem, wave, lane);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  const int fr = lane & 15, fq = lane >> 4;
  for (int t = 0; t < nk; ++t) {
    char* cur = smem + (t & 1) * STAGE_BYTES;
    if (t + 1 < nk)
      stage_tile<AT, BT>(A, B, lda, ldb, m0, n0, (t + 1) * BK, smem + ((t + 1) & 1) * STAGE_BYTES, wave, lane);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 af[8], bfr[4];
#pragma unroll
      for (int m = 0; m < 8; ++m)
        af[m] = read_frag<AT>(cur, wm * 128 + m * 16 + (AT ? 0 : fr), kk, fr, fq);
#pragma unroll
      for (int n = 0; n < 4; ++n)
        bfr[n] = read_frag<BT>(cur + TILE_BYTES, wn * 64 + n * 16 + (BT ? 0 : fr), kk, fr, fq);
#pragma unroll
      for (int m = 0; m < 8; ++m)
#pragma unroll
        for (int n = 0; n < 4; ++n) acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[m], bfr[n], acc[m][n], 0, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  // ---- epilogue: registers -> swizzled bf16 LDS image (per wave 128 x 64) -> 16-B stores ----
  char* wbuf = smem + wave * (128 * 128);
#pragma unroll
  for (int n = 0; n < 4; ++n) {
    const int col = n * 16 + fr;  // column within the wave tile
    float bv = 0.f;
    if constexpr (BIAS) bv = to_f32(bias[n0 + wn * 64 + col]);
    const int ch = col >> 3, co = (col & 7) * 2;
#pragma unroll
    for (int m = 0; m < 8; ++m) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int row = m * 16 + fq * 4 + j;
        float v = acc[m][n][j] * alpha + bv;
        v = act_fn<ACT>(v);
        *reinterpret_cast<__hip_bfloat16*>(wbuf + row * 128 + ((ch ^ (row & 7)) << 4) + co) = __float2bfloat16(v);
      }
    }
  }
  __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's LDS image is complete
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int it = 0; it < 16; ++it) {
    const int id = it * 64 + lane;
    const int row = id >> 3, ch = id & 7;
    uint4 v = *reinterpret_cast<const uint4*>(wbuf + row * 128 + ((ch ^ (row & 7)) << 4));
    const int64_t grow = m0 + wm * 128 + row;
    const int gcol = n0 + wn * 64 + ch * 8;
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
    *reinterpret_cast<uint4*>(C + grow * ldc + gcol) = v;
  }
}

// ---------------------------------------------------------------------------------------------
// 8-phase pipelined variant (cdna_hip_programming.md §5, "256² 8-phase template"; T2/T3+T4/T5).
// Same tile, waves and swizzle as above, but each K-tile (BK = 64) is staged as four 16 KiB
// half-tiles (A rows of m-half 0 / 1 of every wave, B rows of n-half 0 / 1) and consumed in
// four phases of 16 MFMAs (one C-quadrant each):
//   ph1 read A0,B0 -> Q(0,0) | ph2 read B1 -> Q(0,1) | ph3 read A1 -> Q(1,1) | ph4 -> Q(1,0)
// Two K-tiles per loop iteration (even LDS buffer: phases 1-4, odd: 5-8).  Each phase issues ONE
// half-tile of global_load_lds prefetch (2 per lane) into the buffer half that was last read a
// phase earlier, so three half-tiles stay in flight across every barrier: the wait is a counted
// `s_waitcnt vmcnt(6)` at phases 4 and 8 only (never 0 in steady state), barriers are raw
// s_barrier (a __syncthreads() would drain the DMA queue), and all LDS lives in one array.
// Measured on the Llama-2-7B shapes (random data): 6-11 % SLOWER than the 2-buffer loop above
// (profiles/gemm_microbench.json), so variant 0 stays the default; kept for the A/B.
// ---------------------------------------------------------------------------------------------
constexpr int HALF_BYTES = 128 * BK * 2;  // 16 KiB: 128 rows x 128 B

template <int ACT, bool BIAS, bool RES>
__global__ __launch_bounds__(NTHR, 1) void gemm_nt_bf16_8ph_kernel(const __hip_bfloat16* __restrict__ A,
                                                                  const __hip_bfloat16* __restrict__ B,
                                                                  __hip_bfloat16* __restrict__ C,
                                                                  const __hip_bfloat16* __restrict__ bias,
                                                                  const __hip_bfloat16* __restrict__ R, int M, int N,
                                                                  int K, int lda, int ldb, int ldc, int ldr,
                                                                  float alpha) {
  __shared__ __attribute__((aligned(1024))) char smem[8 * HALF_BYTES];  // [buffer 2][part 4] half-tiles

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 2, wn = wave & 3;

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

  // staging: half-tile `part` (0 = A m-half 0, 1 = A m-half 1, 2 = B n-half 0, 3 = B n-half 1) of
  // K-tile kt.  Local row lr of an A part maps to tile row (lr>>6)*128 + part*64 + (lr&63) (wave-row
  // wm = lr>>6 owns local rows 64wm..64wm+63); of a B part to tile column (lr>>5)*64 + h*32 + (lr&31).
  const int sr = lane >> 3, sc = (lane & 7) ^ sr;  // lane's row within an 8-row chunk, swizzled 16-B source chunk
  auto stage = [&](int kt, int part) {
    char* dst = smem + ((kt & 1) * 4 + part) * HALF_BYTES;
    const int k0 = kt * BK + sc * 8;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int chunk = i * 8 + wave;
      const int lr = chunk * 8 + sr;
      const __hip_bfloat16* src;
      if (part < 2) {
        src = A + (int64_t)(m0 + (lr >> 6) * 128 + part * 64 + (lr & 63)) * lda + k0;
      } else {
        src = B + (int64_t)(n0 + (lr >> 5) * 64 + (part - 2) * 32 + (lr & 31)) * ldb + k0;
      }
      __builtin_amdgcn_global_load_lds((const void*)src, (lds_void*)(dst + chunk * 1024), 16, 0, 0);
    }
  };

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int fr = lane & 15, fq = lane >> 4;
  bf16x8 af[4][2], bfr[2][2][2];  // A: 4 m-tiles x 2 k-halves of one part; B: 2 parts x 2 n-tiles x 2 k-halves

  auto read_a = [&](int buf, int part) {
    const char* base = smem + (buf * 4 + part) * HALF_BYTES;
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      const int lr = wm * 64 + m * 16 + fr;
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const int c = kk * 4 + fq;
        af[m][kk] = *reinterpret_cast<const bf16x8*>(base + lr * 128 + ((c ^ (lr & 7)) << 4));
      }
    }
  };
  auto read_b = [&](int buf, int h) {
    const char* base = smem + (buf * 4 + 2 + h) * HALF_BYTES;
#pragma unroll
    for (int n = 0; n < 2; ++n) {
      const int lr = wn * 32 + n * 16 + fr;
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const int c = kk * 4 + fq;
        bfr[h][n][kk] = *reinterpret_cast<const bf16x8*>(base + lr * 128 + ((c ^ (lr & 7)) << 4));
      }
    }
  };
  // C-quadrant (mh, nh): m-tiles 4mh..4mh+3 x n-tiles 2nh, 2nh+1 of the wave's 8x4 accumulator grid
  auto quadrant = [&](int mh, int nh) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int n = 0; n < 2; ++n)
          acc[mh * 4 + m][nh * 2 + n] =
              __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[m][kk], bfr[nh][n][kk], acc[mh * 4 + m][nh * 2 + n], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };
#define LTA_PH_SYNC()                                 \
  __builtin_amdgcn_s_barrier();                       \
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#define LTA_PH_END() __builtin_amdgcn_s_barrier();

  const int nk = K / BK;  // even (K % 128 == 0)
  // prologue: K-tile 0 whole, K-tile 1 but its A m-half 1 (issued in phase 1)
  stage(0, 0);
  stage(0, 2);
  stage(0, 3);
  stage(0, 1);
  stage(1, 0);
  stage(1, 2);
  stage(1, 3);
  asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  __builtin_amdgcn_s_barrier();

  for (int t0 = 0; t0 < nk; t0 += 2) {
    const int t1 = t0 + 1;
    const bool more = t0 + 2 < nk;
    // ---- even buffer (K-tile t0) ----
    read_a(0, 0);
    read_b(0, 0);
    stage(t1, 1);
    LTA_PH_SYNC();
    quadrant(0, 0);
    LTA_PH_END();

    read_b(0, 1);
    if (more) stage(t0 + 2, 0);
    LTA_PH_SYNC();
    quadrant(0, 1);
    LTA_PH_END();

    read_a(0, 1);
    if (more) stage(t0 + 2, 2);
    LTA_PH_SYNC();
    quadrant(1, 1);
    LTA_PH_END();

    if (more) {
      stage(t0 + 2, 3);
      asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    LTA_PH_SYNC();
    quadrant(1, 0);
    LTA_PH_END();

    // ---- odd buffer (K-tile t1) ----
    read_a(1, 0);
    read_b(1, 0);
    if (more) stage(t0 + 2, 1);
    LTA_PH_SYNC();
    quadrant(0, 0);
    LTA_PH_END();

    read_b(1, 1);
    if (more) stage(t1 + 2, 0);
    LTA_PH_SYNC();
    quadrant(0, 1);
    LTA_PH_END();

    read_a(1, 1);
    if (more) stage(t1 + 2, 2);
    LTA_PH_SYNC();
    quadrant(1, 1);
    LTA_PH_END();

    if (more) {
      stage(t1 + 2, 3);
      asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    }
    LTA_PH_SYNC();
    quadrant(1, 0);
    LTA_PH_END();
  }
#undef LTA_PH_SYNC
#undef LTA_PH_END

  // ---- epilogue (as gemm_nt_bf16_kernel): registers -> swizzled bf16 LDS image -> 16-B stores ----
  char* wbuf = smem + wave * (128 * 128);
#pragma unroll
  for (int n = 0; n < 4; ++n) {
    const int col = n * 16 + fr;
    float bv = 0.f;
    if constexpr (BIAS) bv = to_f32(bias[n0 + wn * 64 + col]);
    const int ch = col >> 3, co = (col & 7) * 2;
#pragma unroll
    for (int m = 0; m < 8; ++m) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int row = m * 16 + fq * 4 + j;
        float v = acc[m][n][j] * alpha + bv;
        v = act_fn<ACT>(v);
        *reinterpret_cast<__hip_bfloat16*>(wbuf + row * 128 + ((ch ^ (row & 7)) << 4) + co) = __float2bfloat16(v);
      }
    }
  }
  __builtin_amdgcn_s_waitcnt(0xc07f);
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int it = 0; it < 16; ++it) {
    const int id = it * 64 + lane;
    const int row = id >> 3, ch = id & 7;
    uint4 v = *reinterpret_cast<const uint4*>(wbuf + row * 128 + ((ch ^ (row & 7)) << 4));
    const int64_t grow = m0 + wm * 128 + row;
    const int gcol = n0 + wn * 64 + ch * 8;
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
    *reinterpret_cast<uint4*>(C + grow * ldc + gcol) = v;
  }
}

// ---------------------------------------------------------------------------------------------
// FP8 (OCP e4m3fn / e5m2) NT GEMM on the block-scaled MFMA (v_mfma_scale_f32_16x16x128_f8f6f4,
// 2x the bf16 rate).  Same geometry and LDS image as the bf16 kernel: BK = 128 fp8 = 128-B rows,
// so staging (glds) and the XOR swizzle are byte-identical.  Per-tensor scaling: the operands
// hold x * s_x; the MFMA block scales are 1.0 and alpha = 1 / (s_a * s_b) is applied in the
// epilogue.  Operand k order of the 16x16x128 f8 MFMA (measured, scripts/mx_debug.py): lane group
// g = l>>4 holds k = 16g..16g+15 in its first 16 bytes and k = 64+16g..+15 in its last 16, and the
// E8M0 scale of lane group g applies to k-block g (k = 32g..32g+31) of its row; so lane l reads
// 16-B chunks g and 4+g of the K-step's 128-B row.
// ---------------------------------------------------------------------------------------------
typedef int v8i __attribute__((ext_vector_type(8)));

__device__ __forceinline__ void stage_tile_bytes(const char* __restrict__ A, const char* __restrict__ B, int lda,
                                                 int ldb, int m0, int n0, int k0, char* sbase, int wave, int lane) {
  const int r = lane >> 3, p = lane & 7;
  const int c = p ^ r;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int chunk = i * 8 + wave;
    const int row = chunk * 8 + r;
    __builtin_amdgcn_global_load_lds((const void*)(A + (int64_t)(m0 + row) * lda + k0 + c * 16),
                                     (lds_void*)(sbase + chunk * 1024), 16, 0, 0);
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int chunk = i * 8 + wave;
    const int row = chunk * 8 + r;
    __builtin_amdgcn_global_load_lds((const void*)(B + (int64_t)(n0 + row) * ldb + k0 + c * 16),
                                     (lds_void*)(sbase + TILE_BYTES + chunk * 1024), 16, 0, 0);
  }
}

template <int FA, int FB>
__device__ __forceinline__ f32x4 mfma_fp8(const v8i& a, const v8i& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, FA, FB, 0, 0x7f7f7f7f, 0, 0x7f7f7f7f);
}

// MXFP8: the E8M0 scale in byte 0 of lane l's scale register applies to k-block l>>4 of row l&15
// (lta_fp8_mfma_scale_probe and the k order above pin this)
template <int FA, int FB>
__device__ __forceinline__ f32x4 mfma_mx(const v8i& a, const v8i& b, const f32x4& c, int sa, int sb) {
  return __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, FA, FB, 0, sa, 0, sb);
}

// MX = true: block-scaled operands; SA [M][K/32] / SB [N][K/32] E8M0 scales (sa / sb unused).  Each
// K-step's scales (4 bytes per tile row: 256 A rows + 256 B rows) are staged into LDS by one 4-byte
// global_load_lds per lane beside the operand tiles, and read back as single bytes.
template <int FA, int FB, bool BIAS, bool MX = false>
__global__ __launch_bounds__(NTHR, 1) void gemm_nt_fp8_kernel(const char* __restrict__ A, const char* __restrict__ B,
                                                             __hip_bfloat16* __restrict__ C,
                                                             const __hip_bfloat16* __restrict__ bias, int M, int N,
                                                             int K, int lda, int ldb, int ldc,
                                                             const float* __restrict__ sa,
                                                             const float* __restrict__ sb,
                                                             const uint8_t* __restrict__ SA = nullptr,
                                                             const uint8_t* __restrict__ SB = nullptr) {
  constexpr int SCALE_BYTES = MX ? 2 * 256 * 4 : 0;  // per stage: A rows then B rows, 4 B each
  __shared__ __attribute__((aligned(1024))) char smem[2 * STAGE_BYTES + 2 * SCALE_BYTES];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 2, wn = wave & 3;
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
  constexpr int BKB = 128;  // fp8 elements (= bytes) per K-step

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = K / BKB;
  const int fr = lane & 15, fq = lane >> 4;
  const int ksc = K / 32;  // scale columns
  char* const sc_base = smem + 2 * STAGE_BYTES;
  auto stage_scales = [&](int t, int buf) {
    // wave w: rows 64 (w & 3) + lane of A (w < 4) or B (w >= 4), the K-step's 4 scale bytes each
    const int row = (wave & 3) * 64 + lane;
    const uint8_t* src = wave < 4 ? SA + (int64_t)(m0 + row) * ksc + t * 4 : SB + (int64_t)(n0 + row) * ksc + t * 4;
    __builtin_amdgcn_global_load_lds((const void*)src, (lds_void*)(sc_base + buf * SCALE_BYTES + wave * 256), 4, 0, 0);
  };
  stage_tile_bytes(A, B, lda, ldb, m0, n0, 0, smem, wave, lane);
  if constexpr (MX) stage_scales(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int t = 0; t < nk; ++t) {
    char* cur = smem + (t & 1) * STAGE_BYTES;
    if (t + 1 < nk) {
      stage_tile_bytes(A, B, lda, ldb, m0, n0, (t + 1) * BKB, smem + ((t + 1) & 1) * STAGE_BYTES, wave, lane);
      if constexpr (MX) stage_scales(t + 1, (t + 1) & 1);
    }
    v8i af[8], bfr[4];
#pragma unroll
    for (int m = 0; m < 8; ++m) {
      const int row = wm * 128 + m * 16 + fr;
      const uint4 lo = *reinterpret_cast<const uint4*>(cur + row * 128 + ((fq ^ (row & 7)) << 4));
      const uint4 hi = *reinterpret_cast<const uint4*>(cur + row * 128 + (((4 + fq) ^ (row & 7)) << 4));
      af[m] = v8i{(int)lo.x, (int)lo.y, (int)lo.z, (int)lo.w, (int)hi.x, (int)hi.y, (int)hi.z, (int)hi.w};
    }
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      const int row = wn * 64 + n * 16 + fr;
      const char* base = cur + TILE_BYTES + row * 128;
      const uint4 lo = *reinterpret_cast<const uint4*>(base + ((fq ^ (row & 7)) << 4));
      const uint4 hi = *reinterpret_cast<const uint4*>(base + (((4 + fq) ^ (row & 7)) << 4));
      bfr[n] = v8i{(int)lo.x, (int)lo.y, (int)lo.z, (int)lo.w, (int)hi.x, (int)hi.y, (int)hi.z, (int)hi.w};
    }
    if constexpr (MX) {
      const uint8_t* scs = reinterpret_cast<const uint8_t*>(sc_base + (t & 1) * SCALE_BYTES);
      int ea[8], eb[4];
#pragma unroll
      for (int m = 0; m < 8; ++m) ea[m] = scs[(wm * 128 + m * 16 + fr) * 4 + fq];
#pragma unroll
      for (int n = 0; n < 4; ++n) eb[n] = scs[1024 + (wn * 64 + n * 16 + fr) * 4 + fq];
#pragma unroll
      for (int m = 0; m < 8; ++m)
#pragma unroll
        for (int n = 0; n < 4; ++n) acc[m][n] = mfma_mx<FA, FB>(af[m], bfr[n], acc[m][n], ea[m], eb[n]);
    } else {
#pragma unroll
      for (int m = 0; m < 8; ++m)
#pragma unroll
        for (int n = 0; n < 4; ++n) acc[m][n] = mfma_fp8<FA, FB>(af[m], bfr[n], acc[m][n]);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  const float alpha = MX ? 1.f : 1.f / (*sa * *sb);
  char* wbuf = smem + wave * (128 * 128);
#pragma unroll
  for (int n = 0; n < 4; ++n) {
    const int col = n * 16 + fr;
    float bv = 0.f;
    if constexpr (BIAS) bv = to_f32(bias[n0 + wn * 64 + col]);
    const int ch = col >> 3, co = (col & 7) * 2;
#pragma unroll
    for (int m = 0; m < 8; ++m)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int row = m * 16 + fq * 4 + j;
        *reinterpret_cast<__hip_bfloat16*>(wbuf + row * 128 + ((ch ^ (row & 7)) << 4) + co) =
            __float2bfloat16(acc[m][n][j] * alpha + bv);
      }
  }
  __builtin_amdgcn_s_waitcnt(0xc07f);
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int it = 0; it < 16; ++it) {
    const int id = it * 64 + lane;
    const int row = id >> 3, ch = id & 7;
    const uint4 v = *reinterpret_cast<const uint4*>(wbuf + row * 128 + ((ch ^ (row & 7)) << 4));
    *reinterpret_cast<uint4*>(C + (int64_t)(m0 + wm * 128 + row) * ldc + n0 + wn * 64 + ch * 8) = v;
  }
}

// ---------------------------------------------------------------------------------------------
// MXFP4 (OCP e2m1 elements, E8M0 scale per 32 along K) NT GEMM on the same block-scaled MFMA with
// format 4 (4x the bf16 rate per clock).  Operands are packed two elements per byte (low nibble =
// even k), so a K-step of 256 elements is the same 128-B LDS row as the fp8 kernel's and staging /
// swizzle are byte-identical; each K-step runs two 16x16x128 sub-steps.  e2m1 operand map of the
// MFMA (measured, tests/test_mxfp4.py): lane l holds row l&15, k = 32 (l>>4) + 2 j + nibble in
// byte j of its first four registers, i.e. 16-B chunk 4 s + (l>>4) of sub-step s; the scale of lane
// group g is that of k-block g of the sub-step.  Scales: 8 per row per K-step, staged as two 4-byte
// global_load_lds per lane (halves h = 0, 1 hold k-blocks 4h..4h+3).
// ---------------------------------------------------------------------------------------------
template <bool BIAS>
__global__ __launch_bounds__(NTHR, 1) void gemm_nt_mxfp4_kernel(const char* __restrict__ A, const char* __restrict__ B,
                                                               __hip_bfloat16* __restrict__ C,
                                                               const __hip_bfloat16* __restrict__ bias, int M, int N,
                                                               int K, int lda, int ldb, int ldc,
                                                               const uint8_t* __restrict__ SA,
                                                               const uint8_t* __restrict__ SB) {
  constexpr int SCALE_BYTES = 2 * 2 * 256 * 4;  // per stage: 2 halves x (A rows, B rows) x 4 B
  __shared__ __attribute__((aligned(1024))) char smem[2 * STAGE_BYTES + 2 * SCALE_BYTES];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 2, wn = wave & 3;
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
  constexpr int BKB = 128;  // bytes (= 256 e2m1 elements) per K-step

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = K / 256;
  const int fr = lane & 15, fq = lane >> 4;
  const int ksc = K / 32;
  char* const sc_base = smem + 2 * STAGE_BYTES;
  auto stage_scales = [&](int t, int buf) {
    const int row = (wave & 3) * 64 + lane;
    const uint8_t* src = wave < 4 ? SA + (int64_t)(m0 + row) * ksc + t * 8 : SB + (int64_t)(n0 + row) * ksc + t * 8;
    char* dst = sc_base + buf * SCALE_BYTES + wave * 256;
    __builtin_amdgcn_global_load_lds((const void*)src, (lds_void*)dst, 4, 0, 0);
    __builtin_amdgcn_global_load_lds((const void*)(src + 4), (lds_void*)(dst + 2048), 4, 0, 0);
  };
  stage_tile_bytes(A, B, lda, ldb, m0, n0, 0, smem, wave, lane);
  stage_scales(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int t = 0; t < nk; ++t) {
    char* cur = smem + (t & 1) * STAGE_BYTES;
    if (t + 1 < nk) {
      stage_tile_bytes(A, B, lda, ldb, m0, n0, (t + 1) * BKB, smem + ((t + 1) & 1) * STAGE_BYTES, wave, lane);
      stage_scales(t + 1, (t + 1) & 1);
    }
    const uint8_t* scs = reinterpret_cast<const uint8_t*>(sc_base + (t & 1) * SCALE_BYTES);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int c = 4 * h + fq;
      v8i af[8], bfr[4];
      int ea[8], eb[4];
#pragma unroll
      for (int m = 0; m < 8; ++m) {
        const int row = wm * 128 + m * 16 + fr;
        const uint4 v = *reinterpret_cast<const uint4*>(cur + row * 128 + ((c ^ (row & 7)) << 4));
        af[m] = v8i{(int)v.x, (int)v.y, (int)v.z, (int)v.w, 0, 0, 0, 0};
        ea[m] = scs[h * 2048 + row * 4 + fq];
      }
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        const int row = wn * 64 + n * 16 + fr;
        const uint4 v = *reinterpret_cast<const uint4*>(cur + TILE_BYTES + row * 128 + ((c ^ (row & 7)) << 4));
        bfr[n] = v8i{(int)v.x, (int)v.y, (int)v.z, (int)v.w, 0, 0, 0, 0};
        eb[n] = scs[h * 2048 + 1024 + row * 4 + fq];
      }
#pragma unroll
      for (int m = 0; m < 8; ++m)
#pragma unroll
        for (int n = 0; n < 4; ++n) acc[m][n] = mfma_mx<4, 4>(af[m], bfr[n], acc[m][n], ea[m], eb[n]);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  char* wbuf = smem + wave * (128 * 128);
#pragma unroll
  for (int n = 0; n < 4; ++n) {
    const int col = n * 16 + fr;
    float bv = 0.f;
    if constexpr (BIAS) bv = to_f32(bias[n0 + wn * 64 + col]);
    const int ch = col >> 3, co = (col & 7) * 2;
#pragma unroll
    for (int m = 0; m < 8; ++m)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int row = m * 16 + fq * 4 + j;
        *reinterpret_cast<__hip_bfloat16*>(wbuf + row * 128 + ((ch ^ (row & 7)) << 4) + co) =
            __float2bfloat16(acc[m][n][j] + bv);
      }
  }
  __builtin_amdgcn_s_waitcnt(0xc07f);
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int it = 0; it < 16; ++it) {
    const int id = it * 64 + lane;
    const int row = id >> 3, ch = id & 7;
    const uint4 v = *reinterpret_cast<const uint4*>(wbuf + row * 128 + ((ch ^ (row & 7)) << 4));
    *reinterpret_cast<uint4*>(C + (int64_t)(m0 + wm * 128 + row) * ldc + n0 + wn * 64 + ch * 8) = v;
  }
}

// ---------------------------------------------------------------------------------------------
// K10: grouped NT GEMM for mixture-of-experts: rows [off[g-1], off[g]) of A are multiplied by
// expert g's weight W[g] ([N, K], K-contiguous like nn.Linear), out[M, N] bf16.  The grid is
// sized for the worst case (ceil(M/256) + G row tiles per column tile); each workgroup finds
// its (expert, row tile) by scanning the device offsets, so no host synchronisation is needed.
// Rows past a group's end are clamped on load and masked on store.
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(NTHR, 1) void gemm_grouped_nt_bf16_kernel(const __hip_bfloat16* __restrict__ A,
                                                                       const __hip_bfloat16* __restrict__ W,
                                                                       __hip_bfloat16* __restrict__ C,
                                                                       const int* __restrict__ offs, int G, int M,
                                                                       int N, int K, int64_t wstride) {
  __shared__ __attribute__((aligned(1024))) char smem[2 * STAGE_BYTES];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 2, wn = wave & 3;
  // locate (expert, row tile)
  int slot = blockIdx.x, g = 0, start = 0, end = 0;
  bool found = false;
  for (; g < G; ++g) {
    end = offs[g];
    const int tiles = (end - start + BM - 1) / BM;
    if (slot < tiles) {
      found = true;
      break;
    }
    slot -= tiles;
    start = end;
  }
  if (!found) return;  // uniform across the workgroup: no barrier skipped by part of it
  const int m0 = start + slot * BM, n0 = blockIdx.y * BN;
  const __hip_bfloat16* B = W + (int64_t)g * wstride;
  const int last = end - 1;

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto stage = [&](int k0, char* sbase) {
    const int r = lane >> 3, p = lane & 7;
    const int c = p ^ r;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int chunk = i * 8 + wave;
      const int row = min(m0 + chunk * 8 + r, last);
      __builtin_amdgcn_global_load_lds((const void*)(A + (int64_t)row * K + k0 + c * 8),
                                       (lds_void*)(sbase + chunk * 1024), 16, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int chunk = i * 8 + wave;
      const int row = n0 + chunk * 8 + r;
      __builtin_amdgcn_global_load_lds((const void*)(B + (int64_t)row * K + k0 + c * 8),
                                       (lds_void*)(sbase + TILE_BYTES + chunk * 1024), 16, 0, 0);
    }
  };
  const int nk = K / BK;
  stage(0, smem);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  const int fr = lane & 15, fq = lane >> 4;
  for (int t = 0; t < nk; ++t) {
    char* cur = smem + (t & 1) * STAGE_BYTES;
    if (t + 1 < nk) stage((t + 1) * BK, smem + ((t + 1) & 1) * STAGE_BYTES);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int c = kk * 4 + fq;
      bf16x8 af[8], bfr[4];
#pragma unroll
      for (int m = 0; m < 8; ++m) {
        const int row = wm * 128 + m * 16 + fr;
        af[m] = *reinterpret_cast<const bf16x8*>(cur + row * 128 + ((c ^ (row & 7)) << 4));
      }
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        const int row = wn * 64 + n * 16 + fr;
        bfr[n] = *reinterpret_cast<const bf16x8*>(cur + TILE_BYTES + row * 128 + ((c ^ (row & 7)) << 4));
      }
#pragma unroll
      for (int m = 0; m < 8; ++m)
#pragma unroll
        for (int n = 0; n < 4; ++n) acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[m], bfr[n], acc[m][n], 0, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  char* wbuf = smem + wave * (128 * 128);
#pragma unroll
  for (int n = 0; n < 4; ++n) {
    const int col = n * 16 + fr;
    const int ch = col >> 3, co = (col & 7) * 2;
#pragma unroll
    for (int m = 0; m < 8; ++m)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int row = m * 16 + fq * 4 + j;
        *reinterpret_cast<__hip_bfloat16*>(wbuf + row * 128 + ((ch ^ (row & 7)) << 4) + co) =
            __float2bfloat16(acc[m][n][j]);
      }
  }
  __builtin_amdgcn_s_waitcnt(0xc07f);
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int it = 0; it < 16; ++it) {
    const int id = it * 64 + lane;
    const int row = id >> 3, ch = id & 7;
    const int grow = m0 + wm * 128 + row;
    if (grow < end) {
      const uint4 v = *reinterpret_cast<const uint4*>(wbuf + row * 128 + ((ch ^ (row & 7)) << 4));
      *reinterpret_cast<uint4*>(C + (int64_t)grow * N + n0 + wn * 64 + ch * 8) = v;
    }
  }
}

// ---------------------------------------------------------------------------------------------
// Grouped FP8 NT GEMM for quantized mixture-of-experts inference (reference te_groupedmm_fp8,
// thunder/transforms/te_inference.py:17-113): rows [off[g-1], off[g]) of the e4m3 activations A
// (one per-tensor scale *sa) times expert g's e4m3 weight W[g] ([N, K], per-expert scale sw[g]),
// out bf16 = acc / (sa * sw[g]).  Row-tile search, clamped loads and masked stores as the bf16
// grouped kernel; the K loop, LDS image and fragment map are those of gemm_nt_fp8_kernel.
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(NTHR, 1) void gemm_grouped_nt_fp8_kernel(const char* __restrict__ A,
                                                                      const char* __restrict__ W,
                                                                      __hip_bfloat16* __restrict__ C,
                                                                      const int* __restrict__ offs, int G, int M,
                                                                      int N, int K, int64_t wstride,
                                                                      const float* __restrict__ sa,
                                                                      const float* __restrict__ sw) {
  __shared__ __attribute__((aligned(1024))) char smem[2 * STAGE_BYTES];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 2, wn = wave & 3;
  int slot = blockIdx.x, g = 0, start = 0, end = 0;
  bool found = false;
  for (; g < G; ++g) {
    end = offs[g];
    const int tiles = (end - start + BM - 1) / BM;
    if (slot < tiles) {
      found = true;
      break;
    }
    slot -= tiles;
    start = end;
  }
  if (!found) return;  // uniform across the workgroup
  const int m0 = start + slot * BM, n0 = blockIdx.y * BN;
  const char* B = W + (int64_t)g * wstride;
  const int last = end - 1;
  constexpr int BKB = 128;

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto stage = [&](int k0, char* sbase) {
    const int r = lane >> 3, p = lane & 7;
    const int c = p ^ r;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int chunk = i * 8 + wave;
      const int row = min(m0 + chunk * 8 + r, last);
      __builtin_amdgcn_global_load_lds((const void*)(A + (int64_t)row * K + k0 + c * 16),
                                       (lds_void*)(sbase + chunk * 1024), 16, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int chunk = i * 8 + wave;
      const int row = n0 + chunk * 8 + r;
      __builtin_amdgcn_global_load_lds((const void*)(B + (int64_t)row * K + k0 + c * 16),
                                       (lds_void*)(sbase + TILE_BYTES + chunk * 1024), 16, 0, 0);
    }
  };
  const int nk = K / BKB;
  stage(0, smem);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  const int fr = lane & 15, fq = lane >> 4;
  for (int t = 0; t < nk; ++t) {
    char* cur = smem + (t & 1) * STAGE_BYTES;
    if (t + 1 < nk) stage((t + 1) * BKB, smem + ((t + 1) & 1) * STAGE_BYTES);
    v8i af[8], bfr[4];
#pragma unroll
    for (int m = 0; m < 8; ++m) {
      const int row = wm * 128 + m * 16 + fr;
      const uint4 lo = *reinterpret_cast<const uint4*>(cur + row * 128 + ((fq ^ (row & 7)) << 4));
      const uint4 hi = *reinterpret_cast<const uint4*>(cur + row * 128 + (((4 + fq) ^ (row & 7)) << 4));
      af[m] = v8i{(int)lo.x, (int)lo.y, (int)lo.z, (int)lo.w, (int)hi.x, (int)hi.y, (int)hi.z, (int)hi.w};
    }
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      const int row = wn * 64 + n * 16 + fr;
      const char* base = cur + TILE_BYTES + row * 128;
      const uint4 lo = *reinterpret_cast<const uint4*>(base + ((fq ^ (row & 7)) << 4));
      const uint4 hi = *reinterpret_cast<const uint4*>(base + (((4 + fq) ^ (row & 7)) << 4));
      bfr[n] = v8i{(int)lo.x, (int)lo.y, (int)lo.z, (int)lo.w, (int)hi.x, (int)hi.y, (int)hi.z, (int)hi.w};
    }
#pragma unroll
    for (int m = 0; m < 8; ++m)
#pragma unroll
      for (int n = 0; n < 4; ++n) acc[m][n] = mfma_fp8<0, 0>(af[m], bfr[n], acc[m][n]);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  const float alpha = 1.f / (*sa * sw[g]);
  char* wbuf = smem + wave * (128 * 128);
#pragma unroll
  for (int n = 0; n < 4; ++n) {
    const int col = n * 16 + fr;
    const int ch = col >> 3, co = (col & 7) * 2;
#pragma unroll
    for (int m = 0; m < 8; ++m)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int row = m * 16 + fq * 4 + j;
        *reinterpret_cast<__hip_bfloat16*>(wbuf + row * 128 + ((ch ^ (row & 7)) << 4) + co) =
            __float2bfloat16(acc[m][n][j] * alpha);
      }
  }
  __builtin_amdgcn_s_waitcnt(0xc07f);
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int it = 0; it < 16; ++it) {
    const int id = it * 64 + lane;
    const int row = id >> 3, ch = id & 7;
    const int grow = m0 + wm * 128 + row;
    if (grow < end) {
      const uint4 v = *reinterpret_cast<const uint4*>(wbuf + row * 128 + ((ch ^ (row & 7)) << 4));
      *reinterpret_cast<uint4*>(C + (int64_t)grow * N + n0 + wn * 64 + ch * 8) = v;
    }
  }
}

template <int ACT>
int launch_act(const void* A, const void* B, void* C, const void* bias, const void* R, int M, int N, int K, int lda,
               int ldb, int ldc, int ldr, float alpha, int variant, hipStream_t s) {
  dim3 grid((M / BM) * (N / BN)), block(NTHR);
  const bool eight = variant == 1 && K % (2 * BK) == 0;
#define LTA_GEMM(BI, RE)                                                                                              \
  if (eight)                                                                                                          \
    hipLaunchKernelGGL((gemm_nt_bf16_8ph_kernel<ACT, BI, RE>), grid, block, 0, s, (const __hip_bfloat16*)A,           \
                       (const __hip_bfloat16*)B, (__hip_bfloat16*)C, (const __hip_bfloat16*)bias,                     \
                       (const __hip_bfloat16*)R, M, N, K, lda, ldb, ldc, ldr, alpha);                                 \
  else                                                                                                                \
    hipLaunchKernelGGL((gemm_nt_bf16_kernel<ACT, BI, RE>), grid, block, 0, s, (const __hip_bfloat16*)A,               \
                       (const __hip_bfloat16*)B, (__hip_bfloat16*)C, (const __hip_bfloat16*)bias,                     \
                       (const __hip_bfloat16*)R, M, N, K, lda, ldb, ldc, ldr, alpha)
  if (bias && R) { LTA_GEMM(true, true); }
  else if (bias) { LTA_GEMM(true, false); }
  else if (R) { LTA_GEMM(false, true); }
  else { LTA_GEMM(false, false); }
#undef LTA_GEMM
  return (int)hipGetLastError();
}

}  // namespace

// C[M,N] (bf16) = (A . B^T) / (*sa * *sb) (+ bias); A [M,K], B [N,K] fp8 (fmt 0 = e4m3fn, 1 = e5m2),
// K % 128 == 0; sa / sb are device scalars (the per-tensor scales the operands were cast with).
LTA_EXPORT int lta_gemm_nt_fp8(const void* A, const void* B, void* C, const void* bias, int M, int N, int K, int lda,
                               int ldb, int ldc, int fmt_a, int fmt_b, const void* sa, const void* sb,
                               hipStream_t stream) {
  if (M % BM || N % BN || K % 128) return -2;
  dim3 grid((M / BM) * (N / BN)), block(NTHR);
#define LTA_F8(FA, FB, BI)                                                                                       \
  hipLaunchKernelGGL((gemm_nt_fp8_kernel<FA, FB, BI>), grid, block, 0, stream, (const char*)A, (const char*)B,    \
                     (__hip_bfloat16*)C, (const __hip_bfloat16*)bias, M, N, K, lda, ldb, ldc, (const float*)sa,          \
                     (const float*)sb)
  const bool bi = bias != nullptr;
  if (fmt_a == 0 && fmt_b == 0) { if (bi) LTA_F8(0, 0, true); else LTA_F8(0, 0, false); }
  else if (fmt_a == 1 && fmt_b == 0) { if (bi) LTA_F8(1, 0, true); else LTA_F8(1, 0, false); }
  else if (fmt_a == 0 && fmt_b == 1) { if (bi) LTA_F8(0, 1, true); else LTA_F8(0, 1, false); }
  else return -1;
#undef LTA_F8
  return (int)hipGetLastError();
}

// MXFP8: C[M,N] (bf16) = A . B^T with E8M0 block scales SA [M][K/32], SB [N][K/32] (+ bias);
// A [M,K], B [N,K] fp8 (fmt 0 = e4m3fn, 1 = e5m2), M, N % 256 == 0, K % 128 == 0.
LTA_EXPORT int lta_gemm_nt_mxfp8(const void* A, const void* B, void* C, const void* bias, const void* SA, const void* SB,
                                 int M, int N, int K, int lda, int ldb, int ldc, int fmt_a, int fmt_b,
                                 hipStream_t stream) {
  if (M % BM || N % BN || K % 128) return -2;
  dim3 grid((M / BM) * (N / BN)), block(NTHR);
#define LTA_MX8(FA, FB, BI)                                                                                      \
  hipLaunchKernelGGL((gemm_nt_fp8_kernel<FA, FB, BI, true>), grid, block, 0, stream, (const char*)A,              \
                     (const char*)B, (__hip_bfloat16*)C, (const __hip_bfloat16*)bias, M, N, K, lda, ldb, ldc,       \
                     (const float*)nullptr, (const float*)nullptr, (const uint8_t*)SA, (const uint8_t*)SB)
  const bool bi = bias != nullptr;
  if (fmt_a == 0 && fmt_b == 0) { if (bi) LTA_MX8(0, 0, true); else LTA_MX8(0, 0, false); }
  else if (fmt_a == 1 && fmt_b == 0) { if (bi) LTA_MX8(1, 0, true); else LTA_MX8(1, 0, false); }
  else if (fmt_a == 0 && fmt_b == 1) { if (bi) LTA_MX8(0, 1, true); else LTA_MX8(0, 1, false); }
  else return -1;
#undef LTA_MX8
  return (int)hipGetLastError();
}

// MXFP4: A [M, K/2], B [N, K/2] packed e2m1 (lda / ldb in bytes), SA [M, K/32], SB [N, K/32] E8M0.
LTA_EXPORT int lta_gemm_nt_mxfp4(const void* A, const void* B, void* C, const void* bias, const void* SA, const void* SB,
                                 int M, int N, int K, int lda, int ldb, int ldc, hipStream_t stream) {
  if (M % BM || N % BN || K % 256 || lda % 16 || ldb % 16) return -2;
  dim3 grid((M / BM) * (N / BN)), block(NTHR);
  if (bias != nullptr)
    hipLaunchKernelGGL((gemm_nt_mxfp4_kernel<true>), grid, block, 0, stream, (const char*)A, (const char*)B,
                       (__hip_bfloat16*)C, (const __hip_bfloat16*)bias, M, N, K, lda, ldb, ldc, (const uint8_t*)SA,
                       (const uint8_t*)SB);
  else
    hipLaunchKernelGGL((gemm_nt_mxfp4_kernel<false>), grid, block, 0, stream, (const char*)A, (const char*)B,
                       (__hip_bfloat16*)C, (const __hip_bfloat16*)nullptr, M, N, K, lda, ldb, ldc, (const uint8_t*)SA,
                       (const uint8_t*)SB);
  return (int)hipGetLastError();
}

// out[M, N] = A[rows of g] @ W[g]^T for g in 0..G-1; offs = int32 end offsets (device), W [G, N, K].
LTA_EXPORT int lta_gemm_grouped_nt_bf16(const void* A, const void* W, void* C, const void* offs, int G, int M, int N,
                                        int K, int64_t wstride, hipStream_t stream) {
  if (N % BN || K % BK) return -2;
  dim3 grid((M + BM - 1) / BM + G, N / BN), block(NTHR);
  hipLaunchKernelGGL(gemm_grouped_nt_bf16_kernel, grid, block, 0, stream, (const __hip_bfloat16*)A,
                     (const __hip_bfloat16*)W, (__hip_bfloat16*)C, (const int*)offs, G, M, N, K, wstride);
  return (int)hipGetLastError();
}

// FP8 grouped: A [M, K] e4m3 (scale *sa), W [G, N, K] e4m3 (scales sw[G]), offs int32 row ends ->
// out [M, N] bf16 = (A_g . W[g]^T) / (sa * sw[g]).  N % 256 == 0, K % 128 == 0.
LTA_EXPORT int lta_gemm_grouped_nt_fp8(const void* A, const void* W, void* C, const void* offs, int G, int M, int N,
                                       int K, int64_t wstride, const void* sa, const void* sw, hipStream_t stream) {
  if (N % BN || K % 128) return -2;
  dim3 grid((M + BM - 1) / BM + G, N / BN), block(NTHR);
  hipLaunchKernelGGL(gemm_grouped_nt_fp8_kernel, grid, block, 0, stream, (const char*)A, (const char*)W,
                     (__hip_bfloat16*)C, (const int*)offs, G, M, N, K, wstride, (const float*)sa, (const float*)sw);
  return (int)hipGetLastError();
}

LTA_EXPORT int lta_gemm_tile_m() { return BM; }
LTA_EXPORT int lta_gemm_tile_n() { return BN; }
LTA_EXPORT int lta_gemm_tile_k() { return BK; }

// C = act(alpha * A @ B^T + bias) + R ; A [M,K] (lda), B [N,K] (ldb), C/R [M,N] (ldc/ldr), all bf16.
// Requires M % 256 == 0, N % 256 == 0, K % 64 == 0 and 16-B aligned rows (checked by the caller).
// variant: 0 = 2-buffer loop, 1 = 8-phase pipelined loop (falls back to 0 unless K % 128 == 0).
// C[M,N] (+)= A . B with either operand stored K-major or MN-major (the backward GEMMs):
//   at = 0: A [M][K] (lda = row pitch);   at = 1: A stored [K][M] (A^T row-major, lda = its pitch)
//   bt = 0: B given as [N][K] (B^T);      bt = 1: B stored [K][N] (row-major, ldb = its pitch)
// R (optional, [M][N] with pitch ldr) is added in the epilogue (gradient accumulation).
LTA_EXPORT int lta_gemm_bf16_layout(const void* A, const void* B, void* C, const void* R, int M, int N, int K, int lda,
                                    int ldb, int ldc, int ldr, float alpha, int at, int bt, hipStream_t s) {
  if (M % BM || N % BN || K % BK) return -2;
  dim3 grid((M / BM) * (N / BN)), block(NTHR);
#define LTA_GL(AT_, BT_, RE)                                                                                    \
  hipLaunchKernelGGL((gemm_nt_bf16_kernel<kNone, false, RE, AT_, BT_>), grid, block, 0, s, (const __hip_bfloat16*)A, \
                     (const __hip_bfloat16*)B, (__hip_bfloat16*)C, nullptr, (const __hip_bfloat16*)R, M, N, K, lda, ldb, \
                     ldc, ldr, alpha)
#define LTA_GL2(AT_, BT_) \
  if (R) { LTA_GL(AT_, BT_, true); } else { LTA_GL(AT_, BT_, false); }
  if (!at && !bt) { LTA_GL2(false, false) }
  else if (!at && bt) { LTA_GL2(false, true) }
  else if (at && !bt) { LTA_GL2(true, false) }
  else { LTA_GL2(true, true) }
#undef LTA_GL2
#undef LTA_GL
  return (int)hipGetLastError();
}

LTA_EXPORT int lta_gemm_nt_bf16_v(const void* A, const void* B, void* C, const void* bias, const void* R, int M, int N,
                                  int K, int lda, int ldb, int ldc, int ldr, float alpha, int act, int variant,
                                  hipStream_t stream) {
  if (M % BM || N % BN || K % BK) return -2;
  switch (act) {
    case kNone: return launch_act<kNone>(A, B, C, bias, R, M, N, K, lda, ldb, ldc, ldr, alpha, variant, stream);
    case kGeluTanh: return launch_act<kGeluTanh>(A, B, C, bias, R, M, N, K, lda, ldb, ldc, ldr, alpha, variant, stream);
    case kGeluErf: return launch_act<kGeluErf>(A, B, C, bias, R, M, N, K, lda, ldb, ldc, ldr, alpha, variant, stream);
    case kSilu: return launch_act<kSilu>(A, B, C, bias, R, M, N, K, lda, ldb, ldc, ldr, alpha, variant, stream);
    case kRelu: return launch_act<kRelu>(A, B, C, bias, R, M, N, K, lda, ldb, ldc, ldr, alpha, variant, stream);
  }
  return -1;
}

LTA_EXPORT int lta_gemm_nt_bf16(const void* A, const void* B, void* C, const void* bias, const void* R, int M, int N,
                                int K, int lda, int ldb, int ldc, int ldr, float alpha, int act, hipStream_t stream) {
  return lta_gemm_nt_bf16_v(A, B, C, bias, R, M, N, K, lda, ldb, ldc, ldr, alpha, act, 0, stream);
}
