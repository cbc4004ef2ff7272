// Persistent-tile experiment for the gemm4 main loop (measurement only): every layout of the
// production kernel (csrc/gemm4.hip Stager / read_frag, variant-1 LDS-DMA split), MFMA operands
// swapped so each lane accumulates 4 consecutive COLUMNS of a C row, register epilogue (cvt_pk +
// v_permlane16_swap -> one 16-B store per pair of 16x16 blocks, no LDS).
//   PERSIST = 0: one tile per workgroup (grid = tiles)
//   PERSIST = 1: grid = min(tiles, CUs), each workgroup walks its tiles; the next tile's prologue
//                LDS-DMA is issued BEFORE this tile's epilogue, so the epilogue's conversions and
//                stores run in the shadow of the prologue's HBM/L2 latency.
#include "common.h"

namespace {
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
constexpr int BM = 256, BN = 256, BK = 64, NTHR = 256;
constexpr int OP_BYTES = BM * BK * 2, STAGE = 2 * OP_BYTES;

__device__ __forceinline__ int xcd_tile(int orig, int nwg) {
  const int xcd = orig & 7, q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
}
__device__ __forceinline__ int tr_swz(int k) { return ((k & 3) | (((k >> 3) & 1) << 2)) << 1; }
__device__ __forceinline__ i32x4 make_rsrc(const void* base, int bytes) {
  const uint64_t a = (uint64_t)(uintptr_t)base;
  return i32x4{(int)(uint32_t)a, (int)((uint32_t)(a >> 32) & 0xffffu), bytes, 0x00020000};
}
template <bool MN>
struct Stager {
  i32x4 rsrc;
  int voff[8];
  int istride, kstride;
  __device__ __forceinline__ void init(const __hip_bfloat16* X, int ld, int r0, int K, int wave, int lane, int valid) {
    if constexpr (!MN) {
      rsrc = make_rsrc(X + (int64_t)r0 * ld, (BM - 1) * ld * 2 + K * 2);
      const int r = lane >> 3, c = (lane & 7) ^ r;
#pragma unroll
      for (int i = 0; i < 8; ++i) voff[i] = (min(32 * i + wave * 8 + r, valid - 1) * ld + c * 8) * 2;
      istride = 0;
      kstride = BK * 2;
    } else {
      rsrc = make_rsrc(X + r0, (K - 1) * ld * 2 + BM * 2);
      const int half = lane >> 5, slot = lane & 31, kr = 2 * wave + half;
      const int c0 = slot ^ tr_swz(kr), cmax = (valid >> 3) - 1;
      voff[0] = (kr * ld + min(c0, cmax) * 8) * 2;
      voff[1] = (kr * ld + min(c0 ^ 8, cmax) * 8) * 2;
      istride = 8 * ld * 2;
      kstride = BK * ld * 2;
    }
  }
  __device__ __forceinline__ void issue(int i, int kt, char* img, int wave) const {
    const uint32_t dst = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)(img + (i * 4 + wave) * 1024);
    const int vo = MN ? voff[i & 1] : voff[i];
    const int so = MN ? i * istride + kt * kstride : kt * kstride;
    asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %3 offen lds"
                 :
                 : "s"(dst), "v"(vo), "s"(rsrc), "s"(so)
                 : "memory", "m0");
  }
};
template <bool MN>
__device__ __forceinline__ bf16x8 read_frag(const char* img, int rc, int kk, int fr, int fq) {
  if constexpr (!MN) {
    const int row = rc + fr;
    return *reinterpret_cast<const bf16x8*>(img + row * 128 + (((kk * 4 + fq) ^ (fr & 7)) << 4));
  } else {
    const int q = fr >> 2, p = fr & 3;
    const int k = kk * 32 + fq * 8 + q;
    const int c = (rc >> 3) + (p >> 1);
    const char* a0 = img + k * 512 + ((c ^ tr_swz(k)) << 4) + 8 * (p & 1);
    const char* a1 = img + (k + 4) * 512 + ((c ^ tr_swz(k + 4)) << 4) + 8 * (p & 1);
    const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(__attribute__((address_space(3))) char*)a0);
    const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(__attribute__((address_space(3))) char*)a1);
    union { struct { s16x4 a, b; } s; bf16x8 f; } u;
    u.s.a = lo;
    u.s.b = hi;
    return u.f;
  }
}
// swapped operands: D = B_frag . A_frag^T = C^T block -> lane (fq, fr) holds C[fr][4 fq + j]
__device__ __forceinline__ void mfma_sw(f32x4& acc, const bf16x8& a, const bf16x8& b) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(b), "v"(a));
}
__device__ __forceinline__ uint32_t pk2(float lo, float hi) {
  union { __hip_bfloat16 h[2]; uint32_t u; } p;
  p.h[0] = __float2bfloat16(lo);
  p.h[1] = __float2bfloat16(hi);
  return p.u;
}
__device__ __forceinline__ void tile_coords(int wg, int nTm, int nTn, int& tm, int& tn) {
  constexpr int G = 8;
  const int per_group = G * nTn, group = wg / per_group, first_m = group * G, gm = min(nTm - first_m, G);
  tm = first_m + (wg % per_group) % gm;
  tn = (wg % per_group) / gm;
}
#define FENCE() __builtin_amdgcn_sched_barrier(0)

template <bool AT, bool BT, int PERSIST>
__global__ __launch_bounds__(NTHR, 1) void g5_kernel(const __hip_bfloat16* __restrict__ A, const __hip_bfloat16* __restrict__ B,
                                                    __hip_bfloat16* __restrict__ C, int M, int N, int K, int lda, int ldb,
                                                    int ldc, uint64_t* st) {
  __shared__ __attribute__((aligned(1024))) char smem[2 * STAGE];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1, fr = lane & 15, fq = lane >> 4;
  uint64_t t0 = 0, r0 = 0;
  if (wave == 0) { t0 = __builtin_amdgcn_s_memtime(); r0 = __builtin_amdgcn_s_memrealtime(); }
  const int nTm = (M + BM - 1) / BM, nTn = (N + BN - 1) / BN, nwg = nTm * nTn;
  const int nk = K / BK;
  constexpr int NB2 = 8, NA = 8;
  Stager<AT> sa;
  Stager<BT> sb;
  f32x4 acc[8][8];
  bf16x8 fa0[8], fb0[8], fa1[8], fb1[8];
  auto read_one = [&](const char* stage, int kk, int r, bf16x8* fa, bf16x8* fb) {
    if (r == 0) fa[0] = read_frag<AT>(stage, wm * 128, kk, fr, fq);
    else if (r <= 8) fb[r - 1] = read_frag<BT>(stage + OP_BYTES, wn * 128 + (r - 1) * 16, kk, fr, fq);
    else fa[r - 8] = read_frag<AT>(stage, wm * 128 + (r - 8) * 16, kk, fr, fq);
  };
  auto glds = [&](int j, int kt, char* stage) {
    if (j < 8) sa.issue(j, kt, stage, wave); else sb.issue(j - 8, kt, stage + OP_BYTES, wave);
  };
  auto setup = [&](int v, int& m0, int& n0) {
    int tm, tn;
    tile_coords(xcd_tile(v, nwg), nTm, nTn, tm, tn);
    m0 = tm * BM;
    n0 = tn * BN;
    sa.init(A, lda, m0, K, wave, lane, min(BM, M - m0));
    sb.init(B, ldb, n0, K, wave, lane, min(BN, N - n0));
  };
  auto prologue = [&]() {
#pragma unroll
    for (int j = 0; j < 16; ++j) glds(j, 0, smem);
#pragma unroll
    for (int j = 0; j < NB2; ++j) glds(j, 1, smem + STAGE);
  };
  auto body = [&](int t, auto cur_c) {
    constexpr int CUR = decltype(cur_c)::value;
    char* const bc = smem + CUR * STAGE;
    char* const bn = smem + (CUR ^ 1) * STAGE;
    const int t1 = min(t + 1, nk - 1), t2 = min(t + 2, nk - 1);
#pragma unroll
    for (int i = 0; i < 64; ++i) {
      mfma_sw(acc[i >> 3][i & 7], fa0[i >> 3], fb0[i & 7]);
      if ((i & 3) == 0) read_one(bc, 1, i >> 2, fa1, fb1);
      if ((i & 3) == 2 && (i >> 2) < NA) glds(NB2 + (i >> 2), t1, bn);
      FENCE();
    }
#pragma unroll
    for (int i = 0; i < 32; ++i) {
      mfma_sw(acc[i >> 3][i & 7], fa1[i >> 3], fb1[i & 7]);
      FENCE();
    }
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    FENCE();
#pragma unroll
    for (int i = 32; i < 64; ++i) {
      mfma_sw(acc[i >> 3][i & 7], fa1[i >> 3], fb1[i & 7]);
      const int s = i - 32;
      if ((s & 1) == 0) read_one(bn, 0, s >> 1, fa0, fb0);
      else if ((s & 3) == 1 && (s >> 2) < NB2) glds(s >> 2, t2, bc);
      FENCE();
    }
  };
  const int stride = PERSIST ? (int)gridDim.x : nwg;
  int v = (int)blockIdx.x, m0, n0;
  setup(v, m0, n0);
  prologue();
  // stores of the previous tile still in flight (PERSIST): they are older than this tile's prologue
  int pending_stores = 0;
  uint64_t tl = 0;
  while (true) {
    if (pending_stores)
      asm volatile("s_waitcnt vmcnt(40)" ::: "memory");  // 8 T1 loads + 32 stores may stay in flight
    else
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NB2) : "memory");
    __builtin_amdgcn_s_barrier();
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int r = 0; r < 16; ++r) read_one(smem, 0, r, fa0, fb0);
    for (int t = 0; t < nk; t += 2) {
      body(t, std::integral_constant<int, 0>{});
      body(t + 1, std::integral_constant<int, 1>{});
    }
#pragma unroll
    for (int m = 0; m < 8; ++m)
#pragma unroll
      for (int n = 0; n < 8; ++n) asm volatile("" : "+a"(acc[m][n]));
    asm volatile("s_nop 15\n\ts_nop 15" ::: "memory");
    // the last K-tile's dummy prefetches landed and every wave finished its last LDS reads
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    const int cm0 = m0, cn0 = n0;
    const int vn = v + stride;
    const bool more = PERSIST && vn < nwg;
    if (more) {
      setup(vn, m0, n0);
      prologue();
    }
    // register epilogue: blocks (n, n+1) -> permlane16_swap -> 16 B of one row per lane
    const int rsel = fq & 1, csel = fq >> 1;
#pragma unroll
    for (int m = 0; m < 8; ++m) {
#pragma unroll
      for (int np = 0; np < 4; ++np) {
        const int n = 2 * np;
        const uint32_t x0 = pk2(acc[m][n][0], acc[m][n][1]), x1 = pk2(acc[m][n][2], acc[m][n][3]);
        const uint32_t y0 = pk2(acc[m][n + 1][0], acc[m][n + 1][1]), y1 = pk2(acc[m][n + 1][2], acc[m][n + 1][3]);
        const auto s0 = __builtin_amdgcn_permlane16_swap(x0, y0, false, false);
        const auto s1 = __builtin_amdgcn_permlane16_swap(x1, y1, false, false);
        const uint4 val = make_uint4(s0[0], s1[0], s0[1], s1[1]);
        const int row = cm0 + wm * 128 + m * 16 + fr, col = cn0 + wn * 128 + (n + rsel) * 16 + csel * 8;
        if (row < M && col < N) *reinterpret_cast<uint4*>(C + (int64_t)row * ldc + col) = val;
        FENCE();  // one block pair at a time: bounded VGPR use beside the next tile's stager state
      }
    }
    if (!more) break;
    v = vn;
    pending_stores = 1;
  }
  if (wave == 0 && lane == 0 && st) {
    const uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    st[blockIdx.x * 4 + 0] = t0;
    st[blockIdx.x * 4 + 1] = t1;
    st[blockIdx.x * 4 + 2] = r0;
    st[blockIdx.x * 4 + 3] = r1;
  }
}
}  // namespace

// layout: 0 = NT (fwd), 1 = NN (dgrad: B [K][N]), 2 = TN (wgrad: A [K][M], B [K][N]).  persist: 0 / 1.
LTA_EXPORT int g5_gemm(int layout, int persist, const void* A, const void* B, void* C, int M, int N, int K, int lda,
                       int ldb, int ldc, int cus, void* st, hipStream_t s) {
  if (K % (2 * BK) || N % 8) return -2;
  const int nwg = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  const int grid = persist ? min(nwg, cus) : nwg;
#define L(AT, BT, P)                                                                                          \
  hipLaunchKernelGGL((g5_kernel<AT, BT, P>), dim3(grid), dim3(NTHR), 0, s, (const __hip_bfloat16*)A,            \
                     (const __hip_bfloat16*)B, (__hip_bfloat16*)C, M, N, K, lda, ldb, ldc, (uint64_t*)st)
  if (layout == 0) { if (persist) L(false, false, 1); else L(false, false, 0); }
  else if (layout == 1) { if (persist) L(false, true, 1); else L(false, true, 0); }
  else { if (persist) L(true, true, 1); else L(true, true, 0); }
#undef L
  return (int)hipGetLastError();
}
