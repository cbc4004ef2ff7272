// K3 flash-attention forward, v4 (D = 128, bf16/fp16, causal or full, GQA, any [B,H,T] strides of
// Q / K / V / O with the head dim contiguous; no mask / dropout — those take v1).
// Replaces the reference's cuDNN / aten-flash / FA3 SDPA forward (thunder/executors/cudnn_sdpa.py,
// sdpaex.py, fa3ex.py) on the plain causal training path.
//
// Structure (cdna_hip_programming.md §5.5 T2/T10/T12/T13, §5.7; MI355X_MICROARCH.md §LDS, constants):
//  * one workgroup per CU: 4 waves (one per SIMD, 512-register budget), 64 query rows per wave in
//    two 32-row blocks A and B, so every K fragment read from LDS feeds the MFMAs of a 32-query
//    block and every transposed V read a 32-query PV step;
//  * K / V tiles (64 keys) arrive by LDS-DMA (buffer_load ... lds, no staging VGPRs) into a 4-slot
//    ring two tiles deep: tile t+2 streams in during tile t and the end-of-tile wait is a counted
//    vmcnt(8) for tile t+1 (issued a whole tile earlier: a one-deep ring exposed the DMA latency and
//    ran at half speed), tile t-1's V is still read in tile t (see the skew below).  Images are unpadded 256-B rows (glds writes lane-linearly) with the swizzle applied
//    to the per-lane SOURCE address: K chunk c of row R at slot c ^ (R & 15) (conflict-free
//    ds_read_b128 row reads), V chunk c at slot c ^ ((R & 3) << 2) (conflict-free
//    ds_read_b64_tr_b16 transposed reads);
//  * swapped S^T = K Q^T (each lane owns one query: the softmax row is lane-local + one lane^32
//    partner), O^T += V^T P^T with P^T taken straight from the S accumulator (bf16 pack, no LDS);
//    S in VGPRs (intrinsic MFMAs, this file builds with -amdgpu-mfma-vgpr-form=1), O in the AGPR
//    file (inline-asm MFMAs), Q fragments in VGPRs for the whole kernel;
//  * skewed two-block pipeline, four 16-MFMA phases per tile, each phase's VALU work belonging to
//    the OTHER block (so it runs beside the MFMAs instead of after them):
//        Ph1: QK_A(t)    | finish-softmax B(t-1), second key half; K DMA of tile t+1
//        Ph2: PV_B(t-1)  | start A(t) (row max, rescale decision), finish A(t) first half; V DMA
//        Ph3: QK_B(t)    | finish A(t) second half
//        Ph4: PV_A(t)    | start B(t), finish B(t) first half
//    (B's PV of the wave's last tile drains after the loop.)  One barrier per tile;
//  * scale folded into one FMA per score (p = exp2(s c - m)), row max as a max3 tree with the pair
//    max only on a rescale, O rescale deferred while no row max grows by more than THR log2 units
//    (T13; THR = 0 is the exact online softmax), row sums kept per lane and paired once at the end;
//  * causal: a wave's tiles end at its diagonal tile (64-row waves on 64-key tiles), so only that
//    tile is masked; the workgroup keeps staging for its later waves.
#include <type_traits>

#include "attention.h"
#include "fp8_cvt.h"

using namespace lta;
using namespace lta::attn;

namespace {

constexpr int kD = 128, kBN = 64, kNW = 4, kRows = 64, kBM = kNW * kRows, kThreads = 64 * kNW;
constexpr int kTileB = kBN * kD * 2;  // bytes of one K or V tile image (16 KiB)
constexpr int kNBuf = 4;  // slots: t-1 (V still read), t, and the two tiles in flight
constexpr int kVBase = kNBuf * kTileB;  // V images follow the K images
// epilogue staging per wave: 64 bf16 rows of O (256 B) + their e4m3 copies (128 B)
constexpr int kStageB = 64 * 256 + 64 * 128;
static_assert(kNW * kStageB <= 2 * kNBuf * kTileB, "epilogue staging fits in the K / V ring");

typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

__device__ __forceinline__ i32x4 make_rsrc(const void* base, uint32_t bytes) {
  const uint64_t a = (uint64_t)(uintptr_t)base;
  return i32x4{(int)(uint32_t)a, (int)((uint32_t)(a >> 32) & 0xffffu), (int)bytes, 0x00020000};
}

// one 1-KiB LDS-DMA piece: lane l's 16 bytes at rsrc + voff land at LDS byte dst + 16 l
__device__ __forceinline__ void dma16(uint32_t dst, int voff, i32x4 rsrc) {
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds"
               :
               : "s"(dst), "v"(voff), "s"(rsrc)
               : "memory", "m0");
}

__device__ __forceinline__ float max3f(float a, float b, float c) {
  float r;
  asm("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}
// swap(v, v): element 0 carries lanes 32..63 into lanes 0..31, element 1 lanes 0..31 into 32..63,
// so combining both elements pairs lane l with l ^ 32
__device__ __forceinline__ float pair_max(float v) {
  const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return max3f(v, __uint_as_float(sw[0]), __uint_as_float(sw[1]));
}
__device__ __forceinline__ float pair_sum(float v) {
  const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(sw[0]) + __uint_as_float(sw[1]);
}

// O^T += V^T P^T into the accumulator file.  P (VALU-packed) is always written >= 3 MFMAs before
// the MFMA that reads it (phase layout above), so no wait state is padded here.
__device__ __forceinline__ void pv_mfma(f32x16& acc, const bf16x8& a, const bf16x8& b) {
  asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
}
__device__ __forceinline__ void pv_mfma(f32x16& acc, const f16x8& a, const f16x8& b) {
  asm volatile("v_mfma_f32_32x32x16_f16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
}

// S^T (+)= K Q^T with the Q fragment read from the AGPR file (Q stays there for the whole kernel,
// leaving the 256 VGPRs to S, P, fragments and addresses).  hipcc does not see these MFMAs, so the
// first VALU read of a finished S tile is preceded by an explicit wait-state pad (s_pad_xdl).
__device__ __forceinline__ void qk_mfma(f32x16& acc, const bf16x8& k, const bf16x8& q) {
  asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+v"(acc) : "v"(k), "a"(q));
}
__device__ __forceinline__ void qk_mfma0(f32x16& acc, const bf16x8& k, const bf16x8& q) {
  asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, 0" : "=&v"(acc) : "v"(k), "a"(q));
}
__device__ __forceinline__ void qk_mfma(f32x16& acc, const f16x8& k, const f16x8& q) {
  asm volatile("v_mfma_f32_32x32x16_f16 %0, %1, %2, %0" : "+v"(acc) : "v"(k), "a"(q));
}
__device__ __forceinline__ void qk_mfma0(f32x16& acc, const f16x8& k, const f16x8& q) {
  asm volatile("v_mfma_f32_32x32x16_f16 %0, %1, %2, 0" : "=&v"(acc) : "v"(k), "a"(q));
}
// XDL (16-pass) VGPR write -> VALU read: >= 19 wait states on gfx950 (needed after the asm QK
// variant only; the intrinsic QK MFMAs are padded by hipcc itself)
__device__ __forceinline__ void s_pad_xdl(f32x16& s0, f32x16& s1) {
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 4" : "+v"(s0), "+v"(s1));
}
// the S tile as an operand of an empty asm: no VALU read of it is scheduled above this point
__device__ __forceinline__ void pin2(f32x16& s0, f32x16& s1) {
#ifdef LTA_QK_ASM
  s_pad_xdl(s0, s1);
#else
  asm volatile("" : "+v"(s0), "+v"(s1));
#endif
}
// hipcc moves pure VALU work across sched_barrier at the IR level; an empty volatile asm on the
// value pins it to this point of the (asm-volatile) MFMA stream
template <typename V>
__device__ __forceinline__ void pin(V& v) {
  asm volatile("" : "+v"(v));
}

// acc *= a for an accumulator that lives in the AGPR file: element-wise asm keeps hipcc from
// pulling the whole O tile into VGPRs around every MFMA (which a plain C++ multiply provokes)
__device__ __forceinline__ void scale_acc(f32x16& acc, float a) {
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    float e = acc[i], tmp;
    asm volatile("v_accvgpr_read_b32 %1, %0\n\tv_mul_f32 %1, %1, %2\n\tv_accvgpr_write_b32 %0, %1"
                 : "+a"(e), "=&v"(tmp)
                 : "v"(a));
    acc[i] = e;
  }
}

#define LTA_FENCE() __builtin_amdgcn_sched_barrier(0)
// LDS fragment-read lookahead (MFMAs) of the QK (K rows) and PV (V^T transposed) phases
#ifndef LTA_KLA
#define LTA_KLA 5
#endif
#ifndef LTA_VLA
#define LTA_VLA 3
#endif

template <int N>
using IC = std::integral_constant<int, N>;

// ABL (measurement builds only, impl 11..15): 1 no LDS-DMA in the loop, 2 no softmax-finish VALU,
// 3 no per-tile barrier, 4 no softmax start (results are wrong; timing only), 5 s_memtime stamps of
// workgroup (0, 0) at every phase boundary of its first 64 tiles, written over LSE (diagnostic)
// Q8: O also leaves as e4m3 into q8.q (same element layout as O; AttnQ8 in attention.h)
template <typename T, bool CAUSAL, int THR, int ABL = 0, bool Q8 = false>
__global__ __launch_bounds__(kThreads, 1) void attn_fwd_v4_kernel(const T* __restrict__ Q, const T* __restrict__ K,
                                                                  const T* __restrict__ V, T* __restrict__ O,
                                                                  float* __restrict__ LSE, int Hq, int Hkv, int Tq,
                                                                  int Sk, float c, int64_t so_b, int64_t so_h,
                                                                  int64_t so_t, QKVStrides sx, AttnQ8 q8 = {}) {
  using F = typename Frag<T>::type;
  constexpr int kStampBase = 2 * kNBuf * kTileB;
  __shared__ __attribute__((aligned(1024))) char smem[2 * kNBuf * kTileB + (ABL == 5 ? 4 * 64 * 6 * 8 : 0)];  // the only LDS object

  const int n_qt = (Tq + kBM - 1) / kBM;
  // causal: workgroup y runs query tile n_qt-1-y (heavy) then tile y (light), so every workgroup
  // carries the same number of key tiles and the grid is one balanced wave of workgroups
  const int qt_heavy = n_qt - 1 - (int)blockIdx.y, qt_light = (int)blockIdx.y;
  const int npass = (CAUSAL && qt_light < qt_heavy) ? 2 : 1;
  const int bh = blockIdx.x;                  // x-fastest: all query blocks of a head share an XCD
  const int b = bh / Hq, hq = bh % Hq;
  const int hk = hq / (Hq / Hkv);
  const T* Qb = Q + b * sx.qb + hq * sx.qh;
  const char* Kb = reinterpret_cast<const char*>(K + b * sx.kb + hk * sx.kh);
  const char* Vb = reinterpret_cast<const char*>(V + b * sx.vb + hk * sx.vh);
  const int kst = (int)sx.kt * 2, vst = (int)sx.vt * 2;  // key-row strides in bytes

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 31, h = lane >> 5, g = lane >> 4, l16 = lane & 15;
  [[maybe_unused]] float q8m = 0.f;  // Q8: this lane's max |bf16(O)|
  for (int pass = 0; pass < npass; ++pass) {
  const int qt = pass == 0 ? qt_heavy : qt_light;
  const int q0 = qt * kBM + wave * kRows;  // block X: queries q0 + 32 X + r

  int n_tiles = (Sk + kBN - 1) / kBN;
  if (CAUSAL) n_tiles = min(n_tiles, (min(qt * kBM + kBM, Tq) + kBN - 1) / kBN);
  int nw = n_tiles;  // this wave's tiles [0, nw); only tile nw-1 can need a mask
  if (CAUSAL) nw = min(n_tiles, min(q0 + kRows - 1, Tq - 1) / kBN + 1);
  const bool last_masked = (nw * kBN > Sk) || (CAUSAL && (nw - 1) * kBN + kBN - 1 > q0);

  // ---- LDS-DMA: piece j (0..3 K, 4..7 V) of a tile; instruction j of wave w fills rows
  //      16 (j & 3) + 4 w + (lane >> 4) of the image, slot lane & 15 ------------------------------
  const int drow = 4 * wave + (lane >> 4);
  const int slot = lane & 15;
  const int kch = slot ^ drow;                // K: chunk at slot s of row R is s ^ (R & 15)
  const int vch = slot ^ ((drow & 3) << 2);   // V: chunk at slot s of row R is s ^ ((R & 3) << 2)
  const uint32_t lds0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)smem;
  auto dma = [&](int j, int t) {
    if (ABL == 1 && t > 0) return;
    const int nrem = Sk - t * kBN;  // >= 1
    const int i = j & 3;
    const int row = min(16 * i + drow, nrem - 1);  // clamped rows are real keys; the mask drops them
    const uint32_t dst = lds0 + (j < 4 ? 0 : kVBase) + (t % kNBuf) * kTileB + (4 * i + wave) * 1024;
    if (j < 4)
      dma16(dst, row * kst + kch * 16, make_rsrc(Kb + (int64_t)t * kBN * kst, (uint32_t)nrem * (uint32_t)kst));
    else
      dma16(dst, row * vst + vch * 16, make_rsrc(Vb + (int64_t)t * kBN * vst, (uint32_t)nrem * (uint32_t)vst));
  };

  // ---- fragments ---------------------------------------------------------------------------------
  F qf[2][8];  // B operand of S^T = K Q^T: Q[q0 + 32 X + r][16 s + 8 h .. +7]
#pragma unroll
  for (int x = 0; x < 2; ++x) {
    const int qrow = min(q0 + 32 * x + r, Tq - 1);
#pragma unroll
    for (int s = 0; s < 8; ++s) qf[x][s] = load_frag<F>(Qb + (int64_t)qrow * sx.qt + 16 * s + 8 * h);
  }
  // consume the Q loads here: hipcc then counts them as retired and puts no vmcnt wait for them
  // into the main loop, where the hardware counter also holds the LDS-DMA pieces (a stale
  // vmcnt(N) there would wait for the next tile's DMA in the middle of the MFMA stream)
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int s = 0; s < 8; ++s) pin(qf[x][s]);
  // K fragment (s, kt): row kt * 32 + r, chunk 2 s + h
  auto kfrag = [&](int kimg, int s, int kt) -> F {
    return *reinterpret_cast<const F*>(smem + kimg + (kt * 32 + r) * 256 + (((2 * s + h) ^ (r & 15)) << 4));
  };
  // V^T fragment (dt, kt, s): rows kt*32 + 16 s + 4 h + q (+8), columns dt*32 + 16 (g & 1) + 4 p
  const int vq = l16 >> 2, vp = l16 & 3;
  auto vfrag = [&](int vimg, int dt, int kt, int s) -> F {
    const int row = kt * 32 + 16 * s + 4 * h + vq;
    const int ch = 4 * (dt ^ vq) + 2 * (g & 1) + (vp >> 1);
    const char* a0 = smem + vimg + row * 256 + (ch << 4) + 8 * (vp & 1);
    const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(__attribute__((address_space(3))) char*)a0);
    const s16x4 hi =
        __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(__attribute__((address_space(3))) char*)(a0 + 2048));
    union {
      struct {
        s16x4 a, b;
      } s;
      F f;
    } u;
    u.s.a = lo;
    u.s.b = hi;
    return u.f;
  };

  // ---- state -------------------------------------------------------------------------------------
  f32x16 oacc[2][4];
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int dt = 0; dt < 4; ++dt)
#pragma unroll
      for (int i = 0; i < 16; ++i) oacc[x][dt][i] = 0.f;
  f32x16 sacc[2][2];
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
      for (int i = 0; i < 16; ++i) sacc[x][kt][i] = 0.f;
  // the pipeline enters tile 0 mid-way through B(-1) (a non-existent tile): its P and row sums are
  // finite garbage (P = 1), the PV against the zeroed V slot adds 0 to O_B, and start(B, 0) scales
  // the row sums and O_B by exp2(-inf) = 0 (the first start always rescales: m = -inf)
  F pf[2][2][2];
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
      for (int s = 0; s < 2; ++s) pf[x][kt][s] = F{};  // B(-1): 0 x (zeroed V) must not see NaN bits
  float m[2] = {-INFINITY, -INFINITY};  // running max (log2 units) per block
  float nm[2] = {0.f, 0.f};             // -m once a tile has been started (0 before: see sacc init)
  float lp[2][2] = {{0.f, 0.f}, {0.f, 0.f}};  // per-lane partial row sums (two chains per block)

  // ---- softmax pieces ------------------------------------------------------------------------------
  // start: mask (the wave's last tile), row max, rescale decision (+ O / l rescale when taken)
  auto start = [&](auto xc, auto mc, int t) {
    constexpr int X = decltype(xc)::value;
    if constexpr (ABL == 4) return;
    if constexpr (decltype(mc)::value) {  // the wave's last tile (peeled: no mask code in the loop)
      const int qi = q0 + 32 * X + r;
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int key = t * kBN + kt * 32 + acc_row(i, h);
          if (key >= Sk || (CAUSAL && key > qi)) sacc[X][kt][i] = -INFINITY;
        }
    }
    float mv[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const f32x16& s = sacc[X][q >> 1];
      const int o = 8 * (q & 1);
      float v = max3f(s[o], s[o + 1], s[o + 2]);
      v = max3f(v, s[o + 3], s[o + 4]);
      v = max3f(v, s[o + 5], s[o + 6]);
      mv[q] = max3f(v, s[o + 7], s[o + 7]);
    }
    const float mx = max3f(max3f(mv[0], mv[1], mv[2]), mv[3], mv[3]) * c;  // c > 0 commutes with max
    const bool grow = !(mx - m[X] <= (float)THR);  // true at m = -inf
    if (__builtin_amdgcn_ballot_w64(grow) != 0) {  // wave-uniform
      const float mn = fmaxf(m[X], pair_max(mx));
      const float mu = (mn == -INFINITY) ? 0.f : mn;
      const float alpha = __builtin_amdgcn_exp2f(m[X] - mu);
      m[X] = mu;
      lp[X][0] *= alpha;
      lp[X][1] *= alpha;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) scale_acc(oacc[X][dt], alpha);  // the block's last PV is long complete
    }
    nm[X] = -m[X];
  };
  // finish one score: p = exp2(s c - m), row-sum chain, bf16 pack every 8 scores
  // finish, as a two-stage pipeline over the slots so no result is read by the very next VALU
  // (an exp result or an asm-pinned value read at distance 0 costs an s_nop each):
  //   fstep(e): p_e = exp2(x_e c - m), pinned; x_{e+1} pinned for the next slot's fstep
  //   astep(e): row-sum chain += p_e (one slot later); bf16 pack after p_7 / p_15
  auto fstep = [&](auto xc, int kt, int e) {
    constexpr int X = decltype(xc)::value;
    if constexpr (ABL == 2) return;
    float x = sacc[X][kt][e];
    if (e == 0) pin(x);  // later elements were pinned one slot earlier
    float p = __builtin_amdgcn_exp2f(__builtin_fmaf(x, c, nm[X]));
    pin(p);
    sacc[X][kt][e] = p;
    if (e < 15) {
      float xn = sacc[X][kt][e + 1];
      pin(xn);
      sacc[X][kt][e + 1] = xn;
    }
  };
  auto astep = [&](auto xc, int kt, int e) {
    constexpr int X = decltype(xc)::value;
    if constexpr (ABL == 2) return;
    float ls = lp[X][e & 1] + sacc[X][kt][e];
    pin(ls);
    lp[X][e & 1] = ls;
    if (e == 7) {
      pack_frag(pf[X][kt][0], sacc[X][kt], 0);
      pin(pf[X][kt][0]);
    }
    if (e == 15) {
      pack_frag(pf[X][kt][1], sacc[X][kt], 1);
      pin(pf[X][kt][1]);
    }
  };
  // slot i of a phase whose run is (X, kt) and whose previous run was (XP, KP): the previous run's
  // last element finishes in slots 0 / 1, this run's elements e = i - 1 start from slot 1
  auto fin = [&](auto xc, int kt, auto xpc, int kp, int i, auto&& at_slot1) {
    if (i == 0) {
      fstep(xpc, kp, 15);
      astep(xpc, kp, 14);
    } else if (i == 1) {
      astep(xpc, kp, 15);
      at_slot1();
      fstep(xc, kt, 0);
    } else {
      fstep(xc, kt, i - 1);
      astep(xc, kt, i - 2);
    }
  };
  auto none = [&]() {};

  // ---- the four phase kinds ------------------------------------------------------------------------
  // QK of block X on a K image; slot i = MFMA (s = i >> 1, kt = i & 1); filler(i) after the MFMA
  auto qk_phase = [&](auto xc, int kimg, auto&& filler) {
    constexpr int X = decltype(xc)::value;
    constexpr int L = LTA_KLA;  // fragment reads run L MFMAs ahead
    F kf[L + 1];
#pragma unroll
    for (int i = 0; i < L; ++i) kf[i] = kfrag(kimg, i >> 1, i & 1);
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      if (i + L < 16) kf[(i + L) % (L + 1)] = kfrag(kimg, (i + L) >> 1, (i + L) & 1);
#ifdef LTA_QK_ASM
      if (i < 2)
        qk_mfma0(sacc[X][i & 1], kf[i % (L + 1)], qf[X][i >> 1]);
      else
        qk_mfma(sacc[X][i & 1], kf[i % (L + 1)], qf[X][i >> 1]);
#else
      const f32x16 zero = {};
      sacc[X][i & 1] = mfma(kf[i % (L + 1)], qf[X][i >> 1], i < 2 ? zero : sacc[X][i & 1]);
#endif
      filler(i);
      LTA_FENCE();
    }
  };
  // PV of block X on a V image; slot i = MFMA (dt = i >> 2, kt = (i >> 1) & 1, s = i & 1)
  auto pv_phase = [&](auto xc, int vimg, auto&& filler) {
    constexpr int X = decltype(xc)::value;
    constexpr int L = LTA_VLA;
    F vf[L + 1];
#pragma unroll
    for (int i = 0; i < L; ++i) vf[i] = vfrag(vimg, i >> 2, (i >> 1) & 1, i & 1);
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      if (i + L < 16) vf[(i + L) % (L + 1)] = vfrag(vimg, (i + L) >> 2, ((i + L) >> 1) & 1, (i + L) & 1);
      pv_mfma(oacc[X][i >> 2], vf[i % (L + 1)], pf[X][(i >> 1) & 1][i & 1]);
      filler(i);
      LTA_FENCE();
    }
  };
  auto valu_phase = [&](auto&& filler) {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      filler(i);
      LTA_FENCE();
    }
  };
  auto nothing = [&](int) {};

  const int last = n_tiles - 1;
  // ---- prologue: tiles 0 and 1 in flight; the V image of slot 3 zeroed (the PV of the
  //      non-existent tile B(-1) reads it against P = 0) ----------------------------------------------
#pragma unroll
  for (int j = 0; j < 8; ++j) dma(j, 0);
#pragma unroll
  for (int j = 0; j < 8; ++j) dma(j, min(1, last));
#pragma unroll
  for (int i = 0; i < kTileB / (kThreads * 16); ++i)
    *reinterpret_cast<uint4*>(smem + kVBase + 3 * kTileB + (i * kThreads + tid) * 16) = make_uint4(0, 0, 0, 0);
  asm volatile("s_waitcnt vmcnt(8) lgkmcnt(0)" ::: "memory");  // tile 0 landed (this wave's pieces)
  __builtin_amdgcn_s_barrier();

  // one barrier per tile for every wave: its unmasked tiles, its masked last tile (peeled, so the
  // mask code cannot be hoisted into the main loop), then staging-only tiles for the later waves
  auto stamp = [&](int t, int k) {
    if constexpr (ABL == 5) {
      if (blockIdx.x == 0 && blockIdx.y == 0 && pass == 0 && t < 64) {
        const uint64_t ts = __builtin_amdgcn_s_memtime();
        if (lane == 0) *reinterpret_cast<uint64_t*>(smem + kStampBase + ((wave * 64 + t) * 6 + k) * 8) = ts;
      }
    }
  };
  auto tile = [&](int t, auto mc) {
    stamp(t, 0);
    const int t1 = min(t + 2, last);  // two tiles ahead; past the end: re-stage the last tile into a free slot
    const int kimg = (t % kNBuf) * kTileB;
    const int vimg = kVBase + (t % kNBuf) * kTileB;
    const int vprev = kVBase + ((t + kNBuf - 1) % kNBuf) * kTileB;
    // runs: Ph1 B(t-1) kt1, Ph2 A kt0, Ph3 A kt1, Ph4 B kt0 (each one slot late, see fin)
    qk_phase(IC<0>{}, kimg, [&](int i) {
      fin(IC<1>{}, 1, IC<1>{}, 0, i, none);
      if ((i & 3) == 0) dma(i >> 2, t1);
    });
    stamp(t, 1);
    pv_phase(IC<1>{}, vprev, [&](int i) {
      fin(IC<0>{}, 0, IC<1>{}, 1, i, [&]() {
        pin2(sacc[0][0], sacc[0][1]);
        start(IC<0>{}, mc, t);
      });
      if ((i & 3) == 2) dma(4 + (i >> 2), t1);
    });
    stamp(t, 2);
    qk_phase(IC<1>{}, kimg, [&](int i) { fin(IC<0>{}, 1, IC<0>{}, 0, i, none); });
    stamp(t, 3);
    pv_phase(IC<0>{}, vimg, [&](int i) {
      fin(IC<1>{}, 0, IC<0>{}, 1, i, [&]() {
        pin2(sacc[1][0], sacc[1][1]);
        start(IC<1>{}, mc, t);
      });
    });
    stamp(t, 4);
    if constexpr (ABL != 3) {
      asm volatile("s_waitcnt vmcnt(8) lgkmcnt(0)" ::: "memory");  // tile t+1 landed (this wave's part)
      __builtin_amdgcn_s_barrier();                                 // ... and everyone's; tile t-2 free
    }
    stamp(t, 5);
  };
  const int nplain = last_masked ? nw - 1 : nw;
  int t = 0;
  for (; t < nplain; ++t) tile(t, IC<0>{});
  if (last_masked) tile(t++, IC<1>{});
  for (; t < n_tiles; ++t) {
#pragma unroll
    for (int j = 0; j < 8; ++j) dma(j, min(t + 2, last));
    if (t == nw) {  // drain: B's last tile (its V image is slot (nw - 1) % 4)
      valu_phase([&](int i) { fin(IC<1>{}, 1, IC<1>{}, 0, i, none); });
      fstep(IC<1>{}, 1, 15);
      astep(IC<1>{}, 1, 14);
      astep(IC<1>{}, 1, 15);
      pv_phase(IC<1>{}, kVBase + ((t + kNBuf - 1) % kNBuf) * kTileB, nothing);
    }
    asm volatile("s_waitcnt vmcnt(8) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  }
  // no LDS-DMA may still be writing when the workgroup's LDS is handed to the next workgroup
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (nw == n_tiles) {
    valu_phase([&](int i) { fin(IC<1>{}, 1, IC<1>{}, 0, i, none); });
    fstep(IC<1>{}, 1, 15);
    astep(IC<1>{}, 1, 14);
    astep(IC<1>{}, 1, 15);
    pv_phase(IC<1>{}, kVBase + (last % kNBuf) * kTileB, nothing);
  }

  // the last asm MFMAs' results must be complete before any other instruction reads them
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) asm volatile("" : "+a"(oacc[x][dt]));
  asm volatile("s_nop 15\n\ts_nop 15\n\ts_nop 15" ::: "memory");

  // ---- epilogue: O = O^T / l ; LSE -----------------------------------------------------------------
  if constexpr (!Q8) {
#pragma unroll
  for (int x = 0; x < 2; ++x) {
    const float l = pair_sum(lp[x][0] + lp[x][1]);
    const int qi = q0 + 32 * x + r;
    if (qi >= Tq) continue;
    const float inv = (l > 0.f) ? 1.f / l : 0.f;
    T* orow = O + b * so_b + hq * so_h + qi * so_t;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
#pragma unroll
      for (int a = 0; a < 4; ++a) {
        const int d = dt * 32 + 8 * a + 4 * h;
        union {
          T v[4];
          uint2 u;
        } pk;
#pragma unroll
        for (int e = 0; e < 4; ++e) pk.v[e] = from_f32<T>(oacc[x][dt][4 * a + e] * inv);
        *reinterpret_cast<uint2*>(orow + d) = pk.u;
      }
    }
    if (h == 0 && LSE != nullptr)
      LSE[((int64_t)b * Hq + hq) * Tq + qi] = (l > 0.f) ? (m[x] + log2f(l)) * 0.69314718055994530942f : -INFINITY;
  }
  } else {
  // Q8 (O also as e4m3): a lane holds 4-element pieces of one query row, so direct stores would be 8 B
  // and 4 B at a row stride (32-64 lines per store instruction, issue-bound: cdna_hip_programming.md
  // T21; measured +0.6 ms per 7B step for the e4m3 copy).  Each wave stages its 64 rows in LDS instead
  // (the K / V ring is free now; 16-B chunks XOR-swizzled by row) and stores whole rows with
  // row-contiguous 16-B stores.  (The same staging for the plain bf16 output measured 1 % slower than
  // the direct stores above: scripts/attn_epi_ab.py.)
  [[maybe_unused]] float qs = 0.f;
  if constexpr (Q8) qs = q8.fmax / fmaxf(*q8.amax_in, 1e-12f);
  __syncthreads();  // every wave's last K / V reads are done before the ring is overwritten
  char* const ob = smem + wave * kStageB;
#pragma unroll
  for (int x = 0; x < 2; ++x) {
    const float l = pair_sum(lp[x][0] + lp[x][1]);
    const int row = 32 * x + r, qi = q0 + row;
    const float inv = (l > 0.f) ? 1.f / l : 0.f;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
#pragma unroll
      for (int a = 0; a < 4; ++a) {
        union {
          T v[4];
          uint2 u;
        } pk;
#pragma unroll
        for (int e = 0; e < 4; ++e) pk.v[e] = from_f32<T>(oacc[x][dt][4 * a + e] * inv);
        // bytes 64 dt + 16 a + 8 h of the 256-B row: chunk 4 dt + a, half h
        *reinterpret_cast<uint2*>(ob + row * 256 + (((4 * dt + a) ^ (row & 15)) << 4) + 8 * h) = pk.u;
        if constexpr (Q8) {
          float f[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            f[e] = to_f32(pk.v[e]);  // the bf16 O the unfused cast would read
            if (qi < Tq) q8m = fmaxf(q8m, fabsf(f[e]));
          }
          // bytes 32 dt + 8 a + 4 h of the 128-B e4m3 row: chunk 2 dt + a / 2
          *reinterpret_cast<uint32_t*>(ob + 64 * 256 + row * 128 + (((2 * dt + (a >> 1)) ^ (row & 7)) << 4) +
                                       8 * (a & 1) + 4 * h) = cvt4<false>(f[0] * qs, f[1] * qs, f[2] * qs, f[3] * qs);
        }
      }
    }
    if (h == 0 && LSE != nullptr && qi < Tq)
      LSE[((int64_t)b * Hq + hq) * Tq + qi] = (l > 0.f) ? (m[x] + log2f(l)) * 0.69314718055994530942f : -INFINITY;
  }
  __syncthreads();  // the wave's image is complete (other lanes' writes) before its rows are read back
  {
    T* const obase = O + b * so_b + hq * so_h;
#pragma unroll
    for (int it = 0; it < 16; ++it) {  // 64 rows x 16 chunks of 16 B: 4 rows per instruction
      const int row = 4 * it + (lane >> 4), c = lane & 15, qi = q0 + row;
      const uint4 v = *reinterpret_cast<const uint4*>(ob + row * 256 + ((c ^ (row & 15)) << 4));
      if (qi < Tq) *reinterpret_cast<uint4*>(obase + qi * so_t + 8 * c) = v;
    }
    if constexpr (Q8) {
      uint8_t* const qbase = q8.q + b * so_b + hq * so_h;
#pragma unroll
      for (int it = 0; it < 8; ++it) {  // 64 rows x 8 chunks: 8 rows per instruction
        const int row = 8 * it + (lane >> 3), c = lane & 7, qi = q0 + row;
        const uint4 v = *reinterpret_cast<const uint4*>(ob + 64 * 256 + row * 128 + ((c ^ (row & 7)) << 4));
        if (qi < Tq) *reinterpret_cast<uint4*>(qbase + qi * so_t + 16 * c) = v;
      }
    }
  }
  }  // Q8
  __builtin_amdgcn_s_barrier();  // every wave's LDS reads of this pass precede the next pass's DMA
  }  // pass
  if constexpr (Q8) {
    // after the last pass's barrier the LDS image is free: its first words take the per-wave maxima
    if (blockIdx.x == 0 && blockIdx.y == 0 && tid == 0 && q8.scale_out != nullptr)
      *q8.scale_out = q8.fmax / fmaxf(*q8.amax_in, 1e-12f);
    if (q8.amax_out != nullptr) fp8_amax_out<kNW>(q8m, q8.amax_out, reinterpret_cast<float*>(smem));
  }
  if constexpr (ABL == 5) {
    if (blockIdx.x == 0 && blockIdx.y == 0) {
      uint64_t* dst = reinterpret_cast<uint64_t*>(LSE) + wave * 64 * 6;
      for (int i = lane; i < 64 * 6; i += 64)
        dst[i] = *reinterpret_cast<const uint64_t*>(smem + kStampBase + (wave * 64 * 6 + i) * 8);
    }
  }
}

template <typename T>
int launch(const void* q, const void* k, const void* v, void* o, void* lse, int B, int Hq, int Hkv, int Tq, int Sk,
           float scale, int causal, const int64_t* so, const QKVStrides& sx, int thr, int abl, hipStream_t s,
           const AttnQ8* q8 = nullptr) {
  const float c = scale * 1.44269504088896340736f;
  const int n_qt = (Tq + kBM - 1) / kBM;
  dim3 grid(B * Hq, causal ? (n_qt + 1) / 2 : n_qt), block(kThreads);
  const int64_t sb = so ? so[0] : (int64_t)Hq * Tq * kD, sh = so ? so[1] : (int64_t)Tq * kD, st = so ? so[2] : kD;
  if (q8 != nullptr) {
    // the Q8 epilogue stores whole rows in 16-B pieces (the e4m3 copy: same element offsets)
    if ((uintptr_t)o % 16 || sb % 16 || sh % 16 || st % 16) return -1;  // e4m3 side output: bf16, deferred rescale (the production configuration) only
    if constexpr (!std::is_same<T, __hip_bfloat16>::value) {
      return -1;
    } else {
      if (!thr || abl || ((uintptr_t)q8->q % 16)) return -1;
      if (causal)
        hipLaunchKernelGGL((attn_fwd_v4_kernel<T, true, 8, 0, true>), grid, block, 0, s, (const T*)q, (const T*)k,
                           (const T*)v, (T*)o, (float*)lse, Hq, Hkv, Tq, Sk, c, sb, sh, st, sx, *q8);
      else
        hipLaunchKernelGGL((attn_fwd_v4_kernel<T, false, 8, 0, true>), grid, block, 0, s, (const T*)q, (const T*)k,
                           (const T*)v, (T*)o, (float*)lse, Hq, Hkv, Tq, Sk, c, sb, sh, st, sx, *q8);
      return (int)hipGetLastError();
    }
  }
#ifdef LTA_V4_ONE
#define LTA_V4(CA, TH) if (CA && TH) hipLaunchKernelGGL((attn_fwd_v4_kernel<T, true, 8>), grid, block, 0, s, (const T*)q, (const T*)k, (const T*)v, (T*)o, (float*)lse, Hq, Hkv, Tq, Sk, c, sb, sh, st, sx)
#else
#define LTA_V4(CA, TH)                                                                                            \
  hipLaunchKernelGGL((attn_fwd_v4_kernel<T, CA, TH>), grid, block, 0, s, (const T*)q, (const T*)k, (const T*)v, \
                     (T*)o, (float*)lse, Hq, Hkv, Tq, Sk, c, sb, sh, st, sx)
#endif
#ifdef LTA_ATTN_DIAG  // measurement builds (scripts/attn_v4_ablate.py, attn_v4_stamps.py)
  if (abl) {
#define LTA_V4A(A)                                                                                                   \
  if (causal)                                                                                                        \
    hipLaunchKernelGGL((attn_fwd_v4_kernel<T, true, 8, A>), grid, block, 0, s, (const T*)q, (const T*)k, (const T*)v, \
                       (T*)o, (float*)lse, Hq, Hkv, Tq, Sk, c, sb, sh, st, sx);                                    \
  else                                                                                                               \
    hipLaunchKernelGGL((attn_fwd_v4_kernel<T, false, 8, A>), grid, block, 0, s, (const T*)q, (const T*)k,            \
                       (const T*)v, (T*)o, (float*)lse, Hq, Hkv, Tq, Sk, c, sb, sh, st, sx)
    if (abl == 1) LTA_V4A(1);
    if (abl == 2) LTA_V4A(2);
    if (abl == 3) LTA_V4A(3);
    if (abl == 4) LTA_V4A(4);
    if (abl == 5) LTA_V4A(5);
#undef LTA_V4A
    return (int)hipGetLastError();
  }
#else
  if (abl) return -1;
#endif
  if (causal) {
    if (thr) LTA_V4(true, 8); else LTA_V4(true, 0);
  } else {
    if (thr) LTA_V4(false, 8); else LTA_V4(false, 0);
  }
#undef LTA_V4
  return (int)hipGetLastError();
}

}  // namespace

int lta::attn::attn_fwd_v4_q8(int dtype, const void* q, const void* k, const void* v, void* o, void* lse, int B, int Hq,
                              int Hkv, int Tq, int Sk, int D, float scale, int causal, const int64_t* o_strides,
                              const int64_t* qkv_strides, int defer, const AttnQ8* q8, hipStream_t stream) {
  if (D != kD || Hq % Hkv != 0 || Tq <= 0 || Sk <= 0 || dtype != kBF16) return -1;
  const QKVStrides sx = QKVStrides::from(qkv_strides, Hq, Hkv, Tq, Sk, D);
  if ((double)Sk * (double)(sx.kt > sx.vt ? sx.kt : sx.vt) * 2.0 >= 4294967295.0) return -1;
  return launch<__hip_bfloat16>(q, k, v, o, lse, B, Hq, Hkv, Tq, Sk, scale, causal, o_strides, sx, defer & 1, defer >> 1,
                                stream, q8);
}

// v4 forward entry: D = 128, no mask / dropout.  qkv_strides as lta_attn_fwd_ex2 (null = dense);
// rows must be 16-byte aligned and every key-row offset of a head must fit 32 bits.  defer: rescale
// threshold 8 (log2 units) instead of the exact online softmax.  Returns -1 if unsupported.
LTA_EXPORT int lta_attn_fwd_v4(int dtype, const void* q, const void* k, const void* v, void* o, void* lse, int B,
                               int Hq, int Hkv, int Tq, int Sk, int D, float scale, int causal,
                               const int64_t* o_strides, const int64_t* qkv_strides, int defer, hipStream_t stream) {
  if (D != kD || Hq % Hkv != 0 || Tq <= 0 || Sk <= 0) return -1;
  const QKVStrides sx = QKVStrides::from(qkv_strides, Hq, Hkv, Tq, Sk, D);
  if ((double)Sk * (double)(sx.kt > sx.vt ? sx.kt : sx.vt) * 2.0 >= 4294967295.0) return -1;
  if (dtype == kBF16)
    return launch<__hip_bfloat16>(q, k, v, o, lse, B, Hq, Hkv, Tq, Sk, scale, causal, o_strides, sx, defer & 1,
                                  defer >> 1, stream);
#ifndef LTA_V4_ONE
  if (dtype == kF16) return launch<__half>(q, k, v, o, lse, B, Hq, Hkv, Tq, Sk, scale, causal, o_strides, sx, defer & 1, 0, stream);
#endif
  return -1;
}
