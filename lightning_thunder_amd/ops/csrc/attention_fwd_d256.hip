// K3 flash-attention forward for head dim 256 (Gemma), bf16/fp16, causal or full, grouped-query
// heads, any [B,H,T] strides of Q / K / V / O with the head dim contiguous; no mask / dropout (those
// stay on the generic kernel in attention_fwd.hip).  Replaces the reference's cuDNN SDPA forward at
// d = 256 (thunder/executors/cudnn_sdpa.py:339-363).
//
// Structure (cdna_hip_programming.md §5.5 T2/T10, the D = 128 v4 kernel's data flow without its skew):
//  * one workgroup per CU, 4 waves of 32 query rows (128 per workgroup), grid = (B*Hq, query tiles),
//    heaviest causal tiles first;
//  * 32-key K / V tiles arrive by LDS-DMA (global_load_lds, no staging VGPRs) into a 4-stage ring,
//    three tiles in flight: K [32][512 B] with 16-B chunk c at slot c ^ (row & 15) (conflict-free
//    ds_read_b128 row reads), V [32][512 B] with chunk c at slot c ^ ((row & 3) << 2)
//    (conflict-free ds_read_b64_tr_b16 transposed reads);
//  * swapped S^T = K Q^T (each lane owns one query; its 16 scores + the lane ^ 32 partner's make the
//    row), Q fragments in VGPRs for the whole kernel (64 registers), O^T += V^T P^T with P^T packed
//    straight from the S accumulator and O^T (32 x 256 fp32 per wave) in the AGPR file;
//  * at D = 256 a tile is 32 MFMAs against 16 exponentials per lane, so the softmax fits the MFMA
//    shadow without the v4 skew; the O rescale is deferred while no row max grows by more than 8
//    log2 units (exact: P <= 2^8 and the normaliser use the same offset), so the 128 AGPR rescale
//    multiplies run only on the rare tiles that raise it;
//  * causal: a workgroup's tiles end at its last wave's diagonal; the up to three tiles past an
//    earlier wave's diagonal run fully masked (a per-wave skip branch costs the loop ~220 registers).
#include "attention.h"

using namespace lta;
using namespace lta::attn;

namespace {

typedef __attribute__((address_space(3))) void d256_lds_void;

constexpr int kThreads = 256;
constexpr int kBM = 128;   // queries per workgroup
constexpr int kKT = 32;    // keys per tile
constexpr int kNST = 4;    // ring stages
constexpr int kImg = kKT * 512;
constexpr int kStage = 2 * kImg;

__device__ __forceinline__ void mfma_o(f32x16& acc, const bf16x8& a, const bf16x8& b) {
  asm volatile("s_nop 1\n\tv_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
}
__device__ __forceinline__ void mfma_o(f32x16& acc, const f16x8& a, const f16x8& b) {
  asm volatile("s_nop 1\n\tv_mfma_f32_32x32x16_f16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
}

typedef short d256_s16x4 __attribute__((ext_vector_type(4)));

// acc *= a for the AGPR-resident O tile, element by element (a C++ multiply pulls the whole tile
// into VGPRs)
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

// LDS reads of the DMA'd images as inline asm (as builtins the compiler cannot tell them from the
// stage a DMA in flight is writing and drains the DMA queue in front of them), issued in batches and
// waited with a count so the next batch is in flight under the current batch's MFMAs.
// K row fragments (A operand of S^T = K Q^T): 4 reads at per-lane addresses + immediates
template <int O0, int O1, int O2, int O3, typename F>
__device__ __forceinline__ void kread4(F (&x)[4], uint32_t a0, uint32_t a1, uint32_t a2, uint32_t a3) {
  asm volatile(
      "ds_read_b128 %0, %4 offset:%8\n\tds_read_b128 %1, %5 offset:%9\n\t"
      "ds_read_b128 %2, %6 offset:%10\n\tds_read_b128 %3, %7 offset:%11"
      : "=&v"(x[0]), "=&v"(x[1]), "=&v"(x[2]), "=&v"(x[3])
      : "v"(a0), "v"(a1), "v"(a2), "v"(a3), "i"(O0), "i"(O1), "i"(O2), "i"(O3)
      : "memory");
}
// V^T fragments (A operand of O^T += V^T P^T) of d-blocks at a0, a1 for key steps 0, 1: rows
// 16 s + 4 (lane >> 5) + {0..3} and + 8, i.e. pack_frag's key order
template <typename F>
__device__ __forceinline__ void vread4(F (&x)[4], uint32_t a0, uint32_t a1) {
  d256_s16x4 y[8];
  asm volatile(
      "ds_read_b64_tr_b16 %0, %8\n\tds_read_b64_tr_b16 %1, %8 offset:4096\n\t"
      "ds_read_b64_tr_b16 %2, %8 offset:8192\n\tds_read_b64_tr_b16 %3, %8 offset:12288\n\t"
      "ds_read_b64_tr_b16 %4, %9\n\tds_read_b64_tr_b16 %5, %9 offset:4096\n\t"
      "ds_read_b64_tr_b16 %6, %9 offset:8192\n\tds_read_b64_tr_b16 %7, %9 offset:12288"
      : "=&v"(y[0]), "=&v"(y[1]), "=&v"(y[2]), "=&v"(y[3]), "=&v"(y[4]), "=&v"(y[5]), "=&v"(y[6]), "=&v"(y[7])
      : "v"(a0), "v"(a1)
      : "memory");
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    union {
      struct {
        d256_s16x4 a, b;
      } s;
      F f;
    } u;
    u.s.a = y[2 * i];
    u.s.b = y[2 * i + 1];
    x[i] = u.f;
  }
}
template <int N, typename F>
__device__ __forceinline__ void lds_wait(F (&x)[4]) {
  asm volatile("s_waitcnt lgkmcnt(%4)" : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]) : "n"(N) : "memory");
}

template <typename T, bool CAUSAL>
__global__ __launch_bounds__(kThreads, 1) void attn_fwd_d256_kernel(const T* __restrict__ Q, const T* __restrict__ K,
                                                                    const T* __restrict__ V, T* __restrict__ O,
                                                                    float* __restrict__ LSE, int Hq, int Hkv, int Tq,
                                                                    int Sk, float scale_log2, int64_t so_b, int64_t so_h,
                                                                    int64_t so_t, QKVStrides sx) {
  using F = typename Frag<T>::type;
  constexpr float THR = 8.f;
  __shared__ __attribute__((aligned(1024))) char smem[kNST * kStage];
  const uint32_t lds0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)smem;

  const int n_qt = (Tq + kBM - 1) / kBM;
  const int qt = CAUSAL ? n_qt - 1 - (int)blockIdx.y : (int)blockIdx.y;
  const int bh = blockIdx.x, b = bh / Hq, hq = bh % Hq, hk = hq / (Hq / Hkv);
  const T* Qb = Q + b * sx.qb + hq * sx.qh;
  const T* Kb = K + b * sx.kb + hk * sx.kh;
  const T* Vb = V + b * sx.vb + hk * sx.vh;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 31, h = lane >> 5, g = lane >> 4, l16 = lane & 15, vq = l16 >> 2, vp = l16 & 3;
  const int q0 = qt * kBM + wave * 32, qi = q0 + r;

  int nt = (Sk + kKT - 1) / kKT;
  if (CAUSAL) nt = min(nt, (min(qt * kBM + kBM, Tq) + kKT - 1) / kKT);

  // tile t -> stage st: wave w fills K rows 8 w .. 8 w + 7 and V rows 8 w .. (4 pieces of 2 rows each)
  auto issue = [&](int t, int st) {
    char* kimg = smem + st * kStage;
    char* vimg = kimg + kImg;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int R = 8 * wave + 2 * i + (lane >> 5), slot = lane & 31;
      const int key = min(t * kKT + R, Sk - 1);  // rows past Sk: a clamped copy, masked to P = 0
      __builtin_amdgcn_global_load_lds((const void*)(Kb + (int64_t)key * sx.kt + (slot ^ (R & 15)) * 8),
                                       (d256_lds_void*)(kimg + (4 * wave + i) * 1024), 16, 0, 0);
      __builtin_amdgcn_global_load_lds((const void*)(Vb + (int64_t)key * sx.vt + (slot ^ ((R & 3) << 2)) * 8),
                                       (d256_lds_void*)(vimg + (4 * wave + i) * 1024), 16, 0, 0);
    }
  };

  F qf[16];
  {
    const int qrow = min(qi, Tq - 1);
#pragma unroll
    for (int s = 0; s < 16; ++s) qf[s] = load_frag<F>(Qb + (int64_t)qrow * sx.qt + 16 * s + 8 * h);
  }
  f32x16 oacc[8];
#pragma unroll
  for (int dt = 0; dt < 8; ++dt)
#pragma unroll
    for (int i = 0; i < 16; ++i) oacc[dt][i] = 0.f;

  // per-lane LDS offsets: K chunk (2 s + h) of row r sits at slot (2 s + h) ^ (r & 15) = 2 (s ^ xh) + hb
  // with xh = (r & 15) >> 1, hb = h ^ (r & 1): s = 8 a + b -> 256 a + koff[b]
  uint32_t koff[8], voff[8];
  {
    const int xh = (r & 15) >> 1, hb = h ^ (r & 1);
#pragma unroll
    for (int bb = 0; bb < 8; ++bb) koff[bb] = r * 512 + 32 * (bb ^ xh) + 16 * hb;
#pragma unroll
    for (int dt = 0; dt < 8; ++dt)
      voff[dt] = (4 * h + vq) * 512 + ((4 * (dt ^ vq) + 2 * (g & 1) + (vp >> 1)) << 4) + 8 * (vp & 1);
  }

  float m_use = -INFINITY, l = 0.f;
  const float ninf = -INFINITY;

#pragma unroll
  for (int p = 0; p < kNST - 1; ++p)
    if (p < nt) issue(p, p);
  for (int t = 0; t < nt; ++t) {
    const int later = min(nt - 1 - t, kNST - 2);
    if (later >= 2)
      asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    else if (later == 1)
      asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // tile t landed for every wave; stage (t - 1) % kNST is free
    if (t + kNST - 1 < nt) issue(t + kNST - 1, (t + kNST - 1) % kNST);
    const int kbase = t * kKT;
    // (tiles past this wave's diagonal are fully masked: P = 0)
    const uint32_t kimg = lds0 + (t % kNST) * kStage, vimg = kimg + kImg;

    // ---- S^T = K Q^T (16 k-steps over d; k-step s = 8 a + b reads koff[b] + 256 a) ----
    f32x16 sacc;
#pragma unroll
    for (int i = 0; i < 16; ++i) sacc[i] = 0.f;
    {
      F x[4], y[4];
      kread4<0, 0, 0, 0>(x, kimg + koff[0], kimg + koff[1], kimg + koff[2], kimg + koff[3]);
      kread4<0, 0, 0, 0>(y, kimg + koff[4], kimg + koff[5], kimg + koff[6], kimg + koff[7]);
      lds_wait<4>(x);
#pragma unroll
      for (int i = 0; i < 4; ++i) sacc = mfma(x[i], qf[i], sacc);
      kread4<256, 256, 256, 256>(x, kimg + koff[0], kimg + koff[1], kimg + koff[2], kimg + koff[3]);
      lds_wait<4>(y);
#pragma unroll
      for (int i = 0; i < 4; ++i) sacc = mfma(y[i], qf[4 + i], sacc);
      kread4<256, 256, 256, 256>(y, kimg + koff[4], kimg + koff[5], kimg + koff[6], kimg + koff[7]);
      lds_wait<4>(x);
#pragma unroll
      for (int i = 0; i < 4; ++i) sacc = mfma(x[i], qf[8 + i], sacc);
      lds_wait<0>(y);
#pragma unroll
      for (int i = 0; i < 4; ++i) sacc = mfma(y[i], qf[12 + i], sacc);
    }

    // ---- mask, deferred online softmax (lane-local row + the lane ^ 32 partner) ----
    const bool need_mask = kbase + kKT > Sk || (CAUSAL && kbase + kKT - 1 > q0);
    if (need_mask) {
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int key = kbase + acc_row(i, h);
        if (key >= Sk || (CAUSAL && key > qi)) sacc[i] = ninf;
      }
    }
    float mx = sacc[0];
#pragma unroll
    for (int i = 1; i < 16; ++i) mx = fmaxf(mx, sacc[i]);
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64)) * scale_log2;
    if (__builtin_amdgcn_ballot_w64(mx > m_use + THR || (m_use == ninf && mx != ninf)) != 0) {
      const float m_new = fmaxf(m_use, mx);
      const float alpha = m_use == ninf ? 0.f : __builtin_amdgcn_exp2f(m_use - m_new);
      l *= alpha;
#pragma unroll
      for (int dt = 0; dt < 8; ++dt) scale_acc(oacc[dt], alpha);
      m_use = m_new;
    }
    const float msafe = m_use == ninf ? 0.f : m_use;
    float rs = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const float pv = __builtin_amdgcn_exp2f(__builtin_fmaf(sacc[i], scale_log2, -msafe));
      sacc[i] = pv;
      rs += pv;
    }
    l += rs;
    F pf0, pf1;
    pack_frag(pf0, sacc, 0);
    pack_frag(pf1, sacc, 1);

    // ---- O^T += V^T P^T (8 d-blocks x 2 key steps), d-blocks in pairs ----
    {
      F x[4], y[4];
      vread4(x, vimg + voff[0], vimg + voff[1]);
      vread4(y, vimg + voff[2], vimg + voff[3]);
      lds_wait<8>(x);
      mfma_o(oacc[0], x[0], pf0); mfma_o(oacc[0], x[1], pf1); mfma_o(oacc[1], x[2], pf0); mfma_o(oacc[1], x[3], pf1);
      vread4(x, vimg + voff[4], vimg + voff[5]);
      lds_wait<8>(y);
      mfma_o(oacc[2], y[0], pf0); mfma_o(oacc[2], y[1], pf1); mfma_o(oacc[3], y[2], pf0); mfma_o(oacc[3], y[3], pf1);
      vread4(y, vimg + voff[6], vimg + voff[7]);
      lds_wait<8>(x);
      mfma_o(oacc[4], x[0], pf0); mfma_o(oacc[4], x[1], pf1); mfma_o(oacc[5], x[2], pf0); mfma_o(oacc[5], x[3], pf1);
      lds_wait<0>(y);
      mfma_o(oacc[6], y[0], pf0); mfma_o(oacc[6], y[1], pf1); mfma_o(oacc[7], y[2], pf0); mfma_o(oacc[7], y[3], pf1);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no DMA outlives the workgroup

  // ---- epilogue: O = O^T / l, LSE ----
  l += __shfl_xor(l, 32, 64);
  if (qi < Tq) {
    const float inv = l > 0.f ? 1.f / l : 0.f;
    T* orow = O + b * so_b + hq * so_h + (int64_t)qi * so_t;
#pragma unroll
    for (int dt = 0; dt < 8; ++dt)
#pragma unroll
      for (int a = 0; a < 4; ++a) {
        union {
          T v[4];
          uint2 u;
        } pk;
#pragma unroll
        for (int e = 0; e < 4; ++e) pk.v[e] = from_f32<T>(oacc[dt][4 * a + e] * inv);
        *reinterpret_cast<uint2*>(orow + dt * 32 + 8 * a + 4 * h) = pk.u;
      }
    if (h == 0 && LSE != nullptr)
      LSE[((int64_t)b * Hq + hq) * Tq + qi] = l > 0.f ? (m_use + log2f(l)) * 0.69314718055994530942f : -INFINITY;
  }
}

template <typename T>
int launch_d256(const void* q, const void* k, const void* v, void* o, void* lse, int B, int Hq, int Hkv, int Tq, int Sk,
                float scale, int causal, const int64_t* so, const QKVStrides& sx, hipStream_t s) {
  const float sl2 = scale * 1.44269504088896340736f;
  dim3 grid(B * Hq, (Tq + kBM - 1) / kBM), block(kThreads);
  const int64_t sb = so ? so[0] : (int64_t)Hq * Tq * 256, sh = so ? so[1] : (int64_t)Tq * 256, st = so ? so[2] : 256;
  if (causal)
    hipLaunchKernelGGL((attn_fwd_d256_kernel<T, true>), grid, block, 0, s, (const T*)q, (const T*)k, (const T*)v, (T*)o,
                       (float*)lse, Hq, Hkv, Tq, Sk, sl2, sb, sh, st, sx);
  else
    hipLaunchKernelGGL((attn_fwd_d256_kernel<T, false>), grid, block, 0, s, (const T*)q, (const T*)k, (const T*)v, (T*)o,
                       (float*)lse, Hq, Hkv, Tq, Sk, sl2, sb, sh, st, sx);
  return (int)hipGetLastError();
}

}  // namespace

// D = 256 forward without mask / dropout (strides as lta_attn_fwd_ex2).  -1: not this kernel's case.
LTA_EXPORT int lta_attn_fwd_d256(int dtype, const void* q, const void* k, const void* v, void* o, void* lse, int B,
                                 int Hq, int Hkv, int Tq, int Sk, int D, float scale, int causal,
                                 const int64_t* o_strides, const int64_t* qkv_strides, hipStream_t stream) {
  if (D != 256 || Tq <= 0 || Sk <= 0 || Hkv <= 0 || Hq % Hkv != 0) return -1;
  const QKVStrides sx = QKVStrides::from(qkv_strides, Hq, Hkv, Tq, Sk, D);
  if (dtype == kBF16)
    return launch_d256<__hip_bfloat16>(q, k, v, o, lse, B, Hq, Hkv, Tq, Sk, scale, causal, o_strides, sx, stream);
  if (dtype == kF16) return launch_d256<__half>(q, k, v, o, lse, B, Hq, Hkv, Tq, Sk, scale, causal, o_strides, sx, stream);
  return -1;
}
