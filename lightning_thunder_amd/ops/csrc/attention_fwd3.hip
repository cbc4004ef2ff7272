// K3 flash-attention forward, v3 (D = 128, bf16/fp16, causal or full, GQA, no mask / dropout):
// 64 query rows per wave in two 32-row blocks, one wave per SIMD (4 waves = 256 queries per
// workgroup, one workgroup per CU) — the forward counterpart of the dK/dV v3 kernel
// (attention_bwd.hip) and of cdna_hip_programming.md's one-wave-per-SIMD attention structure.
//  * every K fragment read from LDS feeds both query blocks' S MFMAs and every transposed V read
//    both blocks' PV MFMAs: 64 MFMAs per 64-key tile against 32 in v1, for the same LDS reads;
//  * S = K Q^T ("swapped": the lane owns one query) in VGPRs through the MFMA intrinsic, O^T in
//    the AGPR file through inline-asm MFMAs (this file builds with -amdgpu-mfma-vgpr-form=1), so
//    the 128 O registers do not compete with Q, S and P for the 256 architectural VGPRs;
//  * K / V register-staged one tile ahead into double-buffered padded LDS images (the v1 strides:
//    conflict-free b128 row reads of K, ds_read_b64_tr_b16 reads of V), one barrier per tile;
//  * the scale folds into one FMA per score, row max as a max3 tree + one permlane32 swap, the
//    rescale of O deferred while no row max of a block grows by more than THR (log2 units);
//  * under causal masking only a wave's last tile straddles the diagonal (64-row waves, 64-key
//    tiles, both aligned), so the mask is one wave-uniform branch; past it a wave only stages.
#include "attention.h"

using namespace lta;
using namespace lta::attn;

namespace {

constexpr int kD = 128, kBN = 64, kNW = 4, kRows = 64, kBM = kNW * kRows, kThreads = 64 * kNW;
constexpr int kKSTR = kD + 8, kVSTR = kD + 32;  // padded row strides (elements)
constexpr int kKT = kBN * kKSTR, kVT = kBN * kVSTR;  // elements per K / V tile image
constexpr int kNLD = kBN * (kD / 8) / kThreads;  // 16-B chunks per thread per K (or V) tile

__device__ __forceinline__ float max3f(float a, float b, float c) {
  float r;
  asm("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}

// swap(v, v): element 0 carries lanes 32..63 into lanes 0..31, element 1 lanes 0..31 into 32..63
// (each lane's own value in the other element): max / sum over both pair lane l with l ^ 32
__device__ __forceinline__ float pair_max(float v) {
  const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return max3f(v, __uint_as_float(sw[0]), __uint_as_float(sw[1]));
}
__device__ __forceinline__ float pair_sum(float v) {
  const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(sw[0]) + __uint_as_float(sw[1]);
}

__device__ __forceinline__ float row_max32(const f32x16 (&s)[2]) {
  float m[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const f32x16& x = s[c >> 1];
    const int o = 8 * (c & 1);
    float v = max3f(x[o], x[o + 1], x[o + 2]);
    v = max3f(v, x[o + 3], x[o + 4]);
    v = max3f(v, x[o + 5], x[o + 6]);
    m[c] = max3f(v, x[o + 7], x[o + 7]);
  }
  return pair_max(max3f(max3f(m[0], m[1], m[2]), m[3], m[3]));
}

// O^T += V^T P^T into the accumulator file; `s_nop 1` covers the P pack (VALU) -> MFMA read
__device__ __forceinline__ void pv_mfma(f32x16& acc, const bf16x8& a, const bf16x8& b) {
  asm volatile("s_nop 1\n\tv_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
}
__device__ __forceinline__ void pv_mfma(f32x16& acc, const f16x8& a, const f16x8& b) {
  asm volatile("s_nop 1\n\tv_mfma_f32_32x32x16_f16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
}

template <typename T, bool CAUSAL, int THR>
__global__ __launch_bounds__(kThreads, 1) void attn_fwd_v3_kernel(const T* __restrict__ Q, const T* __restrict__ K,
                                                                  const T* __restrict__ V, T* __restrict__ O,
                                                                  float* __restrict__ LSE, int Hq, int Hkv, int Tq,
                                                                  int Sk, float c, int64_t so_b, int64_t so_h,
                                                                  int64_t so_t) {
  using F = typename Frag<T>::type;
  __shared__ __attribute__((aligned(16))) short smem[2 * kKT + 2 * kVT];

  const int n_qt = (Tq + kBM - 1) / kBM;
  const int qt = n_qt - 1 - (int)blockIdx.y;  // heaviest causal blocks first
  const int bh = blockIdx.x;                  // x-fastest: a head's blocks share one XCD's L2
  const int b = bh / Hq, hq = bh % Hq;
  const int hk = hq / (Hq / Hkv);
  const T* Qb = Q + ((int64_t)b * Hq + hq) * Tq * kD;
  const T* Kb = K + ((int64_t)b * Hkv + hk) * (int64_t)Sk * kD;
  const T* Vb = V + ((int64_t)b * Hkv + hk) * (int64_t)Sk * kD;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 31, h = lane >> 5, g = lane >> 4, l16 = lane & 15;
  const int q0 = qt * kBM + wave * kRows;  // block j: queries q0 + 32 j + r

  int n_tiles = (Sk + kBN - 1) / kBN;
  if (CAUSAL) n_tiles = min(n_tiles, (min(qt * kBM + kBM, Tq) + kBN - 1) / kBN);
  int nw = n_tiles;
  if (CAUSAL) nw = min(n_tiles, min(q0 + kRows - 1, Tq - 1) / kBN + 1);
  const bool last_masked = (nw * kBN > Sk) || (CAUSAL && (nw - 1) * kBN + kBN - 1 > q0);

  F qf[2][8];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int qrow = min(q0 + 32 * j + r, Tq - 1);
#pragma unroll
    for (int s = 0; s < 8; ++s) qf[j][s] = load_frag<F>(Qb + (int64_t)qrow * kD + 16 * s + 8 * h);
  }

  uint4 kreg[kNLD], vreg[kNLD];
  auto gload = [&](int t) {
#pragma unroll
    for (int i = 0; i < kNLD; ++i) {
      const int id = i * kThreads + tid, row = id >> 4, ch = id & 15;
      const int kc = min(t * kBN + row, Sk - 1);  // clamped rows are real keys; the mask drops them
      kreg[i] = *reinterpret_cast<const uint4*>(Kb + (int64_t)kc * kD + ch * 8);
      vreg[i] = *reinterpret_cast<const uint4*>(Vb + (int64_t)kc * kD + ch * 8);
    }
  };
  auto lstore = [&](int buf) {
#pragma unroll
    for (int i = 0; i < kNLD; ++i) {
      const int id = i * kThreads + tid, row = id >> 4, ch = id & 15;
      *reinterpret_cast<uint4*>(smem + buf * kKT + row * kKSTR + ch * 8) = kreg[i];
      *reinterpret_cast<uint4*>(smem + 2 * kKT + buf * kVT + row * kVSTR + ch * 8) = vreg[i];
    }
  };

  f32x16 oacc[2][4];
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int dt = 0; dt < 4; ++dt)
#pragma unroll
      for (int i = 0; i < 16; ++i) oacc[j][dt][i] = 0.f;
  float m_use[2] = {-INFINITY, -INFINITY}, l[2] = {0.f, 0.f};

  const int last = n_tiles - 1;
  gload(0);
  lstore(0);
  __syncthreads();
  for (int t = 0; t < n_tiles; ++t) {
    gload(min(t + 1, last));  // tile t+1 in flight over tile t's math
    if (t < nw) {             // wave-uniform
      const short* Ks = smem + (t & 1) * kKT;
      const __attribute__((address_space(3))) short* Vs3 =
          (const __attribute__((address_space(3))) short*)(smem + 2 * kKT + (t & 1) * kVT);
      // ---- S^T = K Q^T for both query blocks: one K fragment read feeds two MFMAs --------------
      f32x16 sacc[2][2];
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int kt = 0; kt < 2; ++kt)
#pragma unroll
          for (int i = 0; i < 16; ++i) sacc[j][kt][i] = 0.f;
#pragma unroll
      for (int s = 0; s < 8; ++s)
#pragma unroll
        for (int kt = 0; kt < 2; ++kt) {
          const F ka = load_frag<F>(Ks + (kt * 32 + r) * kKSTR + 16 * s + 8 * h);
          sacc[0][kt] = mfma(ka, qf[0][s], sacc[0][kt]);
          sacc[1][kt] = mfma(ka, qf[1][s], sacc[1][kt]);
        }
      if (t == nw - 1 && last_masked) {
        const int kbase = t * kBN;
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int kt = 0; kt < 2; ++kt)
#pragma unroll
            for (int i = 0; i < 16; ++i) {
              const int key = kbase + kt * 32 + acc_row(i, h);
              if (key >= Sk || (CAUSAL && key > q0 + 32 * j + r)) sacc[j][kt][i] = -INFINITY;
            }
      }
      // ---- online softmax per block; P fragments for the PV MFMAs ---------------------------------
      F pf[2][2][2];
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const float mx = row_max32(sacc[j]) * c;  // c > 0: the max commutes with the scale
        const bool grow = !(mx - m_use[j] <= (float)THR);  // true at m_use = -inf
        if (__builtin_amdgcn_ballot_w64(grow) != 0) {       // wave-uniform
          const float mn = fmaxf(m_use[j], mx);
          const float mu = (mn == -INFINITY) ? 0.f : mn;
          const float alpha = __builtin_amdgcn_exp2f(m_use[j] - mu);
          m_use[j] = mu;
          l[j] *= alpha;
#pragma unroll
          for (int dt = 0; dt < 4; ++dt)
#pragma unroll
            for (int i = 0; i < 16; ++i) oacc[j][dt][i] *= alpha;  // PV of tile t-1 long complete
        }
        const float nm = -m_use[j];
        float rs0 = 0.f, rs1 = 0.f;
#pragma unroll
        for (int kt = 0; kt < 2; ++kt)
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            const float p = __builtin_amdgcn_exp2f(__builtin_fmaf(sacc[j][kt][i], c, nm));
            sacc[j][kt][i] = p;
            if (i & 1) rs1 += p; else rs0 += p;
          }
        l[j] += pair_sum(rs0 + rs1);
#pragma unroll
        for (int kt = 0; kt < 2; ++kt) {
          pack_frag(pf[j][kt][0], sacc[j][kt], 0);
          pack_frag(pf[j][kt][1], sacc[j][kt], 1);
        }
      }
      // ---- O^T += V^T P^T: one transposed V fragment feeds both blocks ------------------------------
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        const int col0 = dt * 32 + 16 * (g & 1);
#pragma unroll
        for (int kt = 0; kt < 2; ++kt)
#pragma unroll
          for (int s = 0; s < 2; ++s) {
            const F va = tr_frag<F>(Vs3, kt * 32 + 16 * s + 4 * h, col0, kVSTR, l16);
            pv_mfma(oacc[0][dt], va, pf[0][kt][s]);
            pv_mfma(oacc[1][dt], va, pf[1][kt][s]);
          }
      }
    }
    lstore((t + 1) & 1);  // over tile t-1 (read before the last barrier)
    __syncthreads();
  }
  // the last asm MFMAs' results must be complete before any other instruction reads them
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) asm volatile("s_nop 15\n\ts_nop 15" : "+a"(oacc[j][dt]));

  // ---- epilogue: O = O^T / l ; LSE ------------------------------------------------------------------
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int qi = q0 + 32 * j + r;
    if (qi >= Tq) continue;
    const float inv = (l[j] > 0.f) ? 1.f / l[j] : 0.f;
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
        for (int e = 0; e < 4; ++e) pk.v[e] = from_f32<T>(oacc[j][dt][4 * a + e] * inv);
        *reinterpret_cast<uint2*>(orow + d) = pk.u;
      }
    }
    if (h == 0 && LSE != nullptr)
      LSE[((int64_t)b * Hq + hq) * Tq + qi] =
          (l[j] > 0.f) ? (m_use[j] + log2f(l[j])) * 0.69314718055994530942f : -INFINITY;
  }
}

template <typename T>
int launch(const void* q, const void* k, const void* v, void* o, void* lse, int B, int Hq, int Hkv, int Tq, int Sk,
           float scale, int causal, const int64_t* so, int defer, hipStream_t s) {
  const float c = scale * 1.44269504088896340736f;
  dim3 grid(B * Hq, (Tq + kBM - 1) / kBM), block(kThreads);
  const int64_t sb = so ? so[0] : (int64_t)Hq * Tq * kD, sh = so ? so[1] : (int64_t)Tq * kD, st = so ? so[2] : kD;
#define LTA_V3(CA, TH)                                                                                            \
  hipLaunchKernelGGL((attn_fwd_v3_kernel<T, CA, TH>), grid, block, 0, s, (const T*)q, (const T*)k, (const T*)v, \
                     (T*)o, (float*)lse, Hq, Hkv, Tq, Sk, c, sb, sh, st)
  if (causal) {
    if (defer) LTA_V3(true, 8); else LTA_V3(true, 0);
  } else {
    if (defer) LTA_V3(false, 8); else LTA_V3(false, 0);
  }
#undef LTA_V3
  return (int)hipGetLastError();
}

}  // namespace

// v3 forward entry (D = 128, no mask / dropout); o_strides as lta_attn_fwd_ex.  defer: rescale
// threshold 8 (log2 units) instead of exact.  Returns -1 for unsupported shapes / dtypes.
LTA_EXPORT int lta_attn_fwd_v3(int dtype, const void* q, const void* k, const void* v, void* o, void* lse, int B,
                               int Hq, int Hkv, int Tq, int Sk, int D, float scale, int causal,
                               const int64_t* o_strides, int defer, hipStream_t stream) {
  if (D != kD || Hq % Hkv != 0 || Tq <= 0 || Sk <= 0) return -1;
  if (dtype == kBF16)
    return launch<__hip_bfloat16>(q, k, v, o, lse, B, Hq, Hkv, Tq, Sk, scale, causal, o_strides, defer, stream);
  if (dtype == kF16) return launch<__half>(q, k, v, o, lse, B, Hq, Hkv, Tq, Sk, scale, causal, o_strides, defer, stream);
  return -1;
}
