// K3 flash-attention forward for CDNA4 (gfx950), bf16/fp16, head dim 64 or 128, causal or full,
// grouped-query heads.  Replaces the reference's cuDNN/aten-flash/FA3 SDPA executors
// (thunder/executors/{cudnn_sdpa,sdpaex,fa3ex}.py).
//
// Structure (see attention.h for the MFMA operand maps):
//  * workgroup = 4 waves = 128 query rows (32 per wave), grid = (query tiles, batch*heads),
//    heaviest causal tiles first;
//  * per 64-key tile: K and V are staged global -> registers -> LDS (padded rows: K rows read
//    with ds_read_b128 are conflict-free at stride 68 dwords, V rows read with
//    ds_read_b64_tr_b16 are conflict-free at stride 80 dwords) with the next tile's global
//    loads issued before the current tile's math (async-STAGE split, T14);
//  * "swapped" S^T = K * Q^T: each lane owns one query, so the online-softmax row max/sum is
//    16 register ops + one lane^32 exchange, and O^T = V^T * P^T keeps the rescale lane-local;
//  * P^T goes from the S accumulator straight into the PV MFMA as the B operand (no LDS
//    round trip), V^T comes from transposed LDS reads.
// Outputs O [B,H,T,D] and LSE [B,H,T] (natural-log log-sum-exp of the scaled scores).
#include "attention.h"

using namespace lta;
using namespace lta::attn;

namespace {

constexpr int kBM = 128;  // queries per workgroup
constexpr int kBN = 64;   // keys per tile
constexpr int kThreads = 256;

template <int D> struct Cfg {
  // D = 256 (Gemma): 32-key tiles and one workgroup per CU, so Q (64 VGPRs), O (128 accumulators)
  // and the staged K / V tile fit the 512-entry VGPR + AGPR file of a lone wave without spilling
  static constexpr int BN = D > 128 ? 32 : kBN;    // keys per tile
  static constexpr int NKT = BN / 32;              // 32-key sub-tiles
  static constexpr int OCC = D > 128 ? 1 : 2;      // workgroups per CU (launch bound)
  static constexpr int KSTR = D + 8;               // K tile row stride (elements)
  static constexpr int VSTR = D + 32;              // V tile row stride
  static constexpr int CH = D / 8;                 // 16-byte chunks per row
  static constexpr int LOADS = BN * CH / kThreads;  // chunks per thread per tile
  static constexpr int KS = D / 16;                // MFMA k-steps over D
  static constexpr int DT = D / 32;                // 32-wide d tiles
};

template <typename T, int D, bool CAUSAL, int EX = 0>
__global__ __launch_bounds__(kThreads, Cfg<D>::OCC) void attn_fwd_kernel(const T* __restrict__ Q, const T* __restrict__ K,
                                                               const T* __restrict__ V, T* __restrict__ O,
                                                               float* __restrict__ LSE, int Hq, int Hkv, int Tq,
                                                               int Sk, float scale_log2, int64_t so_b, int64_t so_h,
                                                               int64_t so_t, AttnExtra ex) {
  constexpr bool MASK = EX & kExMask, DROP = EX & kExDrop;
  using C = Cfg<D>;
  using F = typename Frag<T>::type;
  __shared__ __attribute__((aligned(16))) short smem[C::BN * C::KSTR + C::BN * C::VSTR];
  __shared__ __attribute__((aligned(16))) unsigned ktab[DROP ? 4 * C::BN : 4];  // per-wave key terms (dropout)
  short* Ks = smem;
  short* Vs = smem + C::BN * C::KSTR;
  const __attribute__((address_space(3))) short* Vs3 = (const __attribute__((address_space(3))) short*)Vs;

  const int n_qt = (Tq + kBM - 1) / kBM;
  // grid = (B*H, tiles): dispatch is x-fastest and round-robins workgroups over the 8 XCDs, so
  // every XCD receives the same mix of causal tile weights and the heaviest tiles start first.
  const int qt = n_qt - 1 - (int)blockIdx.y;
  const int bh = blockIdx.x;
  const int b = bh / Hq, hq = bh % Hq;
  const int hk = hq / (Hq / Hkv);
  const T* Qb = Q + b * ex.sx.qb + hq * ex.sx.qh;
  const T* Kb = K + b * ex.sx.kb + hk * ex.sx.kh;
  const T* Vb = V + b * ex.sx.vb + hk * ex.sx.vh;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // provably wave-uniform
  const int r = lane & 31, h = lane >> 5, g = lane >> 4, l16 = lane & 15;
  const int q0 = qt * kBM + wave * 32;
  const int qi = q0 + r;  // this lane's query
  const float* mrow = nullptr;
  if constexpr (MASK) mrow = ex.mask + b * ex.mb + hq * ex.mh + (int64_t)min(qi, Tq - 1) * ex.mq;
  unsigned qterm = 0;
  if constexpr (DROP) qterm = rng_q(rng_head(ex, bh), qi);

  // Q fragments (B operand of S^T = K Q^T): Q[qi][16s + 8h .. +7]
  F qf[C::KS];
  {
    const int qrow = min(qi, Tq - 1);
#pragma unroll
    for (int s = 0; s < C::KS; ++s) qf[s] = load_frag<F>(Qb + (int64_t)qrow * ex.sx.qt + 16 * s + 8 * h);
  }

  f32x16 oacc[C::DT];
#pragma unroll
  for (int dt = 0; dt < C::DT; ++dt)
#pragma unroll
    for (int i = 0; i < 16; ++i) oacc[dt][i] = 0.f;
  float m = -INFINITY, l = 0.f;

  int n_tiles = (Sk + C::BN - 1) / C::BN;
  if (CAUSAL) n_tiles = min(n_tiles, (min(qt * kBM + kBM, Tq) + C::BN - 1) / C::BN);

  // register staging of one K/V tile
  uint4 kreg[C::LOADS], vreg[C::LOADS];
  auto gload = [&](int t) {
#pragma unroll
    for (int c = 0; c < C::LOADS; ++c) {
      const int id = c * kThreads + tid;
      const int row = id / C::CH, ch = id % C::CH;
      const int key = t * C::BN + row;
      const int kc = min(key, Sk - 1);  // branch-free: clamp the address, zero the data
      uint4 kx = *reinterpret_cast<const uint4*>(Kb + (int64_t)kc * ex.sx.kt + ch * 8);
      uint4 vx = *reinterpret_cast<const uint4*>(Vb + (int64_t)kc * ex.sx.vt + ch * 8);
      const bool ok = key < Sk;
      kreg[c] = ok ? kx : make_uint4(0, 0, 0, 0);
      vreg[c] = ok ? vx : make_uint4(0, 0, 0, 0);
    }
  };
  auto lstore = [&]() {
#pragma unroll
    for (int c = 0; c < C::LOADS; ++c) {
      const int id = c * kThreads + tid;
      const int row = id / C::CH, ch = id % C::CH;
      *reinterpret_cast<uint4*>(Ks + row * C::KSTR + ch * 8) = kreg[c];
      *reinterpret_cast<uint4*>(Vs + row * C::VSTR + ch * 8) = vreg[c];
    }
  };

  if (n_tiles > 0) gload(0);
  for (int t = 0; t < n_tiles; ++t) {
    __syncthreads();  // previous tile fully consumed
    lstore();
    __syncthreads();
    if (t + 1 < n_tiles) gload(t + 1);  // next tile's HBM traffic overlaps this tile's math

    // ---- S^T = K Q^T : two 32-key sub-tiles -------------------------------------------------
    f32x16 sacc[C::NKT];
#pragma unroll
    for (int kt = 0; kt < C::NKT; ++kt)
#pragma unroll
      for (int i = 0; i < 16; ++i) sacc[kt][i] = 0.f;
#pragma unroll
    for (int s = 0; s < C::KS; ++s) {
#pragma unroll
      for (int kt = 0; kt < C::NKT; ++kt) {
        const F ka = load_frag<F>(Ks + (kt * 32 + r) * C::KSTR + 16 * s + 8 * h);
        sacc[kt] = mfma(ka, qf[s], sacc[kt]);
      }
    }

    // ---- scale, mask, online softmax (lane-local row = query qi) --------------------------------
    const int kbase = t * C::BN;
    const bool need_mask = (kbase + C::BN > Sk) || (CAUSAL && kbase + C::BN - 1 > q0);
    float mx = -INFINITY;
    if constexpr (MASK) {  // additive mask, 4 consecutive keys per 16-B load (key dim padded to 64)
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
        float v = MASK ? sacc[kt][i] : sacc[kt][i] * scale_log2;
        if (need_mask) {  // wave-uniform branch; per-element select
          const int key = kbase + kt * 32 + acc_row(i, h);
          v = (key >= Sk || (CAUSAL && key > qi)) ? -INFINITY : v;
        }
        sacc[kt][i] = v;
        mx = fmaxf(mx, v);
      }
    }
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    const float m_new = fmaxf(m, mx);
    const float m_use = (m_new == -INFINITY) ? 0.f : m_new;
    const float alpha = __builtin_amdgcn_exp2f(m - m_use);
    float rs = 0.f;
#pragma unroll
    for (int kt = 0; kt < C::NKT; ++kt) {
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const float p = __builtin_amdgcn_exp2f(sacc[kt][i] - m_use);
        sacc[kt][i] = p;
        rs += p;
      }
    }
    rs += __shfl_xor(rs, 32, 64);
    l = l * alpha + rs;
    m = m_new;
    if constexpr (DROP) {  // the normalizer keeps every probability; only P.V sees the dropped ones
      unsigned* krow = ktab + wave * C::BN;
      if (lane < C::BN) krow[lane] = rng_k(kbase + lane);
#pragma unroll
      for (int kt = 0; kt < C::NKT; ++kt)
#pragma unroll
        for (int a = 0; a < 4; ++a) {
          const uint4 kv = rng_tab4(krow + kt * 32, a, h);
          const unsigned kk[4] = {kv.x, kv.y, kv.z, kv.w};
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const bool keep = rng_keep(ex, qterm, kk[e]);
            sacc[kt][4 * a + e] = keep ? sacc[kt][4 * a + e] * ex.keep_scale : 0.f;
          }
        }
    }
#pragma unroll
    for (int dt = 0; dt < C::DT; ++dt)
#pragma unroll
      for (int i = 0; i < 16; ++i) oacc[dt][i] *= alpha;

    // ---- O^T += V^T P^T ----------------------------------------------------------------------
    F pf[C::NKT][2];
#pragma unroll
    for (int kt = 0; kt < C::NKT; ++kt) {
      pack_frag(pf[kt][0], sacc[kt], 0);
      pack_frag(pf[kt][1], sacc[kt], 1);
    }
#pragma unroll
    for (int dt = 0; dt < C::DT; ++dt) {
      const int col0 = dt * 32 + 16 * (g & 1);
#pragma unroll
      for (int kt = 0; kt < C::NKT; ++kt) {
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          const F va = tr_frag<F>(Vs3, kt * 32 + 16 * s + 4 * h, col0, C::VSTR, l16);
          oacc[dt] = mfma(va, pf[kt][s], oacc[dt]);
        }
      }
    }
  }

  // ---- epilogue: O = O^T / l ; LSE --------------------------------------------------------------
  if (qi < Tq) {
    const float inv = (l > 0.f) ? 1.f / l : 0.f;
    T* orow = O + b * so_b + hq * so_h + qi * so_t;  // any [B,H,T] strides (e.g. [B,T,H,D] storage)
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
        for (int e = 0; e < 4; ++e) pk.v[e] = from_f32<T>(oacc[dt][4 * a + e] * inv);
        *reinterpret_cast<uint2*>(orow + d) = pk.u;
      }
    }
    if (h == 0 && LSE != nullptr) {
      // natural-log LSE of the scaled scores: (m + log2 l) * ln 2
      LSE[((int64_t)b * Hq + hq) * Tq + qi] = (l > 0.f) ? (m + log2f(l)) * 0.69314718055994530942f : -INFINITY;
    }
  }
}

// D = 128 without mask / dropout: 10 = v4 with the deferred O rescale (default), 9 = v4 exact online
// softmax, 0 = v1 (the plain-HIP kernel every other configuration runs; profiles/attn_v4_*, retired
// v2 / v3 kernels: profiles/attn_v2_ab.json, profiles/attn_fwd_pmc.json).  11..15 select the v4
// measurement builds, compiled only with -DLTA_ATTN_DIAG.
int g_fwd_impl = 10;
// D = 256 without mask / dropout: 1 = the LDS-DMA ring kernel (attention_fwd_d256.hip), 0 = the
// generic kernel below (A/B: lta_attn_fwd_set_ring; a D = 64 port of the ring kernel measured no faster
// than the generic kernel, profiles/attn_d256_bench.txt)
int g_fwd_ring = 1;

template <typename T, int D, int EX>
int launch_ex(const void* q, const void* k, const void* v, void* o, void* lse, int B, int Hq, int Hkv, int Tq, int Sk,
              float scale, int causal, const int64_t* so, const AttnExtra& ex, hipStream_t s) {
  const float sl2 = scale * 1.44269504088896340736f;
  dim3 grid(B * Hq, (Tq + kBM - 1) / kBM), block(kThreads);
  const int64_t sb = so ? so[0] : (int64_t)Hq * Tq * D, sh = so ? so[1] : (int64_t)Tq * D, st = so ? so[2] : D;
  if (causal)
    hipLaunchKernelGGL((attn_fwd_kernel<T, D, true, EX>), grid, block, 0, s, (const T*)q, (const T*)k, (const T*)v,
                       (T*)o, (float*)lse, Hq, Hkv, Tq, Sk, sl2, sb, sh, st, ex);
  else
    hipLaunchKernelGGL((attn_fwd_kernel<T, D, false, EX>), grid, block, 0, s, (const T*)q, (const T*)k, (const T*)v,
                       (T*)o, (float*)lse, Hq, Hkv, Tq, Sk, sl2, sb, sh, st, ex);
  return (int)hipGetLastError();
}

template <typename T, int D>
int launch(const void* q, const void* k, const void* v, void* o, void* lse, int B, int Hq, int Hkv, int Tq, int Sk,
           float scale, int causal, const int64_t* so, const AttnExtra& ex, int exf, hipStream_t s) {
  switch (exf) {
    case 0: return launch_ex<T, D, 0>(q, k, v, o, lse, B, Hq, Hkv, Tq, Sk, scale, causal, so, ex, s);
    case kExMask: return launch_ex<T, D, kExMask>(q, k, v, o, lse, B, Hq, Hkv, Tq, Sk, scale, causal, so, ex, s);
    case kExDrop: return launch_ex<T, D, kExDrop>(q, k, v, o, lse, B, Hq, Hkv, Tq, Sk, scale, causal, so, ex, s);
    case kExMask | kExDrop:
      return launch_ex<T, D, kExMask | kExDrop>(q, k, v, o, lse, B, Hq, Hkv, Tq, Sk, scale, causal, so, ex, s);
  }
  return -1;
}

}  // namespace

LTA_EXPORT int lta_attn_fwd_d256(int dtype, const void* q, const void* k, const void* v, void* o, void* lse, int B,
                                 int Hq, int Hkv, int Tq, int Sk, int D, float scale, int causal,
                                 const int64_t* o_strides, const int64_t* qkv_strides, hipStream_t stream);

LTA_EXPORT int lta_attn_fwd_v4(int dtype, const void* q, const void* k, const void* v, void* o, void* lse, int B,
                               int Hq, int Hkv, int Tq, int Sk, int D, float scale, int causal,
                               const int64_t* o_strides, const int64_t* qkv_strides, int defer, hipStream_t stream);

// o_strides: optional int64[3] (batch, head, token) element strides of O (head dim contiguous);
// null = contiguous [B,H,T,D].  [B,T,H,D] storage lets the output projection read O without a copy.
// mask: optional fp32 additive mask [Bm][Hm][Tq][Skp] (Bm in {1,B}, Hm in {1,Hq}, Skp = Sk rounded up
// to 64, padding -inf); dropout_p > 0: counter-based dropout of P (seed, offset: the generator state).
// qkv_strides: optional int64[9] = (batch, head, token) element strides of Q, K, V (head dim
// contiguous, 16-byte aligned rows); null = contiguous [B,H,T,D].
LTA_EXPORT int lta_attn_fwd_ex2(int dtype, const void* q, const void* k, const void* v, void* o, void* lse, int B,
                                int Hq, int Hkv, int Tq, int Sk, int D, float scale, int causal,
                                const int64_t* o_strides, const void* mask, int mask_b, int mask_h, float dropout_p,
                                uint64_t seed, uint64_t offset, const int64_t* qkv_strides, hipStream_t stream) {
  const long long* rng = take_attn_rng();
  const AttnQ8 q8 = take_attn_q8();
  if (Hq % Hkv != 0 || dropout_p < 0.f || dropout_p >= 1.f) return -2;
  AttnExtra ex{};
  ex.sx = QKVStrides::from(qkv_strides, Hq, Hkv, Tq, Sk, D);
  int exf = 0;
  if (mask) {
    const int64_t skp = (int64_t)(Sk + 63) / 64 * 64;
    ex.mask = (const float*)mask;
    ex.mq = skp;
    ex.mh = mask_h ? (int64_t)Tq * skp : 0;
    ex.mb = mask_b ? (int64_t)(mask_h ? Hq : 1) * Tq * skp : 0;
    exf |= kExMask;
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
  if (D == 128 && exf == 0 && g_fwd_impl >= 9 && Tq > 0 && Sk > 0) {  // v4 (attention_fwd4.hip)
    const int defer = g_fwd_impl == 9 ? 0 : (g_fwd_impl == 10 ? 1 : 1 | ((g_fwd_impl - 10) << 1));
    if (q8.q != nullptr) {
      const int rc = attn_fwd_v4_q8(dtype, q, k, v, o, lse, B, Hq, Hkv, Tq, Sk, D, scale, causal, o_strides,
                                    qkv_strides, defer, &q8, stream);
      if (rc != -1) {
        g_attn_q8_used = rc == 0;
        return rc;
      }
    }
    const int rc = lta_attn_fwd_v4(dtype, q, k, v, o, lse, B, Hq, Hkv, Tq, Sk, D, scale, causal, o_strides,
                                   qkv_strides, defer, stream);
    if (rc != -1) return rc;
  }
  if (D == 256 && exf == 0 && g_fwd_ring) {  // LDS-DMA ring kernel (attention_fwd_d256.hip)
    const int rc = lta_attn_fwd_d256(dtype, q, k, v, o, lse, B, Hq, Hkv, Tq, Sk, D, scale, causal, o_strides,
                                     qkv_strides, stream);
    if (rc != -1) return rc;
  }
  if (dtype == kBF16) {
    if (D == 128) return launch<__hip_bfloat16, 128>(q, k, v, o, lse, B, Hq, Hkv, Tq, Sk, scale, causal, o_strides, ex, exf, stream);
    if (D == 64) return launch<__hip_bfloat16, 64>(q, k, v, o, lse, B, Hq, Hkv, Tq, Sk, scale, causal, o_strides, ex, exf, stream);
    if (D == 96) return launch<__hip_bfloat16, 96>(q, k, v, o, lse, B, Hq, Hkv, Tq, Sk, scale, causal, o_strides, ex, exf, stream);
    if (D == 256) return launch<__hip_bfloat16, 256>(q, k, v, o, lse, B, Hq, Hkv, Tq, Sk, scale, causal, o_strides, ex, exf, stream);
  } else if (dtype == kF16) {
    if (D == 128) return launch<__half, 128>(q, k, v, o, lse, B, Hq, Hkv, Tq, Sk, scale, causal, o_strides, ex, exf, stream);
    if (D == 64) return launch<__half, 64>(q, k, v, o, lse, B, Hq, Hkv, Tq, Sk, scale, causal, o_strides, ex, exf, stream);
    if (D == 96) return launch<__half, 96>(q, k, v, o, lse, B, Hq, Hkv, Tq, Sk, scale, causal, o_strides, ex, exf, stream);
    if (D == 256) return launch<__half, 256>(q, k, v, o, lse, B, Hq, Hkv, Tq, Sk, scale, causal, o_strides, ex, exf, stream);
  }
  return -1;
}

// graph-safe dropout: the device RNG state (int64 [seed, base]) the next lta_attn_fwd_ex2 / lta_attn_bwd_ex3
// call of this thread reads (its seed / offset arguments then relative to it)
LTA_EXPORT void lta_attn_set_rng_state(const void* state) { g_attn_rng = (const long long*)state; }

// FP8 side output (AttnQ8, attention.h) for the next lta_attn_fwd_ex2 call of this thread
LTA_EXPORT void lta_attn_set_fp8_out(void* q, const void* amax_in, float fmax, void* scale_out, void* amax_out) {
  g_attn_q8 = AttnQ8{(uint8_t*)q, (const float*)amax_in, fmax, (float*)scale_out, (float*)amax_out};
  g_attn_q8_used = 0;
}
// 1 when the last lta_attn_fwd_ex2 call of this thread wrote the requested FP8 side output (then cleared)
LTA_EXPORT int lta_attn_fp8_out_used() {
  const int u = g_attn_q8_used;
  g_attn_q8_used = 0;
  return u;
}

LTA_EXPORT int lta_attn_fwd_ex(int dtype, const void* q, const void* k, const void* v, void* o, void* lse, int B, int Hq,
                               int Hkv, int Tq, int Sk, int D, float scale, int causal, const int64_t* o_strides,
                               const void* mask, int mask_b, int mask_h, float dropout_p, uint64_t seed,
                               uint64_t offset, hipStream_t stream) {
  return lta_attn_fwd_ex2(dtype, q, k, v, o, lse, B, Hq, Hkv, Tq, Sk, D, scale, causal, o_strides, mask, mask_b, mask_h,
                          dropout_p, seed, offset, nullptr, stream);
}

LTA_EXPORT int lta_attn_fwd_s(int dtype, const void* q, const void* k, const void* v, void* o, void* lse, int B, int Hq,
                              int Hkv, int Tq, int Sk, int D, float scale, int causal, const int64_t* o_strides,
                              hipStream_t stream) {
  return lta_attn_fwd_ex(dtype, q, k, v, o, lse, B, Hq, Hkv, Tq, Sk, D, scale, causal, o_strides, nullptr, 0, 0, 0.f,
                         0, 0, stream);
}

LTA_EXPORT int lta_attn_fwd(int dtype, const void* q, const void* k, const void* v, void* o, void* lse, int B, int Hq,
                            int Hkv, int Tq, int Sk, int D, float scale, int causal, hipStream_t stream) {
  return lta_attn_fwd_s(dtype, q, k, v, o, lse, B, Hq, Hkv, Tq, Sk, D, scale, causal, nullptr, stream);
}

// forward kernel selection for D = 128 without mask / dropout (A/B measurement hook)
LTA_EXPORT int lta_attn_fwd_set_impl(int impl) {
  const int old = g_fwd_impl;
  if (impl >= 0 && impl <= 15) g_fwd_impl = impl;
  return old;
}

// D = 256 forward kernel selection (A/B measurement hook): 1 = LDS-DMA ring kernel, 0 = generic
LTA_EXPORT int lta_attn_fwd_set_ring(int on) {
  const int old = g_fwd_ring;
  if (on == 0 || on == 1) g_fwd_ring = on;
  return old;
}
