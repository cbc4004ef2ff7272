// MXFP4 weight-only GEMV for decode: y[M, N] = x[M, K] . dequant(W)[N, K]^T with W packed e2m1
// [N, K/2] (low nibble = even k) and E8M0 scales S [N, K/32]; x / y bf16, M <= 8 rows.
//
// Decode is weight-streaming bound: the weight is read once per token, so 4-bit storage streams a
// quarter of the bf16 bytes.  Each lane owns whole 32-element blocks (16 weight bytes + 1 scale):
// one 16-B load, the gfx950 scaled conversion v_cvt_scalef32_pk_f32_fp4 (two scaled fp32 values
// per instruction, the E8M0 scale folded in) and fp32 FMAs against the block's x values, which
// every wave re-reads from L2/L1 (x is a few KB).  A wave computes NPW output columns so each x
// load feeds NPW weight rows (x bytes per weight byte = 4 / NPW); lanes of a wave walk consecutive blocks of the rows (1 KiB per
// wave-instruction, coalesced), and a butterfly reduces the 64 partial sums.
#include "common.h"

using namespace lta;

namespace {

typedef float f2 __attribute__((ext_vector_type(2)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

constexpr int WAVES = 4;   // waves per workgroup
constexpr int MAXM = 8;

__device__ __forceinline__ float e8m0_to_f32(uint32_t be) {
  return be == 0 ? __uint_as_float(0x00400000u) : __uint_as_float(be << 23);  // 2^(be - 127)
}

template <int M, int NPW>
__global__ __launch_bounds__(WAVES * 64) void gemv_mxfp4_kernel(const __hip_bfloat16* __restrict__ x,
                                                                 const uint8_t* __restrict__ w,
                                                                 const uint8_t* __restrict__ s,
                                                                 const __hip_bfloat16* __restrict__ bias,
                                                                 __hip_bfloat16* __restrict__ y, int N, int K, int ldx,
                                                                 int ldy) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int n0 = (blockIdx.x * WAVES + wave) * NPW;
  if (n0 >= N) return;  // whole waves only; no barrier below
  const int nb = K / 32;
  float acc[M][NPW];
#pragma unroll
  for (int m = 0; m < M; ++m)
#pragma unroll
    for (int j = 0; j < NPW; ++j) acc[m][j] = 0.f;

#pragma unroll 2
  for (int b = lane; b < nb; b += 64) {
    u32x4 wq[NPW];
    uint32_t se[NPW];
#pragma unroll
    for (int j = 0; j < NPW; ++j) {  // all loads of the iteration in flight together
      const int n = min(n0 + j, N - 1);
      wq[j] = *reinterpret_cast<const u32x4*>(w + (int64_t)n * (K / 2) + b * 16);
      se[j] = s[(int64_t)n * nb + b];
    }
#pragma unroll
    for (int m = 0; m < M; ++m) {
      // the block's 32 activations of row m (bf16 pairs), then every column's scaled conversion
      const __hip_bfloat16* xr = x + (int64_t)m * ldx + b * 32;
      float xf[32];
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const Vec16<__hip_bfloat16> xv = load16(xr + c * 8);
#pragma unroll
        for (int e = 0; e < 8; ++e) xf[c * 8 + e] = to_f32(xv.v[e]);
      }
#pragma unroll
      for (int j = 0; j < NPW; ++j) {
        const float sc = e8m0_to_f32(se[j]);
        const uint32_t d[4] = {wq[j].x, wq[j].y, wq[j].z, wq[j].w};
        float a = acc[m][j];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
#define LTA_CVT(BS)                                                       \
  {                                                                       \
    const f2 v = __builtin_amdgcn_cvt_scalef32_pk_f32_fp4(d[q], sc, BS);   \
    a = fmaf(xf[q * 8 + BS * 2], v.x, a);                                 \
    a = fmaf(xf[q * 8 + BS * 2 + 1], v.y, a);                             \
  }
          LTA_CVT(0) LTA_CVT(1) LTA_CVT(2) LTA_CVT(3)
#undef LTA_CVT
        }
        acc[m][j] = a;
      }
    }
  }
#pragma unroll
  for (int m = 0; m < M; ++m) {
#pragma unroll
    for (int j = 0; j < NPW; ++j) {
      const float v = wave_sum(acc[m][j]);
      if (lane == 0 && n0 + j < N) {
        const float bv = bias != nullptr ? to_f32(bias[n0 + j]) : 0.f;
        y[(int64_t)m * ldy + n0 + j] = __float2bfloat16(v + bv);
      }
    }
  }
}

}  // namespace

// x [M, K] bf16 (row stride ldx), w [N, K/2] packed e2m1, s [N, K/32] E8M0 -> y [M, N] bf16 (ldy).
LTA_EXPORT int lta_gemv_mxfp4(const void* x, const void* w, const void* s, const void* bias, void* y, int M, int N,
                              int K, int ldx, int ldy, hipStream_t stream) {
  if (M < 1 || M > MAXM || K % 32 || ldx % 8) return -2;
  if (reinterpret_cast<uintptr_t>(x) % 16) return -2;  // x is read with 16-B vector loads
  // columns per wave: 8 amortise each activation load over more weight rows (the kernel is
  // bound by L1 traffic otherwise); 4 keep enough workgroups in flight for narrow outputs
  const bool wide = N >= 8192;
  const int cols_per_wg = WAVES * (wide ? 8 : 4);
  dim3 grid((N + cols_per_wg - 1) / cols_per_wg), block(WAVES * 64);
#define LTA_G4(MM)                                                                                             \
  case MM:                                                                                                     \
    if (wide)                                                                                                  \
      hipLaunchKernelGGL((gemv_mxfp4_kernel<MM, 8>), grid, block, 0, stream, (const __hip_bfloat16*)x,          \
                         (const uint8_t*)w, (const uint8_t*)s, (const __hip_bfloat16*)bias, (__hip_bfloat16*)y, N, K, \
                         ldx, ldy);                                                                            \
    else                                                                                                       \
      hipLaunchKernelGGL((gemv_mxfp4_kernel<MM, 4>), grid, block, 0, stream, (const __hip_bfloat16*)x,          \
                         (const uint8_t*)w, (const uint8_t*)s, (const __hip_bfloat16*)bias, (__hip_bfloat16*)y, N, K, \
                         ldx, ldy);                                                                            \
    break;
  switch (M) {
    LTA_G4(1) LTA_G4(2) LTA_G4(3) LTA_G4(4) LTA_G4(5) LTA_G4(6) LTA_G4(7) LTA_G4(8)
  }
#undef LTA_G4
  return (int)hipGetLastError();
}
