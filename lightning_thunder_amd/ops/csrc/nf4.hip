// K9: NF4 (4-bit NormalFloat, block-wise absmax) weight dequantisation for CDNA4.
// (reference: bitsandbytes dequantize_4bit behind thunder/transforms/quantization.py:19-44)
//
// Packed layout (bitsandbytes-compatible): byte i holds element 2i in its high nibble and
// element 2i+1 in its low nibble; absmax[b] scales block b of `blocksize` elements.
// One lane turns 8 packed bytes (16 weights) into two 16-byte bf16/fp16 stores; the 16-entry
// code book lives in registers (LDS would serialise the lookups on bank conflicts).
#include "common.h"

using namespace lta;

namespace {

template <typename T>
__global__ __launch_bounds__(256) void nf4_dequant_kernel(const uint8_t* __restrict__ q, const float* __restrict__ absmax,
                                                         const float* __restrict__ code, T* __restrict__ out, int64_t n,
                                                         int blocksize) {
  float cb[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) cb[i] = code[i];
  const int64_t nchunks = n / 16;
  for (int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; c < nchunks; c += (int64_t)gridDim.x * blockDim.x) {
    const uint2 p = *reinterpret_cast<const uint2*>(q + c * 8);
    const float s = absmax[(c * 16) / blocksize];
    Vec16<T> o0, o1;
    const uint32_t w[2] = {p.x, p.y};
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      const uint32_t byte = (w[b >> 2] >> (8 * (b & 3))) & 0xffu;
      const float hi = cb[byte >> 4] * s, lo = cb[byte & 15u] * s;
      T* dst = (b < 4) ? o0.v : o1.v;
      const int j = (b & 3) * 2;
      dst[j] = from_f32<T>(hi);
      dst[j + 1] = from_f32<T>(lo);
    }
    store16(out + c * 16, o0);
    store16(out + c * 16 + 8, o1);
  }
}

}  // namespace

LTA_EXPORT int lta_nf4_dequant(int dtype, const void* q, const void* absmax, const void* code, void* out, int64_t n,
                               int blocksize, hipStream_t stream) {
  if (n % 16 != 0 || blocksize % 16 != 0) return -2;
  const int64_t chunks = n / 16;
  const unsigned grid = (unsigned)std::min<int64_t>((chunks + 255) / 256, 8192);
  if (dtype == kBF16)
    hipLaunchKernelGGL(nf4_dequant_kernel<__hip_bfloat16>, dim3(grid), dim3(256), 0, stream, (const uint8_t*)q,
                       (const float*)absmax, (const float*)code, (__hip_bfloat16*)out, n, blocksize);
  else if (dtype == kF16)
    hipLaunchKernelGGL(nf4_dequant_kernel<__half>, dim3(grid), dim3(256), 0, stream, (const uint8_t*)q,
                       (const float*)absmax, (const float*)code, (__half*)out, n, blocksize);
  else
    return -1;
  return (int)hipGetLastError();
}
