// Probe of gfx950's ds_read_b64_tr_b8 (transposing LDS read of 8-bit data): LDS byte (row R, column C)
// of a 256-B-pitch image holds (R & 15) << 4 | (C & 15); every lane passes the byte address given by
// the host and returns the 8 bytes it received.  scripts/exp/tr8_probe.py checks the lane mapping.
#include <hip/hip_runtime.h>

typedef int v2i __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) v2i lds_v2i;

__global__ void tr8_probe_kernel(const unsigned* addr_bytes, unsigned* out) {
  __shared__ __attribute__((aligned(16))) unsigned char s[8192];
  for (int i = threadIdx.x; i < 8192; i += 64) s[i] = (unsigned char)((((i >> 8) & 15) << 4) | (i & 15));
  __syncthreads();
  const unsigned a = addr_bytes[threadIdx.x];
  const v2i r = __builtin_amdgcn_ds_read_tr8_b64_v2i32((lds_v2i*)((__attribute__((address_space(3))) char*)s + a));
  out[2 * threadIdx.x] = (unsigned)r[0];
  out[2 * threadIdx.x + 1] = (unsigned)r[1];
}

extern "C" int tr8_probe(const unsigned* addr, unsigned* out, hipStream_t s) {
  hipLaunchKernelGGL(tr8_probe_kernel, dim3(1), dim3(64), 0, s, addr, out);
  return (int)hipGetLastError();
}
