// Hardware-behaviour probes run by tests on the GPU (not on any hot path).
//
// lta_probe_lds_dma_oob: what an out-of-range lane of an LDS-DMA load (buffer_load_dwordx4 ... lds)
// writes into LDS.  One wave DMAs 64 x 16 B from a buffer whose descriptor covers only the first
// `valid_bytes` (voffset = 16 * lane); LDS is pre-filled with 0xA5 bytes; the 1 KiB LDS image is
// copied out.  The grouped wgrad GEMM relies on out-of-range rows arriving as zeros.
#include "common.h"

namespace {

typedef int i32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(64) void probe_lds_dma_oob_kernel(const uint4* __restrict__ src, uint4* __restrict__ out,
                                                              int valid_bytes) {
  __shared__ __attribute__((aligned(1024))) uint4 img[64];
  const int lane = threadIdx.x;
  img[lane] = make_uint4(0xA5A5A5A5u, 0xA5A5A5A5u, 0xA5A5A5A5u, 0xA5A5A5A5u);
  __syncthreads();
  const uint64_t a = (uint64_t)(uintptr_t)src;
  const i32x4 rsrc = i32x4{(int)(uint32_t)a, (int)((uint32_t)(a >> 32) & 0xffffu), valid_bytes, 0x00020000};
  const uint32_t dst = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint4*)img;
  const int voff = lane * 16;
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds\n\ts_waitcnt vmcnt(0)"
               :
               : "s"(dst), "v"(voff), "s"(rsrc)
               : "memory", "m0");
  __syncthreads();
  out[lane] = img[lane];
}

}  // namespace

LTA_EXPORT int lta_probe_lds_dma_oob(const void* src, void* out, int valid_bytes, hipStream_t s) {
  hipLaunchKernelGGL(probe_lds_dma_oob_kernel, dim3(1), dim3(64), 0, s, (const uint4*)src, (uint4*)out, valid_bytes);
  return (int)hipGetLastError();
}

// lta_cu_occupy: n_wg workgroups that each hold a CU slot for `ticks` of the 100 MHz real-time
// counter, then exit (every wave reaches the exit: bounded by the counter, no flags).  Used to
// emulate the workgroups an overlapped RCCL collective keeps resident (one per channel) while the
// compute stream runs: `lds_bytes` of dynamic LDS and `threads` per workgroup set how much of a CU
// each one takes (an RCCL channel workgroup's shape is read from a kernel trace), so the GEMMs'
// one-tile-per-CU waves can be timed with 0 / 8 / 16 / 32 CUs taken (scripts/cu_contention.py).
namespace {

__global__ __launch_bounds__(1024) void cu_occupy_kernel(uint64_t ticks, int lds_bytes) {
  extern __shared__ char lds_hold[];
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
  if (ticks == 0 && (int)threadIdx.x < lds_bytes) lds_hold[threadIdx.x] = 0;  // keeps the LDS allocation referenced
}

}  // namespace

LTA_EXPORT int lta_cu_occupy(int n_wg, int threads, int lds_bytes, uint64_t ticks, hipStream_t s) {
  if (n_wg <= 0 || threads <= 0 || threads > 1024 || lds_bytes < 0 || lds_bytes > 160 * 1024) return -1;
  if (lds_bytes > 64 * 1024)
    hipFuncSetAttribute((const void*)cu_occupy_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, lds_bytes);
  hipLaunchKernelGGL(cu_occupy_kernel, dim3(n_wg), dim3(threads), lds_bytes, s, ticks, lds_bytes);
  return (int)hipGetLastError();
}
