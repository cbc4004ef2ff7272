"""User HIP kernels registered as operators (reference parity:
``notebooks/extend_thunder_with_cuda_python.ipynb`` — an NVRTC kernel registered as a Thunder
operator, replacing a torch function and given a gradient)."""
import os
import struct

import pytest
import torch

import lightning_thunder_amd as thunder
from lightning_thunder_amd.core.proxies import TensorProxy
from lightning_thunder_amd.extend import OperatorExecutor
from lightning_thunder_amd.extend.hip_kernel import HipKernel, register_hip_kernel

LIB = os.path.join(os.path.dirname(thunder.__file__), "ops", "_lta_kernels.so")

SCALE_ADD = r"""
extern "C" __global__ void scale_add(const float* x, const float* y, float* out, float a, long n) {
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = a * x[i] + y[i];
}
"""

# y = x * sigmoid(x) in bf16 storage, fp32 math; TILE elements per thread (a define).
SILU = r"""
extern "C" __global__ void silu_bf16(const __hip_bfloat16* x, __hip_bfloat16* y, long n) {
  long base = ((long)blockIdx.x * blockDim.x + threadIdx.x) * TILE;
  #pragma unroll
  for (int j = 0; j < TILE; ++j) {
    long i = base + j;
    if (i < n) { float v = __bfloat162float(x[i]); y[i] = __float2bfloat16(v / (1.f + __expf(-v))); }
  }
}
extern "C" __global__ void silu_bwd_bf16(const __hip_bfloat16* x, const __hip_bfloat16* g, __hip_bfloat16* dx, long n) {
  long base = ((long)blockIdx.x * blockDim.x + threadIdx.x) * TILE;
  #pragma unroll
  for (int j = 0; j < TILE; ++j) {
    long i = base + j;
    if (i < n) {
      float v = __bfloat162float(x[i]), s = 1.f / (1.f + __expf(-v));
      dx[i] = __float2bfloat16(__bfloat162float(g[i]) * s * (1.f + v * (1.f - s)));
    }
  }
}
"""


def test_pack_natural_alignment():
    k = HipKernel(SCALE_ADD, "scale_add", ("ptr", "ptr", "ptr", "f32", "i64"))
    buf = k.pack(0x1000, None, 0x3000, 2.5, 7)
    assert len(buf) == 40  # 3 pointers, f32 at 24, i64 aligned up to 32
    assert struct.unpack_from("<QQQ", buf, 0) == (0x1000, 0, 0x3000)
    assert struct.unpack_from("<f", buf, 24)[0] == 2.5
    assert struct.unpack_from("<q", buf, 32)[0] == 7
    k2 = HipKernel("", "f", ("i32", "ptr", "i32"))
    assert len(k2.pack(1, 0, 2)) == 24  # the pointer aligns to 8, the struct rounds up to 8
    with pytest.raises(TypeError):
        k.pack(1, 2)
    with pytest.raises(ValueError):
        HipKernel("", "f", ("float",))


@pytest.mark.skipif(not os.path.exists(LIB), reason="native library not built")
def test_compiles_for_gfx950_without_gpu():
    k = HipKernel(SILU, "silu_bf16", ("ptr", "ptr", "i64"), defines={"TILE": 4})
    code = k.compile()
    assert code[:4] == b"\x7fELF" and len(code) > 500
    # a different define is a different code object
    assert HipKernel(SILU, "silu_bf16", ("ptr", "ptr", "i64"), defines={"TILE": 2}).compile() != code


def _silu_executor():
    fwd = HipKernel(SILU, "silu_bf16", ("ptr", "ptr", "i64"), defines={"TILE": 4})
    bwd = HipKernel(SILU, "silu_bwd_bf16", ("ptr", "ptr", "ptr", "i64"), defines={"TILE": 4})
    calls = []

    def silu_impl(x):
        x = x.contiguous()
        y = torch.empty_like(x)
        n = x.numel()
        fwd(((n + 1023) // 1024,), (256,), x, y, n)
        calls.append("fwd")
        return y

    def silu_bwd_impl(x, g):
        x, g = x.contiguous(), g.contiguous()
        dx = torch.empty_like(x)
        n = x.numel()
        bwd(((n + 1023) // 1024,), (256,), x, g, dx, n)
        calls.append("bwd")
        return dx

    ex = OperatorExecutor("user_hip_silu")
    silu_bwd = register_hip_kernel(ex, "user_silu_bwd", silu_bwd_impl, meta=lambda x, g: TensorProxy(like=x))

    def silu_vjp(x):
        y = silu(x)
        return y, lambda g: (silu_bwd(x, g),)

    silu = register_hip_kernel(ex, "user_silu", silu_impl, meta=lambda x: TensorProxy(like=x),
                               replaces=torch.nn.functional.silu,
                               checker=lambda x: x.dtype == thunder.dtypes.bfloat16, vjp=silu_vjp)
    return ex, calls


def test_registered_op_traces_and_replaces_torch_function():
    """Tracing only (CPU): the user operator replaces F.silu and owns the backward."""
    ex, _ = _silu_executor()

    def f(x):
        return torch.nn.functional.silu(x) * 2

    x = torch.randn(8, 16, dtype=torch.bfloat16, requires_grad=True)

    jf = thunder.jit(f, executors=[ex, *thunder.get_default_executors()])
    try:
        jf(x)
    except Exception:
        pass  # no GPU: the kernel launch fails, the traces exist
    fw = str(thunder.last_traces(jf)[-1])
    assert "user_silu" in fw


@pytest.mark.gpu
def test_user_hip_kernel_fwd_bwd_gpu():
    ex, calls = _silu_executor()

    def f(x):
        return torch.nn.functional.silu(x) * 2

    x = torch.randn(333, 129, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    jf = thunder.jit(f, executors=[ex, *thunder.get_default_executors()])
    out = jf(x)
    g = torch.randn_like(out)
    out.backward(g)
    assert "fwd" in calls and "bwd" in calls
    x64 = x.detach().double().requires_grad_()
    ref = f(x64)
    ref.backward(g.double())
    torch.testing.assert_close(out.double(), ref, atol=2e-2, rtol=2e-2)
    torch.testing.assert_close(x.grad.double(), x64.grad, atol=3e-2, rtol=3e-2)


@pytest.mark.gpu
def test_hip_kernel_direct_launch_gpu():
    k = HipKernel(SCALE_ADD, "scale_add", ("ptr", "ptr", "ptr", "f32", "i64"))
    x = torch.randn(100_003, device="cuda")
    y = torch.randn_like(x)
    out = torch.empty_like(x)
    k(((x.numel() + 255) // 256,), (256,), x, y, out, 1.5, x.numel())
    torch.testing.assert_close(out, 1.5 * x + y)
