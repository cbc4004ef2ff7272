"""Numerics of the hand-written HIP kernels vs plain PyTorch fp32 references (MI355X only)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

DT = [torch.bfloat16, torch.float16, torch.float32]
TOL = {torch.bfloat16: 2e-2, torch.float16: 2e-3, torch.float32: 1e-5}


@pytest.fixture(scope="module", autouse=True)
def _lib():
    from lightning_thunder_amd.ops import require

    require()


@pytest.mark.parametrize("dtype", DT)
@pytest.mark.parametrize("shape", [(4, 4096), (3, 7, 4096), (5, 1000), (2, 11008), (16, 64)])
def test_rmsnorm_fwd_bwd(dtype, shape):
    from lightning_thunder_amd.ops.rmsnorm import rms_norm_fwd, rms_norm_bwd

    torch.manual_seed(0)
    x = torch.randn(shape, device="cuda", dtype=dtype)
    w = torch.randn(shape[-1], device="cuda", dtype=dtype)
    dy = torch.randn(shape, device="cuda", dtype=dtype)
    eps = 1e-5
    y, rstd = rms_norm_fwd(x, w, eps)
    xf, wf = x.float().requires_grad_(True), w.float().requires_grad_(True)
    ref = xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps) * wf
    torch.testing.assert_close(y.float(), ref.detach(), atol=TOL[dtype] * 4, rtol=TOL[dtype])
    ref.backward(dy.float())
    dx, dw = rms_norm_bwd(dy, x, w, rstd)
    torch.testing.assert_close(dx.float(), xf.grad, atol=TOL[dtype] * 4, rtol=TOL[dtype] * 2)
    torch.testing.assert_close(dw.float(), wf.grad, atol=TOL[dtype] * shape[0] * 4, rtol=TOL[dtype] * 4)
