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


@pytest.mark.parametrize("dtype", DT)
@pytest.mark.parametrize("nh,ng,hs,rope_n", [(4, 4, 64, 64), (8, 2, 128, 128), (4, 4, 64, 16)])
@pytest.mark.parametrize("cos_dtype", [torch.float32, None])
def test_qkv_rope(dtype, nh, ng, hs, rope_n, cos_dtype):
    from lightning_thunder_amd.ops.fused import qkv_rope_fwd, qkv_rope_bwd
    from lightning_thunder_amd.models.litgpt import qkv_split_rope, build_rope_cache

    torch.manual_seed(0)
    B, T = 2, 33
    cos, sin = build_rope_cache(T, rope_n, device="cuda")
    cd = cos_dtype or dtype
    cos, sin = cos.to(cd), sin.to(cd)
    qkv = torch.randn(B, T, (nh + 2 * ng) * hs, device="cuda", dtype=dtype)
    q, k, v = qkv_rope_fwd(qkv, cos, sin, nh, ng, hs, rope_n)
    x = qkv.float().requires_grad_(True)
    rq, rk, rv = qkv_split_rope(x, cos.float(), sin.float(), nh, ng, hs, rope_n)
    for a, b in ((q, rq), (k, rk), (v, rv)):
        torch.testing.assert_close(a.float(), b.detach(), atol=TOL[dtype] * 4, rtol=TOL[dtype])
    gq, gk, gv = (torch.randn_like(t) for t in (q, k, v))
    torch.autograd.backward((rq, rk, rv), (gq.float(), gk.float(), gv.float()))
    dqkv = qkv_rope_bwd(gq, gk, gv, cos, sin, nh, ng, hs, rope_n)
    torch.testing.assert_close(dqkv.float(), x.grad, atol=TOL[dtype] * 4, rtol=TOL[dtype])


@pytest.mark.parametrize("dtype", DT)
@pytest.mark.parametrize("n", [(4, 11008), (3, 5, 7)])
def test_swiglu(dtype, n):
    from lightning_thunder_amd.ops.fused import swiglu_fwd, swiglu_bwd

    torch.manual_seed(0)
    a = torch.randn(n, device="cuda", dtype=dtype)
    b = torch.randn(n, device="cuda", dtype=dtype)
    g = torch.randn(n, device="cuda", dtype=dtype)
    y = swiglu_fwd(a, b)
    af, bf = a.float().requires_grad_(True), b.float().requires_grad_(True)
    ref = torch.nn.functional.silu(af) * bf
    torch.testing.assert_close(y.float(), ref.detach(), atol=TOL[dtype] * 4, rtol=TOL[dtype])
    ref.backward(g.float())
    da, db = swiglu_bwd(g, a, b)
    torch.testing.assert_close(da.float(), af.grad, atol=TOL[dtype] * 4, rtol=TOL[dtype])
    torch.testing.assert_close(db.float(), bf.grad, atol=TOL[dtype] * 4, rtol=TOL[dtype])


@pytest.mark.parametrize("dtype", DT)
@pytest.mark.parametrize("rows,V", [(64, 32000), (7, 1000), (16, 1003)])
@pytest.mark.parametrize("reduction", ["mean", "sum", "none"])
@pytest.mark.parametrize("ls", [0.0, 0.1])
def test_cross_entropy(dtype, rows, V, reduction, ls):
    from lightning_thunder_amd.ops.fused import cross_entropy_fwd, cross_entropy_bwd

    torch.manual_seed(0)
    x = torch.randn(rows, V, device="cuda", dtype=dtype) * 3
    t = torch.randint(0, V, (rows,), device="cuda")
    t[1] = -100
    loss, lse, stats = cross_entropy_fwd(x, t, -100, reduction, ls)
    xf = x.float().requires_grad_(True)
    ref = torch.nn.functional.cross_entropy(xf, t, ignore_index=-100, reduction=reduction, label_smoothing=ls)
    torch.testing.assert_close(loss.float(), ref.detach().to(dtype).float(), atol=TOL[dtype] * 8, rtol=TOL[dtype] * 2)
    g = torch.randn_like(ref)
    ref.backward(g)
    dl = cross_entropy_bwd(g.to(dtype), x, t, lse, stats, -100, reduction, ls)
    torch.testing.assert_close(dl.float(), xf.grad, atol=TOL[dtype] * 2, rtol=TOL[dtype] * 4)
