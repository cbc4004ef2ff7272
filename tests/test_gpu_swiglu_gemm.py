"""Fused SwiGLU GEMMs (csrc/gemm4.hip EPI 1 / 2) against fp32 PyTorch references.

gate-up forward: a = x W1^T, b = x W2^T, y = silu(a) b in one launch (B staged from two weights);
backward: g = dY W kept on chip, da = g b silu'(a), db = g silu(a) in the store pass.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _fused_on(monkeypatch):
    monkeypatch.setenv("LTA_FUSED_SWIGLU", "1")  # opt-in epilogues (ops/gemm.py _fused_swiglu_on)


def _rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


@pytest.mark.parametrize("M,K,Nh", [(512, 256, 384), (256, 512, 128), (1024, 384, 640)])
def test_gate_up_swiglu_vs_fp32(M, K, Nh):
    from lightning_thunder_amd.ops import gemm as G

    torch.manual_seed(0)
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    w1 = torch.randn(Nh, K, device="cuda", dtype=torch.bfloat16) / K ** 0.5
    w2 = torch.randn(Nh, K, device="cuda", dtype=torch.bfloat16) / K ** 0.5
    assert G.gate_up_supported(x, w1, w2)
    a, b, y = G.gate_up_swiglu(x, w1, w2)
    ar = x.float() @ w1.float().t()
    br = x.float() @ w2.float().t()
    yr = torch.nn.functional.silu(ar) * br
    assert _rel(a, ar) < 1e-2 and _rel(b, br) < 1e-2, (_rel(a, ar), _rel(b, br))
    assert _rel(y, yr) < 2e-2, _rel(y, yr)
    # y is computed from the bf16-rounded a, b exactly as the unfused swiglu kernel does
    yb = (torch.nn.functional.silu(a.float()) * b.float()).bfloat16()
    assert (y.float() - yb.float()).abs().max().item() <= 1e-2 * yb.float().abs().max().item()
    # y-only launch (inference) writes the same y
    _, _, y2 = G.gate_up_swiglu(x, w1, w2, need_ab=False)
    assert torch.equal(y, y2)


@pytest.mark.parametrize("M,K,N", [(512, 256, 768), (256, 384, 256)])
def test_matmul_swiglu_bwd_vs_fp32(M, K, N):
    from lightning_thunder_amd.ops import gemm as G

    torch.manual_seed(1)
    dy = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(K, N, device="cuda", dtype=torch.bfloat16) / K ** 0.5  # the proj weight [out, in] = [K, N]
    a = torch.randn(M, N, device="cuda", dtype=torch.bfloat16)
    b = torch.randn(M, N, device="cuda", dtype=torch.bfloat16)
    da, db = G.matmul_swiglu_bwd(dy, w, a, b)
    g = dy.float() @ w.float()
    s = torch.sigmoid(a.float())
    dar = g * b.float() * s * (1 + a.float() * (1 - s))
    dbr = g * a.float() * s
    assert _rel(da, dar) < 2e-2 and _rel(db, dbr) < 2e-2, (_rel(da, dar), _rel(db, dbr))
    # same as the unfused pair (dgrad GEMM, then the swiglu backward kernel)
    from lightning_thunder_amd.ops.fused import swiglu_bwd

    ua, ub = swiglu_bwd(G.matmul(dy, w), a, b)
    assert _rel(da, ua) < 1e-2 and _rel(db, ub) < 1e-2


@pytest.mark.parametrize("B,T,nh,ng,K", [(1, 512, 4, 4, 256), (2, 256, 4, 2, 384)])
def test_linear_qkv_rope_vs_fp32(B, T, nh, ng, K):
    """qkv projection with the RoPE split in the epilogue (EPI 3) vs fp32 projection + rotate-half."""
    from lightning_thunder_amd.ops import gemm as G
    from lightning_thunder_amd.ops.fused import qkv_rope_fwd

    torch.manual_seed(2)
    D = 128
    x = torch.randn(B, T, K, device="cuda", dtype=torch.bfloat16)
    w = torch.randn((nh + 2 * ng) * D, K, device="cuda", dtype=torch.bfloat16) / K ** 0.5
    pos = torch.arange(T + 16, device="cuda", dtype=torch.float32)
    inv = 1.0 / (10000 ** (torch.arange(0, D // 2, device="cuda", dtype=torch.float32) * 2 / D))
    ang = torch.outer(pos, inv).repeat(1, 2)
    cos, sin = ang.cos(), ang.sin()
    q, k, v = G.linear_qkv_rope(x, w, cos, sin, nh, ng, D, D)
    qkv = (x.float() @ w.float().t()).view(B, T, nh + 2 * ng, D).transpose(1, 2)
    qr, kr, vr = qkv[:, :nh], qkv[:, nh:nh + ng], qkv[:, nh + ng:]

    def rope(t):
        x1, x2 = t[..., :D // 2], t[..., D // 2:]
        return t * cos[:T] + torch.cat((-x2, x1), -1) * sin[:T]

    assert q.shape == (B, nh, T, D) and k.shape == (B, ng, T, D) and v.shape == (B, ng, T, D)
    assert _rel(q, rope(qr)) < 1e-2 and _rel(k, rope(kr)) < 1e-2 and _rel(v, vr) < 1e-2
    # bitwise the unfused pair's result (same GEMM, same rounding points as csrc/rope.hip)
    uq, uk, uv = qkv_rope_fwd(G.linear(x, w), cos, sin, nh, ng, D, D)
    assert torch.equal(v, uv)
    assert _rel(q, uq) < 1e-3 and _rel(k, uk) < 1e-3
