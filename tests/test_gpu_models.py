"""End-to-end compiled LitGPT-style models on the GPU vs eager (reference analogue: test_networks.py)."""
import pytest
import torch

import lightning_thunder_amd as thunder
from lightning_thunder_amd.models.litgpt import GPT, init_weights

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


@pytest.mark.parametrize("name", ["llama2-like", "llama3-like", "gpt-neox-like", "gemma-like"])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_litgpt_fwd_bwd_gpu(name, dtype):
    """Compiled model vs an fp32 eager reference (bf16 runs must be as accurate as bf16 eager, up to 3x)."""
    torch.manual_seed(0)
    dev = torch.device("cuda")
    m32 = GPT.from_name(name).to(device=dev)
    init_weights(m32)
    m32.set_rope_cache(64, device=dev)
    m = GPT.from_name(name).to(device=dev)
    m.load_state_dict(m32.state_dict())
    m = m.to(dtype)
    m.set_rope_cache(64, device=dev)
    idx = torch.randint(0, 320, (2, 64), device=dev)
    tm = thunder.jit(m)
    out = tm(idx)
    ref32 = m32(idx)
    eager = m(idx)
    g = torch.randn_like(ref32)
    base_fwd = max(_rel(eager, ref32), 1e-6)
    assert _rel(out, ref32) <= 3 * base_fwd + 1e-5, (_rel(out, ref32), base_fwd)
    out.backward(g.to(dtype))
    got = {n: p.grad.clone() for n, p in m.named_parameters()}
    for p in m.parameters():
        p.grad = None
    eager.backward(g.to(dtype))
    eg = {n: p.grad.clone() for n, p in m.named_parameters()}
    ref32.backward(g)
    for n, p in m32.named_parameters():
        base = max(_rel(eg[n], p.grad), 1e-6)
        err = _rel(got[n], p.grad)
        assert err <= 3 * base + 1e-5, (n, err, base)
    src = str(thunder.last_traces(tm)[-1])
    if name not in ("gpt-neox-like", "gemma-like"):
        assert "hip_rms_norm_fwd" in src and "hip_qkv_rope" in src and "hip_swiglu" in src
    if name == "gemma-like" and dtype == torch.bfloat16:  # head_size 256: the D = 256 attention kernels in a model
        assert "hip_rms_norm_fwd" in src and "hip_flash_attn" in src, src


def test_train_step_with_fused_loss_gpu():
    torch.manual_seed(0)
    dev = torch.device("cuda")
    m = GPT.from_name("llama2-like").to(device=dev, dtype=torch.bfloat16)
    init_weights(m)
    m.set_rope_cache(64, device=dev)
    V = m.config.padded_vocab_size

    class TS(torch.nn.Module):
        def __init__(self, m):
            super().__init__()
            self.m = m

        def forward(self, x, y):
            return torch.nn.functional.cross_entropy(self.m(x).reshape(-1, V), y.reshape(-1))

    ts = TS(m)
    tm = thunder.jit(ts)
    x = torch.randint(0, 320, (2, 64), device=dev)
    y = torch.randint(0, 320, (2, 64), device=dev)
    loss = tm(x, y)
    loss.backward()
    got = {n: p.grad.float().clone() for n, p in m.named_parameters()}
    for p in m.parameters():
        p.grad = None
    ref = ts(x, y)
    ref.backward()
    torch.testing.assert_close(loss.float(), ref.float(), atol=2e-2, rtol=2e-2)
    for n, p in m.named_parameters():
        torch.testing.assert_close(got[n], p.grad.float(), atol=5e-2, rtol=5e-2, msg=n)
    assert "hip_cross_entropy_fwd" in str(thunder.last_traces(tm)[-1])


@pytest.mark.gpu
def test_hip_linear_residual_epilogue_fusion():
    import lightning_thunder_amd as thunder
    from lightning_thunder_amd.executors.hipex import hip_linear

    torch.manual_seed(0)

    class M(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.fc = torch.nn.Linear(512, 1024, bias=False)
            self.proj = torch.nn.Linear(1024, 512, bias=True)

        def forward(self, x):
            return self.proj(torch.nn.functional.gelu(self.fc(x))) + x

    m = M().cuda().bfloat16()
    x = torch.randn(2, 128, 512, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    jm = thunder.jit(m)
    out = jm(x)
    ref = m(x)
    torch.testing.assert_close(out, ref, rtol=2e-2, atol=2e-2)
    tr = thunder.last_traces(jm)[-1]
    lin = [b for b in tr.bound_symbols if b.sym is hip_linear]
    assert len(lin) == 2
    assert any(len(b.args) > 3 and b.args[3] is not None for b in lin), "residual add not fused into the GEMM"
    g = torch.randn_like(out)
    (gx,) = torch.autograd.grad(out, (x,), g)
    (rx,) = torch.autograd.grad(ref, (x,), g)
    torch.testing.assert_close(gx, rx, rtol=2e-2, atol=2e-2)


@pytest.mark.gpu
def test_grouped_mm_kernel():
    from lightning_thunder_amd.ops.gemm import grouped_mm, grouped_nt_supported

    torch.manual_seed(0)
    G, M, K, N = 5, 900, 256, 512
    a = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(G, N, K, device="cuda", dtype=torch.bfloat16) / 16
    ends = torch.tensor([0, 37, 300, 300, 900], device="cuda", dtype=torch.int32)  # an empty group too
    b = w.transpose(1, 2)
    assert grouped_nt_supported(a, b, ends)
    out = grouped_mm(a, b, ends)
    starts = [0] + ends.tolist()[:-1]
    ref = torch.zeros(M, N, device="cuda")
    for g, (s, e) in enumerate(zip(starts, ends.tolist())):
        ref[s:e] = a[s:e].float() @ w[g].float().t()
    torch.testing.assert_close(out.float(), ref, rtol=2e-2, atol=5e-2)


@pytest.mark.gpu
def test_moe_model_fp32_matches_eager():
    torch.manual_seed(0)
    dev = torch.device("cuda")
    m = GPT.from_name("mixtral-like").to(device=dev)
    m.set_rope_cache(64, device=dev)
    idx = torch.randint(0, 320, (2, 64), device=dev)
    tm = thunder.jit(m)
    out = tm(idx)
    ref = m(idx)
    torch.testing.assert_close(out, ref, rtol=1e-4, atol=1e-4)
    g = torch.randn_like(out)
    gj = torch.autograd.grad(out, list(m.parameters()), g)
    gr = torch.autograd.grad(ref, list(m.parameters()), g)
    for a, b in zip(gj, gr):
        torch.testing.assert_close(a, b, rtol=1e-3, atol=1e-4)


@pytest.mark.gpu
def test_moe_model_bf16_uses_grouped_kernel():
    torch.manual_seed(0)
    dev = torch.device("cuda")
    m = GPT.from_name("mixtral-like").to(device=dev, dtype=torch.bfloat16)
    m.set_rope_cache(64, device=dev)
    idx = torch.randint(0, 320, (2, 64), device=dev)
    tm = thunder.jit(m)
    out = tm(idx)
    assert torch.isfinite(out).all()
    out.float().sum().backward()
    assert all(p.grad is not None and torch.isfinite(p.grad).all() for p in m.parameters())
    assert "hip_grouped_mm" in str(thunder.last_traces(tm)[-1])
