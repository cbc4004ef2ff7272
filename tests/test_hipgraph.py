"""HipGraphTransform tests (reference: ``thunder/tests/test_transforms.py`` CUDAGraph tests)."""
import pytest
import torch

import lightning_thunder_amd as thunder
from lightning_thunder_amd.transforms.hipgraph import HipGraphTransform, default_capturable


def test_region_structure_cpu():
    """Regions are formed (with a permissive capturability predicate on CPU) and run eagerly."""
    from lightning_thunder_amd.transforms import hipgraph as hg

    t = HipGraphTransform(is_capturable=lambda b: b.sym.id not in hg._NOT_CAPTURABLE_IDS and not hg._is_unpack(b))
    m = torch.nn.Sequential(torch.nn.Linear(8, 16), torch.nn.ReLU(), torch.nn.Linear(16, 4))
    jm = thunder.jit(m, transforms=[t])
    x = torch.randn(3, 8)
    y = jm(x)
    torch.testing.assert_close(y, m(x))
    y.sum().backward()
    fw = thunder.last_traces(jm)[-1]
    bw = thunder.last_backward_traces(jm)[-1]
    assert any(b.sym.name.startswith("HipGraph") for b in fw.bound_symbols)
    assert any(b.sym.name.startswith("HipGraph") for b in bw.bound_symbols)


def test_cpu_ops_not_capturable():
    m = torch.nn.Linear(4, 4)
    jm = thunder.jit(m, transforms=[HipGraphTransform()])
    jm(torch.randn(2, 4))
    assert not any(b.sym.name.startswith("HipGraph") for b in thunder.last_traces(jm)[-1].bound_symbols)


@pytest.mark.gpu
def test_hipgraph_training_matches_eager_gpu():
    torch.manual_seed(0)

    def make():
        torch.manual_seed(0)
        return torch.nn.Sequential(torch.nn.Linear(64, 256), torch.nn.GELU(), torch.nn.Linear(256, 64)).cuda()

    m_ref, m_g = make(), make()
    t = HipGraphTransform()
    jm = thunder.jit(m_g, transforms=[t])
    opt_r = torch.optim.SGD(m_ref.parameters(), lr=0.1)
    opt_g = torch.optim.SGD(m_g.parameters(), lr=0.1)
    for step in range(5):
        x = torch.randn(32, 64, device="cuda")
        lr = m_ref(x).square().mean()
        lg = jm(x).square().mean()
        lr.backward()
        lg.backward()
        opt_r.step(); opt_r.zero_grad(set_to_none=True)
        opt_g.step(); opt_g.zero_grad(set_to_none=True)
        torch.testing.assert_close(lg, lr, rtol=1e-4, atol=1e-5)
    for pr, pg in zip(m_ref.parameters(), m_g.parameters()):
        torch.testing.assert_close(pg, pr, rtol=1e-4, atol=1e-5)
    assert sum(r.replays for r in t.runners) >= 4
    assert sum(r.captures for r in t.runners) >= 2


@pytest.mark.gpu
def test_hipgraph_with_hip_kernels_gpu():
    """A LitGPT block step (HIP attention / RMSNorm / RoPE / SwiGLU kernels) replays correctly."""
    from lightning_thunder_amd.models.litgpt import GPT, Config

    torch.manual_seed(0)
    cfg = Config.from_name("llama2-like", n_layer=2)
    m = GPT(cfg).cuda().to(torch.bfloat16)
    m.set_rope_cache(128, device="cuda")
    t = HipGraphTransform()
    jm = thunder.jit(m, transforms=[t])
    jplain = thunder.jit(m)
    for _ in range(3):
        x = torch.randint(0, cfg.vocab_size, (2, 128), device="cuda")
        out = jm(x)
        ref = jplain(x)
        torch.testing.assert_close(out, ref)
        out.float().sum().backward()
    assert sum(r.replays for r in t.runners) >= 1
