"""Counter-based RNG (``uniform_philox``) and the RNG state of traced programs, on CPU.

Parity: the reference's ``thunder/tests/test_randomness.py`` (uniform_philox value range and dtype,
reproducibility from (seed, offset), distinct streams per offset / seed, RNG-state reproducibility
of jitted programs, a module with dropout matching itself under the same seed).  On the GPU the
same prim is a hipfuse Philox region (tests/test_hipfuse.py, tests/test_hipgraph.py).
"""
import pytest
import torch

import lightning_thunder_amd as thunder
from lightning_thunder_amd import torch as ltorch


def _philox(shape, seed, offset, dtype=torch.float32, lo=0.0, hi=1.0):
    return ltorch.uniform_philox(shape, lo, hi, device="cpu", dtype=dtype, seed=seed, offset=offset)


@pytest.mark.parametrize("dtype", [torch.float32, torch.float64, torch.bfloat16])
def test_uniform_philox_range_dtype_moments(dtype):
    jf = thunder.jit(lambda s, o: _philox((256, 129), s, o, dtype=dtype))
    u = jf(3, 0)
    assert u.shape == (256, 129) and u.dtype == dtype
    assert u.min().item() >= 0.0 and u.max().item() <= 1.0
    uf = u.double()
    assert abs(uf.mean().item() - 0.5) < 0.01
    assert abs(uf.var().item() - 1.0 / 12) < 0.005


def test_uniform_philox_bounds():
    jf = thunder.jit(lambda s, o: _philox((4096,), s, o, lo=-2.0, hi=3.0))
    u = jf(1, 0)
    assert u.min().item() >= -2.0 and u.max().item() <= 3.0
    assert abs(u.mean().item() - 0.5) < 0.1


def test_uniform_philox_reproducible_per_seed_and_offset():
    jf = thunder.jit(lambda s, o: _philox((64, 33), s, o))
    a, b = jf(7, 0), jf(7, 0)
    assert torch.equal(a, b)                 # (seed, offset) fixes the stream
    assert not torch.equal(a, jf(7, 4))      # another offset: another stream
    assert not torch.equal(a, jf(8, 0))      # another seed: another stream


def test_jitted_dropout_follows_the_global_seed():
    jg = thunder.jit(lambda x: torch.nn.functional.dropout(x, 0.5, training=True))
    x = torch.ones(1000, 100)
    torch.manual_seed(0)
    o1 = jg(x)
    torch.manual_seed(0)
    o2 = jg(x)
    o3 = jg(x)
    assert torch.equal(o1, o2)               # same seed -> same mask
    assert not torch.equal(o1, o3)           # the state advanced between calls
    assert set(o1.unique().tolist()) <= {0.0, 2.0}
    assert abs((o1 == 0).float().mean().item() - 0.5) < 0.01


def test_dropout_backward_reuses_the_forward_mask():
    jg = thunder.jit(lambda x: torch.nn.functional.dropout(x, 0.3, training=True) * 3.0)
    x = torch.randn(64, 64, dtype=torch.float64, requires_grad=True)
    out = jg(x)
    out.sum().backward()
    keep = out != 0
    expected = torch.where(keep, torch.full_like(x, 3.0 / 0.7), torch.zeros_like(x))
    torch.testing.assert_close(x.grad, expected)


def test_module_with_dropout_reproducible_under_seed():
    m = torch.nn.Sequential(torch.nn.Linear(16, 32), torch.nn.Dropout(0.25), torch.nn.Linear(32, 4))
    m.train()
    jm = thunder.jit(m)
    x = torch.randn(8, 16)
    torch.manual_seed(123)
    a = jm(x)
    torch.manual_seed(123)
    b = jm(x)
    torch.testing.assert_close(a, b, atol=0, rtol=0)
    m.eval()
    jm_eval = thunder.jit(m)
    torch.testing.assert_close(jm_eval(x), m(x))   # eval: dropout is the identity
