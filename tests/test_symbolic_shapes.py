"""cache="symbolic values" with symbolic tensor dims (ports of the reference's
thunder/tests/test_jit_general.py:1533-1625 plus model-level checks).  The design is in
lightning_thunder_amd/core/symbolic.py."""
import pytest
import torch
from torch.testing import assert_close

import lightning_thunder_amd as thunder
from lightning_thunder_amd.core import prims
from lightning_thunder_amd.core.proxies import IntegerProxy
from lightning_thunder_amd.core.symbolic import SymInt


def test_cache_symbolic_values_dynamic_shape():
    def foo(a):
        return a.relu()

    jfoo = thunder.jit(foo, cache="symbolic values")
    a = torch.randn((2, 2, 2))
    assert_close(jfoo(a), foo(a))
    assert thunder.cache_misses(jfoo) == 1
    assert thunder.cache_hits(jfoo) == 0
    a = torch.randn((3, 4, 5))
    assert_close(jfoo(a), foo(a))
    assert thunder.cache_misses(jfoo) == 1
    assert thunder.cache_hits(jfoo) == 1


def test_cache_symbolic_values_reshape_numel():
    def foo(a):
        a = torch.reshape(a, [a.numel()])
        return a.relu()

    jfoo = thunder.jit(foo, cache="symbolic values")
    a = torch.randn(2, 3, 8, requires_grad=True)
    assert_close(jfoo(a), foo(a))
    # the reshape target is printed as the product of the dims: a new size reuses the program
    b = torch.randn(4, 5, 6, requires_grad=True)
    assert_close(jfoo(b), foo(b))
    assert thunder.cache_misses(jfoo) == 1 and thunder.cache_hits(jfoo) == 1


def test_cache_symbolic_values_slice():
    def foo(a):
        a = a[..., : a.shape[-1]]
        return a.relu()

    jfoo = thunder.jit(foo, cache="symbolic values")
    a = torch.randn(2, 3, 8, requires_grad=True)
    assert_close(jfoo(a), foo(a))
    b = torch.randn(2, 3, 9, requires_grad=True)
    assert_close(jfoo(b), foo(b))


def test_cache_symbolic_values_dict():
    def foo(a, v):
        return a[v].relu()

    jfoo = thunder.jit(foo, cache="symbolic values")
    a = {
        2: torch.randn(2, 3, 8, requires_grad=True),
        5: torch.randn(4, 8, requires_grad=True),
    }
    assert_close(jfoo(a, 2), foo(a, 2))
    b = {
        "a": torch.randn(2, 8, requires_grad=True),
        "b": torch.randn(7, requires_grad=True),
    }
    assert_close(jfoo(b, "b"), foo(b, "b"))


def test_cache_symbolic_values_nn_parameter_static_shape():
    linear = torch.nn.Linear(2, 2)
    x = torch.randn(2, 2)
    jlinear = thunder.jit(linear, cache="symbolic values")
    jlinear(x)
    comp = thunder.last_traces(jlinear)[0]
    by_name = {a.name: a for a in comp.args}
    params = [a for n, a in by_name.items() if "weight" in n or "bias" in n]
    assert params and all(not any(isinstance(s, SymInt) for s in p.shape) for p in params)
    inputs = [a for n, a in by_name.items() if "weight" not in n and "bias" not in n]
    assert inputs and all(isinstance(s, SymInt) for s in inputs[0].shape)


def test_symbolic_guards_broadcasting_specializes_size_one():
    """A dim that is 1 at trace time stays static (broadcasting semantics depend on it), so a call where
    it is not 1 misses the cache and retraces instead of broadcasting wrongly."""

    def foo(a, b):
        return a + b

    jfoo = thunder.jit(foo, cache="symbolic values")
    a, b = torch.randn(4, 1), torch.randn(4, 5)
    assert_close(jfoo(a, b), foo(a, b))
    a, b = torch.randn(6, 1), torch.randn(6, 3)
    assert_close(jfoo(a, b), foo(a, b))
    assert thunder.cache_misses(jfoo) == 1
    a, b = torch.randn(6, 3), torch.randn(6, 3)
    assert_close(jfoo(a, b), foo(a, b))
    assert thunder.cache_misses(jfoo) == 2


def test_symbolic_guards_equal_dims():
    """Two dims compared equal while tracing (matmul's inner dims) must stay equal: a call where they
    differ is a cache miss that raises the shape error of eager PyTorch."""

    def foo(a, b):
        return a @ b

    jfoo = thunder.jit(foo, cache="symbolic values")
    x, w = torch.randn(3, 4), torch.randn(4, 5)
    assert_close(jfoo(x, w), x @ w)
    x, w = torch.randn(7, 6), torch.randn(6, 2)
    assert_close(jfoo(x, w), x @ w)
    assert thunder.cache_misses(jfoo) == 1
    with pytest.raises(Exception):
        jfoo(torch.randn(3, 4), torch.randn(5, 2))


def test_symbolic_values_training_one_entry():
    """Forward + backward of an MLP over three batch sizes through one cache entry."""
    torch.manual_seed(0)
    m = torch.nn.Sequential(torch.nn.Linear(8, 16), torch.nn.GELU(), torch.nn.Linear(16, 4))
    jm = thunder.jit(m, cache="symbolic values")
    for n in (3, 5, 9):
        x = torch.randn(n, 8)
        out = jm(x)
        ref = m(x)
        assert_close(out, ref)
        g = torch.randn_like(ref)
        out.backward(g)
        got = [p.grad.clone() for p in m.parameters()]
        m.zero_grad()
        ref.backward(g)
        for a, p in zip(got, m.parameters()):
            assert_close(a, p.grad)
        m.zero_grad()
    assert thunder.cache_misses(jm) == 1 and thunder.cache_hits(jm) == 2


def _rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["llama2-like", "llama3-like"])
def test_symbolic_litgpt_three_lengths_one_entry_gpu(name):
    """A small LitGPT (bf16, HIP executors) trains at three sequence lengths through ONE cache entry:
    no re-trace and no new generated / hiprtc-compiled kernel after the first length; at every length
    the forward and every parameter gradient are as close to an fp32 eager reference as bf16 eager is
    (3x band, as tests/test_gpu_models.py)."""
    from lightning_thunder_amd.executors import hipfuse
    from lightning_thunder_amd.models.litgpt import GPT, init_weights

    torch.manual_seed(0)
    dev = torch.device("cuda")
    m32 = GPT.from_name(name).to(device=dev)
    init_weights(m32)
    m32.set_rope_cache(512, device=dev)
    m = GPT.from_name(name).to(device=dev)
    m.load_state_dict(m32.state_dict())
    m = m.to(torch.bfloat16)
    m.set_rope_cache(512, device=dev)
    jm = thunder.jit(m, cache="symbolic values")
    counts = None
    # lengths with the same residues the claim rules test (token rows % 256 for the hand GEMMs): one
    # program; a length with another residue is a guarded cache miss, not a wrong kernel
    for T in (128, 256, 384):
        x = torch.randint(0, 320, (2, T), device=dev)
        out = jm(x)
        eager = m(x)
        ref = m32(x)
        base = max(_rel(eager, ref), 1e-6)
        assert _rel(out, ref) <= 3 * base + 1e-5, (T, _rel(out, ref), base)
        g = torch.randn_like(ref)
        out.backward(g.to(torch.bfloat16))
        got = {n: p.grad.float().clone() for n, p in m.named_parameters()}
        m.zero_grad()
        eager.backward(g.to(torch.bfloat16))
        eg = {n: p.grad.float().clone() for n, p in m.named_parameters()}
        m.zero_grad()
        ref.backward(g)
        for n, p in m32.named_parameters():
            b = max(_rel(eg[n], p.grad), 1e-6)
            e = _rel(got[n], p.grad)
            assert e <= 3 * b + 1e-5, (T, n, e, b)
        m32.zero_grad()
        if counts is None:
            counts = dict(hipfuse.RTC_STATS)
    assert thunder.cache_misses(jm) == 1 and thunder.cache_hits(jm) == 2
    assert hipfuse.RTC_STATS == counts, (hipfuse.RTC_STATS, counts)
    src = str(thunder.last_traces(jm)[-1])
    assert "hip_" in src, src  # the HIP kernels (GEMM, attention, norms) serve every length
