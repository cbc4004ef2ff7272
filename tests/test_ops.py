"""OpInfo-driven operator tests (reference: ``thunder/tests/test_ops.py`` ``test_core_vs_torch_consistency``
and ``thunder/tests/test_grad.py`` ``test_vjp_correctness``).

* consistency: ``jit(op)`` vs eager torch, per op x dtype, on CPU (torch executor claims) and on
  the MI355X (``@pytest.mark.gpu``: the HIP executors — hipex kernels and the hipfuse code
  generator — claim what they support);
* gradients: the compiled VJP against a float64 central finite difference of the eager op,
  ``<v, J u>`` computed both ways.
"""
import pytest
import torch

import lightning_thunder_amd as thunder
from opinfos import OPS, OpInfo

TOL = {torch.float32: (1e-5, 1.3e-6), torch.bfloat16: (2e-2, 1.6e-2), torch.float16: (2e-3, 1e-3),
       torch.float64: (1e-7, 1e-7)}


def _compare(a, b, opinfo: OpInfo, dtype):
    fa, _ = torch.utils._pytree.tree_flatten(a)
    fb, _ = torch.utils._pytree.tree_flatten(b)
    assert len(fa) == len(fb)
    for x, y in zip(fa, fb):
        if isinstance(x, torch.Tensor):
            assert isinstance(y, torch.Tensor)
            assert x.shape == y.shape, (x.shape, y.shape)
            assert x.dtype == y.dtype, (x.dtype, y.dtype)
            if x.dtype.is_floating_point:
                atol, rtol = TOL.get(dtype, (1e-5, 1e-5))
                if opinfo.atol is not None and dtype != torch.float32:
                    atol, rtol = max(atol, opinfo.atol), max(rtol, opinfo.rtol)
                torch.testing.assert_close(x, y, atol=atol, rtol=rtol, equal_nan=True)
            else:
                assert torch.equal(x.cpu(), y.cpu())
        else:
            assert x == y


def _cases(device):
    out = []
    for o in OPS:
        for dt in o.dtypes:
            if device == "cpu" and dt == torch.float16 and not o.differentiable:
                continue
            out.append(pytest.param(o, dt, id=f"{o.name}-{str(dt).split('.')[-1]}"))
    return out


def _run_consistency(opinfo: OpInfo, dtype, device):
    torch.manual_seed(1234)
    jfn = thunder.jit(opinfo.op)
    n = 0
    for sample in opinfo.samples(device, dtype, False):
        expected = opinfo.op(*sample.args, **sample.kwargs)
        got = jfn(*sample.args, **sample.kwargs)
        _compare(got, expected, opinfo, dtype)
        n += 1
    assert n > 0


@pytest.mark.parametrize("opinfo,dtype", _cases("cpu"))
def test_core_vs_torch_consistency(opinfo, dtype):
    _run_consistency(opinfo, dtype, "cpu")


@pytest.mark.gpu
@pytest.mark.parametrize("opinfo,dtype", _cases("cuda"))
def test_core_vs_torch_consistency_gpu(opinfo, dtype):
    if opinfo.skip_gpu:
        pytest.skip("not supported on the GPU path")
    _run_consistency(opinfo, dtype, "cuda")


# ---------------------------------------------------------------------------------------------
# VJP correctness against finite differences (float64)
# ---------------------------------------------------------------------------------------------
def _float_outputs(out):
    flat, _ = torch.utils._pytree.tree_flatten(out)
    return [o for o in flat if isinstance(o, torch.Tensor) and o.dtype.is_floating_point]


def _check_vjp(opinfo: OpInfo, sample, eps=1e-6):
    args, kwargs = sample.args, sample.kwargs
    flat, spec = torch.utils._pytree.tree_flatten((args, kwargs))
    diff_pos = [i for i, x in enumerate(flat) if isinstance(x, torch.Tensor) and x.dtype.is_floating_point]
    if not diff_pos:
        return False

    def call(vals):
        a, k = torch.utils._pytree.tree_unflatten(vals, spec)
        return a, k

    inputs = [flat[i].detach().clone().requires_grad_(True) for i in diff_pos]
    dirs = [torch.randn_like(x) for x in inputs]
    vals = list(flat)
    for i, x in zip(diff_pos, inputs):
        vals[i] = x
    a, k = call(vals)
    jfn = thunder.jit(opinfo.op)
    out = _float_outputs(jfn(*a, **k))
    if not out:
        return False
    cot = [torch.randn_like(o) for o in out]
    grads = torch.autograd.grad(out, inputs, cot, allow_unused=True)
    analytic = sum((g * u).sum() for g, u in zip(grads, dirs) if g is not None)

    def f_at(sign):
        v2 = list(flat)
        for i, x, u in zip(diff_pos, inputs, dirs):
            v2[i] = (x.detach() + sign * eps * u)
        a2, k2 = call(v2)
        return _float_outputs(opinfo.op(*a2, **k2))

    plus, minus = f_at(1.0), f_at(-1.0)
    numeric = sum(((p - m) / (2 * eps) * c).sum() for p, m, c in zip(plus, minus, cot))
    torch.testing.assert_close(analytic.detach(), numeric.detach(), atol=max(opinfo.grad_atol, 1e-5), rtol=1e-4)
    return True


@pytest.mark.parametrize("opinfo", [pytest.param(o, id=o.name) for o in OPS if o.differentiable])
def test_vjp_correctness(opinfo):
    torch.manual_seed(0)
    checked = 0
    for sample in opinfo.samples("cpu", torch.float64, False):
        checked += _check_vjp(opinfo, sample)
    assert checked > 0


@pytest.fixture
def hipfuse_on_cpu():
    from lightning_thunder_amd.executors import hipfuse

    old = hipfuse.ex.allow_cpu
    hipfuse.ex.allow_cpu = True
    yield
    hipfuse.ex.allow_cpu = old


@pytest.mark.parametrize("opinfo,dtype", [pytest.param(o, dt, id=f"{o.name}-{str(dt).split('.')[-1]}")
                                          for o in OPS for dt in (torch.float32, torch.bfloat16) if dt in o.dtypes])
def test_hipfuse_partition_consistency(opinfo, dtype, hipfuse_on_cpu):
    """The hipfuse fusion pass (partitioning, index maps) on every op; regions run through the
    torch reference path on the CPU, so partition bugs surface without a GPU."""
    torch.manual_seed(1234)
    jfn = thunder.jit(opinfo.op, executors=["hipfuse", "torch"])
    for requires_grad in ((False, True) if opinfo.differentiable else (False,)):
        for sample in opinfo.samples("cpu", dtype, requires_grad):
            expected = opinfo.op(*sample.args, **sample.kwargs)
            got = jfn(*sample.args, **sample.kwargs)
            _compare(got, expected, opinfo, dtype)


@pytest.mark.skipif(not __import__("os").path.exists("/opt/rocm/lib/libhiprtc.so"), reason="needs ROCm hiprtc")
@pytest.mark.parametrize("opinfo", [pytest.param(o, id=o.name) for o in OPS if torch.float32 in o.dtypes])
def test_hipfuse_codegen_cpu(opinfo):
    """Every op through the hipfuse partitioner on CPU (regions run by the reference path, checked
    against eager) with each region's generated HIP kernel compiled by hiprtc for gfx950 — the
    GPU-side codegen checked without a GPU."""
    from lightning_thunder_amd.executors import hipfuse

    old = hipfuse.ex.allow_cpu
    hipfuse.ex.allow_cpu = True
    try:
        torch.manual_seed(1234)
        jfn = thunder.jit(opinfo.op, executors=["hipfuse", "torch"])
        for sample in opinfo.samples("cpu", torch.float32, False):
            expected = opinfo.op(*sample.args, **sample.kwargs)
            got = jfn(*sample.args, **sample.kwargs)
            _compare(got, expected, opinfo, torch.float32)
            hipfuse.precompile(thunder.last_traces(jfn)[-1])
    finally:
        hipfuse.ex.allow_cpu = old
