"""Gradient registration and functional transform APIs (reference ``thunder/core/transforms.py``:
``register_grad`` :620 with ``get_grad``/``put_grad``, ``vjp`` :3041, ``value_and_grad`` :3068)."""
import torch

import lightning_thunder_amd as thunder
from lightning_thunder_amd.core import prims
from lightning_thunder_amd.core.proxies import TensorProxy
from lightning_thunder_amd.core.transforms import get_grad, put_grad, register_grad, value_and_grad, vjp
from lightning_thunder_amd.extend import OperatorExecutor, register_executor


def _sincos_executor():
    ex = OperatorExecutor("test_joint_grad_ex")
    register_executor(ex)
    calls = {"fwd": 0}

    def impl(a, b):
        calls["fwd"] += 1
        return torch.sin(a) * b

    op = ex.register_operator("sin_mul", meta=lambda a, b: TensorProxy(like=a), fn=impl)

    def sin_mul_grad(a, b):
        # joint style: forward, then read the output's cotangent and put the inputs' gradients
        out = op(a, b)
        g = get_grad(out)
        put_grad(a, g * b * prims.cos(a))
        put_grad(b, g * prims.sin(a))
        return out

    register_grad(op, sin_mul_grad)
    return ex, op, calls


def test_register_grad_joint_style():
    ex, op, calls = _sincos_executor()

    def f(x, y):
        return op(x * 2, y).sum() * 3

    x = torch.randn(5, 7, requires_grad=True)
    y = torch.randn(5, 7, requires_grad=True)
    jf = thunder.jit(f, executors=[ex])
    out = jf(x, y)
    out.backward()
    xr, yr = x.detach().requires_grad_(), y.detach().requires_grad_()
    ref = (torch.sin(xr * 2) * yr).sum() * 3
    ref.backward()
    torch.testing.assert_close(out, ref)
    torch.testing.assert_close(x.grad, xr.grad)
    torch.testing.assert_close(y.grad, yr.grad)
    bw = str(thunder.last_backward_traces(jf)[-1])
    assert "cos" in bw  # the registered backward ran in the backward trace
    fw = str(thunder.last_traces(jf)[-1])
    assert "cos" not in fw  # and none of it leaked into the forward


def test_value_and_grad_and_vjp():
    def f(x, y):
        return (x * y).sin().sum()

    x, y = torch.randn(4, 3), torch.randn(4, 3)
    v, (gx, gy) = value_and_grad(f)(x, y)
    xr, yr = x.clone().requires_grad_(), y.clone().requires_grad_()
    r = f(xr, yr)
    r.backward()
    torch.testing.assert_close(v.detach(), r.detach())
    torch.testing.assert_close(gx, xr.grad)
    torch.testing.assert_close(gy, yr.grad)

    ct = torch.randn(4, 3)
    out, (g,) = vjp(lambda a: a.exp() * 2)((x,), (ct,))
    torch.testing.assert_close(g, x.exp() * 2 * ct)
    # non-differentiable primals get None
    out, grads = vjp(lambda a, n: a * n)((x, 3), (ct,))
    assert grads[1] is None
    torch.testing.assert_close(grads[0], ct * 3)
