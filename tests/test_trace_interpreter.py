"""Trace interpreter, substitution processor and vjp_utils (parity: reference
``thunder/tests/test_interpreter.py`` trace-interpreter cases and ``test_grad.py`` vjp helpers)."""
import torch

import lightning_thunder_amd as thunder
from lightning_thunder_amd.core.proxies import TensorProxy
from lightning_thunder_amd.core.trace import TraceCtx, tracectx
from lightning_thunder_amd.core.trace_interpreter import (
    interpret_trace, interpret_trace_to_trace, TraceSubstitutionProcessor,
)
from lightning_thunder_amd.core.vjp_utils import (
    make_aug_forward_and_backward, get_saved_for_backward_tensors, set_saved_for_backward_tensors,
)


def _f(x, w):
    return torch.nn.functional.gelu(x @ w).sum()


def test_interpret_trace_concrete_and_to_trace():
    x, w = torch.randn(4, 8), torch.randn(8, 8)
    tr = thunder.trace(_f, x, w)
    torch.testing.assert_close(interpret_trace(tr, x, w), _f(x, w))
    t2 = interpret_trace_to_trace(tr, x, w)
    torch.testing.assert_close(interpret_trace(t2, x, w), _f(x, w))


def test_substitution_processor_replaces_symbol():
    x, w = torch.randn(4, 8), torch.randn(8, 8)
    tr = thunder.trace(_f, x, w)

    class GeluToRelu(TraceSubstitutionProcessor):
        def process_bsym(self, bsym):
            if bsym.sym.name == "gelu":
                self.set_result(self.add_bsyms_from_function(thunder.torch.relu, bsym.args[0]))
            else:
                self.add_processed_bsyms([bsym])
                self.set_result(bsym.output)

    nt, _ = GeluToRelu(tr)()
    assert any(b.sym.name == "relu" for b in nt.bound_symbols)
    torch.testing.assert_close(interpret_trace(nt, x, w), torch.relu(x @ w).sum())


def test_make_aug_forward_and_backward():
    x, w = torch.randn(4, 8), torch.randn(8, 8, requires_grad=True)
    tr = thunder.trace(_f, x, w)
    b = next(b for b in tr.bound_symbols if b.sym.name == "gelu")
    fw, bw = make_aug_forward_and_backward(b)
    t = TraceCtx(None)
    with tracectx(t):
        a = TensorProxy(like=b.args[0])
        out, saved = fw(a)
        grads = bw(*saved, TensorProxy(like=out))
    assert isinstance(out, TensorProxy) and out.shape == b.output.shape
    g = grads[0] if isinstance(grads, (tuple, list)) else grads
    assert isinstance(g, TensorProxy) and g.shape == a.shape
    # helpers on an augmented forward trace
    jf = thunder.jit(_f)
    jf(x, w)
    fwt = thunder.last_traces(jf)[-1]
    saved = get_saved_for_backward_tensors(fwt)
    set_saved_for_backward_tensors(fwt, saved)
    assert get_saved_for_backward_tensors(fwt) == saved
