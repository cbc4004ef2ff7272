"""Trace pattern matching (reference thunder/core/patterns.py semantics: matchers with context
updates, repetition ranges, non-connected (reorderable) steps, bind_names)."""
import torch

import lightning_thunder_amd as thunder
from lightning_thunder_amd.core.patterns import Pattern, bind_names, numbered_ancestors


def _trace(fn, *args):
    jf = thunder.jit(fn)
    jf(*args)
    return thunder.last_traces(jf)[0]


def _is(name):
    return lambda b: b.sym.name == name


def test_chain_with_context_and_bind_names():
    def f(x, w, b):
        return torch.relu(torch.nn.functional.linear(x, w) + b)

    tr = _trace(f, torch.randn(2, 3), torch.randn(4, 3), torch.randn(4))
    def is_linear(b):
        if b.sym.name != "linear":
            return False
        names = bind_names(b)
        return True, {"weight": names.get("weight", names.get("w", b.args[1]))}

    p = (Pattern()
         .match(is_linear)
         .match(lambda b: b.sym.name in ("add", "torch_add"),
                lambda prev, b, ctx: ctx["weight"] is prev[0].args[1])
         .match(_is("relu")))
    m = p(tr)
    assert len(m) == 1 and [b.sym.name for _, b in m[0]][0] == "linear" and len(m[0]) == 3
    assert p.contexts[0]["weight"].shape == (4, 3)


def test_repetition_ranges():
    def f(x):
        return torch.exp(torch.sin(torch.sin(torch.sin(x))))

    tr = _trace(f, torch.randn(5))
    m = Pattern().match(_is("sin"), min_times=1, max_times=-1).match(_is("exp"))(tr)
    assert len(m) == 1 and [b.sym.name for _, b in m[0]] == ["sin", "sin", "sin", "exp"]
    m = Pattern().match(_is("sin"), min_times=1, max_times=2)(tr)
    assert [len(x) for x in m] == [2, 1]  # greedy, non-overlapping
    # min_times larger than what is there: no match
    assert Pattern().match(_is("sin"), min_times=4, max_times=5)(tr) == []
    # an optional step (min_times=0) may be skipped
    def g(x):
        return torch.exp(torch.cos(x))

    tr2 = _trace(g, torch.randn(5))
    m = Pattern().match(_is("cos")).match(_is("sin"), min_times=0).match(_is("exp"))(tr2)
    assert len(m) == 1 and [b.sym.name for _, b in m[0]] == ["cos", "exp"]


def test_non_connected_step_matches_sibling_linears():
    """Two linears reading the same input (a horizontal-fusion candidate) are not dataflow
    connected: ``connected=False`` matches the second one."""
    def f(x, w1, w2):
        a = torch.nn.functional.linear(x, w1)
        b = torch.nn.functional.linear(x, w2)
        return a * b

    tr = _trace(f, torch.randn(2, 3), torch.randn(4, 3), torch.randn(4, 3))
    assert Pattern().match(_is("linear")).match(_is("linear"))(tr) == []
    m = Pattern().match(_is("linear")).match(
        _is("linear"), lambda prev, b: b.args[0] is prev[0].args[0], connected=False)(tr)
    assert len(m) == 1 and len(m[0]) == 2


def test_skipped_consumer_blocks_match():
    """A symbol between the matched ones that consumes the partial match blocks it (the group could
    not be replaced at its last member's position)."""
    def f(x):
        a = torch.sin(x)
        c = torch.cos(a)  # consumes the partial match
        b = torch.exp(torch.tanh(x))  # independent
        return torch.exp(a) + c + b

    tr = _trace(f, torch.randn(5))
    anc = numbered_ancestors(tr)
    assert len(anc) == len(tr.bound_symbols)
    m = Pattern().match(_is("sin")).match(_is("exp"))(tr)
    assert m == []  # sin -> exp(a) has cos(a) in between
    m = Pattern().match(_is("tanh")).match(_is("exp"))(tr)
    assert len(m) == 1
