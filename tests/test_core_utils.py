"""Trace utility layer (core/utils.py) and bound-symbol DAG utilities (core/dag.py).

Reference: thunder/core/utils.py (ProxyDict, producers, consumers, find_producer_symbols,
OrderedSet) and thunder/core/transforms.py (bsym_list_to_dag, toposort_bsym_dag,
insert_inplace, visitor_transform); tests modelled on thunder/tests/test_core.py.
"""
import torch

import lightning_thunder_amd as thunder
from lightning_thunder_amd.core import dag, prims
from lightning_thunder_amd.core import utils as U
from lightning_thunder_amd.core.prims import PrimIDs


def _trace():
    def f(a, b):
        c = a + b
        d = c.sin()
        e = a * 2.0
        return d + e, c

    jf = thunder.jit(f)
    jf(torch.randn(4), torch.randn(4))
    return thunder.last_traces(jf)[0]


def test_ordered_set():
    s = U.OrderedSet([3, 1, 3, 2])
    assert list(s) == [3, 1, 2]
    s.add(0)
    s.discard(1)
    assert list(s) == [3, 2, 0] and 2 in s and 1 not in s
    assert list(s | [5, 3]) == [3, 2, 0, 5]
    assert list(s - [2]) == [3, 0]
    assert list(s & [0, 3]) == [3, 0]


def test_frozen_dict_and_hashable():
    h = U.make_hashable({"a": [1, 2], "b": {"c": 3}})
    assert hash(h) == hash(U.make_hashable({"b": {"c": 3}, "a": [1, 2]}))
    assert U.is_hashable(h) and not U.is_hashable([1])


def test_producers_consumers_and_slice():
    tr = _trace()
    prod, cons = U.producers_and_consumers(tr)
    bs = tr.bound_symbols
    # every consumer list is in program order and every produced proxy maps to its producer
    for b in bs:
        for o in b.flat_proxy_outs:
            if o.name in prod:
                assert prod[o] is not None
    ret = bs[-1]
    out = ret.args[0][0] if isinstance(ret.args[0], (tuple, list)) else ret.args[0]
    sl = U.find_producer_symbols(tr, [out], stop_proxies=[])
    pos = [next(i for i, x in enumerate(bs) if x is b) for b in sl]
    assert pos == sorted(pos)  # program order
    assert any("sin" in b.sym.name for b in sl)
    # every consumer of an input reads it
    a = tr.args[0] if tr.args else None
    if a is not None and a in cons:
        assert all(any(x.name == a.name for x in c.flat_proxy_args) for c in cons[a])
    last = U.get_symbols_to_last_used_variables(bs, ignore=())
    assert sum(len(v) for v in last.values()) >= 3


def test_toposort_default_keeps_program_order_and_bottom_up():
    tr = _trace()
    bs = tr.bound_symbols
    _, _, nodes = dag.bsym_list_to_dag(bs)
    assert [b for b in dag.toposort_bsym_dag(nodes)] == list(bs)
    bu = dag.toposort_bsym_dag(nodes, dag.TOPOSORT_ORDER.BOTTOM_UP)
    pos = {id(b): i for i, b in enumerate(bu)}
    for n in nodes:
        for c in n.children:
            assert pos[id(n.bsym)] < pos[id(c.bsym)]


def test_toposort_selector_prefers_priority():
    tr = _trace()
    bs = [b for b in tr.bound_symbols if b.sym.id != PrimIDs.RETURN]
    # schedule multiplications as early as possible: the independent `a * 2` moves up
    out = dag.toposort_with_priority(bs, lambda n: 0 if "mul" in n.bsym.sym.name else 1)
    names = [b.sym.name for b in out]
    first_mul = min(i for i, n in enumerate(names) if "mul" in n)
    first_sin = min(i for i, n in enumerate(names) if "sin" in n)
    assert first_mul < first_sin
    _, _, nodes = dag.bsym_list_to_dag(bs)
    pos = {id(b): i for i, b in enumerate(out)}
    for n in nodes:
        for c in n.children:
            assert pos[id(n.bsym)] < pos[id(c.bsym)]


def test_visitor_transform_and_insert_inplace():
    tr = _trace()

    def visit(b):
        if b.sym.name == "sin":
            prims.cos(b.args[0])  # recorded after the sin
            return dag.VISIT_TYPE.INSERT_AFTER
        return dag.VISIT_TYPE.NO_OP

    new = dag.visitor_transform(tr, visit, provenance="test visitor")
    names = [b.sym.name for b in new.bound_symbols]
    i = names.index([n for n in names if "sin" in n][0])
    assert "cos" in names[i + 1]
    assert len(names) == len(tr.bound_symbols) + 1
    x = tr.bound_symbols[0].flat_proxy_outs[0] if tr.bound_symbols[0].flat_proxy_outs else None
    if x is not None:
        n0 = len(new.bound_symbols)
        dag.insert_inplace(new, 1, prims.neg, x)
        assert len(new.bound_symbols) == n0 + 1 and "neg" in new.bound_symbols[1].sym.name
