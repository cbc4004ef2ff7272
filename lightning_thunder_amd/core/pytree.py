"""Minimal, dependency-free pytree (parity: reference ``thunder/core/pytree.py:17-135``, which uses optree).

Containers: tuple, list, dict (incl. OrderedDict/defaultdict), namedtuple and
dataclass instances.  ``torch.Size``, slices and proxies are leaves.
"""
from __future__ import annotations

import dataclasses
from collections import OrderedDict
from typing import Any, Callable

import torch


class TreeSpec:
    __slots__ = ("kind", "ctx", "children")

    def __init__(self, kind: str, ctx: Any, children: list["TreeSpec"]):
        self.kind = kind
        self.ctx = ctx
        self.children = children

    @property
    def num_leaves(self) -> int:
        if self.kind == "leaf":
            return 1
        return sum(c.num_leaves for c in self.children)

    def __eq__(self, other):
        return (
            isinstance(other, TreeSpec)
            and self.kind == other.kind
            and self.ctx == other.ctx
            and self.children == other.children
        )

    def __hash__(self):
        return hash((self.kind, repr(self.ctx), tuple(self.children)))

    def __repr__(self):
        if self.kind == "leaf":
            return "*"
        return f"{self.kind}({self.ctx}, {self.children})"


LEAF = TreeSpec("leaf", None, [])


def _is_namedtuple(x) -> bool:
    return isinstance(x, tuple) and hasattr(type(x), "_fields") and type(x) is not tuple


# exact types that are always leaves: checked first, so flattening a call's arguments (every
# compiled call does it) costs one set lookup per tensor / number
_FAST_LEAF = frozenset({torch.Tensor, torch.nn.Parameter, int, float, bool, str, type(None), torch.dtype,
                        torch.device})


def tree_flatten(tree, is_leaf: Callable | None = None) -> tuple[list, TreeSpec]:
    leaves: list = []

    def rec(x) -> TreeSpec:
        t = type(x)
        if is_leaf is None:
            if t in _FAST_LEAF:
                leaves.append(x)
                return LEAF
            if t is tuple:
                return TreeSpec("tuple", None, [rec(v) for v in x])
            if t is list:
                return TreeSpec("list", None, [rec(v) for v in x])
        elif is_leaf(x):
            leaves.append(x)
            return LEAF
        if isinstance(x, torch.Size):
            leaves.append(x)
            return LEAF
        if _is_namedtuple(x):
            return TreeSpec("namedtuple", type(x), [rec(v) for v in x])
        if isinstance(x, tuple) and hasattr(type(x), "n_fields"):  # torch.return_types structseqs
            return TreeSpec("structseq", type(x), [rec(v) for v in x])
        if t is tuple:
            return TreeSpec("tuple", None, [rec(v) for v in x])
        if t is list:
            return TreeSpec("list", None, [rec(v) for v in x])
        if t is dict:
            keys = list(x)
            return TreeSpec("dict", (dict, tuple(keys)), [rec(x[k]) for k in keys])
        if isinstance(x, dict):
            keys = list(x.keys())
            # a dataclass that subclasses dict (diffusers / HF model outputs): fields that are not
            # (yet) keys travel as extra children so the rebuilt object has every attribute
            extra = ()
            if dataclasses.is_dataclass(x) and not isinstance(x, type):
                extra = tuple(f.name for f in dataclasses.fields(x) if f.name not in x)
            ctx = (type(x), tuple(keys)) if not extra else (type(x), tuple(keys), extra)
            return TreeSpec("dict", ctx, [rec(x[k]) for k in keys] + [rec(getattr(x, f, None)) for f in extra])
        if dataclasses.is_dataclass(x) and not isinstance(x, type):
            fields = [f.name for f in dataclasses.fields(x)]
            return TreeSpec("dataclass", (type(x), tuple(fields)), [rec(getattr(x, f)) for f in fields])
        leaves.append(x)
        return LEAF

    spec = rec(tree)
    return leaves, spec


def tree_unflatten(leaves, spec: TreeSpec):
    it = iter(leaves)

    def rec(s: TreeSpec):
        if s.kind == "leaf":
            return next(it)
        vals = [rec(c) for c in s.children]
        if s.kind == "tuple":
            return tuple(vals)
        if s.kind == "list":
            return vals
        if s.kind == "namedtuple":
            return s.ctx(*vals)
        if s.kind == "structseq":
            return s.ctx(vals)
        if s.kind == "dict":
            typ, keys = s.ctx[0], s.ctx[1]
            extra = s.ctx[2] if len(s.ctx) > 2 else ()
            extra_vals = dict(zip(extra, vals[len(keys):]))
            vals = vals[:len(keys)]
            d = OrderedDict(zip(keys, vals)) if typ is OrderedDict else dict(zip(keys, vals))
            if typ not in (dict, OrderedDict):
                if dataclasses.is_dataclass(typ):  # e.g. transformers ModelOutput (OrderedDict + dataclass)
                    try:
                        return typ(**d, **extra_vals)
                    except Exception:
                        pass
                try:
                    nd = typ.__new__(typ)
                    dict.__init__(nd)
                    nd.update(d)
                    for f, v in extra_vals.items():
                        object.__setattr__(nd, f, v)
                    return nd
                except Exception:
                    return d
            return d
        if s.kind == "dataclass":
            typ, fields = s.ctx
            obj = object.__new__(typ)
            for f, v in zip(fields, vals):
                object.__setattr__(obj, f, v)
            return obj
        raise ValueError(s.kind)

    out = rec(spec)
    return out


def tree_map(fn: Callable, tree, is_leaf: Callable | None = None):
    leaves, spec = tree_flatten(tree, is_leaf=is_leaf)
    return tree_unflatten([fn(x) for x in leaves], spec)


def tree_iter(tree):
    leaves, _ = tree_flatten(tree)
    return iter(leaves)
