"""Trace utility layer: proxy-keyed maps, producer/consumer analysis, ordered sets.

Parity: reference ``thunder/core/utils.py`` (``OrderedSet`` :712-786, ``ProxyDict`` :966-1014,
``producers`` / ``consumers`` / ``producers_and_consumers`` :1016-1092, ``find_producer_symbols``
:1094-1156, ``get_symbols_to_last_used_variables`` :1158-1192, ``safe_map`` / ``safe_zip`` /
``partition`` / ``make_hashable``).  Passes that need def-use information (remat, fusion,
distributed scheduling, the DAG utilities in :mod:`core.dag`) build it here once instead of
re-deriving it ad hoc.
"""
from __future__ import annotations

from collections.abc import Hashable, Iterable, Iterator, Mapping, MutableSet, Sequence
from typing import Any, Callable

from .proxies import Proxy
from .pytree import tree_flatten


class OrderedSet(MutableSet):
    """A set that iterates in insertion order (a dict with None values underneath)."""

    __slots__ = ("_d",)

    def __init__(self, items: Iterable = ()):
        self._d: dict = dict.fromkeys(items)

    def __contains__(self, x) -> bool:
        return x in self._d

    def __iter__(self) -> Iterator:
        return iter(self._d)

    def __len__(self) -> int:
        return len(self._d)

    def __repr__(self) -> str:
        return f"OrderedSet({list(self._d)})"

    def add(self, x) -> None:
        self._d[x] = None

    def discard(self, x) -> None:
        self._d.pop(x, None)

    def update(self, *its: Iterable) -> None:
        for it in its:
            for x in it:
                self._d[x] = None

    def union(self, *its: Iterable) -> "OrderedSet":
        r = OrderedSet(self)
        r.update(*its)
        return r

    def intersection(self, other: Iterable) -> "OrderedSet":
        o = set(other)
        return OrderedSet(x for x in self if x in o)

    def difference(self, other: Iterable) -> "OrderedSet":
        o = set(other)
        return OrderedSet(x for x in self if x not in o)

    __or__ = union
    __and__ = intersection
    __sub__ = difference


class FrozenDict(Mapping):
    """An immutable, hashable mapping (used for hashable kwargs in cache keys)."""

    __slots__ = ("_d", "_h")

    def __init__(self, *args, **kwargs):
        self._d = dict(*args, **kwargs)
        self._h = None

    def __getitem__(self, k):
        return self._d[k]

    def __iter__(self):
        return iter(self._d)

    def __len__(self):
        return len(self._d)

    def __hash__(self):
        if self._h is None:
            self._h = hash(tuple(sorted((hash(k), hash(v)) for k, v in self._d.items())))
        return self._h

    def __repr__(self):
        return f"FrozenDict({self._d})"


def make_hashable(x: Any):
    """Tuples for sequences, FrozenDict for dicts, recursively; other values unchanged."""
    if isinstance(x, dict):
        return FrozenDict({k: make_hashable(v) for k, v in x.items()})
    if isinstance(x, (list, tuple)):
        return tuple(make_hashable(v) for v in x)
    return x


def is_hashable(x: Any) -> bool:
    try:
        hash(x)
    except TypeError:
        return False
    return isinstance(x, Hashable)


def safe_zip(*args):
    """zip that raises on length mismatch."""
    lens = {len(a) for a in args}
    if len(lens) > 1:
        raise ValueError(f"safe_zip: lengths differ {[len(a) for a in args]}")
    return zip(*args)


def safe_map(f: Callable, *args) -> list:
    return [f(*xs) for xs in safe_zip(*args)]


def partition(pred: Callable, iterable: Iterable) -> tuple[list, list]:
    """(items where pred is False, items where pred is True)."""
    f, t = [], []
    for x in iterable:
        (t if pred(x) else f).append(x)
    return f, t


def unzip2(pairs: Iterable) -> tuple[tuple, tuple]:
    a, b = [], []
    for x, y in pairs:
        a.append(x)
        b.append(y)
    return tuple(a), tuple(b)


class ProxyDict:
    """Dict keyed by proxies (by NAME: two proxy objects with one name are one key)."""

    __slots__ = ("_d",)

    def __init__(self):
        self._d: dict[str, Any] = {}

    @staticmethod
    def _k(p) -> str:
        if isinstance(p, Proxy):
            return p.name
        if isinstance(p, str):
            return p
        raise TypeError(f"ProxyDict keys are proxies, got {type(p).__name__}")

    def __setitem__(self, p, v) -> None:
        self._d[self._k(p)] = v

    def __getitem__(self, p):
        return self._d[self._k(p)]

    def __contains__(self, p) -> bool:
        return isinstance(p, (Proxy, str)) and self._k(p) in self._d

    def __len__(self) -> int:
        return len(self._d)

    def get(self, p, default=None):
        return self._d.get(self._k(p), default)

    def get_by_name(self, name: str, default=None):
        return self._d.get(name, default)

    def append(self, p, v) -> None:
        """Append ``v`` to the list stored under ``p`` (creating it)."""
        self._d.setdefault(self._k(p), []).append(v)

    def remove(self, p, v) -> None:
        self._d[self._k(p)].remove(v)

    def keys(self):
        return self._d.keys()

    def items(self):
        return self._d.items()

    def __repr__(self) -> str:
        return f"ProxyDict({self._d})"


def _bsyms(trace_or_bsyms) -> Sequence:
    return trace_or_bsyms.bound_symbols if hasattr(trace_or_bsyms, "bound_symbols") else trace_or_bsyms


def _flat_proxies(x) -> list:
    return [p for p in tree_flatten(x)[0] if isinstance(p, Proxy)]


def producers(trace_or_bsyms, *, _map_to_numbers: bool = False) -> ProxyDict:
    """proxy -> the bound symbol (or its index, ``_map_to_numbers``) that FIRST produces it.  Trace
    inputs (unpacked by the prologue) have no producer entry unless a bound symbol outputs them."""
    pd = ProxyDict()
    for i, b in enumerate(_bsyms(trace_or_bsyms)):
        args = {a.name for a in _flat_proxies((b.args, b.kwargs))}
        for o in _flat_proxies(b.output):
            if o.name in pd or o.name in args:  # in-place / pass-through outputs keep their producer
                continue
            pd[o] = i if _map_to_numbers else b
    return pd


def consumers(trace_or_bsyms, *, _map_to_numbers: bool = False) -> ProxyDict:
    """proxy -> list of the bound symbols (or indices) that read it, in program order."""
    cd = ProxyDict()
    for i, b in enumerate(_bsyms(trace_or_bsyms)):
        seen = set()
        for a in _flat_proxies((b.args, b.kwargs)):
            if a.name in seen:
                continue
            seen.add(a.name)
            cd.append(a, i if _map_to_numbers else b)
    return cd


def producers_and_consumers(trace_or_bsyms) -> tuple[ProxyDict, ProxyDict]:
    return producers(trace_or_bsyms), consumers(trace_or_bsyms)


def find_producer_symbols(trace, proxies: Sequence[Proxy], stop_proxies: Sequence[Proxy] = ()) -> tuple:
    """The bound symbols (in program order) needed to compute ``proxies`` from ``stop_proxies`` and
    the trace inputs: a backward slice over the def-use graph."""
    bsyms = _bsyms(trace)
    prod = producers(bsyms, _map_to_numbers=True)
    stop = {p.name for p in stop_proxies}
    need: set[int] = set()
    work = [p.name for p in proxies if isinstance(p, Proxy)]
    seen: set[str] = set()
    while work:
        n = work.pop()
        if n in seen or n in stop:
            continue
        seen.add(n)
        i = prod.get_by_name(n)
        if i is None or i in need:
            continue
        need.add(i)
        work.extend(a.name for a in _flat_proxies((bsyms[i].args, bsyms[i].kwargs)))
    return tuple(bsyms[i] for i in sorted(need))


def get_symbols_to_last_used_variables(symbols: Sequence, ignore: Iterable = ()) -> dict:
    """bound symbol -> tuple of the proxies whose LAST use is that symbol (what ``del`` frees after it)."""
    ignore = {p.name if isinstance(p, Proxy) else p for p in ignore}
    last: dict[str, int] = {}
    objs: dict[str, Proxy] = {}
    for i, b in enumerate(symbols):
        for p in _flat_proxies((b.args, b.kwargs)) + _flat_proxies(b.output):
            if p.name in ignore:
                continue
            last[p.name] = i
            objs[p.name] = p
    out: dict = {id(b): [] for b in symbols}
    for n, i in last.items():
        out[id(symbols[i])].append(objs[n])
    return {b: tuple(out[id(b)]) for b in symbols}
