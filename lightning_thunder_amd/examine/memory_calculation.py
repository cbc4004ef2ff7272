"""Static memory estimate of an execution trace (reference: ``thunder/examine/memory_calculation.py``).

Walks the bound symbols in program order with a model of the caching allocator's view of the
program: every tensor output that is not an alias starts a new allocation of ``numel * itemsize``
bytes; outputs of view-like symbols (reshape / transpose / slice / broadcast / squeeze ... of a
live tensor) share their source's storage; an allocation is released when the last name that
refers to it is ``del``-ed.  Returns the peak and, optionally, the live bytes after every symbol
(the memory timeline).  Inputs are counted as live from the start (the reference does the same:
arguments are held by the caller).
"""
from __future__ import annotations

from ..core.prims import PrimIDs, OpTags
from ..core.proxies import TensorProxy

_VIEW_IDS = {PrimIDs.TRANSPOSE, PrimIDs.RESHAPE, PrimIDs.BROADCAST_IN_DIM, PrimIDs.SQUEEZE, PrimIDs.SLICE}
_VIEW_NAMES = {"transpose", "reshape", "view", "expand", "broadcast", "broadcast_in_dim", "squeeze", "unsqueeze",
               "slice", "permute", "t", "getitem", "split", "chunk", "as_strided", "narrow", "flatten", "view_as",
               "expand_as", "unflatten", "movedim", "swapaxes", "diagonal"}


def is_view_bsym(b) -> bool:
    """True when the outputs of ``b`` may alias its first tensor input (no new allocation)."""
    if b.sym.id in _VIEW_IDS or OpTags.SHAPE_OP in (b.sym.tags or ()):
        return True
    nm = str(b.sym.name)
    base = nm[:-5] if nm.endswith("_prim") else nm
    return base in _VIEW_NAMES


def _nbytes(p: TensorProxy) -> int:
    n = p.numel
    return int(n) * p.dtype.itemsize if isinstance(n, int) else 0


def get_alloc_memory(trace, *, timeline: bool = False):
    """Peak bytes of live tensor storage while executing ``trace``.

    Returns ``(peak, live)`` where ``live`` maps one name per storage alive at the end to its bytes;
    with ``timeline=True`` a third element lists ``(bound symbol name, live bytes after it)``.
    """
    storage_of: dict[str, int] = {}   # tensor name -> storage id
    size: dict[int, int] = {}         # storage id -> bytes
    refs: dict[int, int] = {}         # storage id -> number of live names
    nxt = 0
    cur = 0

    def alloc(name, nbytes):
        nonlocal nxt, cur
        sid = nxt
        nxt += 1
        storage_of[name] = sid
        size[sid] = nbytes
        refs[sid] = 1
        cur += nbytes

    def alias(name, src):
        sid = storage_of[src]
        storage_of[name] = sid
        refs[sid] += 1

    def release(name):
        nonlocal cur
        sid = storage_of.pop(name, None)
        if sid is None:
            return
        refs[sid] -= 1
        if refs[sid] == 0:
            cur -= size.pop(sid)
            del refs[sid]

    for a in trace.args:
        if isinstance(a, TensorProxy) and a.name not in storage_of:
            alloc(a.name, _nbytes(a))
    peak = cur
    tl = []
    for b in trace.bound_symbols:
        if b.sym.id == PrimIDs.DEL or b.sym.name == "python_del":
            for p in b.flat_proxy_args:
                release(p.name)
            if timeline:
                tl.append((str(b.sym.name), cur))
            continue
        src = next((a.name for a in b.flat_proxy_args if isinstance(a, TensorProxy) and a.name in storage_of), None)
        view = src is not None and is_view_bsym(b)
        for o in b.flat_proxy_outs:
            if not isinstance(o, TensorProxy) or o.name in storage_of:
                continue
            if view:
                alias(o.name, src)
            else:
                alloc(o.name, _nbytes(o))
        peak = max(peak, cur)
        if timeline:
            tl.append((str(b.sym.name), cur))
    # one entry per live storage (its first live name): views / aliases of a storage are not counted
    # again, so ``sum(live.values())`` is the live byte count at the end
    live, seen = {}, set()
    for n, s in storage_of.items():
        if s not in seen:
            seen.add(s)
            live[n] = size[s]
    assert sum(live.values()) == cur
    return (peak, live, tl) if timeline else (peak, live)


__all__ = ["get_alloc_memory", "is_view_bsym"]
