"""In-place ops and aliasing during acquisition (parity: reference ``thunder/core/update_aliases.py``
``insert_alias_updates`` :143, ``thunder/core/functionalization.py`` and the alias-aware cache
entries in ``thunder/__init__.py`` (``alias_tensor_indices``)).

The reference keeps in-place ops in the trace and threads ``update_aliases`` bound symbols
through it, relying on the runtime tensors really sharing storage.  Here the trace is made
*functional while it is acquired*, which keeps every later pass (autodiff, hipfuse fusion,
rematerialisation, hipGraph capture) free of aliasing hazards:

* every top-level bound symbol that contains ``prims.copy_`` into a pre-existing tensor is
  replaced by its out-of-place decomposition; the mutated Python object (the proxy the user
  code holds) is *re-bound* to the new value: prior trace references are moved to a copy of
  the proxy carrying the old name, and the object takes the new value's name;
* view ops (``view``, ``reshape``, basic ``__getitem__``, ``transpose``, ``split`` ...) record
  ``(base, view chain)``; mutating a view scatters the new value into the base
  (``view_scatter``) and bumps the base's version; other views of that base are lazily
  re-derived from the new base the next time they are used (version check);
* mutated *inputs* (arguments, parameters, buffers, captured tensors) get one real
  ``prims.copy_`` write-back into the caller's tensor at the end of the computation;
* arguments passed more than once (same tensor) are identity views of the first one, and the
  cache entry records the input storage-aliasing pattern so a call with a different pattern
  re-traces.
"""
from __future__ import annotations

import copy
from typing import Any

import torch

from .proxies import Proxy, TensorProxy, NumberProxy, pyval
from .pytree import tree_flatten, tree_map

# ltorch symbol id -> torch.Tensor method that reproduces the view on a real tensor
VIEW_METHODS = {
    "torch.view": "view",
    "torch.reshape": "reshape",
    "torch.Tensor.__getitem__": "__getitem__",
    "torch.transpose": "transpose",
    "torch.permute": "permute",
    "torch.expand": "expand",
    "torch.expand_as": "expand_as",
    "torch.squeeze": "squeeze",
    "torch.unsqueeze": "unsqueeze",
    "torch.split": "split",
    "torch.chunk": "chunk",
    "torch.unbind": "unbind",
    "torch.tensor_split": "tensor_split",
    "torch.narrow": "narrow",
    "torch.select": "select",
    "torch.flatten": "flatten",
    "torch.unflatten": "unflatten",
    "torch.movedim": "movedim",
    "torch.t": "t",
    "torch.view_as": "view_as",
    "torch.contiguous": "contiguous",
    "torch.detach": "detach",
}


def _is_basic_key(key) -> bool:
    ks = key if isinstance(key, tuple) else (key,)
    for k in ks:
        if k is None or k is Ellipsis or isinstance(k, (int, slice, NumberProxy)):
            continue
        return False
    return True


def _const(x):
    """Chain arguments must be printable constants."""
    def f(v):
        if isinstance(v, NumberProxy):
            return pyval(v)
        if isinstance(v, slice):
            return slice(f(v.start), f(v.stop), f(v.step))
        if isinstance(v, torch.Size):
            return tuple(v)
        return v

    if isinstance(x, tuple):
        return tuple(_const(v) for v in x)
    if isinstance(x, list):
        return [_const(v) for v in x]
    if isinstance(x, dict):
        return {k: _const(v) for k, v in x.items()}
    return f(x)


def _apply_view(v, name, args, kwargs):
    if name == "as_strided_rel":  # an argument that is a strided window of another argument
        size, stride, rel = args
        return v.as_strided(size, stride, v.storage_offset() + rel)
    return getattr(v, name)(*args, **kwargs)


def _view_scatter_impl(base, src, chain):
    out = base.clone()
    v = out
    for name, args, kwargs, idx in chain:
        v = _apply_view(v, name, args, kwargs)
        if idx is not None:
            v = v[idx]
    v.copy_(src)
    return out


_view_scatter_impl.__qualname__ = "view_scatter"
_view_scatter_impl.__module__ = "thunder"


def _replay_impl(base, chain):
    v = base
    for name, args, kwargs, idx in chain:
        v = _apply_view(v, name, args, kwargs)
        if idx is not None:
            v = v[idx]
    return v


def storage_alias_pattern(flat_args) -> tuple:
    """Canonical storage-sharing pattern of the tensor arguments (cache key part)."""
    groups: dict = {}
    exact: dict = {}
    first: dict = {}
    pat = []
    for x in flat_args:
        if not isinstance(x, torch.Tensor) or isinstance(x, Proxy) or x.device.type == "meta":
            continue
        try:
            sp = x.untyped_storage().data_ptr()
        except Exception:  # noqa: BLE001 - tensors without storage (e.g. sparse)
            sp = id(x)
        g = groups.setdefault(sp, len(groups))
        e = exact.setdefault((sp, x.storage_offset(), tuple(x.shape), tuple(x.stride())), len(exact))
        x0 = first.setdefault(sp, x)
        if x0 is x:
            pat.append((g, e))
        else:  # a window of an earlier argument: the program replays it at this relative offset
            pat.append((g, e, x.storage_offset() - x0.storage_offset(), tuple(x.shape), tuple(x.stride())))
    return tuple(pat)


class _ViewInfo:
    __slots__ = ("obj", "base", "chain", "version")

    def __init__(self, obj, base, chain, version):
        self.obj = obj
        self.base = base
        self.chain = chain
        self.version = version


class AliasTracker:
    """Attached to the computation trace while the frontend acquires it."""

    def __init__(self, trace):
        self.trace = trace
        self.views: dict[int, _ViewInfo] = {}
        self.version: dict[int, int] = {}
        self.input_objs: dict[int, TensorProxy] = {}
        self.mutated_inputs: dict[int, tuple[TensorProxy, TensorProxy]] = {}
        self.partial_alias: set[int] = set()
        self.input_specs = None
        self.any_mutation = False
        self.busy = 0

    # --- registration -----------------------------------------------------------------------
    def register_input(self, p: TensorProxy) -> None:
        self.input_objs[id(p)] = p

    def register_identity_alias(self, p: TensorProxy, base: TensorProxy) -> None:
        self.views[id(p)] = _ViewInfo(p, base, (), self.version.setdefault(id(base), 0))

    def register_window_alias(self, p: TensorProxy, base: TensorProxy, size, stride, rel: int) -> None:
        """``p`` is a strided window (``as_strided`` at element offset ``rel``) of the argument ``base``."""
        chain = (("as_strided_rel", (tuple(size), tuple(stride), int(rel)), {}, None),)
        self.views[id(p)] = _ViewInfo(p, base, chain, self.version.setdefault(id(base), 0))

    def original(self, p: TensorProxy) -> TensorProxy:
        """The proxy naming the caller's tensor for an input that may have been re-bound."""
        hit = self.mutated_inputs.get(id(p))
        return hit[1] if hit is not None else p

    def _root(self, p):
        vi = self.views.get(id(p))
        if vi is None:
            return p, ()
        return vi.base, vi.chain

    # --- hooks called by Symbol.__call__ at the top-level scope -----------------------------
    def before_call(self, args, kwargs) -> None:
        if self.busy:
            return
        flat, _ = tree_flatten((args, kwargs))
        for x in flat:
            if isinstance(x, TensorProxy):
                self.refresh(x)

    def after_call(self, bsym, result):
        if self.busy:
            return result
        muts = []
        _find_copies(bsym, set(id(o) for o in bsym.flat_proxy_outs), muts, _produced_inside(bsym))
        if not muts:
            self._maybe_register_view(bsym, result)
            return result
        trc = self.trace
        assert trc.bound_symbols and trc.bound_symbols[-1] is bsym
        trc.bound_symbols.pop()
        stripped = _strip_copies(bsym, _produced_inside(bsym))
        trc.bound_symbols.extend(stripped)
        produced = set()
        for b in stripped:
            _collect_outputs(b, produced)
        out_map = {}
        for src, dst, out in muts:
            out_map[id(out)] = dst
            self.mutate(dst, src, produced)
        if out_map:
            self._replace_everywhere(dict(out_map))
        return tree_map(lambda x: out_map.get(id(x), x) if isinstance(x, Proxy) else x, result)

    def _maybe_register_view(self, bsym, result) -> None:
        method = VIEW_METHODS.get(bsym.sym.id)
        if method is None or not bsym.args or not isinstance(bsym.args[0], TensorProxy):
            return
        if method == "__getitem__" and not _is_basic_key(bsym.args[1] if len(bsym.args) > 1 else None):
            return
        src = bsym.args[0]
        base, chain = self._root(src)
        ver = self.version.setdefault(id(base), 0)
        rest = _const(tuple(bsym.args[1:]))
        kw = _const(dict(bsym.kwargs))
        if isinstance(result, (tuple, list)):
            for i, o in enumerate(result):
                if isinstance(o, TensorProxy):
                    self.views[id(o)] = _ViewInfo(o, base, chain + ((method, rest, kw, i),), ver)
        elif isinstance(result, TensorProxy):
            self.views[id(result)] = _ViewInfo(result, base, chain + ((method, rest, kw, None),), ver)

    # --- core operations ------------------------------------------------------------------
    def refresh(self, p: TensorProxy) -> None:
        vi = self.views.get(id(p))
        if vi is None:
            return
        cur = self.version.get(id(vi.base), 0)
        if vi.version == cur:
            return
        from ..torch.default_torch_ops import opaque_symbol

        self.busy += 1
        try:
            if vi.chain:
                nv = opaque_symbol(_replay_impl, "view_replay")(vi.base, vi.chain)
            else:
                from . import prims

                nv = prims.shallow_copy(vi.base)
        finally:
            self.busy -= 1
        self.rebind(p, nv)
        vi.version = cur

    def mutate(self, dst: TensorProxy, src: TensorProxy, produced: set) -> None:
        from . import prims
        from ..torch.default_torch_ops import opaque_symbol

        self.any_mutation = True
        base, chain = self._root(dst)
        if id(base) in self.partial_alias:
            raise NotImplementedError(
                "in-place update of an input whose storage partially overlaps another input is not supported"
            )
        if torch.is_grad_enabled() and id(base) in self.input_objs and base.requires_grad and "parameter" in base.tags:
            raise RuntimeError("a leaf Variable that requires grad is being used in an in-place operation.")
        self.busy += 1
        try:
            if id(src) not in produced or src is dst:
                src = prims.shallow_copy(src)
                produced.add(id(src))
            if base is not dst:
                nb = opaque_symbol(_view_scatter_impl, "view_scatter")(base, src, chain)
        finally:
            self.busy -= 1
        if base is not dst:
            self.rebind(base, nb)
        self.rebind(dst, src)
        v = self.version.get(id(base), 0) + 1
        self.version[id(base)] = v
        vi = self.views.get(id(dst))
        if vi is not None:
            vi.version = v

    def rebind(self, d: TensorProxy, v: TensorProxy) -> None:
        """Makes the Python object ``d`` denote the value ``v`` from now on."""
        old = copy.copy(d)
        d._name = v.name
        d.requires_grad = v.requires_grad
        self._replace_everywhere({id(d): old, id(v): d})
        if id(d) in self.input_objs:
            self.input_objs[id(old)] = old
            if id(d) not in self.mutated_inputs:
                self.mutated_inputs[id(d)] = (d, old)

    def _replace_everywhere(self, m: dict) -> None:
        def sub(x):
            return m.get(id(x), x) if isinstance(x, Proxy) else x

        def fix(b):
            hit = any(id(x) in m for x in b.flat_args) or any(id(x) in m for x in b.flat_outs)
            if hit:
                b.args = tree_map(sub, b.args)
                b.kwargs = tree_map(sub, b.kwargs)
                b.output = tree_map(sub, b.output)
                b._flat_args = None
                b._flat_outs = None
            for s in b.subsymbols:
                fix(s)

        for b in self.trace.bound_symbols:
            fix(b)
        if self.input_specs is not None:
            for s in self.input_specs:
                if s.proxy is not None and id(s.proxy) in m:
                    s.proxy = m[id(s.proxy)]

    # --- end of acquisition ------------------------------------------------------------
    def finish(self, result):
        """Refreshes stale outputs and emits input write-backs; returns the fixed result."""
        from . import prims

        def fresh(x):
            if isinstance(x, TensorProxy):
                self.refresh(x)
            return x

        result = tree_map(fresh, result)
        for d, old in list(self.mutated_inputs.values()):
            if id(d) in self.views:  # views of another input: the base's write-back covers them
                continue
            self.busy += 1
            try:
                prims.copy_(d, old)
            finally:
                self.busy -= 1
        return result


def _produced_inside(bsym) -> set:
    s = set()
    for sub in bsym.subsymbols:
        _collect_outputs(sub, s)
    return s


def _collect_outputs(b, acc: set) -> None:
    for o in b.flat_proxy_outs:
        acc.add(id(o))
    for s in b.subsymbols:
        _collect_outputs(s, acc)


def _find_copies(bsym, outs, acc, produced) -> None:
    from .prims import PrimIDs

    if bsym.sym.id == PrimIDs.COPY_:
        src, dst = bsym.args[0], bsym.args[1]
        if isinstance(dst, TensorProxy) and id(dst) not in produced:
            acc.append((src, dst, bsym.output))
        return
    for s in bsym.subsymbols:
        _find_copies(s, outs, acc, produced)


def _contains_copy(bsym) -> bool:
    from .prims import PrimIDs

    if bsym.sym.id == PrimIDs.COPY_:
        return True
    return any(_contains_copy(s) for s in bsym.subsymbols)


def _strip_copies(bsym, produced: set) -> list:
    """The decomposition of ``bsym`` without its copies into pre-existing tensors."""
    from .prims import PrimIDs

    out = []
    for s in bsym.subsymbols:
        if s.sym.id == PrimIDs.COPY_ and id(s.args[1]) not in produced:
            continue
        if _contains_copy(s):
            out.extend(_strip_copies(s, produced))
        else:
            out.append(s)
    return out
