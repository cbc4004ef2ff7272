"""Reverse-mode autodiff on traces (parity: reference ``thunder/transforms/autodiff.py``
``grad_transform_on_trace`` :28-449, ``split_into_forward_and_backward`` :465-602).

The reference builds a joint forward+backward trace and then splits it.  Here the
split is constructed directly: walking the computation trace forward, each
differentiable bound symbol is replaced by its VJP rule's forward part in the
*forward* trace while its backward closure is queued; replaying the queue in
reverse inside a fresh *backward* trace accumulates cotangents.  Proxies that the
backward closures capture are exactly the saved-for-backward tensors.

Rule lookup order for a bound symbol:
1. the grad transform of the first executor that can execute it (e.g. HIP flash
   attention saving its LSE),
2. a registered VJP rule (``core/transforms.py`` for prims, below for ltorch ops),
3. a generic ``torch.autograd`` rule for auto-registered opaque ops,
4. otherwise the bound symbol's decomposition (subsymbols) is differentiated.

Bound symbols tagged ``RECOMPUTE_IN_BACKWARD`` (activation checkpointing) are
replayed in the backward trace instead of being saved.
"""
from __future__ import annotations

import inspect
import math
import time
from typing import Any, Callable

import torch

from ..core import dtypes, prims
from ..core.prims import PrimIDs, OpTags
from ..core.proxies import Proxy, TensorProxy, DTensorProxy, NumberProxy, pyval
from ..core.pytree import tree_flatten, tree_unflatten, tree_map
from ..core.symbol import BoundSymbol, BoundSymbolTag, Symbol, NON_DIFFERENTIABLE_TAG, register_symbol, _LAYOUT_IDENTITIES
from ..core.trace import TraceCtx, tracectx, from_trace, TraceProvenance, get_tracectx
from ..core.transforms import get_vjp_rule, register_vjp, _vjp_rules, grad_like, sum_to_shape, linear_backward, _requires
from ..core.transform_common import dce
from ..common import get_compile_option


class GradsWithKwargs:
    """A backward closure's result when keyword-only tensor arguments also receive gradients."""

    def __init__(self, args, kwargs):
        self.args = args
        self.kwargs = kwargs


class _Record:
    __slots__ = ("bwd", "outs", "args", "kwargs", "name")

    def __init__(self, bwd, outs, args, kwargs, name):
        self.bwd = bwd
        self.outs = outs
        self.args = args
        self.kwargs = kwargs
        self.name = name


def _is_differentiable_bsym(bsym: BoundSymbol) -> bool:
    if NON_DIFFERENTIABLE_TAG in bsym.sym.tags or BoundSymbolTag.NO_GRAD in bsym.tags:
        return False
    if bsym.sym.id in (PrimIDs.RETURN, PrimIDs.DEL, PrimIDs.COMMENT):
        return False
    if not any(isinstance(a, TensorProxy) and a.requires_grad for a in bsym.flat_args):
        return False
    if not any(isinstance(o, TensorProxy) and dtypes.is_inexact_dtype(o.dtype) for o in bsym.flat_outs):
        return False
    return True


def _canonicalize_args(sym: Symbol, args, kwargs):
    """Bind kwargs to positional parameters where possible (so rules see a canonical signature)."""
    meta = sym.meta
    if meta is None or not kwargs:
        return args, kwargs
    try:
        sig = inspect.signature(meta)
        bound = sig.bind(*args, **kwargs)
    except (TypeError, ValueError):
        return args, kwargs
    new_args = []
    new_kwargs = {}
    for name, param in sig.parameters.items():
        if name not in bound.arguments:
            if param.kind in (param.POSITIONAL_ONLY, param.POSITIONAL_OR_KEYWORD) and param.default is not param.empty:
                # keep positional alignment only if later positional args are bound
                later = [n for n in list(sig.parameters)[list(sig.parameters).index(name) + 1:] if n in bound.arguments and sig.parameters[n].kind in (param.POSITIONAL_ONLY, param.POSITIONAL_OR_KEYWORD)]
                if later:
                    new_args.append(param.default)
            continue
        v = bound.arguments[name]
        if param.kind == param.VAR_POSITIONAL:
            new_args.extend(v)
        elif param.kind == param.VAR_KEYWORD:
            new_kwargs.update(v)
        elif param.kind == param.KEYWORD_ONLY:
            new_kwargs[name] = v
        else:
            new_args.append(v)
    return tuple(new_args), new_kwargs


def _zip_grads(args, grads, acc):
    """Walks args and their grads (same structure; None covers a subtree)."""
    if grads is None:
        return
    if isinstance(args, TensorProxy):
        acc.append((args, grads))
        return
    if isinstance(args, (list, tuple)):
        if not isinstance(grads, (list, tuple)):
            return
        for a, g in zip(args, grads):
            _zip_grads(a, g, acc)
        return
    if isinstance(args, dict) and isinstance(grads, dict):
        for k, a in args.items():
            _zip_grads(a, grads.get(k), acc)


def _executor_grad_transforms(bsym: BoundSymbol, executors) -> list:
    """Grad transforms of the executors (in priority order, always-executors last) able to run ``bsym``.

    A grad transform may return ``None`` to decline (e.g. unsupported layout), in which case the
    next candidate is tried.
    """
    from ..extend import get_always_executors

    out = []
    seen = set()
    for ex in list(executors or ()) + list(get_always_executors()):
        if ex.name in seen:
            continue
        seen.add(ex.name)
        gt = ex.get_grad_transform(bsym.sym)
        if gt is not None and ex.can_execute_directly(bsym):
            out.append(gt)
    return out


# ---- generic torch.autograd rule for opaque (auto-registered) ops -------------------------
def _torch_vjp_impl(fn, args, kwargs, cotangents):
    flat, spec = tree_flatten((args, kwargs))
    inputs = []
    new_flat = []
    for x in flat:
        if isinstance(x, torch.Tensor) and (x.is_floating_point() or x.is_complex()):
            y = x.detach().requires_grad_(True)
            inputs.append(y)
            new_flat.append(y)
        else:
            new_flat.append(x)
    a, k = tree_unflatten(new_flat, spec)
    with torch.enable_grad():
        out = fn(*a, **k)
        outs, _ = tree_flatten(out)
        # expanded cotangents (e.g. from sum's backward: stride 0) are made dense — some
        # backward kernels (grouped_mm) reject zero strides
        pairs = [(o, c if c.is_contiguous() else c.contiguous())
                 for o, c in zip([o for o in outs if isinstance(o, torch.Tensor)], cotangents)
                 if c is not None and o.requires_grad]
        if not pairs:
            return tuple(None for _ in inputs)
        grads = torch.autograd.grad([p[0] for p in pairs], inputs, [p[1] for p in pairs], allow_unused=True)
    return tuple(grads)


def _torch_vjp_meta(fn, args, kwargs, cotangents):
    flat, _ = tree_flatten((args, kwargs))
    return tuple(x.replace(requires_grad=False) if isinstance(x, DTensorProxy) else TensorProxy(like=x, requires_grad=False)
                 for x in flat if isinstance(x, TensorProxy) and dtypes.is_inexact_dtype(x.dtype))


torch_vjp = Symbol("torch_autograd_vjp", _torch_vjp_meta, id="autodiff.torch_autograd_vjp", is_prim=True)
register_symbol(torch_vjp)


def _register_torch_vjp_impl():
    from ..executors import torchex

    op = torchex.ex.register_operator("torch_autograd_vjp", like=torch_vjp, fn=_torch_vjp_impl)
    torchex.ex.register_implementation(torch_vjp, op)


def _opaque_rule(sym):
    def rule(*args, **kwargs):
        out = sym(*args, **kwargs)

        def bwd(*cts):
            grads = torch_vjp(sym.torch_fn, args, kwargs, list(cts))
            # map flat grads back onto args structure
            flat, spec = tree_flatten((args, kwargs))
            it = iter(grads)
            gflat = []
            for x in flat:
                if isinstance(x, TensorProxy) and dtypes.is_inexact_dtype(x.dtype):
                    gflat.append(next(it))
                else:
                    gflat.append(None)
            ga, gk = tree_unflatten(gflat, spec)
            return GradsWithKwargs(ga, gk) if gk else ga

        return out, bwd

    return rule


# -----------------------------------------------------------------------------------------
# The pass
# -----------------------------------------------------------------------------------------
class ForwardBackward:
    def __init__(self, forward_trace, backward_trace, saved_tensors, saved_other, grad_input_indices, diff_output_mask):
        self.forward_trace = forward_trace
        self.backward_trace = backward_trace
        self.saved_tensors = saved_tensors
        self.saved_other = saved_other
        self.grad_input_indices = grad_input_indices
        self.diff_output_mask = diff_output_mask


_EXPENSIVE_NAME_PARTS = ("matmul", "linear", "scaled_dot_product", "attention", "grouped_mm", "conv", "bmm", "einsum")


def _never_auto_recompute(b: BoundSymbol) -> bool:
    """Ops ``auto_recompute_intermediates`` leaves saved: GEMM/attention-shaped and random ops
    (reference: ``DONT_AUTO_RECOMPUTE_IN_BACKWARD`` on sdpa/matmul, ``RANDOM_OP``)."""
    tags = set(b.sym.tags or ())
    if tags & {OpTags.RANDOM_OP, OpTags.MATMUL_OP, OpTags.DONT_AUTO_RECOMPUTE_IN_BACKWARD}:
        return True
    if BoundSymbolTag.DONT_AUTO_RECOMPUTE_IN_BACKWARD in b.tags:
        return True
    name = b.sym.name.lower()
    return any(part in name for part in _EXPENSIVE_NAME_PARTS)


def forward_and_backward_from_trace(trace: TraceCtx, *, executors=()) -> ForwardBackward:
    start = time.perf_counter_ns()
    fw = from_trace(trace)
    fw.bound_symbols = []
    fw.scopes = [fw.bound_symbols]
    swap: dict[str, Proxy] = {}
    records: list[_Record] = []
    recompute_bsyms: list[BoundSymbol] = []

    def sw(x):
        if isinstance(x, Proxy):
            seen = 0
            while x.name in swap and seen < 100:
                nx = swap[x.name]
                if nx is x:
                    break
                x = nx
                seen += 1
        return x

    ret_bsym = None
    auto_recompute = bool(get_compile_option(
        "auto_recompute_intermediates",
        "Recompute the intermediates of differentiated decompositions in the backward instead of "
        "saving them (fewer saved tensors, more compute); matmul/attention/random ops are never recomputed"))

    def process(bsym: BoundSymbol, recompute: bool = False):
        nonlocal ret_bsym
        b = bsym.swap_proxies(swap, skip_output=True)
        if b.sym.id == PrimIDs.RETURN:
            ret_bsym = b
            return
        if bsym.sym.id == "torch.checkpoint":
            for s in bsym.subsymbols:
                s2 = s.from_bsym(tags=set(s.tags) | {BoundSymbolTag.RECOMPUTE_IN_BACKWARD})
                process(s2, recompute=True)
            return
        if BoundSymbolTag.RECOMPUTE_IN_BACKWARD in bsym.tags:
            recompute = True
        if not _is_differentiable_bsym(b):
            if recompute and not (recompute == "auto" and _never_auto_recompute(b)):
                b.tags.add(BoundSymbolTag.RECOMPUTE_IN_BACKWARD)
            fw.bound_symbols.append(b)
            return
        in_names = {a.name for a in bsym.flat_proxy_args}
        if (not bsym.subsymbols and bsym.sym.name not in _LAYOUT_IDENTITIES
                and all(o.name in in_names for o in bsym.flat_proxy_outs)):
            # identity (e.g. cat with an empty operand): the output *is* an input, whose name the
            # swap table already maps; the gradient flows through the shared name.  (contiguous is
            # kept: it has a rule producing a fresh proxy, needed for the run-time memory layout)
            return
        candidates = _executor_grad_transforms(b, executors)
        registered = _vjp_rules.get(b.sym.id, "missing")
        if registered is None and not candidates:  # explicitly non-differentiable
            fw.bound_symbols.append(b)
            return
        if registered not in (None, "missing"):
            candidates.append(registered)
        if OpTags.AUTO_REGISTERED in b.sym.tags:
            candidates.append(_opaque_rule(b.sym))
        args, kwargs = _canonicalize_args(b.sym, b.args, b.kwargs)
        n_before = len(fw.bound_symbols)
        res = None
        for rule in candidates:
            res = rule(*args, **kwargs)
            if res is not None:
                break
            del fw.bound_symbols[n_before:]  # the rule declined (unsupported options)
        if res is None:  # differentiate the decomposition
            if b.subsymbols:
                auto = auto_recompute and not recompute and not _never_auto_recompute(b)
                for s in b.subsymbols:
                    process(s, "auto" if auto else recompute)
                if auto:
                    # auto_recompute_intermediates (reference trace_interpreter.py:204-222): the
                    # decomposition's intermediates are recomputed in the backward instead of
                    # saved; the decomposed op's own outputs stay ordinary forward values.
                    finals = {sw(o).name for o in bsym.flat_proxy_outs}
                    for nb in fw.bound_symbols[n_before:]:
                        if any(o.name in finals for o in nb.flat_proxy_outs):
                            nb.tags.discard(BoundSymbolTag.RECOMPUTE_IN_BACKWARD)
                return
            raise NotImplementedError(f"No VJP rule for {b.sym.name} ({b.sym.id}) and it has no decomposition")
        out, bwd = res
        if recompute and not (recompute == "auto" and _never_auto_recompute(b)):
            for nb in fw.bound_symbols[n_before:]:
                nb.tags.add(BoundSymbolTag.RECOMPUTE_IN_BACKWARD)
        old_flat = [o for o in tree_flatten(bsym.output)[0]]
        new_flat = [o for o in tree_flatten(out)[0]]
        for o_old, o_new in zip(old_flat, new_flat):
            if isinstance(o_old, Proxy) and isinstance(o_new, Proxy) and o_old is not o_new:
                swap[o_old.name] = o_new
                if isinstance(o_new, TensorProxy) and isinstance(o_old, TensorProxy):
                    o_new.requires_grad = o_old.requires_grad or o_new.requires_grad
        in_ids = {id(x) for x in tree_flatten((args, kwargs))[0] if isinstance(x, Proxy)}
        if all(id(o) in in_ids for o in new_flat if isinstance(o, Proxy)):
            return  # identity (e.g. contiguous, same-dtype .to): gradient flows through the shared name
        records.append(_Record(bwd, [o for o in new_flat], args, kwargs, b.sym.name))

    with tracectx(fw):
        for bsym in trace.bound_symbols:
            process(bsym)

    # outputs of the forward
    orig_out = ret_bsym.args[0] if ret_bsym is not None and len(ret_bsym.args) == 1 else (ret_bsym.args if ret_bsym else None)
    fw_out = tree_map(sw, orig_out)
    flat_out, out_spec = tree_flatten(fw_out)

    # ---- backward ------------------------------------------------------------------
    bw = TraceCtx(None)
    bw.fn_name = "backward_fn"
    bw.names = set(fw.names)
    bw._counters = type(fw._counters)(int, fw._counters)
    grads: dict[str, TensorProxy] = {}
    cotangent_args = []
    diff_output_mask = []
    with tracectx(bw):
        for o in flat_out:
            if isinstance(o, TensorProxy) and o.requires_grad and dtypes.is_inexact_dtype(o.dtype):
                ct = TensorProxy(like=o, requires_grad=False, prefix="ct")
                cotangent_args.append(ct)
                diff_output_mask.append(True)
                prev = grads.get(o.name)
                grads[o.name] = ct if prev is None else prims.add(prev, ct)
            else:
                diff_output_mask.append(False)

        def acc(p: TensorProxy, g):
            if g is None or not isinstance(p, TensorProxy):
                return
            if not p.requires_grad and p.name not in grads:
                # still accumulate: intermediate proxies may have stale flags
                pass
            g = grad_like(g, p)
            if g is None:
                return
            prev = grads.get(p.name)
            grads[p.name] = g if prev is None else _ltorch_add(prev, g)

        for rec in reversed(records):
            cts = []
            any_ct = False
            for o in rec.outs:
                if isinstance(o, TensorProxy):
                    g = grads.get(o.name)
                    if g is not None:
                        any_ct = True
                    cts.append(g)
                else:
                    cts.append(None)
            if not any_ct:
                continue
            # missing cotangents of multi-output ops become zeros (only for float outputs)
            cts = [
                (c if c is not None else (prims.full(tuple(o.shape), 0, device=o.device, dtype=o.dtype) if isinstance(o, TensorProxy) and dtypes.is_inexact_dtype(o.dtype) else None))
                for c, o in zip(cts, rec.outs)
            ]
            tensor_cts = [c for c, o in zip(cts, rec.outs) if isinstance(o, TensorProxy)]
            res = rec.bwd(*tensor_cts)
            pairs: list = []
            if isinstance(res, GradsWithKwargs):
                _zip_grads(tuple(rec.args), tuple(res.args), pairs)
                _zip_grads(rec.kwargs, res.kwargs, pairs)
            else:
                _zip_grads(tuple(rec.args), tuple(res) if isinstance(res, (list, tuple)) else (res,), pairs)
            for p, g in pairs:
                acc(p, g)

        # input gradients
        grad_input_indices = []
        input_grads = []
        for i, a in enumerate(trace.args):
            if isinstance(a, TensorProxy) and a.requires_grad:
                grad_input_indices.append(i)
                input_grads.append(grads.get(a.name))
        prims.python_return(tuple(input_grads))

    # ---- saved-for-backward = free variables of the backward ----------------------------------
    bw = dce(bw)
    produced = {p.name for p in cotangent_args}
    free: dict[str, Proxy] = {}
    for b in bw.bound_symbols:
        for a in b.flat_proxy_args:
            if a.name not in produced and a.name not in free:
                free[a.name] = a
        for o in b.flat_proxy_outs:
            produced.add(o.name)

    # activation checkpointing: recompute tagged forward ops inside the backward
    recompute_names = {o.name for b in fw.bound_symbols if BoundSymbolTag.RECOMPUTE_IN_BACKWARD in b.tags for o in b.flat_proxy_outs}
    if recompute_names & set(free):
        bw, free = _insert_recomputation(fw, bw, free, recompute_names, cotangent_args)

    saved_tensors = [p for p in free.values() if isinstance(p, TensorProxy)]
    saved_other = [p for p in free.values() if not isinstance(p, TensorProxy)]
    saved_tensors = _protect_saved_from_writeback(fw, bw, saved_tensors)
    bw.args = saved_tensors + saved_other + cotangent_args
    bw.set_provenance(TraceProvenance(f"Backward pass (took {(time.perf_counter_ns() - start) // 1000000} milliseconds)"))

    with tracectx(fw):
        prims.python_return((fw_out, tuple(saved_tensors), tuple(saved_other)))
    fw.fn_name = "augmented_forward_fn"
    fw = dce(fw)
    fw.set_provenance(TraceProvenance(f"Augmented forward pass (took {(time.perf_counter_ns() - start) // 1000000} milliseconds)"))
    return ForwardBackward(fw, bw, saved_tensors, saved_other, grad_input_indices, diff_output_mask)


def _protect_saved_from_writeback(fw: TraceCtx, bw: TraceCtx, saved: list) -> list:
    """Inputs mutated by the forward (functionalized in-place ops end in one ``copy_`` write-back,
    see ``core/functionalization.py``) keep their pre-mutation value for the backward: the saved
    tensor becomes a clone taken just before the write-back."""
    names = {p.name for p in saved}
    swap: dict[str, Proxy] = {}
    i = 0
    while i < len(fw.bound_symbols):
        b = fw.bound_symbols[i]
        if b.sym.id == PrimIDs.COPY_ and isinstance(b.args[1], TensorProxy) and b.args[1].name in names:
            dst = b.args[1]
            if dst.name not in swap:
                from .. import torch as ltorch

                base = f"{dst.name}_saved"
                name, k = base, 0
                while name in fw.names or name in bw.names:
                    k += 1
                    name = f"{base}{k}"
                with tracectx(fw):
                    c = TensorProxy(name, like=dst)
                bw.names.add(name)
                sub = prims.shallow_copy.bind(dst, output=c)
                fw.bound_symbols.insert(i, ltorch.clone.bind(dst, output=c, subsymbols=[sub]))
                i += 1
                swap[dst.name] = c
        i += 1
    if not swap:
        return saved
    bw.bound_symbols = [b.swap_proxies(swap) for b in bw.bound_symbols]
    bw.scopes = [bw.bound_symbols]
    return [swap.get(p.name, p) for p in saved]

def _insert_recomputation(fw, bw, free, recompute_names, cotangent_args):
    """Moves RECOMPUTE_IN_BACKWARD producers needed by the backward into the backward (reference :363-432)."""
    producers = {}
    for b in fw.bound_symbols:
        for o in b.flat_proxy_outs:
            producers[o.name] = b
    needed: list[BoundSymbol] = []
    needed_set: set[int] = set()
    new_free: dict[str, Proxy] = {}

    def visit(name):
        b = producers.get(name)
        if b is None or name not in recompute_names:
            return False
        if id(b) in needed_set:
            return True
        for a in b.flat_proxy_args:
            if a.name in recompute_names:
                visit(a.name)
            else:
                new_free.setdefault(a.name, a)
        needed_set.add(id(b))
        needed.append(b)
        return True

    for name, p in list(free.items()):
        if not visit(name):
            new_free.setdefault(name, p)
    order = {id(b): i for i, b in enumerate(fw.bound_symbols)}
    needed.sort(key=lambda b: order[id(b)])
    bw2 = from_trace(bw)
    bw2.bound_symbols = needed + list(bw.bound_symbols)
    bw2.scopes = [bw2.bound_symbols]
    produced = {p.name for p in cotangent_args}
    free2: dict[str, Proxy] = {}
    for b in bw2.bound_symbols:
        for a in b.flat_proxy_args:
            if a.name not in produced and a.name not in free2:
                free2[a.name] = a
        for o in b.flat_proxy_outs:
            produced.add(o.name)
    return bw2, free2


def _upcast(x):
    """Computation dtype for gradient math: at least fp32 (fp64 stays fp64)."""
    if isinstance(x, TensorProxy) and (x.dtype in (torch.bfloat16, torch.float16) or dtypes.is_float8_dtype(x.dtype)):
        return prims.convert_element_type(x, torch.float32)
    return x


def _ltorch_add(a, b):
    if a.dtype != b.dtype:
        b = prims.convert_element_type(b, a.dtype)
    return prims.add(a, b)


# =========================================================================================
# ltorch-level VJP rules: keep high-level ops intact so executors can claim them
# =========================================================================================
def _lt():
    from .. import torch as ltorch

    return ltorch


def _install_ltorch_rules():
    ltorch = _lt()
    from .. import clang

    def rg(x):
        return isinstance(x, TensorProxy) and x.requires_grad

    @register_vjp(ltorch.add)
    def _add(a, b, *, alpha=None):
        out = ltorch.add(a, b, alpha=alpha)

        def bwd(g):
            gb = None
            if rg(b):
                gb = g if alpha is None or alpha == 1 else ltorch.mul(g, alpha)
            return (g if rg(a) else None), gb

        return out, bwd

    @register_vjp(ltorch.sub)
    def _sub(a, b, *, alpha=None):
        out = ltorch.sub(a, b, alpha=alpha)

        def bwd(g):
            gb = None
            if rg(b):
                gb = ltorch.neg(g) if alpha is None or alpha == 1 else ltorch.mul(g, -alpha)
            return (g if rg(a) else None), gb

        return out, bwd

    def _cj(t):
        if isinstance(t, TensorProxy) and dtypes.is_complex_dtype(t.dtype):
            from ..torch.default_torch_ops import opaque_symbol

            return opaque_symbol(torch.conj_physical)(t)
        if isinstance(t, complex):
            return t.conjugate()
        return t

    @register_vjp(ltorch.mul)
    def _mul(a, b):
        out = ltorch.mul(a, b)

        def bwd(g):
            # complex operands: PyTorch's convention is grad_a = g * conj(b)
            return (ltorch.mul(g, _cj(b)) if rg(a) else None), (ltorch.mul(g, _cj(a)) if rg(b) else None)

        return out, bwd

    @register_vjp(ltorch.dropout)
    def _dropout(a, p=0.5, training=True, inplace=False):
        """The mask is recomputed from (seed, offset) in the backward (K13): nothing but two
        integers is saved, and hipfuse fuses the regenerated mask into the gradient kernel."""
        from ..core import prims as _prims
        from .. import clang as _clang

        pv = pyval(p)
        if not training or pv == 0.0:
            return a, lambda g: (g,)
        if pv == 1.0:
            out = ltorch.mul(a, 0.0)
            return out, lambda g: (ltorch.mul(g, 0.0),)
        scale = 1.0 / (1.0 - pv)
        n = 1
        for d in a.shape:
            n *= d
        seed, offset = _prims.get_rng_seed_offset(n)

        def apply(t):
            keep = ltorch.philox_keep_mask(t, pv, seed, offset)
            compute = _clang.compute_dtype(t.dtype)
            x = _clang.maybe_convert_to_dtype(t, compute)
            y = _prims.mul(_prims.mul(x, _clang.maybe_convert_to_dtype(keep, compute)), scale)
            return _clang.maybe_convert_to_dtype(y, t.dtype)

        out = apply(a)
        return out, lambda g: (apply(g),)

    @register_vjp(ltorch.true_divide)
    def _div(a, b):
        out = ltorch.true_divide(a, b)

        def bwd(g):
            ga = ltorch.true_divide(g, b) if rg(a) else None
            gb = ltorch.neg(ltorch.true_divide(ltorch.mul(g, out), b)) if rg(b) else None
            return ga, gb

        return out, bwd

    @register_vjp(ltorch.neg)
    def _neg(a):
        return ltorch.neg(a), lambda g: (ltorch.neg(g),)

    # complex parts (PyTorch's convention: real(z) -> g + 0j, imag(z) -> g * 1j)
    from ..core import prims as _prims

    @register_vjp(_prims.real)
    def _real(a):
        return _prims.real(a), lambda g: (clang.maybe_convert_to_dtype(g, a.dtype),)

    @register_vjp(_prims.imag)
    def _imag(a):
        return _prims.imag(a), lambda g: (ltorch.mul(clang.maybe_convert_to_dtype(g, a.dtype), 1j),)

    @register_vjp(ltorch.exp)
    def _exp(a):
        out = ltorch.exp(a)
        return out, lambda g: (ltorch.mul(g, out),)

    @register_vjp(ltorch.tanh)
    def _tanh(a):
        out = ltorch.tanh(a)
        return out, lambda g: (ltorch.mul(g, ltorch.rsub(ltorch.mul(out, out), 1.0)),)

    @register_vjp(ltorch.sigmoid)
    def _sigmoid(a):
        out = ltorch.sigmoid(a)
        return out, lambda g: (ltorch.mul(g, ltorch.mul(out, ltorch.rsub(out, 1.0))),)

    @register_vjp(ltorch.relu)
    def _relu(a, inplace=False):
        out = ltorch.relu(a)
        return out, lambda g: (ltorch.where(ltorch.gt(out, 0), g, 0.0),)

    @register_vjp(ltorch.silu)
    def _silu(a, inplace=False):
        out = ltorch.silu(a)

        def bwd(g):
            x = _upcast(a)
            s = ltorch.sigmoid(x)
            d = ltorch.mul(s, ltorch.add(ltorch.mul(x, ltorch.rsub(s, 1.0)), 1.0))
            return (clang.maybe_convert_to_dtype(ltorch.mul(_upcast(g), d), a.dtype),)

        return out, bwd

    @register_vjp(ltorch.gelu)
    def _gelu(a, approximate="none"):
        out = ltorch.gelu(a, approximate=approximate)

        def bwd(g):
            x = _upcast(a)
            gf = _upcast(g)
            if approximate == "tanh":
                k = math.sqrt(2.0 / math.pi)
                x3 = ltorch.mul(ltorch.mul(x, x), x)
                inner = ltorch.mul(ltorch.add(x, ltorch.mul(x3, 0.044715)), k)
                t = ltorch.tanh(inner)
                dinner = ltorch.mul(ltorch.add(ltorch.mul(ltorch.mul(x, x), 3 * 0.044715), 1.0), k)
                d = ltorch.add(ltorch.mul(ltorch.add(t, 1.0), 0.5), ltorch.mul(ltorch.mul(ltorch.mul(x, 0.5), ltorch.rsub(ltorch.mul(t, t), 1.0)), dinner))
            else:
                cdf = ltorch.mul(ltorch.add(ltorch.erf(ltorch.mul(x, 1.0 / math.sqrt(2.0))), 1.0), 0.5)
                pdf = ltorch.mul(ltorch.exp(ltorch.mul(ltorch.mul(x, x), -0.5)), 1.0 / math.sqrt(2.0 * math.pi))
                d = ltorch.add(cdf, ltorch.mul(x, pdf))
            return (clang.maybe_convert_to_dtype(ltorch.mul(gf, d), a.dtype),)

        return out, bwd

    @register_vjp(ltorch.linear)
    def _linear(a, w, bias=None):
        out = ltorch.linear(a, w, bias)
        return out, lambda g: linear_backward(a, w, bias, g)

    @register_vjp(ltorch._grouped_mm)
    def _grouped_mm_vjp(a, b, offs=None, bias=None, out_dtype=None):
        """MoE expert GEMM: out[rows of g] = a[rows of g] @ b[g] (2-D x 3-D form)."""
        out = ltorch._grouped_mm(a, b, offs)

        def bwd(g):
            ga = ltorch._grouped_mm(g, ltorch.transpose(b, -1, -2), offs) if rg(a) else None
            gb = ltorch._grouped_mm(ltorch.transpose(a, 0, 1), g, offs) if rg(b) else None
            return ga, gb

        return out, bwd

    @register_vjp(ltorch.matmul)
    def _matmul(a, b):
        from ..core.transforms import _vjp_rules as R

        return R[PrimIDs.MATMUL](a, b)

    def _shape_rule(fn):
        def rule(a, *args, **kwargs):
            out = fn(a, *args, **kwargs)
            return out, lambda g: (clang.reshape(g, a.shape),)

        return rule

    for f in (ltorch.reshape, ltorch.view, ltorch.flatten, ltorch.unsqueeze, ltorch.squeeze, ltorch.view_as, ltorch.unflatten):
        register_vjp(f)(_shape_rule(f))

    @register_vjp(ltorch.transpose)
    def _transpose(a, dim0, dim1):
        out = ltorch.transpose(a, dim0, dim1)
        return out, lambda g: (ltorch.transpose(g, dim0, dim1),)

    @register_vjp(ltorch.permute)
    def _permute(a, *dims):
        from ..torch import _shape_args

        d = clang.canonicalize_dims(a.ndim, _shape_args(dims))
        out = ltorch.permute(a, d)
        inv = [0] * len(d)
        for i, p in enumerate(d):
            inv[p] = i
        return out, lambda g: (ltorch.permute(g, inv),)

    @register_vjp(ltorch.expand)
    def _expand(a, *shape):
        out = ltorch.expand(a, *shape)
        return out, lambda g: (sum_to_shape(g, a.shape),)

    for f in (ltorch.contiguous, ltorch.clone):
        register_vjp(f)(lambda a, *args, _f=f, **kw: (_f(a, *args, **kw), lambda g: (g,)))

    def _cast_rule(fn):
        def rule(a, *args, **kwargs):
            out = fn(a, *args, **kwargs)

            def bwd(g):
                gg = g
                if gg.dtype != a.dtype:
                    gg = clang.maybe_convert_to_dtype(gg, a.dtype)
                if isinstance(out, TensorProxy) and out.device != a.device:
                    gg = clang.device_put(gg, a.device)
                return (gg,)

            return out, bwd

        return rule

    for f in (ltorch.to, ltorch.type_as, ltorch.tensor_float, ltorch.bfloat16, ltorch.half, ltorch.double):
        register_vjp(f)(_cast_rule(f))

    @register_vjp(ltorch.softmax)
    def _softmax(a, dim, dtype=None, **kw):
        out = ltorch.softmax(a, dim, dtype=dtype)

        def bwd(g):
            d = clang.canonicalize_dim(a.ndim, dim)
            gf = _upcast(g)
            of = _upcast(out)
            go = ltorch.mul(gf, of)
            s = ltorch.sum(go, d, True)
            r = ltorch.sub(go, ltorch.mul(of, s))
            return (clang.maybe_convert_to_dtype(r, a.dtype),)

        return out, bwd

    @register_vjp(ltorch.log_softmax)
    def _log_softmax(a, dim, dtype=None, **kw):
        out = ltorch.log_softmax(a, dim, dtype=dtype)

        def bwd(g):
            d = clang.canonicalize_dim(a.ndim, dim)
            gf = _upcast(g)
            of = _upcast(out)
            r = ltorch.sub(gf, ltorch.mul(ltorch.exp(of), ltorch.sum(gf, d, True)))
            return (clang.maybe_convert_to_dtype(r, a.dtype),)

        return out, bwd

    @register_vjp(ltorch.sum)
    def _sum(a, dim=None, keepdim=False, *, dtype=None):
        out = ltorch.sum(a, dim, keepdim, dtype=dtype)

        def bwd(g):
            dims = ltorch._dim_list(dim, a.ndim)
            gg = g
            if not keepdim:
                shape = [1 if i in dims else s for i, s in enumerate(a.shape)]
                gg = clang.reshape(gg, tuple(shape))
            return (clang.maybe_convert_to_dtype(clang.expand(gg, a.shape), a.dtype),)

        return out, bwd

    @register_vjp(ltorch.mean)
    def _mean(a, dim=None, keepdim=False, *, dtype=None):
        out = ltorch.mean(a, dim, keepdim, dtype=dtype)

        def bwd(g):
            dims = ltorch._dim_list(dim, a.ndim)
            n = math.prod(a.shape[d] for d in dims) if a.ndim else 1
            gg = g
            if not keepdim:
                shape = [1 if i in dims else s for i, s in enumerate(a.shape)]
                gg = clang.reshape(gg, tuple(shape))
            return (clang.maybe_convert_to_dtype(ltorch.true_divide(clang.expand(gg, a.shape), float(n)), a.dtype),)

        return out, bwd

    @register_vjp(ltorch.embedding)
    def _embedding(a, weight, padding_idx=None, max_norm=None, norm_type=2.0, scale_grad_by_freq=False, sparse=False):
        out = ltorch.embedding(a, weight, padding_idx, max_norm, norm_type, scale_grad_by_freq, sparse)

        def bwd(g):
            pidx = -1 if padding_idx is None else padding_idx
            return None, prims.embedding_backward(g, a, weight.shape[0], pidx, scale_grad_by_freq, sparse)

        return out, bwd

    @register_vjp(ltorch.rms_norm)
    def _rms_norm(a, normalized_shape, weight=None, eps=None):
        if eps is None:
            eps = torch.finfo(a.dtype).eps
        nd = len(normalized_shape)
        dims = tuple(range(a.ndim - nd, a.ndim))
        out = ltorch.rms_norm(a, normalized_shape, weight, eps)

        def bwd(g):
            x = _upcast(a)
            gf = _upcast(g)
            n = math.prod(normalized_shape)
            rstd = ltorch.rsqrt(ltorch.add(ltorch.mean(ltorch.mul(x, x), dims, True), eps))
            xhat = ltorch.mul(x, rstd)
            gw = None
            gy = gf
            if weight is not None:
                wf = _upcast(weight)
                if rg(weight):
                    lead = tuple(range(a.ndim - nd))
                    gw = clang.maybe_convert_to_dtype(ltorch.sum(ltorch.mul(gf, xhat), lead) if lead else ltorch.mul(gf, xhat), weight.dtype)
                gy = ltorch.mul(gf, wf)
            dot = ltorch.mean(ltorch.mul(gy, xhat), dims, True)
            gx = ltorch.mul(ltorch.sub(gy, ltorch.mul(xhat, dot)), rstd)
            return clang.maybe_convert_to_dtype(gx, a.dtype), None, gw

        return out, bwd

    @register_vjp(ltorch.layer_norm)
    def _layer_norm(a, normalized_shape, weight=None, bias=None, eps=1e-5):
        nd = len(normalized_shape)
        dims = tuple(range(a.ndim - nd, a.ndim))
        out = ltorch.layer_norm(a, normalized_shape, weight, bias, eps)

        def bwd(g):
            x = _upcast(a)
            gf = _upcast(g)
            mu = ltorch.mean(x, dims, True)
            xc = ltorch.sub(x, mu)
            rstd = ltorch.rsqrt(ltorch.add(ltorch.mean(ltorch.mul(xc, xc), dims, True), eps))
            xhat = ltorch.mul(xc, rstd)
            lead = tuple(range(a.ndim - nd))
            gw = gb = None
            gy = gf
            if weight is not None:
                if rg(weight):
                    gw = clang.maybe_convert_to_dtype(ltorch.sum(ltorch.mul(gf, xhat), lead) if lead else ltorch.mul(gf, xhat), weight.dtype)
                gy = ltorch.mul(gf, _upcast(weight))
            if bias is not None and rg(bias):
                gb = clang.maybe_convert_to_dtype(ltorch.sum(gf, lead) if lead else gf, bias.dtype)
            m1 = ltorch.mean(gy, dims, True)
            m2 = ltorch.mean(ltorch.mul(gy, xhat), dims, True)
            gx = ltorch.mul(ltorch.sub(ltorch.sub(gy, m1), ltorch.mul(xhat, m2)), rstd)
            return clang.maybe_convert_to_dtype(gx, a.dtype), None, gw, gb

        return out, bwd

    @register_vjp(ltorch.cross_entropy)
    def _cross_entropy(a, target, weight=None, size_average=None, ignore_index=-100, reduce=None, reduction="mean", label_smoothing=0.0):
        if weight is not None or label_smoothing != 0.0 or a.ndim != 2:
            return None  # fall back to decomposition
        out = ltorch.cross_entropy(a, target, None, None, ignore_index, None, reduction, 0.0)

        def bwd(g):
            x = _upcast(a)
            p = ltorch.softmax(x, 1)
            valid = ltorch.ne(target, ignore_index)
            safe = ltorch.where(valid, target, 0)
            oh = clang.maybe_convert_to_dtype(clang.eq(clang.unsqueeze(safe, 1), prims.iota(a.shape[1], start=0, step=1, device=a.device, dtype=torch.int64)), torch.float32)
            d = ltorch.sub(p, oh)
            vf = clang.unsqueeze(clang.maybe_convert_to_dtype(valid, torch.float32), 1)
            d = ltorch.mul(d, vf)
            gf = _upcast(g)
            if reduction == "mean":
                n = ltorch.sum(clang.maybe_convert_to_dtype(valid, torch.float32))
                d = ltorch.mul(d, ltorch.true_divide(gf, n))
            elif reduction == "sum":
                d = ltorch.mul(d, gf)
            else:
                d = ltorch.mul(d, clang.unsqueeze(gf, 1))
            return (clang.maybe_convert_to_dtype(d, a.dtype),)

        return out, bwd

    @register_vjp(ltorch.scaled_dot_product_attention)
    def _sdpa(query, key, value, attn_mask=None, dropout_p=0.0, is_causal=False, *, scale=None, enable_gqa=False):
        if dropout_p != 0.0:
            return None
        out = ltorch.scaled_dot_product_attention(query, key, value, attn_mask, 0.0, is_causal, scale=scale, enable_gqa=enable_gqa)

        def bwd(g):
            return sdpa_reference_backward(query, key, value, attn_mask, is_causal, scale, g)

        return out, bwd


def sdpa_reference_backward(q, k, v, attn_mask, is_causal, scale, g):
    """Math backward of softmax attention (recomputes the probabilities; used when no fused kernel claims SDPA)."""
    ltorch = _lt()
    from .. import clang

    E = q.shape[-1]
    sc = scale if scale is not None else 1.0 / math.sqrt(E)
    rep = q.shape[-3] // k.shape[-3]
    kk = ltorch.repeat_interleave(k, rep, -3) if rep > 1 else k
    vv = ltorch.repeat_interleave(v, rep, -3) if rep > 1 else v
    qf = _upcast(q)
    kf = _upcast(kk)
    vf = _upcast(vv)
    gf = _upcast(g)
    s = ltorch.mul(ltorch.matmul(qf, ltorch.transpose(kf, -2, -1)), sc)
    L, S = q.shape[-2], k.shape[-2]
    if is_causal:
        mask = ltorch.tril(ltorch.ones(L, S, dtype=torch.bool, device=q.device))
        s = ltorch.masked_fill(s, ltorch.logical_not(mask), -math.inf)
    if attn_mask is not None:
        s = ltorch.masked_fill(s, ltorch.logical_not(attn_mask), -math.inf) if attn_mask.dtype == torch.bool else ltorch.add(s, attn_mask)
    p = ltorch.softmax(s, -1)
    dv = ltorch.matmul(ltorch.transpose(p, -2, -1), gf)
    dp = ltorch.matmul(gf, ltorch.transpose(vf, -2, -1))
    ds = ltorch.mul(p, ltorch.sub(dp, ltorch.sum(ltorch.mul(dp, p), -1, True)))
    dq = ltorch.mul(ltorch.matmul(ds, kf), sc)
    dk = ltorch.mul(ltorch.matmul(ltorch.transpose(ds, -2, -1), qf), sc)
    if rep > 1:
        shp = list(k.shape)
        dk = ltorch.sum(ltorch.reshape(dk, tuple(shp[:-3]) + (shp[-3], rep) + tuple(shp[-2:])), -3)
        dv = ltorch.sum(ltorch.reshape(dv, tuple(shp[:-3]) + (shp[-3], rep) + tuple(shp[-2:])), -3)
    grads = (clang.maybe_convert_to_dtype(dq, q.dtype), clang.maybe_convert_to_dtype(dk, k.dtype),
             clang.maybe_convert_to_dtype(dv, v.dtype))
    if attn_mask is not None and attn_mask.dtype != torch.bool and attn_mask.requires_grad:
        # an additive float mask enters the scores unscaled: its gradient is dS, reduced over the
        # dimensions the mask was broadcast along
        from ..core.transforms import sum_to_shape

        grads += (clang.maybe_convert_to_dtype(sum_to_shape(ds, attn_mask.shape), attn_mask.dtype),)
    return grads


_installed = False


def install():
    global _installed
    if _installed:
        return
    _installed = True
    _install_ltorch_rules()
    _register_torch_vjp_impl()
