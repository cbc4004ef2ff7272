"""Program acquisition: run the user's callable on proxies and record a trace (parity: reference
``thunder/core/jit_ext.py`` — ``thunder_general_jit`` :2149-2272, ``unpack_inputs`` :1649-1972,
``process_recorded_modifications`` :1973).

The reference acquires programs with a CPython bytecode interpreter
(``interpreter.py``).  This frontend acquires them by *execution*: module
parameters, buffers and tensor attributes are swapped for proxies, tensor
arguments become proxies, and every torch call is routed through a
``TorchFunctionMode`` to the ``ltorch`` language (or auto-registered as an opaque
op).  Python control flow runs natively and is specialised, exactly like the
reference's "constant values" cache mode.  Provenance of every input is
recorded, so the prologue re-fetches inputs and checks guards on each call,
and attribute writes made during tracing are replayed by the epilogue.
"""
from __future__ import annotations

import contextlib
import math
from numbers import Number
from typing import Any, Callable

import torch
from torch.overrides import TorchFunctionMode

from . import prims
from .codeutils import sanitize_name
from .proxies import Proxy, TensorProxy, DTensorProxy, NumberProxy, AnyProxy, tensorproxy, ProxyTag
from .pytree import tree_flatten, tree_unflatten, tree_map
from .trace import TraceCtx, tracectx, get_tracectx, TraceProvenance
from .symbol import BoundSymbol
from .functionalization import AliasTracker, storage_alias_pattern
from .symbolic import current_env


# -----------------------------------------------------------------------------------------
# Torch function dispatch while tracing
# -----------------------------------------------------------------------------------------
class _AcquisitionState:
    """Per-trace bookkeeping of external (captured) tensors."""

    def __init__(self):
        self.constants: dict[int, tuple[torch.Tensor, TensorProxy]] = {}
        self.lookasides: dict[Callable, Callable] = {}

    def proxify_constant(self, t: torch.Tensor) -> TensorProxy:
        hit = self.constants.get(id(t))
        if hit is not None and hit[0] is t:
            return hit[1]
        p = tensorproxy(t, prefix="tc")
        p.requires_grad = False if not t.requires_grad else True
        p.tags.add(ProxyTag.STATIC_MEMORY_LOCATION)
        self.constants[id(t)] = (t, p)
        trc = get_tracectx()
        if trc is not None and trc.alias_tracker is not None:
            trc.alias_tracker.register_input(p)
        return p


_state_stack: list[_AcquisitionState] = []


def _current_state() -> _AcquisitionState | None:
    return _state_stack[-1] if _state_stack else None


_RANDOM_OR_FACTORY = None


def _random_or_factory_fns():
    global _RANDOM_OR_FACTORY
    if _RANDOM_OR_FACTORY is None:
        names = [
            "rand", "randn", "randint", "rand_like", "randn_like", "randint_like", "randperm", "normal", "bernoulli",
            "multinomial", "empty", "empty_like", "zeros", "zeros_like", "ones", "ones_like", "full", "full_like",
            "arange", "linspace", "tensor",
        ]
        s = set()
        for n in names:
            f = getattr(torch, n, None)
            if f is not None:
                s.add(f)
        f = getattr(torch.nn.functional, "dropout", None)
        if f is not None:
            s.add(f)
        _RANDOM_OR_FACTORY = s
    return _RANDOM_OR_FACTORY


_PASSTHROUGH_NAMES = {"__get__", "__set__", "__repr__", "__format__", "__str__", "__hash__", "__len__", "__bool__"}


def dispatch_torch_function(func, args, kwargs):
    """Routes a torch callable with (possibly) proxy arguments to the ltorch language."""
    from .. import torch as ltorch
    from ..torch.default_torch_ops import opaque_symbol

    trc = get_tracectx()
    flat, spec = tree_flatten((args, kwargs))
    has_proxy = any(isinstance(x, Proxy) for x in flat)
    state = _current_state()

    if state is not None:
        la = state.lookasides.get(func)
        if la is not None:
            return la(*args, **kwargs)

    sym = ltorch._torch_to_thunder_function_map.get(func)
    if trc is None or (not has_proxy and (sym is None or func not in _random_or_factory_fns())):
        # Eager computation on real tensors (constant folding of trace-independent values)
        with _disabled_mode():
            return func(*args, **kwargs)

    name = getattr(func, "__name__", "")
    if name in _PASSTHROUGH_NAMES and not has_proxy:
        return func(*args, **kwargs)

    # Proxify captured real tensors that meet traced values
    if state is not None:
        changed = False
        nflat = []
        for x in flat:
            if isinstance(x, torch.Tensor) and not isinstance(x, Proxy):
                nflat.append(state.proxify_constant(x))
                changed = True
            else:
                nflat.append(x)
        if changed:
            args, kwargs = tree_unflatten(nflat, spec)

    if has_proxy and any(isinstance(x, DTensorProxy) for x in flat):
        from ..distributed.dtensor import dtensor_symbol

        return dtensor_symbol(func)(*args, **kwargs)

    if sym is None:
        from ..torch.custom_op import opdef_of, custom_op_symbol

        od = opdef_of(func)
        if od is not None:  # torch.library custom op: its own symbol, fake-impl meta, registered autograd
            return custom_op_symbol(od)(*args, **kwargs)
    if sym is not None:
        from .symbol import CALLED_TORCH_FN

        prev = CALLED_TORCH_FN[0]
        CALLED_TORCH_FN[0] = func
        try:
            return sym(*args, **kwargs)
        finally:
            CALLED_TORCH_FN[0] = prev
    return opaque_symbol(func)(*args, **kwargs)


class ThunderTorchFunctionMode(TorchFunctionMode):
    def __torch_function__(self, func, types, args=(), kwargs=None):
        from .symbol import META_DEPTH

        if META_DEPTH[0] > 0:
            return func(*args, **(kwargs or {}))
        return dispatch_torch_function(func, args, kwargs or {})


@contextlib.contextmanager
def user_code_tracing():
    """Re-enables tracing of user code called from inside a symbol meta (e.g. activation checkpointing)."""
    from .symbol import META_DEPTH

    prev = META_DEPTH[0]
    META_DEPTH[0] = 0
    try:
        yield
    finally:
        META_DEPTH[0] = prev


@contextlib.contextmanager
def _disabled_mode():
    with torch._C.DisableTorchFunction():
        yield


# -----------------------------------------------------------------------------------------
# Input provenance
# -----------------------------------------------------------------------------------------
class InputSpec:
    """Where a computation input comes from at call time."""

    __slots__ = ("kind", "path", "proxy", "value", "module_path", "attr")

    def __init__(self, kind, path=None, proxy=None, value=None, module_path=None, attr=None):
        self.kind = kind  # "arg" | "param" | "buffer" | "attr" | "const"
        self.path = path
        self.proxy = proxy
        self.value = value
        self.module_path = module_path
        self.attr = attr


def _named_tensor_attrs(module: torch.nn.Module):
    """(module_path, submodule, attr_name, tensor) for plain tensor attributes (not params/buffers)."""
    for mpath, m in module.named_modules(remove_duplicate=True):
        for k, v in list(vars(m).items()):
            if isinstance(v, torch.Tensor) and not isinstance(v, torch.nn.Parameter) and not k.startswith("__"):
                yield mpath, m, k, v


class AcquiredProgram:
    def __init__(self):
        self.prologue_trace: TraceCtx | None = None
        self.computation_trace: TraceCtx | None = None
        self.epilogue_trace: TraceCtx | None = None
        self.input_specs: list[InputSpec] = []
        self.arg_spec = None
        self.param_accessors: list[tuple[torch.nn.Module, str, str]] = []  # (module, name, kind)
        self.constants: list[torch.Tensor] = []
        self.output_spec = None
        self.output_arg_refs: list[tuple[int, int]] = []
        self.epilogue_writes: list[tuple[torch.nn.Module, str]] = []
        self.alias_pattern = None
        self.guards: list = []  # (Prov, value) read by the program through module/global/closure state
        self.guard_roots: list = []
        self.interpreter_log = None
        self.sharp_edges: list[str] = []
        self.n_instructions = 0
        self.symbolic_args: dict[int, NumberProxy] = {}  # flat-arg index -> symbolic number input
        self.specialized_args: set[int] = set()  # symbolic inputs whose value the program read
        self.symbolic_shapes: dict[int, tuple] = {}  # flat-arg index -> shape pattern (None = symbolic dim)


def acquire(fn: Callable, args: tuple, kwargs: dict, *, module: torch.nn.Module | None = None,
            lookasides: dict | None = None, prune_param_checks: bool = True,
            python_lookasides: list | None = None, interpretation: str = "python interpreter",
            record_history: bool | str = False, sharp_edges: str = "allow", show_progress: bool = False,
            symbolic_numbers: bool = False) -> AcquiredProgram:
    """Traces ``fn(*args, **kwargs)`` and builds prologue / computation / epilogue traces.

    ``symbolic_numbers`` (``cache="symbolic values"``): int / float arguments become number inputs
    of the computation, checked by type only, unless the program reads their value (see
    ``NumberProxy.concrete``), in which case that input is specialized and value-checked.

    ``interpretation``: ``"python interpreter"`` (default) runs the user's Python on the bytecode
    interpreter (:mod:`.interpreter`: provenance guards, lookasides on any callable, sharp
    edges, interpreter log); ``"torch function mode"`` runs it natively.  Torch operations are
    captured by the ``TorchFunctionMode`` in both cases."""
    if interpretation not in ("python interpreter", "torch function mode"):
        raise ValueError(f"unknown interpretation {interpretation!r}")
    patched = []
    for owner, attr, repl in python_lookasides or ():
        if hasattr(owner, attr):
            orig = getattr(owner, attr)
            repl.__wrapped_original__ = orig
            patched.append((owner, attr, orig))
            setattr(owner, attr, repl)
    try:
        return _acquire(fn, args, kwargs, module=module, lookasides=lookasides, prune_param_checks=prune_param_checks,
                        symbolic_numbers=symbolic_numbers,
                        interp_options=None if interpretation != "python interpreter" else dict(
                            record_history=record_history, sharp_edges=sharp_edges, show_progress=show_progress))
    finally:
        for owner, attr, orig in reversed(patched):
            setattr(owner, attr, orig)


def _needs_restructure(spec) -> bool:
    """True if the output contains containers the printed trace cannot rebuild (dict subclasses,
    dataclasses, namedtuples such as HF ``ModelOutput``)."""
    if spec.kind == "dict" and spec.ctx[0] is not dict:
        return True
    if spec.kind in ("dataclass", "namedtuple", "structseq"):
        return True
    return any(_needs_restructure(c) for c in spec.children)


def _is_window_of(x: torch.Tensor, x0: torch.Tensor) -> bool:
    """Every element of ``x`` lies inside the (contiguous) argument ``x0``."""
    if not x0.is_contiguous() or x.dtype != x0.dtype or x.numel() == 0:
        return False
    lo = x.storage_offset()
    hi = lo + sum((n - 1) * st for n, st in zip(x.shape, x.stride()) if n > 0)
    return x0.storage_offset() <= lo and hi < x0.storage_offset() + x0.numel() and min(x.stride(), default=1) >= 0


def _has_opaque_container(spec) -> bool:
    if spec.kind in ("dataclass", "namedtuple", "structseq") or (spec.kind == "dict" and len(spec.ctx) > 2):
        return True
    return any(_has_opaque_container(c) for c in spec.children)


def _argument_provenance(args, kwargs):
    """``Prov("input", key=flat_index)`` for every top-level argument that is a pytree leaf."""
    from .interpreter import Prov
    from .pytree import LEAF

    off = 0
    aprov = []
    for a in args:
        leaves, spec = tree_flatten(a)
        aprov.append(Prov("input", key=off) if spec is LEAF and not isinstance(a, (torch.Tensor, Proxy)) else None)
        off += len(leaves)
    kprov = {}
    for k, v in kwargs.items():
        leaves, spec = tree_flatten(v)
        if spec is LEAF and not isinstance(v, (torch.Tensor, Proxy)):
            kprov[k] = Prov("input", key=off)
        off += len(leaves)
    return aprov, kprov


def _annotate_with_interpreted_stack(e: Exception, stack: list[str]) -> None:
    """Appends the interpreted (user-code) call stack to an exception raised while tracing."""
    if not stack or getattr(e, "_lta_annotated", False):
        return
    try:
        e._lta_annotated = True
        if e.args and isinstance(e.args[0], str):
            e.args = (e.args[0] + "\n\nwhile tracing (innermost last):\n  " + "\n  ".join(reversed(stack)),) + e.args[1:]
    except Exception:  # exceptions with read-only args
        pass


def _storage_ptr(x: torch.Tensor):
    if x.device.type == "meta" or type(x) is not torch.Tensor and not isinstance(x, torch.nn.Parameter):
        return None
    try:
        return x.untyped_storage().data_ptr()
    except (RuntimeError, NotImplementedError):
        return None


def _acquire(fn: Callable, args: tuple, kwargs: dict, *, module: torch.nn.Module | None = None,
             lookasides: dict | None = None, prune_param_checks: bool = True,
             interp_options: dict | None = None, symbolic_numbers: bool = False) -> AcquiredProgram:
    prog = AcquiredProgram()
    comp = TraceCtx(fn if not isinstance(fn, torch.nn.Module) else type(fn).forward)
    comp.fn_name = "computation"
    from ..transforms.autocast import current_autocast_dtype

    comp.autocast_dtype = current_autocast_dtype()
    state = _AcquisitionState()
    if lookasides:
        state.lookasides.update(lookasides)

    flat_args, arg_spec = tree_flatten((args, kwargs))
    prog.arg_spec = arg_spec
    swapped: list[tuple[dict, str, Any]] = []
    attr_swaps: list[tuple[torch.nn.Module, str, Any]] = []
    tracker = AliasTracker(comp)
    tracker.input_specs = prog.input_specs
    comp.alias_tracker = tracker

    with tracectx(comp):
        # 1. tensor arguments (a tensor passed twice is an identity view of its first occurrence;
        #    partially overlapping arguments may not be mutated)
        proxied_flat = []
        arg_proxies = []
        by_view: dict = {}
        by_storage: dict = {}
        for i, x in enumerate(flat_args):
            if isinstance(x, torch.Tensor):
                p = tensorproxy(x)
                env = current_env()
                if symbolic_numbers and env is not None and not isinstance(x, torch.nn.Parameter) and x.ndim:
                    # cache="symbolic values": every dim >= 2 of a non-parameter tensor argument is a
                    # symbol (core/symbolic.py); 0 / 1 stay static (broadcasting depends on them)
                    p._shape = tuple(env.new_symbol(n, i, d) if n >= 2 else n for d, n in enumerate(x.shape))
                    prog.symbolic_shapes[i] = tuple(None if n >= 2 else n for n in x.shape)
                arg_proxies.append((i, p))
                proxied_flat.append(p)
                prog.input_specs.append(InputSpec("arg", path=i, proxy=p))
                tracker.register_input(p)
                sp = _storage_ptr(x)
                if sp is not None:
                    key = (sp, x.storage_offset(), tuple(x.shape), tuple(x.stride()), x.dtype)
                    if key in by_view:
                        tracker.register_identity_alias(p, by_view[key])
                    else:
                        by_view[key] = p
                        if sp in by_storage:
                            x0, p0 = by_storage[sp]
                            if _is_window_of(x, x0):
                                # a strided window of an earlier argument (e.g. ``f(a, a[1:])``): an
                                # in-place write to either is seen by the other through the view
                                tracker.register_window_alias(p, p0, x.shape, x.stride(),
                                                              x.storage_offset() - x0.storage_offset())
                            else:
                                tracker.partial_alias.update((id(p), id(p0)))
                        by_storage.setdefault(sp, (x, p))
            elif symbolic_numbers and type(x) in (int, float):
                from .proxies import IntegerProxy, FloatProxy

                cls = IntegerProxy if type(x) is int else FloatProxy
                p = cls(x, name=comp.make_unique_name("i" if type(x) is int else "f"))

                def _specialize(i=i):
                    prog.specialized_args.add(i)

                p._on_value = _specialize
                prog.symbolic_args[i] = p
                env = current_env()
                if env is not None and type(x) is int and x >= 2:
                    # an int size argument is a dim symbol like a tensor's (core/symbolic.py): the program
                    # sees a SymInt, the number input only carries the value the program binds it from
                    si = env.new_symbol(x, i, None)
                    p._sym = si.expr
                    proxied_flat.append(si)
                else:
                    proxied_flat.append(p)
                prog.input_specs.append(InputSpec("arg", path=i, proxy=p))
            else:
                proxied_flat.append(x)
        pargs, pkwargs = tree_unflatten(proxied_flat, arg_spec)

        # 2. module state
        if module is not None:
            seen: dict[int, TensorProxy] = {}
            for mpath, m in module.named_modules(remove_duplicate=False):
                for pname, param in list(m._parameters.items()):
                    if param is None:
                        continue
                    full = f"{mpath}.{pname}" if mpath else pname
                    if id(param) in seen:
                        p = seen[id(param)]
                    else:
                        p = tensorproxy(param, name=comp.make_unique_name("t_" + full))
                        full_shape = getattr(param, "_lc_full_shape", None)
                        if full_shape is not None:
                            # sharded (FSDP) parameter: the model code sees the full shape; the
                            # FSDP transform re-types the input as the local shard + all-gather.
                            p._shape = tuple(full_shape)
                            p.tags.add("sharded")
                        tp_kind = getattr(param, "_lc_tp_kind", None)
                        if tp_kind in ("head_qkv", "head_proj"):
                            # head-parallel attention weight: traced with its LOCAL shape (the
                            # attention module's config was localized to this rank's heads)
                            p.tags.add("tp_" + tp_kind)
                        p.tags.add(ProxyTag.STATIC_MEMORY_LOCATION)
                        p.tags.add("parameter")
                        seen[id(param)] = p
                        prog.input_specs.append(InputSpec("param", path=full, proxy=p, module_path=mpath, attr=pname))
                        tracker.register_input(p)
                        prog.param_accessors.append((m, pname, "param"))
                    swapped.append((m._parameters, pname, param))
                    m._parameters[pname] = p
                for bname, buf in list(m._buffers.items()):
                    if buf is None:
                        continue
                    full = f"{mpath}.{bname}" if mpath else bname
                    if id(buf) in seen:
                        p = seen[id(buf)]
                    else:
                        p = tensorproxy(buf, name=comp.make_unique_name("t_" + full))
                        p.tags.add(ProxyTag.STATIC_MEMORY_LOCATION)
                        seen[id(buf)] = p
                        prog.input_specs.append(InputSpec("buffer", path=full, proxy=p, module_path=mpath, attr=bname))
                        tracker.register_input(p)
                        prog.param_accessors.append((m, bname, "buffer"))
                    swapped.append((m._buffers, bname, buf))
                    m._buffers[bname] = p
            for mpath, m, k, v in list(_named_tensor_attrs(module)):
                full = f"{mpath}.{k}" if mpath else k
                if id(v) in seen:
                    p = seen[id(v)]
                else:
                    p = tensorproxy(v, name=comp.make_unique_name("t_" + full))
                    p.tags.add(ProxyTag.STATIC_MEMORY_LOCATION)
                    seen[id(v)] = p
                    prog.input_specs.append(InputSpec("attr", path=full, proxy=p, module_path=mpath, attr=k))
                    tracker.register_input(p)
                    prog.param_accessors.append((m, k, "attr"))
                attr_swaps.append((m, k, v))
                object.__setattr__(m, k, p)

        # snapshot of module attribute identity to detect writes made during tracing
        before = {}
        before_buffers = {}
        if module is not None:
            for mpath, m in module.named_modules(remove_duplicate=True):
                before[id(m)] = dict(vars(m))
                before_buffers[id(m)] = dict(m._buffers)

        interp = None
        if interp_options is not None:
            from .interpreter import Interpreter

            prov_inputs: dict[int, tuple] = {}

            def _capture(t, prov):
                """A real tensor read through Python state becomes a computation input: re-fetched
                along its provenance by the prologue when the chain starts at an argument, a global,
                a closure cell or the module; otherwise captured as a constant."""
                if isinstance(t, Proxy):
                    return t
                hit = prov_inputs.get(id(t))
                if hit is not None and hit[0] is t:
                    return hit[1]
                root = prov.root().kind if prov is not None else None
                if root in ("input", "global", "cell") or (root == "module" and module is not None):
                    c = state.constants.get(id(t))
                    if c is not None and c[0] is t:
                        return c[1]
                    p = tensorproxy(t, name=comp.make_unique_name("tp"))
                    if isinstance(t, torch.nn.Parameter):
                        p.tags.add("nn_parameter")  # isinstance(.., nn.Parameter) holds for user code
                    if root != "input":
                        # module / global / closure state lives across calls; tensors reached through
                        # an argument (a cache object handed in per call) belong to the caller
                        p.tags.add(ProxyTag.STATIC_MEMORY_LOCATION)
                    tracker.register_input(p)
                    prov_inputs[id(t)] = (t, p, prov)
                    return p
                return state.proxify_constant(t)

            interp = Interpreter(lookasides=lookasides, module=module, tensor_hook=_capture, **interp_options)
            # provenance of top-level (leaf) arguments: their index in the flattened inputs
            arg_provs, kw_provs = _argument_provenance(args, kwargs)
        _state_stack.append(state)
        try:
            with ThunderTorchFunctionMode():
                target = module if module is not None else fn
                if interp is not None:
                    try:
                        result = interp.call(target, pargs, pkwargs, arg_provs=arg_provs, kw_provs=kw_provs)
                    except Exception as e:
                        _annotate_with_interpreted_stack(e, interp.error_stack)
                        raise
                else:
                    result = target(*pargs, **pkwargs)
        finally:
            _state_stack.pop()
            # detect attribute writes (epilogue) before restoring
            writes = []
            if module is not None:
                for mpath, m in module.named_modules(remove_duplicate=True):
                    old = before.get(id(m), {})
                    for k, v in vars(m).items():
                        if isinstance(v, TensorProxy) and old.get(k) is not v:
                            writes.append((m, k, v))
                    old_b = before_buffers.get(id(m), {})
                    for k, v in m._buffers.items():  # `self.buf = new` rebinds a registered buffer
                        if isinstance(v, TensorProxy) and old_b.get(k) is not v:
                            writes.append((m, k, v))
            for d, k, v in swapped:
                d[k] = v
            for m, k, v in attr_swaps:
                # if the attribute was overwritten during tracing keep the write for the epilogue
                object.__setattr__(m, k, v)

        # 3. captured constants become inputs
        for t, p in state.constants.values():
            prog.constants.append(t)
            prog.input_specs.append(InputSpec("const", proxy=tracker.original(p), value=t))

        # 4. epilogue writes are returned from the computation
        prog.epilogue_writes = [(m, k) for m, k, v in writes]
        epi_values = [v for m, k, v in writes]

        # outputs: real tensors in the result are constants
        def fix_out(x):
            if isinstance(x, torch.Tensor) and not isinstance(x, Proxy):
                return state.proxify_constant(x)
            return x

        result = tree_map(fix_out, result)
        out_leaves, out_spec = tree_flatten(result)
        # non-tensor objects returned from the inputs (an HF cache passed in and handed back in the
        # ModelOutput) must be the caller's objects of *this* call, not the ones seen while tracing
        arg_ids = {id(a): j for j, a in enumerate(flat_args)
                   if not isinstance(a, (torch.Tensor, Proxy, bool, int, float, str, type(None)))}
        prog.output_arg_refs = [(i, arg_ids[id(v)]) for i, v in enumerate(out_leaves) if id(v) in arg_ids]
        epi_values = [tracker.refresh(v) or v for v in epi_values]
        result = tracker.finish(result)
        comp.alias_tracker = None
        prog.alias_pattern = storage_alias_pattern(flat_args) if tracker.any_mutation else None
        for t, p in state.constants.values():
            if all(t is not c for c in prog.constants):
                prog.constants.append(t)
                prog.input_specs.append(InputSpec("const", proxy=tracker.original(p), value=t))
        if _has_opaque_container(out_spec):
            # dataclasses / namedtuples are not printable in the program: it returns the flat
            # leaves and the runtime rebuilds the container from ``output_spec``
            result = tuple(tree_flatten(result)[0])
        if epi_values:
            prims.python_return((result, tuple(epi_values)))
        else:
            prims.python_return(result)

    if interp is not None:
        for t, p, prov in prov_inputs.values():
            prog.input_specs.append(InputSpec("prov", proxy=tracker.original(p), value=prov))
        prog.guards = list(interp.guards.values())
        prog.interpreter_log = interp.history
        prog.sharp_edges = interp.sharp_edges_seen
        prog.n_instructions = interp.n_instructions
    comp.args = [s.proxy for s in prog.input_specs]
    comp.set_provenance(TraceProvenance(
        "Acquisition (bytecode interpreter)" if interp is not None else "Acquisition (torch function mode)"))
    prog.computation_trace = comp
    prog.output_spec = out_spec if _needs_restructure(out_spec) else None
    prog.prologue_trace = build_prologue(prog, flat_args, prune_param_checks=prune_param_checks, module_root=module)
    if prog.epilogue_writes:
        prog.epilogue_trace = None  # epilogue is applied by the runtime (see common.run_epilogue)
    return prog


def _emit_provenance_guards(prog: AcquiredProgram, roots_proxy, module_root, unpacked_args) -> list:
    """Prologue checks for Python values the program read through module/global/closure state.

    Each guard re-fetches its value along its provenance chain (``unpack_attr``/``unpack_key``
    from a guard root: the compiled module, a globals dict or a closure cell) and checks it
    (reference: provenance-driven ``unpack_inputs``, ``thunder/core/jit_ext.py:1649-1972``)."""
    roots: list = []
    root_ids: dict[int, int] = {}

    def root_index(obj):
        i = root_ids.get(id(obj))
        if i is None:
            i = len(roots)
            root_ids[id(obj)] = i
            roots.append(obj)
        return i

    prov_specs = [s for s in prog.input_specs if s.kind == "prov"]
    chains = []
    for prov, value in list(prog.guards) + [(s.value, s) for s in prov_specs]:
        r = prov.root()
        if r.kind == "module":
            if module_root is None:
                continue
            root_index(module_root)
        elif r.kind == "global":
            root_index(r.parent)
        elif r.kind == "cell":
            root_index(r.parent)
        chains.append((prov, value))
    if not chains:
        return []
    root_vals = prims.unpack_sequence(roots_proxy, len(roots)) if roots else []
    memo: dict = {}

    def key_of(p):
        if p.kind == "module":
            return ("module", p.key)
        if p.kind == "input":
            return ("input", p.key)
        if p.kind in ("global", "cell"):
            return (p.kind, id(p.parent), p.key)
        return (key_of(p.parent), p.kind, p.key)

    def emit(p):
        k = key_of(p)
        hit = memo.get(k)
        if hit is not None:
            return hit
        if p.kind == "module":
            out = root_vals[root_ids[id(module_root)]]
            path = ""
            for part in (p.key.split(".") if p.key else ()):
                path = f"{path}.{part}" if path else part
                sub = memo.get(("module", path))
                out = sub if sub is not None else prims.unpack_attr(out, part)
                memo[("module", path)] = out
        elif p.kind == "input":
            out = unpacked_args[p.key]
        elif p.kind == "global":
            out = prims.unpack_key(root_vals[root_ids[id(p.parent)]], p.key)
        elif p.kind == "cell":
            out = prims.unpack_attr(root_vals[root_ids[id(p.parent)]], "cell_contents")
        elif p.kind == "attr":
            out = prims.unpack_attr(emit(p.parent), p.key)
        else:
            out = prims.unpack_key(emit(p.parent), p.key)
        memo[k] = out
        return out

    fetched = []
    for prov, value in chains:
        v = emit(prov)
        if isinstance(value, InputSpec):  # a tensor input re-fetched along its provenance
            t = value.proxy
            prims.check_tensor_shape_and_metadata(v, tuple(t.shape), str(t.device), t.dtype, t.requires_grad)
            fetched.append(v)
            continue
        if value is None:
            prims.check_none(v)
        elif isinstance(value, str):
            prims.check_string_value(v, value)
        elif isinstance(value, (bool, int, float)):
            prims.check_number_type_and_value(v, value)
        else:
            prims.check_literal_like(v, value)
    prog.guard_roots = roots
    return fetched


def build_prologue(prog: AcquiredProgram, flat_args: list, *, prune_param_checks: bool,
                   module_root: torch.nn.Module | None = None) -> TraceCtx:
    """Prologue: flattened args -> checks -> computation inputs (reference ``unpack_inputs`` :1649)."""
    pro = TraceCtx(None)
    pro.fn_name = "prologue"
    with tracectx(pro):
        fa = AnyProxy(None, name="flat_args")
        st = AnyProxy(None, name="module_state")
        cs = AnyProxy(None, name="constants")
        gr = AnyProxy(None, name="guard_roots")
        pro.args = [fa, st, cs, gr]
        n = len(flat_args)
        unpacked = prims.unpack_sequence(fa, n)
        for i, (u, x) in enumerate(zip(unpacked, flat_args)):
            if isinstance(x, torch.Tensor):
                # symbolic dims are checked by the guards of the cache entry (core/symbolic.py)
                shape = prog.symbolic_shapes.get(i, tuple(x.shape))
                prims.check_tensor_shape_and_metadata(u, shape, str(x.device), x.dtype, x.requires_grad)
            elif x is None:
                prims.check_none(u)
            elif isinstance(x, str):
                prims.check_string_value(u, x)
            elif i in prog.symbolic_args and i not in prog.specialized_args:
                prims.check_number_type(u, type(x))
            elif isinstance(x, (bool, int, float, complex)):
                prims.check_number_type_and_value(u, x)
            elif isinstance(x, (torch.dtype, torch.device)):
                prims.check_literal_like(u, x)
        arg_outs = [unpacked[s.path] for s in prog.input_specs if s.kind == "arg"]
        n_state = len(prog.param_accessors)
        state_vals = prims.unpack_sequence(st, n_state) if n_state else []
        if not prune_param_checks:
            j = 0
            for s in prog.input_specs:
                if s.kind in ("param", "buffer", "attr"):
                    p = s.proxy
                    prims.check_tensor_shape_and_metadata(state_vals[j], tuple(p.shape), str(p.device), p.dtype, p.requires_grad)
                    j += 1
        fetched = []
        if prog.guards or any(s.kind == "prov" for s in prog.input_specs):
            fetched = _emit_provenance_guards(prog, gr, module_root, unpacked)
        n_const = len(prog.constants)
        const_vals = prims.unpack_sequence(cs, n_const) if n_const else []
        prims.python_return(list(arg_outs) + list(state_vals) + list(const_vals) + list(fetched))
    pro.set_provenance(TraceProvenance("Prologue construction"))
    return pro
