"""lightning_thunder_amd — an MI355X-native source-to-source compiler for PyTorch.

Public API parity with the reference's ``thunder/__init__.py`` (``jit`` :315-921,
``compile`` :274-311, introspection :924-1100).  Typical use::

    import lightning_thunder_amd as thunder
    tm = thunder.jit(model)                       # or thunder.compile(model, plugins=["fsdp", "reduce-overhead"])
    loss = tm(x).sum(); loss.backward()
    print(thunder.last_traces(tm)[-1])            # the executed program (printable python)
"""
from __future__ import annotations

import os
import time
from typing import Any, Callable, Sequence

import torch as _torch

from .core import dtypes, devices, prims
from .core.proxies import (
    Proxy, TensorProxy, NumberProxy, IntegerProxy, FloatProxy, ComplexProxy, StringProxy, TupleProxy,
    ListProxy, DictProxy, AnyProxy, FutureTensorProxy, DistParallelType,
)
from .core.trace import TraceCtx, tracectx, _set_execution_file
from .core.transform_common import Transform, dce
from .core.pytree import tree_flatten, tree_unflatten
from .common import (
    CACHE_OPTIONS, SHARP_EDGES_OPTIONS, CompileData, CompileStats, DebugOptions, resolve_cache_option,
    resolve_sharp_edges_option, get_compile_data, _compile_data_ctx,
)
from . import extend
from .extend import (
    resolve_executors, add_executor_lists, get_executor, get_all_executors, get_default_executors,
    get_always_executors, add_default_executor,
)
from . import clang
from . import torch as ltorch
from .core.module import ThunderModule

__version__ = "0.1.0"

bool8 = dtypes.bool8
uint8 = dtypes.uint8
int8 = dtypes.int8
int16 = dtypes.int16
int32 = dtypes.int32
int64 = dtypes.int64
bfloat16 = dtypes.bfloat16
float8_e5m2 = dtypes.float8_e5m2
float8_e5m2fnuz = dtypes.float8_e5m2fnuz
float8_e4m3fn = dtypes.float8_e4m3fn
float8_e4m3fnuz = dtypes.float8_e4m3fnuz
float16 = dtypes.float16
float32 = dtypes.float32
float64 = dtypes.float64
complex32 = dtypes.complex32
complex64 = dtypes.complex64
complex128 = dtypes.complex128

set_execution_callback_file = _set_execution_file

# executors: importing registers them and the default list
extend._ensure_builtin_executors()
pytorch_executor = get_executor("torch")
python_executor = get_executor("python")
hipex_executor = get_executor("hipex")
hipfuse_executor = get_executor("hipfuse")

from .transforms import autodiff as _autodiff  # noqa: E402

_autodiff.install()


from .core.profile import annotate_for_profile as _annotate_for_profile  # noqa: E402


def _default_executor_list():
    return get_default_executors()


# =========================================================================================
# Cache entries
# =========================================================================================
class CacheEntry:
    def __init__(self):
        self.prologue_fn = None
        self.computation_fn = None
        self.forward_fn = None
        self.backward_fn = None
        self.overlap_optimizer = None  # transforms/optimizer_overlap.py
        self.epilogue_writes = []
        self.param_accessors = []
        self.constants = []
        self.grad_enabled = False
        self.uses_autograd = False
        self.no_grad_sync = False
        self.alias_pattern = None
        self.grad_input_indices = []
        self.diff_output_mask = []
        self.diff_output_meta = []
        self.prologue_traces = []
        self.computation_traces = []
        self.backward_traces = []
        self._last_out_spec = None
        self._last_flat_out = None
        self.has_epilogue = False
        self.autocast_key = None
        self.guard_roots = []
        self.output_spec = None
        self.output_arg_refs = []
        self.interpreter_log = None
        self.sharp_edges = []

    def module_state(self):
        out = []
        for m, n, kind in self.param_accessors:
            if kind == "param":
                out.append(m._parameters[n])
            elif kind == "buffer":
                out.append(m._buffers[n])
            else:
                out.append(getattr(m, n))
        return out


def _autocast_key():
    if _torch.is_autocast_enabled("cuda") if _has_device_autocast() else _torch.is_autocast_enabled():
        return ("cuda", _torch.get_autocast_dtype("cuda") if hasattr(_torch, "get_autocast_dtype") else _torch.get_autocast_gpu_dtype())
    if _torch.is_autocast_enabled("cpu") if _has_device_autocast() else False:
        return ("cpu", _torch.get_autocast_dtype("cpu") if hasattr(_torch, "get_autocast_dtype") else _torch.get_autocast_cpu_dtype())
    return None


def _has_device_autocast():
    global _HAS_DEVICE_AUTOCAST
    if _HAS_DEVICE_AUTOCAST is None:
        try:
            _torch.is_autocast_enabled("cuda")
            _HAS_DEVICE_AUTOCAST = True
        except TypeError:
            _HAS_DEVICE_AUTOCAST = False
    return _HAS_DEVICE_AUTOCAST


_HAS_DEVICE_AUTOCAST = None


def _check_traces(traces, cd):
    if cd.debug_options.check_traces:
        from .dev_utils.check_trace import check_trace

        for t in traces:
            check_trace(t)


from .core.functionalization import storage_alias_pattern  # noqa: E402


def _overlap_allowed(cd: CompileData) -> bool:
    """Optimizer-in-backward hooks: single process only, and not inside captured hipGraphs."""
    import torch.distributed as dist

    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        return False
    from .transforms.hipgraph import HipGraphTransform

    return not any(isinstance(t, HipGraphTransform) for t in cd.transforms)


def _post_transforms(cd: CompileData) -> list:
    """User transforms, plus the kernel-sync debug transform when requested."""
    ts = list(cd.transforms)
    if cd.debug_options.sync_after_each_kernel:
        from .dev_utils.numerics_check import SyncAfterEachKernelTransform

        ts.append(SyncAfterEachKernelTransform())
    return ts


def _build_cache_entry(cd: CompileData, cs: CompileStats, module, args, kwargs) -> CacheEntry:
    from .core.jit_ext import acquire
    from .executors.passes import transform_for_execution, del_last_used
    from .transforms.autodiff import forward_and_backward_from_trace
    from .distributed.utils import maybe_sort_waits

    entry = CacheEntry()
    entry.grad_enabled = _torch.is_grad_enabled()
    entry.autocast_key = _autocast_key()
    from .distributed import get_skip_data_parallel_grad_sync

    entry.no_grad_sync = get_skip_data_parallel_grad_sync()

    cs.last_trace_tracing_start = time.perf_counter_ns()
    tok = _compile_data_ctx.set(cd)
    from .core.symbolic import ShapeEnv, current_env, _env as _shape_env_var

    senv = ShapeEnv() if cd.cache_option is CACHE_OPTIONS.SYMBOLIC_VALUES else None
    senv_tok = _shape_env_var.set(senv)
    try:
        lookasides = {}
        python_lookasides = []
        for ex in cd.executors_list:
            lookasides.update(ex._lookasides)
            python_lookasides.extend(getattr(ex, "_python_lookasides", ()))
        if _torch.distributed.is_available():
            from .distributed.dtensor import python_lookasides as _dt_lookasides

            python_lookasides.extend(_dt_lookasides())
        from .transforms.autocast import autocast_ctx

        default_dtype = _torch.get_default_dtype()
        with autocast_ctx(entry.autocast_key):
            dbg = cd.debug_options
            record = cd.get_compile_option("record_interpreter_history", "Record the interpreter log", None)
            if record is None:
                record = dbg.record_interpreter_history
            prog = acquire(cd.fn if module is None else module, args, kwargs, module=module, lookasides=lookasides,
                           prune_param_checks=cd.compile_options.get("prune_prologue_checks", True),
                           python_lookasides=python_lookasides,
                           interpretation=cd.get_compile_option(
                               "interpretation", "'python interpreter' (bytecode interpreter, default) or "
                               "'torch function mode'", "python interpreter"),
                           record_history=record, sharp_edges=cd.sharp_edges.value,
                           show_progress=dbg.show_interpreter_progress,
                           symbolic_numbers=cd.cache_option is CACHE_OPTIONS.SYMBOLIC_VALUES)
        cs.last_trace_tracing_stop = time.perf_counter_ns()
        # global modes user code flipped while it was being interpreted: grad mode is recorded per
        # op (BoundSymbolTag.NO_GRAD) and restored; a changed default dtype would make the program
        # disagree with the cache key (reference: same error in thunder/__init__.py)
        _torch.set_grad_enabled(entry.grad_enabled)
        if _torch.get_default_dtype() != default_dtype:
            _torch.set_default_dtype(default_dtype)
            raise RuntimeError("Default dtype is changed during the execution of jitted function. "
                               "This is currently unsupported.")
        pro, comp, epi = prog.prologue_trace, prog.computation_trace, prog.epilogue_trace
        computation_traces = [comp]
        for t in cd.transforms:
            pro, comp, epi = t.transform_traces_pre_prologue(pro, comp, epi, compile_data=cd)
            comp.set_provenance(f"{type(t).__name__}.transform_traces_pre_prologue")
            computation_traces.append(comp)
        comp = dce(comp)
        computation_traces.append(comp)

        entry.output_spec = prog.output_spec
        entry.output_arg_refs = prog.output_arg_refs
        entry.guard_roots = prog.guard_roots
        entry.interpreter_log = prog.interpreter_log
        entry.sharp_edges = prog.sharp_edges
        cs.last_interpreter_log = prog.interpreter_log
        entry.param_accessors = prog.param_accessors
        entry.alias_pattern = prog.alias_pattern
        entry.constants = prog.constants
        entry.epilogue_writes = prog.epilogue_writes
        entry.has_epilogue = bool(prog.epilogue_writes)
        entry._same_input_positions = [s.path for s in prog.input_specs if s.kind == "arg"]
        entry.has_prov_inputs = any(s.kind == "prov" for s in prog.input_specs)
        from .executors.pythonex import ex as pyex

        pro_exec = transform_for_execution(pro, [pyex])[-1]
        entry.prologue_fn = pro_exec.python_callable()
        entry.prologue_traces = [pro, pro_exec]
        specialized_at_prologue = set(prog.specialized_args)

        requires_grad = (
            entry.grad_enabled
            and not cd.disable_torch_autograd
            and any(isinstance(a, TensorProxy) and a.requires_grad for a in comp.args)
        )
        executors = cd.executors_list
        if requires_grad:
            fb = forward_and_backward_from_trace(comp, executors=executors)
            if cd.compile_options.get("rematerialize", True):
                from .transforms.rematerialization import rematerialize_forward_and_backward
                from .core.symbolic import no_guards

                with no_guards():  # a cut is valid for every size: its weights record no shape guards
                    fb = rematerialize_forward_and_backward(fb)
            from .distributed.utils import lower_tp_syncs

            fw_traces = [fb.forward_trace] + transform_for_execution(lower_tp_syncs(fb.forward_trace), executors)
            bw_traces = [fb.backward_trace] + transform_for_execution(lower_tp_syncs(fb.backward_trace), executors)
            fw = fw_traces[-1]
            bw = bw_traces[-1]
            fw = maybe_sort_waits(fw)
            bw = maybe_sort_waits(bw)
            window = cd.compile_options.get("lta_fsdp_allgather_window")
            if window:
                from .distributed.utils import schedule_allgathers

                fw = schedule_allgathers(fw, int(window))
                bw = schedule_allgathers(bw, int(window))
            opt = getattr(cd, "overlap_optimizer", None)
            if opt is not None and _overlap_allowed(cd):
                from .transforms.optimizer_overlap import insert_grad_ready_hooks

                names = [comp.args[i].name if isinstance(comp.args[i], TensorProxy) else None
                         for i in fb.grad_input_indices]
                bw = insert_grad_ready_hooks(bw, names, getattr(cd, "overlap_bucket_bytes", 128 << 20), fw=fw)
                entry.overlap_optimizer = opt
            fw = del_last_used(fw)
            bw = del_last_used(bw)
            bw.unpack_list_arg = True
            for t in _post_transforms(cd):
                fw = t.transform_trace_post_optimization(fw, compile_data=cd)
                bw = t.transform_trace_post_optimization(bw, compile_data=cd)
            fw_traces.append(fw)
            bw_traces.append(bw)
            _check_traces(fw_traces + bw_traces, cd)
            entry.forward_fn = fw.python_callable()
            entry.backward_fn = bw.python_callable()
            entry.uses_autograd = True
            entry.grad_input_indices = fb.grad_input_indices
            entry.diff_output_mask = fb.diff_output_mask
            flat_out, _ = tree_flatten(fb.forward_trace.output[0] if fb.forward_trace.output is not None else None)
            entry.diff_output_meta = [
                (tuple(o.shape), o.dtype, o.device) for o, d in zip(flat_out, fb.diff_output_mask) if d
            ]
            entry.computation_traces = computation_traces + fw_traces
            entry.backward_traces = bw_traces
        else:
            if cd.compile_options.get("inplace_index_copy", True):
                from .transforms.inplace_index_copy import inplace_index_copy

                comp2 = inplace_index_copy(comp)
                if comp2 is not comp:
                    comp = comp2
                    computation_traces.append(comp)
            from .distributed.utils import lower_tp_syncs

            ex_traces = transform_for_execution(lower_tp_syncs(comp), executors)
            c = ex_traces[-1]
            c = maybe_sort_waits(c)
            window = cd.compile_options.get("lta_fsdp_allgather_window")
            if window:
                from .distributed.utils import schedule_allgathers

                c = schedule_allgathers(c, int(window))
            c = del_last_used(c)
            for t in _post_transforms(cd):
                c = t.transform_trace_post_optimization(c, compile_data=cd)
            ex_traces.append(c)
            _check_traces(ex_traces, cd)
            entry.computation_fn = c.python_callable()
            entry.computation_traces = computation_traces + ex_traces
        late = prog.specialized_args - specialized_at_prologue
        if late:
            # a transform read a symbolic number's value after the prologue was built: the program
            # is specialized on it, so the cache entry must check that value too
            from .executors.pythonex import _check_number

            flat_now, _ = tree_flatten((args, kwargs))
            vals = {i: flat_now[i] for i in late}
            base = entry.prologue_fn

            def prologue_with_late_checks(fa, *rest, _base=base, _vals=vals):
                for i, v in _vals.items():
                    _check_number(fa[i], v)
                return _base(fa, *rest)

            entry.prologue_fn = prologue_with_late_checks
        if senv is not None and senv.symbols:
            # symbolic tensor dims: the prologue checked ranks and static dims; the guards recorded
            # while tracing, transforming and claiming (core/symbolic.py) decide the rest
            from .executors.pythonex import ThunderCacheMiss

            guards = senv.guard_fn()
            base2 = entry.prologue_fn

            def prologue_with_shape_guards(fa, *rest, _base=base2, _g=guards):
                out = _base(fa, *rest)
                if not _g(fa):
                    raise ThunderCacheMiss("symbolic shape guards")
                return out

            entry.prologue_fn = prologue_with_shape_guards
            entry.shape_guards = guards
    finally:
        _shape_env_var.reset(senv_tok)
        _compile_data_ctx.reset(tok)
        _torch.set_grad_enabled(entry.grad_enabled)
    return entry


def _run_entry(entry: CacheEntry, inps, flat_args=None):
    if entry.uses_autograd:
        from .executors.torch_autograd import connect_to_autograd

        out = connect_to_autograd(entry, inps)
    else:
        out = entry.computation_fn(*inps)
    if entry.has_epilogue:
        out, epi_vals = out
        for (m, k), v in zip(entry.epilogue_writes, epi_vals):
            if k in m._buffers:
                m._buffers[k] = v
            else:
                object.__setattr__(m, k, v)
    if entry.output_arg_refs and flat_args is not None:  # input objects handed back: this call's
        leaves, spec = tree_flatten(out)
        for i, j in entry.output_arg_refs:
            leaves[i] = flat_args[j]
        out = tree_unflatten(leaves, spec)
    if entry.output_spec is not None:  # rebuild ModelOutput / dataclass / namedtuple results
        out = tree_unflatten(tree_flatten(out)[0], entry.output_spec)
    return out


def jit(
    fn: Callable,
    /,
    *,
    langctx: Any = None,
    executors: Sequence | None = None,
    sharp_edges: Any = None,
    cache: Any = None,
    disable_torch_autograd: bool = False,
    transforms: list | None = None,
    debug_options: DebugOptions | None = None,
    **compile_options,
) -> Callable:
    """Just-in-time compile a function or ``nn.Module`` (reference ``thunder.jit`` :315).

    Keyword Args:
        executors: executor list (names or objects); defaults to ``get_default_executors()``
            (``hipex → hipfuse → torch``), always amended with the always-executors.
        cache: ``"constant values"`` (default), ``"same input"`` or ``"no caching"``.
        transforms: list of :class:`Transform` instances (DDP/FSDP/TP/autocast/FP8/hipGraph/...).
        disable_torch_autograd: compile forward only.
        **compile_options: free-form options read with ``get_compile_option``.
    """
    if "executors_list" in compile_options and executors is None:
        executors = compile_options.pop("executors_list")
    transforms = list(transforms or [])
    executors_list = resolve_executors(executors)
    is_module = isinstance(fn, _torch.nn.Module)
    cd = CompileData(
        fn=fn,
        executors_list=executors_list,
        cache_option=resolve_cache_option(cache),
        sharp_edges=resolve_sharp_edges_option(sharp_edges),
        disable_torch_autograd=disable_torch_autograd,
        transforms=transforms,
        debug_options=debug_options,
        compile_options=compile_options,
        is_module=is_module,
    )
    cs = CompileStats()
    holder: dict[str, Any] = {"module": None}
    from .executors.pythonex import ThunderCacheMiss
    from .distributed import get_skip_data_parallel_grad_sync
    from .core.pytree import _FAST_LEAF

    @_annotate_for_profile("get_computation_and_inputs")
    def get_computation_and_inputs(args, kwargs):
        cs.last_trace_cache_start = time.perf_counter_ns()
        if not kwargs and all(type(a) in _FAST_LEAF for a in args):
            flat_args = list(args)  # the common call: tensors / numbers only, nothing to flatten
        else:
            flat_args, _ = tree_flatten((args, kwargs))
        grad_enabled = _torch.is_grad_enabled()
        ac = _autocast_key()
        nosync = get_skip_data_parallel_grad_sync()
        if cd.cache_option is not CACHE_OPTIONS.NO_CACHING:
            for entry in reversed(cs.interpreter_cache):
                if entry.grad_enabled != grad_enabled or entry.autocast_key != ac or entry.no_grad_sync != nosync:
                    continue
                if entry.alias_pattern is not None and storage_alias_pattern(flat_args) != entry.alias_pattern:
                    continue
                if cd.cache_option is CACHE_OPTIONS.SAME_INPUT and not entry.has_prov_inputs:
                    inps = _same_input(entry, flat_args)
                    cs.cache_hits += 1
                    cs.last_trace_cache_stop = time.perf_counter_ns()
                    return entry, inps
                try:
                    inps = entry.prologue_fn(flat_args, entry.module_state(), entry.constants, entry.guard_roots)
                except ThunderCacheMiss:
                    continue
                cs.cache_hits += 1
                cs.last_trace_cache_stop = time.perf_counter_ns()
                return entry, inps
        cs.cache_misses += 1
        cs.last_trace_cache_stop = time.perf_counter_ns()
        entry = _build_cache_entry(cd, cs, holder["module"], args, kwargs)
        cs.interpreter_cache.append(entry)
        cs.last_traces = entry.computation_traces
        cs.last_backward_traces = entry.backward_traces
        cs.last_prologue_traces = entry.prologue_traces
        inps = entry.prologue_fn(flat_args, entry.module_state(), entry.constants, entry.guard_roots)
        return entry, inps

    @_annotate_for_profile("fn_")
    def fn_(*args, **kwargs):
        cs.calls += 1
        cs.last_trace_host_start = time.perf_counter_ns()
        entry, inps = get_computation_and_inputs(args, kwargs)
        cs.last_traces = entry.computation_traces
        cs.last_backward_traces = entry.backward_traces
        cs.last_prologue_traces = entry.prologue_traces
        cs.last_interpreter_log = entry.interpreter_log
        cs.last_executed = entry
        cs.last_trace_host_execution_start = time.perf_counter_ns()
        out = _run_entry(entry, inps, tree_flatten((args, kwargs))[0] if entry.output_arg_refs else None)
        cs.last_trace_host_execution_stop = time.perf_counter_ns()
        cs.last_trace_host_stop = cs.last_trace_host_execution_stop
        return out

    fn_._lc_cd = cd
    fn_._lc_cs = cs
    if is_module:
        tm = ThunderModule(fn, fn_)
        holder["module"] = fn
        tm._lc_cd = cd
        tm._lc_cs = cs
        for t in transforms:
            t.transform_module(tm)
        return tm
    return fn_


def _same_input(entry, flat_args):
    return [flat_args[i] for i in entry._same_input_positions] + entry.module_state() + list(entry.constants)


def compile(fn, recipe=None, plugins=None):
    """Recipe/plugin entry point (reference ``thunder.compile`` :274-311)."""
    from .core.recipe import Recipe, Plugin
    from .recipes import BaseRecipe, get_recipe_class
    from .plugins import get_plugin

    if plugins is not None and not isinstance(plugins, (list, tuple)):
        plugins = [plugins]
    plugins = [get_plugin(p)() if isinstance(p, str) else p for p in (plugins or [])]
    if recipe is None or recipe == "auto":
        recipe = Recipe.get_for_model(fn) if isinstance(fn, _torch.nn.Module) else BaseRecipe()
    elif isinstance(recipe, str):
        recipe = get_recipe_class(recipe)()
    recipe.add_plugins(plugins)
    return recipe.apply(fn)


# =========================================================================================
# Introspection
# =========================================================================================
def _cs(fn) -> CompileStats:
    cs = getattr(fn, "_lc_cs", None)
    if cs is None:
        raise TypeError(f"{fn} was not compiled with lightning_thunder_amd.jit")
    return cs


def compile_data(fn) -> CompileData | None:
    return getattr(fn, "_lc_cd", None)


def compile_stats(fn) -> CompileStats | None:
    return getattr(fn, "_lc_cs", None)


def last_traces(fn) -> list[TraceCtx]:
    cs = _cs(fn)
    if cs.last_traces is None:
        raise TypeError(f"{fn} has not been called yet")
    return cs.last_traces


def last_backward_traces(fn) -> list[TraceCtx]:
    return _cs(fn).last_backward_traces or []


def last_prologue_traces(fn) -> list[TraceCtx]:
    return _cs(fn).last_prologue_traces


def cache_option(fn) -> CACHE_OPTIONS:
    return compile_data(fn).cache_option


def cache_hits(fn) -> int:
    return _cs(fn).cache_hits


def cache_misses(fn) -> int:
    return _cs(fn).cache_misses


def list_transforms(fn) -> list:
    return compile_data(fn).transforms


def last_compile_options(fn) -> None:
    cd = compile_data(fn)
    used = cd._compile_options_used
    print("Compile options used:", sorted(used))
    print("Compile options passed:", sorted(cd.compile_options))


def get_auto_registered_torch_op_names(fn=None) -> set[str]:
    from .torch.default_torch_ops import get_auto_registered_torch_op_names as g

    return g()


def last_interpreter_log(fn):
    return _cs(fn).last_interpreter_log


def print_last_interpreter_log(fn, *, max_lines: int | None = None, **kwargs):
    """Prints the interpreter log of the last compilation (``record_interpreter_history=True``)."""
    log = last_interpreter_log(fn)
    if log is None:
        print("no interpreter log recorded: pass record_interpreter_history=True (or DebugOptions)")
        return
    for item in log[:max_lines]:
        print(item)


def last_sharp_edges(fn) -> list[str]:
    """Sharp edges (global reads/writes, non-deterministic calls) seen by the last compilation."""
    e = _cs(fn).last_executed
    return [] if e is None else list(e.sharp_edges)


def grad(fn):
    """Returns a function computing grads of ``fn``'s (scalar) output w.r.t. its tensor inputs."""

    def wrapper(*args, **kwargs):
        args = [a.detach().requires_grad_(True) if isinstance(a, _torch.Tensor) and a.is_floating_point() else a for a in args]
        jfn = jit(fn)
        out = jfn(*args, **kwargs)
        ins = [a for a in args if isinstance(a, _torch.Tensor) and a.requires_grad]
        return _torch.autograd.grad(out, ins)

    return wrapper


def trace(fn, *args, interpretation: str = "python interpreter", **kwargs) -> TraceCtx:
    """Acquires the computation trace of ``fn(*args, **kwargs)`` without executing it."""
    from .core.jit_ext import acquire

    prog = acquire(fn, args, kwargs, module=fn if isinstance(fn, _torch.nn.Module) else None,
                   interpretation=interpretation)
    return prog.computation_trace


from . import distributed  # noqa: E402,F401
from .torch import einops_backend as _einops_backend  # noqa: E402,F401  (einops on traced tensors)
from .transforms import *  # noqa: E402,F401,F403

__all__ = [
    "jit", "compile", "trace", "last_traces", "last_backward_traces", "last_prologue_traces", "compile_data",
    "compile_stats", "cache_option", "cache_hits", "cache_misses", "list_transforms", "last_compile_options",
    "get_auto_registered_torch_op_names", "DebugOptions", "last_interpreter_log", "print_last_interpreter_log",
    "last_sharp_edges", "set_execution_callback_file", "Transform",
    "ThunderModule", "resolve_executors", "add_executor_lists", "get_executor", "get_all_executors",
    "get_default_executors", "get_always_executors", "grad", "Proxy", "TensorProxy", "NumberProxy",
]
