"""Execution passes: claiming, fusion, del-last-used (parity: reference ``thunder/executors/passes.py``
``_transform_for_operator_executor_execution`` :32-104, ``transform_for_execution`` :107-146,
``del_last_used`` :215-288).
"""
from __future__ import annotations

import time
from typing import Sequence

from ..core import prims
from ..core.prims import PrimIDs
from ..core.proxies import Proxy, TensorProxy
from ..core.pytree import tree_flatten
from ..core.symbol import BoundSymbol
from ..core.trace import TraceCtx, from_trace, tracectx, TraceProvenance
from ..core.transform_common import dce, cse
from ..extend import Executor, FusionExecutor, get_always_executors


class ClaimError(RuntimeError):
    pass


def _transform_for_operator_executor_execution(trace: TraceCtx, executors: Sequence[Executor]) -> TraceCtx:
    start = time.perf_counter_ns()
    new = from_trace(trace)
    new.bound_symbols = []
    new.scopes = [new.bound_symbols]
    swap: dict[str, Proxy] = {}

    def visit(bsym: BoundSymbol):
        b = bsym.swap_proxies(swap, skip_output=True)
        if b.sym.executor is not None or b.sym.is_fusion:
            new.bound_symbols.append(b)
            return
        for ex in executors:
            if isinstance(ex, FusionExecutor):
                if ex.can_fuse(b):
                    new.bound_symbols.append(b)
                    return
                continue
            if not ex.can_execute_directly(b):
                continue
            impl = ex.implmap[b.sym.id]
            if impl.execution_transform is not None:
                scope: list = []
                with tracectx(new):
                    new.push_scope(scope)
                    try:
                        out = impl.execution_transform(*b.args, **b.kwargs)
                    finally:
                        new.pop_scope()
                old_flat, _ = tree_flatten(b.output)
                new_flat, _ = tree_flatten(out)
                for o_old, o_new in zip(old_flat, new_flat):
                    if isinstance(o_old, Proxy) and isinstance(o_new, Proxy) and o_old.name != o_new.name:
                        swap[o_old.name] = o_new
                for s in scope:
                    visit(s)
                return
            if impl.symbol is not None:
                nb = impl.symbol.bind(*b.args, output=b.output, subsymbols=b.subsymbols, **b.kwargs)
                nb.tags = set(b.tags)
                nb = ex.bind_call_ctx(nb, b)
                new.bound_symbols.append(nb)
                return
        if b.subsymbols:
            for s in b.subsymbols:
                visit(s)
            return
        raise ClaimError(f"Could not find an executor for bound symbol {b.sym.name} ({b.sym.id}); executors: {list(executors)}")

    for bsym in trace.bound_symbols:
        visit(bsym)
    new.set_provenance(TraceProvenance(f"Transform for operator executor execution (took {(time.perf_counter_ns() - start) // 1000000} milliseconds)"))
    return new


def transform_for_execution(trace: TraceCtx, executors: Sequence[Executor]) -> list[TraceCtx]:
    """DCE → claiming → fusion passes → always-executors; returns the list of intermediate traces."""
    traces = []
    executors = list(executors)
    for ex in get_always_executors():
        if ex not in executors:
            executors.append(ex)
    from ..distributed.bucketing import has_grad_syncs, bucket_grad_syncs

    if has_grad_syncs(trace):
        from ..common import get_compile_option

        trace = bucket_grad_syncs(trace, get_compile_option("lta_bucket_size_mb", "DDP/FSDP gradient bucket size (MiB)"))
        traces.append(trace)
    from ..distributed.bucketing import has_fsdp_param_gathers, bucket_fsdp_all_gathers

    if has_fsdp_param_gathers(trace):
        from ..common import get_compile_option

        strategy = get_compile_option("lta_fsdp_bucketing", "FSDP parameter all-gather buckets: none|layer|block")
        if strategy in ("layer", "block"):
            trace = bucket_fsdp_all_gathers(trace, strategy)
            traces.append(trace)
    trace = dce(trace)
    traces.append(trace)
    trace = _transform_for_operator_executor_execution(trace, executors)
    traces.append(trace)
    trace = dce(cse(trace))
    # executor-specific rewrites of the claimed program before fusion (e.g. hipex folds residual
    # adds into its GEMM epilogue, which beats fusing them into a separate elementwise kernel)
    for ex in executors:
        hook = getattr(ex, "post_claim_pass", None)
        if hook is not None:
            new = hook(trace)
            if new is not trace:
                trace = new
                traces.append(trace)
    for ex in executors:
        if isinstance(ex, FusionExecutor):
            trace = ex.fusion_pass(trace)
            traces.append(trace)
    # whatever the fusion executors left unclaimed goes to the always executors
    trace = _transform_for_operator_executor_execution(trace, [e for e in executors if not isinstance(e, FusionExecutor)])
    trace = dce(trace)
    traces.append(trace)
    return traces


def del_last_used(trace: TraceCtx, *, clear_mutable_collections: bool = False) -> TraceCtx:
    """Inserts ``del`` after each proxy's last use so memory is released early."""
    start = time.perf_counter_ns()
    out_names = set()
    ret = trace.bound_symbols[-1] if trace.bound_symbols else None
    if ret is not None and ret.sym.id == PrimIDs.RETURN:
        for p in ret.flat_proxy_args:
            out_names.add(p.name)
    handled: set[str] = set(out_names)
    new_bsyms: list[BoundSymbol] = []
    for bsym in reversed(trace.bound_symbols):
        if bsym.sym.id == PrimIDs.RETURN:
            new_bsyms.append(bsym)
            continue
        to_del = []
        for p in bsym.flat_proxy_args + bsym.flat_proxy_outs:
            if p.name not in handled:
                handled.add(p.name)
                to_del.append(p)
        if to_del:
            new_bsyms.append(prims.python_del.bind(*to_del, output=None))
        new_bsyms.append(bsym)
    new_bsyms.reverse()
    new = from_trace(trace)
    new.bound_symbols = new_bsyms
    new.scopes = [new.bound_symbols]
    new.set_provenance(TraceProvenance(f"Delete Last Used (took {(time.perf_counter_ns() - start) // 1000000} milliseconds)"))
    return new
