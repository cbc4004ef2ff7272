"""``examine``: which torch operations does a program use, and can this framework run it?
(reference ``thunder/examine/__init__.py``: ``examine``, ``get_fusions``, ``get_fusion_symbols``,
``make_trace_dot``; ``memory_calculation.py``).
"""
from __future__ import annotations

import collections
import traceback
from typing import Callable

import torch
from torch.overrides import TorchFunctionMode, resolve_name

from ..core.trace import TraceCtx


class _CollectFunctionsUsed(TorchFunctionMode):
    def __init__(self):
        super().__init__()
        self.calls: dict[str, int] = collections.Counter()
        self.funcs: dict[str, Callable] = {}

    def __torch_function__(self, func, types, args=(), kwargs=None):
        name = resolve_name(func) or getattr(func, "__qualname__", str(func))
        self.calls[name] += 1
        self.funcs[name] = func
        return func(*args, **(kwargs or {}))


def examine(fn: Callable, *args, show_call_stack: bool = False, **kwargs):
    """Runs ``fn`` eagerly recording the torch operations it calls, reports which of them have
    a language-level symbol here (``ltorch``) vs. which would be auto-registered as opaque
    ops, then compiles and runs ``fn`` and compares the result with eager."""
    from .. import jit, torch as ltorch
    from ..torch import _torch_to_thunder_function_map as _torch_to_thunder_map

    mode = _CollectFunctionsUsed()
    with mode:
        eager = fn(*args, **kwargs)
    known, opaque = [], []
    for name, f in mode.funcs.items():
        (known if f in _torch_to_thunder_map else opaque).append(name)
    print(f"Found {len(mode.calls)} distinct operations, of which {len(known)} ({100.0 * len(known) / max(1, len(mode.calls)):.1f}%) "
          f"have a language-level symbol; {len(opaque)} will run as opaque (torch-executed) symbols:")
    for n in sorted(opaque):
        print(f"  {n}")
    try:
        jfn = jit(fn)
        out = jfn(*args, **kwargs)
    except Exception as e:  # noqa: BLE001
        print("Compiling or running the program failed:")
        if show_call_stack:
            traceback.print_exc()
        else:
            print(f"  {type(e).__name__}: {e}")
        return None
    ok = _close(out, eager)
    print("The compiled program runs and its result matches eager." if ok else
          "The compiled program runs but its result differs from eager!")
    return jfn


def _close(a, b) -> bool:
    fa, _ = torch.utils._pytree.tree_flatten(a)
    fb, _ = torch.utils._pytree.tree_flatten(b)
    for x, y in zip(fa, fb):
        if isinstance(x, torch.Tensor):
            if not torch.allclose(x.detach().float(), y.detach().float(), rtol=1e-3, atol=1e-3, equal_nan=True):
                return False
    return True


def get_fusion_symbols(trace: TraceCtx) -> list:
    return [b for b in trace.bound_symbols if b.sym.is_fusion]


def get_fusions(trace: TraceCtx) -> list[tuple[str, Callable]]:
    out = []
    for b in get_fusion_symbols(trace):
        name = b.sym.name
        out.append((name, (b._call_ctx or {}).get(name)))
    return out


def get_hipfuse_source(trace: TraceCtx, name: str) -> str:
    """HIP source of a hipfuse region for the contiguous-input call signature (repro aid)."""
    from ..executors import hipfuse_codegen as cg
    from ..core.proxies import TensorProxy

    for b in get_fusion_symbols(trace):
        if b.sym.name == name:
            f = b._call_ctx[name]
            targs = {p.name: cg.TensorArg(tuple(p.shape), tuple(torch.empty(p.shape, device="meta").stride()), p.dtype, True)
                     for p in f.inputs if isinstance(p, TensorProxy)}
            return cg.generate(f.plan, f.inputs, f.outputs, targs).src
    raise KeyError(name)


def make_trace_dot(trace: TraceCtx, show_metadata: bool = False) -> str:
    """Graphviz DOT text of a trace's dataflow (render with ``dot -Tsvg``)."""
    lines = ["digraph trace {", "  rankdir=TB;"]
    producers = {}
    for i, b in enumerate(trace.bound_symbols):
        label = b.sym.name
        if show_metadata:
            label += "\\n" + ", ".join(o.type_string() for o in b.flat_proxy_outs if hasattr(o, "type_string"))
        lines.append(f'  n{i} [label="{label}"];')
        for a in b.flat_proxy_args:
            if a.name in producers:
                lines.append(f"  n{producers[a.name]} -> n{i} [label=\"{a.name}\"];")
        for o in b.flat_proxy_outs:
            producers[o.name] = i
    lines.append("}")
    return "\n".join(lines)


from .memory_calculation import get_alloc_memory  # noqa: E402
