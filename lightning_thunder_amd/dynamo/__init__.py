"""ThunderFX: a ``torch.compile`` backend that hands FX graphs to the lightning_thunder_amd compiler.

Reference parity: ``thunder/dynamo/{compiler,splitter,utils,report}.py`` (``ThunderCompiler``,
``thunderfx``, ``_splitter``, ``SubgraphInfo``, ``SplitReason``).

* Dynamo captures the program (handling graph breaks, guards and Python control flow); the
  backend receives each FX ``GraphModule``.
* ``_split`` marks every node as supported or not by *executing it symbolically*: the node's
  target is called under this framework's tracing mode on proxies built from the node's fake
  example values (``node.meta["example_value"]``).  Maximal runs of supported nodes become
  submodules compiled with :func:`lightning_thunder_amd.jit` (the HIP executors run there);
  unsupported nodes stay in the outer graph and run eagerly on PyTorch-ROCm (there is no
  Triton/Inductor fallback on this stack by design).
* ``thunderfx(fn)`` is the convenience wrapper; ``ThunderCompiler.subgraph_infos`` records the
  splits and their reasons for reports (``split_report``).
"""
from __future__ import annotations

import dataclasses
import enum
import operator
from typing import Any, Callable

import torch
from torch.fx.passes.split_module import split_module

__all__ = ["ThunderCompiler", "thunderfx", "SubgraphInfo", "SplitReason", "SplitReasonType", "split_report"]


class SplitReasonType(enum.Enum):
    UNSUPPORTED_NODE = enum.auto()
    EXCEPTION_PROXY_THUNDER_OP = enum.auto()
    EXCEPTION_META_THUNDER_OP = enum.auto()


@dataclasses.dataclass
class SplitReason:
    reason_type: SplitReasonType
    info: str
    exception: str | None = None


@dataclasses.dataclass
class SubgraphInfo:
    original_graph_module: torch.fx.GraphModule
    split_graph_module: torch.fx.GraphModule | None
    thunder_compiled_fns: list
    submodule_to_compiled_functions: dict
    split_reasons: list
    original_split_modules: dict = None  # split module name -> the GraphModule before jit (graph benchmarking)


_ALWAYS_EAGER = {
    "_local_scalar_dense", "item", "tolist", "nonzero", "unique", "masked_select", "manual_seed", "set_grad_enabled",
    "print",
}
# context-manager nodes: supported as a whole region (the interpreter applies the autocast inside the
# compiled program), or the whole region runs eagerly (reference get_nodes_in_unsupported_ctx_regions)
_CTX_ENTER, _CTX_EXIT = "_enter_autocast", "_exit_autocast"


def _target_name(node) -> str:
    t = node.target
    return t if isinstance(t, str) else getattr(t, "__name__", str(t))


def _hint(v):
    """Concrete example value of a symbolic scalar (dynamo's hint for the traced size)."""
    if isinstance(v, (torch.SymInt, torch.SymFloat, torch.SymBool)):
        node = v.node
        h = getattr(node, "hint", None)
        if h is None:
            h = node.shape_env.size_hint(node.expr) if getattr(node, "shape_env", None) is not None else None
        if h is None:
            raise ValueError(f"symbolic value {v} has no hint")
        if isinstance(v, torch.SymBool):
            return bool(h)
        return float(h) if isinstance(v, torch.SymFloat) else int(h)
    return v


def _proxy_of(v, trc):
    from ..core.proxies import TensorProxy

    if isinstance(v, torch.Tensor):
        # symbolic sizes (dynamic=True graphs) are checked at their example (hint) values: the op's
        # support does not depend on the size, and the compiled submodule re-specializes per shape
        shape = tuple(_hint(d) for d in v.shape)
        return TensorProxy(trc.make_unique_name("fx"), shape=shape, device=v.device, dtype=v.dtype,
                           requires_grad=v.requires_grad)
    return _hint(v)


def _is_dynamic(gm: torch.fx.GraphModule) -> bool:
    for n in gm.graph.nodes:
        if n.op != "placeholder":
            continue
        ev = n.meta.get("example_value", n.meta.get("val"))
        if isinstance(ev, (torch.SymInt, torch.SymFloat, torch.SymBool)):
            return True
        if isinstance(ev, torch.Tensor) and any(isinstance(d, torch.SymInt) for d in ev.shape):
            return True
    return False


def _is_checkpoint_hop(node) -> bool:
    return node.op == "call_function" and _target_name(node) == "tag_activation_checkpoint"


def _checkpoint_hop_call(body, *args, **kwargs):
    """What a ``tag_activation_checkpoint`` node becomes inside a compiled submodule: the region
    through ``torch.utils.checkpoint`` (the framework's checkpoint symbol recomputes it in the
    backward; reference ``thunder/dynamo/utils.py:741-792`` checkpoint_converter)."""
    from .. import torch as ltorch

    return ltorch.checkpoint(body, *args)


def _fx_enter_autocast(*vals):
    """A compiled region's ``_enter_autocast`` node: sets the trace's autocast dtype."""
    from ..core.interpreter import _AUTOCAST, _autocast_enter

    return _autocast_enter(None, _AUTOCAST(*vals))


def _fx_exit_autocast(mode):
    from ..core.interpreter import _autocast_exit

    return _autocast_exit(None, mode, None, None, None)


def _convert_checkpoints(gm: torch.fx.GraphModule, part: dict) -> None:
    """Rewrite the nodes a compiled submodule cannot run natively: checkpoint regions and autocast
    enter / exit (inside a thunder submodule they set the program's autocast state)."""
    for n in gm.graph.nodes:
        if n not in part or not part[n][1]:
            continue  # nodes of eager partitions keep their torch targets
        if _is_checkpoint_hop(n):
            n.target = _checkpoint_hop_call
            n.kwargs = {}
        elif n.op == "call_function" and _target_name(n) == _CTX_ENTER:
            n.target = _fx_enter_autocast
        elif n.op == "call_function" and _target_name(n) == _CTX_EXIT:
            n.target = _fx_exit_autocast
    gm.recompile()


def is_node_supported(node: torch.fx.Node) -> tuple[bool, SplitReason | None]:
    """Symbolically runs ``node`` through the framework's torch-function dispatch on proxies."""
    if node.op in ("placeholder", "output", "get_attr"):
        return True, None
    name = _target_name(node)
    if name in (_CTX_ENTER, _CTX_EXIT):
        return True, None  # decided per region in _split
    if _is_checkpoint_hop(node):
        # an activation-checkpointed region is supported when every node of its body is
        body = getattr(node.graph.owning_module, node.args[0].target, None)
        if not isinstance(body, torch.fx.GraphModule):
            return False, SplitReason(SplitReasonType.UNSUPPORTED_NODE, "checkpoint body is not a GraphModule")
        for bn in body.graph.nodes:
            ok, why = is_node_supported(bn)
            if not ok:
                return False, why
        return True, None
    if name in _ALWAYS_EAGER:
        return False, SplitReason(SplitReasonType.UNSUPPORTED_NODE, f"{name} needs host values / side effects")
    if node.op == "call_module":
        return True, None  # submodules are traced through (their own nodes were checked by dynamo's inlining)
    from ..core.trace import TraceCtx, tracectx
    from ..core.jit_ext import ThunderTorchFunctionMode

    def example(n):
        if isinstance(n, torch.fx.Node):
            ev = n.meta.get("example_value", n.meta.get("val"))
            return ev
        return n

    args = torch.fx.node.map_arg(node.args, example)
    kwargs = torch.fx.node.map_arg(node.kwargs, example)
    trc = TraceCtx()
    try:
        with tracectx(trc):
            pargs = torch.utils._pytree.tree_map(lambda v: _proxy_of(v, trc), args)
            pkwargs = torch.utils._pytree.tree_map(lambda v: _proxy_of(v, trc), kwargs)
            with ThunderTorchFunctionMode():
                if node.op == "call_method":
                    getattr(pargs[0], node.target)(*pargs[1:], **pkwargs)
                else:
                    node.target(*pargs, **pkwargs)
    except Exception as e:  # noqa: BLE001 - any failure means "run this node eagerly"
        return False, SplitReason(SplitReasonType.EXCEPTION_META_THUNDER_OP, f"{name} failed to trace",
                                  exception=f"{type(e).__name__}: {e}")
    return True, None


def _split(gm: torch.fx.GraphModule):
    """Partition id per node: supported runs get even ids, unsupported nodes odd ids."""
    reasons = []
    part = {}
    cur = 0
    prev_supported = None
    nodes = [n for n in gm.graph.nodes if n.op not in ("placeholder", "output")]
    support = {}
    for node in nodes:
        ok, why = is_node_supported(node)
        if why is not None:
            reasons.append(why)
        support[node] = ok
    # an autocast region with any unsupported node runs eagerly as a whole
    stack = []
    for i, node in enumerate(nodes):
        name = _target_name(node)
        if name == _CTX_ENTER:
            stack.append(i)
        elif name == _CTX_EXIT and stack:
            j = stack.pop()
            region = nodes[j:i + 1]
            if not all(support[n] for n in region):
                for n in region:
                    support[n] = False
                reasons.append(SplitReason(SplitReasonType.UNSUPPORTED_NODE,
                                           "autocast region with an unsupported node runs eagerly"))
    for node in nodes:
        ok = support[node]
        if prev_supported is None or ok != prev_supported:
            cur += 1
        part[node] = (cur, ok)
        prev_supported = ok
    return part, reasons


class ThunderCompiler:
    """``torch.compile(model, backend=ThunderCompiler(**jit_options))``."""

    def __init__(self, **thunder_options):
        self.thunder_options = thunder_options
        self.subgraph_infos: list[SubgraphInfo] = []

    def _options(self, gm) -> dict:
        """Per-graph jit options (reference ``thunder/dynamo/compiler.py:51-84,132-154``): the
        dataflow fusion partitioner, and — for static graphs, whose input shapes / dtypes / devices
        dynamo already guards — an extraction-only prologue (no redundant per-call checks).  Dynamic
        graphs keep the checks: a new size must miss the cache and re-specialize."""
        from ..transforms.prune_prologue_checks import ExtractionOnlyPrologueTransform

        opts = dict(self.thunder_options)
        opts.setdefault("fusion_type", "dataflow")
        if not _is_dynamic(gm) and opts.pop("extraction_only_prologue", True):
            ts = list(opts.get("transforms") or [])
            if not any(isinstance(t, ExtractionOnlyPrologueTransform) for t in ts):
                ts.append(ExtractionOnlyPrologueTransform())
            opts["transforms"] = ts
        else:
            opts.pop("extraction_only_prologue", None)
            # dynamic graphs: symbolic tensor dims and size arguments (core/symbolic.py), so one
            # compiled program serves every size dynamo's own graph serves
            opts.setdefault("cache", "symbolic values")
        return opts

    def __call__(self, gm: torch.fx.GraphModule, sample_args):
        from .. import jit

        part, reasons = _split(gm)
        if not part:
            return gm
        if any((_is_checkpoint_hop(n) or _target_name(n) in (_CTX_ENTER, _CTX_EXIT)) and part[n][1]
               for n in gm.graph.nodes if n in part):
            _convert_checkpoints(gm, part)
        compiled = []
        mapping = {}
        originals = {}
        if all(ok for _, ok in part.values()):
            fn = jit(gm, **self._options(gm))
            compiled.append(fn)
            self.subgraph_infos.append(SubgraphInfo(gm, None, compiled, {"whole": fn}, reasons))
            return fn
        split_gm = split_module(gm, None, lambda n: part[n][0], keep_original_order=True)
        for n in split_gm.graph.nodes:
            if n.op != "call_module":
                continue
            idx = int(n.target.split("_")[-1])
            sub = getattr(split_gm, n.target)
            supported = any(ok for (i, ok) in part.values() if i == idx)
            if supported:
                originals[n.target] = sub
                fn = jit(sub, **self._options(gm))
                setattr(split_gm, n.target, fn)
                compiled.append(fn)
                mapping[n.target] = fn
        split_gm.recompile()
        self.subgraph_infos.append(SubgraphInfo(gm, split_gm, compiled, mapping, reasons, originals))
        return split_gm


class ThunderFXCompiledObject:
    def __init__(self, fn, backend: ThunderCompiler, **compile_kwargs):
        self._backend = backend
        self._fn = torch.compile(fn, backend=backend, **compile_kwargs)

    def __call__(self, *args, **kwargs):
        return self._fn(*args, **kwargs)

    @property
    def subgraph_infos(self):
        return self._backend.subgraph_infos

    @property
    def last_traces(self):
        from .. import last_traces

        return [last_traces(f) for info in self._backend.subgraph_infos for f in info.thunder_compiled_fns]


def thunderfx(fn: Callable, /, **kwargs) -> ThunderFXCompiledObject:
    """``torch.compile(fn, backend=ThunderCompiler(**kwargs))`` with access to the split info."""
    torch_kw = {k: kwargs.pop(k) for k in ("dynamic", "fullgraph", "mode") if k in kwargs}
    torch_kw.setdefault("dynamic", False)
    return ThunderFXCompiledObject(fn, ThunderCompiler(**kwargs), **torch_kw)


def split_report(compiled) -> str:
    """Human-readable summary of the graph splits (reference ``thunder/dynamo/report.py``)."""
    infos = compiled.subgraph_infos if hasattr(compiled, "subgraph_infos") else compiled
    lines = []
    for i, info in enumerate(infos):
        n_nodes = sum(1 for n in info.original_graph_module.graph.nodes if n.op not in ("placeholder", "output"))
        lines.append(f"graph {i}: {n_nodes} nodes, {len(info.thunder_compiled_fns)} thunder submodule(s)")
        for r in info.split_reasons:
            lines.append(f"  split: {r.reason_type.name}: {r.info}" + (f" ({r.exception})" if r.exception else ""))
    return "\n".join(lines)
