"""Tensor parallelism: column-/row-wise sharded ``nn.Linear`` / ``nn.Embedding`` (#48).

Reference parity: ``thunder/distributed/tensor_parallel/{common,column_wise,row_wise,optimize_comm}.py``
(``column_parallel(tm, target_modules, process_group)``, ``row_parallel(...)``, pre/post-process
pairs around the sharded op, redundant-communication removal).

Design (MI355X, RCCL over xGMI):
* ``transform_module`` shards the target modules' weights in place (column: dim 0, row: dim 1;
  column biases are sharded, row biases stay whole and are added once after the reduction).
  The program is still acquired with full shapes (``_lc_full_shape``), exactly like FSDP.
* ``transform_traces_pre_prologue`` retypes each sharded weight as its local shard and rewrites
  the consuming ``linear`` / ``embedding``:
    column linear : y = all_gather_lastdim(linear(x, W_r, b_r))      (bwd: slice; dx all-reduced)
    row linear    : y = all_reduce(linear(slice_lastdim(x), W_r)) + b (bwd: all-gather of dx)
    column embed  : y = all_reduce(mask(embedding(idx - r*V_r, W_r)))
    row embed     : y = all_gather_lastdim(embedding(idx, W_r))
  The rewrite happens before autodiff, so the backward's collectives come from the VJPs of the
  TP sync prims (``distributed/prims.py``).
* ``remove_redundant_comms`` then deletes all_gather -> slice pairs between a column-parallel and
  a row-parallel linear, *including through elementwise chains* (e.g. ``silu(fc_1) * fc_2`` between
  ``fc_1``/``fc_2`` column-parallel and ``proj`` row-parallel: the chain is recomputed on the
  local shards, which is the Megatron MLP with a single all-reduce per block — the reference only
  removes directly adjacent pairs).
"""
from __future__ import annotations

from typing import Sequence

import torch
import torch.distributed as tdist

from ...core.proxies import TensorProxy, DistParallelType
from ...core.symbol import BoundSymbol
from ...core.trace import from_trace, tracectx, TraceProvenance
from ...core.transform_common import Transform, dce
from .. import prims as dist_prims
from ..prims import TPLayerType

__all__ = ["column_parallel", "row_parallel", "TensorParallelTransform", "remove_redundant_comms", "TPLayerType"]

COLUMN, ROW = "column", "row"


class TensorParallelTransform(Transform):
    """Shards ``target_modules`` (name -> 'column' | 'row') over ``process_group``."""

    def __init__(self, target_modules: dict[str, str], process_group=None, optimize_comms: bool = True):
        self.targets = dict(target_modules)
        self.process_group = process_group
        self.optimize_comms = optimize_comms
        self.param_kinds: dict[str, tuple[str, type]] = {}  # "mod.weight" -> (kind, module type)
        self.original_shapes: dict[str, torch.Size] = {}

    def _group(self):
        return self.process_group if self.process_group is not None else tdist.distributed_c10d._get_default_group()

    def merge(self, target_modules: dict[str, str]):
        for k, v in target_modules.items():
            if k in self.targets and self.targets[k] != v:
                raise ValueError(f"module {k} is already {self.targets[k]}-parallel")
            self.targets[k] = v

    # --- module ------------------------------------------------------------------------------
    def transform_module(self, model) -> None:
        group = self._group()
        rank, world = tdist.get_rank(group), tdist.get_world_size(group)
        inner = model._model
        mods = dict(inner.named_modules())
        with torch.no_grad():
            for name, kind in self.targets.items():
                m = mods.get(name)
                if m is None:
                    raise ValueError(f"{name} is not a submodule of the model")
                if not isinstance(m, (torch.nn.Linear, torch.nn.Embedding)):
                    raise ValueError(f"tensor parallel supports nn.Linear / nn.Embedding, got {type(m).__name__} for {name}")
                w = m.weight
                if getattr(w, "_lc_tp_kind", None) is not None:
                    continue
                dim = 0 if kind == COLUMN else 1
                if w.shape[dim] % world:
                    raise ValueError(f"{name}.weight dim {dim} ({w.shape[dim]}) is not divisible by {world}")
                n = w.shape[dim] // world
                shard = w.detach().narrow(dim, rank * n, n).clone()
                newp = torch.nn.Parameter(shard, requires_grad=w.requires_grad)
                newp._lc_full_shape = tuple(w.shape)
                newp._lc_tp_kind = kind
                newp.distparallel_type = DistParallelType.COLUMN_WISE if kind == COLUMN else DistParallelType.ROW_WISE
                self.original_shapes[f"{name}.weight"] = w.shape
                m._parameters["weight"] = newp
                self.param_kinds[f"{name}.weight"] = (kind, type(m))
                b = getattr(m, "bias", None)
                if b is not None and kind == COLUMN:
                    nb = b.shape[0] // world
                    bp = torch.nn.Parameter(b.detach().narrow(0, rank * nb, nb).clone(), requires_grad=b.requires_grad)
                    bp._lc_full_shape = tuple(b.shape)
                    bp._lc_tp_kind = "column_bias"
                    bp.distparallel_type = DistParallelType.COLUMN_WISE
                    self.original_shapes[f"{name}.bias"] = b.shape
                    m._parameters["bias"] = bp

    # --- trace ---------------------------------------------------------------------------------
    def transform_traces_pre_prologue(self, prologue_trace, computation_trace, epilogue_trace, **kwargs):
        from ... import torch as ltorch

        group = self._group()
        rank, world = tdist.get_rank(group), tdist.get_world_size(group)
        comp = computation_trace
        # local-shard proxies for the sharded parameters
        local: dict[str, TensorProxy] = {}
        kinds: dict[str, str] = {}
        for a in comp.args:
            if not isinstance(a, TensorProxy) or a.distparallel_type not in (DistParallelType.COLUMN_WISE,
                                                                               DistParallelType.ROW_WISE):
                continue
            if "sharded" not in a.tags:
                continue
            shape = list(a.shape)
            if a.distparallel_type is DistParallelType.COLUMN_WISE:
                shape[0] //= world
                kinds[a.name] = COLUMN
            else:
                shape[1] //= world
                kinds[a.name] = ROW
            p = TensorProxy(like=a, shape=tuple(shape), name=comp.make_unique_name(a.name + "_tp"))
            p.tags = set(a.tags)
            local[a.name] = p
        if not local:
            return prologue_trace, computation_trace, epilogue_trace

        new = from_trace(comp)
        new.bound_symbols = []
        new.scopes = [new.bound_symbols]
        new.args = [local.get(a.name, a) if isinstance(a, TensorProxy) else a for a in comp.args]
        swap: dict = {}
        col_inputs: dict[str, TensorProxy] = {}  # one identity/all-reduce sync per shared input
        with tracectx(new):
            for b in comp.bound_symbols:
                w = b.args[1] if len(b.args) > 1 and isinstance(b.args[1], TensorProxy) else None
                name = b.sym.name
                if w is not None and w.name in local and name in ("linear", "embedding"):
                    nb = b.swap_proxies(swap, skip_output=True)
                    x = nb.args[0]
                    wl = local[w.name]
                    kind = kinds[w.name]
                    bias = nb.args[2] if name == "linear" and len(nb.args) > 2 else nb.kwargs.get("bias")
                    if bias is not None and bias.name in local:
                        bias = local[bias.name]
                    if name == "linear" and kind == COLUMN:
                        x2 = col_inputs.get(x.name)
                        if x2 is None:
                            x2 = dist_prims.synchronize_tensor_parallel_input(x, group, TPLayerType.COLUMN_LINEAR)
                            col_inputs[x.name] = x2
                        y = ltorch.linear(x2, wl, bias)
                        y = dist_prims.synchronize_tensor_parallel_output(y, group, TPLayerType.COLUMN_LINEAR)
                    elif name == "linear":
                        x2 = dist_prims.synchronize_tensor_parallel_input(x, group, TPLayerType.ROW_LINEAR)
                        y = ltorch.linear(x2, wl, None)
                        y = dist_prims.synchronize_tensor_parallel_output(y, group, TPLayerType.ROW_LINEAR)
                        if bias is not None:
                            y = ltorch.add(y, bias)
                    elif kind == COLUMN:  # vocab-sharded embedding
                        v_local = wl.shape[0]
                        start = rank * v_local
                        idx = ltorch.sub(x, start)
                        oob = ltorch.logical_or(ltorch.lt(idx, 0), ltorch.ge(idx, v_local))
                        idx = ltorch.masked_fill(idx, oob, 0)
                        y = ltorch.embedding(idx, wl, *nb.args[2:], **nb.kwargs)
                        y = ltorch.masked_fill(y, ltorch.unsqueeze(oob, -1), 0.0)
                        y = dist_prims.synchronize_tensor_parallel_output(y, group, TPLayerType.COLUMN_EMBED)
                    else:  # embedding-dim sharded
                        y = ltorch.embedding(x, wl, *nb.args[2:], **nb.kwargs)
                        y = dist_prims.synchronize_tensor_parallel_output(y, group, TPLayerType.ROW_EMBED)
                    swap[b.output.name] = y
                    continue
                for a in b.flat_proxy_args:
                    if a.name in local:
                        raise NotImplementedError(
                            f"tensor-parallel weight {a.name} is used by {b.sym.name}; only linear/embedding consumers are supported")
                new.bound_symbols.append(b.swap_proxies(swap))
        if self.optimize_comms:
            new = remove_redundant_comms(new)
        new.set_provenance(TraceProvenance("Tensor parallel (column/row-wise)"))
        return prologue_trace, new, epilogue_trace

    # --- state dict ------------------------------------------------------------------------------
    def transform_state_dict_for_submodule(self, model, submodule_name, state_dict):
        group = self._group()
        rank, world = tdist.get_rank(group), tdist.get_world_size(group)
        out = {}
        for k, v in state_dict.items():
            full = f"{submodule_name}.{k}" if submodule_name else k
            if full in self.original_shapes and isinstance(v, torch.Tensor):
                kind = self.param_kinds.get(full, (COLUMN, None))[0]
                dim = 0 if (kind == COLUMN or k.endswith("bias")) else 1
                n = v.shape[dim] // world
                out[k] = v.narrow(dim, rank * n, n).clone()
            else:
                out[k] = v
        return out

    def reverse_transform_state_dict_for_submodule(self, model, submodule_name, state_dict):
        group = self._group()
        world = tdist.get_world_size(group)
        out = {}
        for k, v in state_dict.items():
            full = f"{submodule_name}.{k}" if submodule_name else k
            if full in self.original_shapes and isinstance(v, torch.Tensor):
                kind = self.param_kinds.get(full, (COLUMN, None))[0]
                dim = 0 if (kind == COLUMN or k.endswith("bias")) else 1
                parts = [torch.empty_like(v) for _ in range(world)]
                tdist.all_gather(parts, v.contiguous(), group=group)
                out[k] = torch.cat(parts, dim)
            else:
                out[k] = v
        return out


# ---------------------------------------------------------------------------------------------
# Communication optimisation
# ---------------------------------------------------------------------------------------------
_ELEMENTWISE_NAMES = {
    "silu", "gelu", "relu", "tanh", "sigmoid", "mul", "add", "sub", "true_divide", "div", "neg", "exp", "hip_swiglu",
    "swiglu", "square", "pow", "abs", "leaky_relu", "erf", "to", "type_as", "convert_element_type", "tensor_float",
}


def _is_tp(b, layer_type, out: bool) -> bool:
    sym = dist_prims.synchronize_tensor_parallel_output if out else dist_prims.synchronize_tensor_parallel_input
    return b.sym is sym and b.args[2] is layer_type


def remove_redundant_comms(trace):
    """Removes column all-gather -> (elementwise chain) -> row slice round trips."""
    from ...core.pytree import tree_flatten

    producers: dict[str, BoundSymbol] = {}
    for b in trace.bound_symbols:
        for o in b.flat_proxy_outs:
            producers[o.name] = b

    def local_of(p, cache) -> bool:
        """True if tensor ``p`` (full width) can be recomputed from column-local shards."""
        if p.name in cache:
            return cache[p.name] is not False
        b = producers.get(p.name)
        ok = False
        if b is not None:
            if _is_tp(b, TPLayerType.COLUMN_LINEAR, out=True):
                ok = True
            elif b.sym.name in _ELEMENTWISE_NAMES:
                tens = [a for a in b.flat_proxy_args if isinstance(a, TensorProxy)]
                ok = bool(tens) and all(tuple(a.shape) == tuple(p.shape) and local_of(a, cache) for a in tens)
        cache[p.name] = ok if ok else False
        return ok

    changed = False
    new = from_trace(trace)
    new.bound_symbols = []
    new.scopes = [new.bound_symbols]
    swap: dict = {}
    with tracectx(new):
        for b in trace.bound_symbols:
            nb = b.swap_proxies(swap, skip_output=True)
            if _is_tp(nb, TPLayerType.ROW_LINEAR, out=False):
                x = nb.args[0]
                cache: dict = {}
                if isinstance(x, TensorProxy) and local_of(x, cache):
                    memo: dict[str, TensorProxy] = {}

                    def rebuild(p):
                        if p.name in memo:
                            return memo[p.name]
                        pb = producers[p.name]
                        if _is_tp(pb, TPLayerType.COLUMN_LINEAR, out=True):
                            r = swap.get(pb.args[0].name, pb.args[0])
                        else:
                            args = [rebuild(a) if isinstance(a, TensorProxy) else a for a in pb.args]
                            kwargs = {k: (rebuild(v) if isinstance(v, TensorProxy) else v) for k, v in pb.kwargs.items()}
                            r = pb.sym(*args, **kwargs)
                        memo[p.name] = r
                        return r

                    y = rebuild(x)
                    if tuple(y.shape) == tuple(nb.output.shape):
                        swap[nb.output.name] = y
                        changed = True
                        continue
            new.bound_symbols.append(nb)
    if not changed:
        return trace
    new = dce(new)
    new.set_provenance(TraceProvenance("Remove redundant tensor-parallel communication"))
    return new


# ---------------------------------------------------------------------------------------------
# User API
# ---------------------------------------------------------------------------------------------
def _apply(thunder_module, targets: dict[str, str], process_group):
    from ...core.module import ThunderModule
    from ...core.transforms import add_transform
    from ... import jit

    if not tdist.is_initialized():
        raise RuntimeError("tensor parallelism requires torch.distributed to be initialized")
    if not isinstance(thunder_module, ThunderModule):
        thunder_module = jit(thunder_module)
    cd = thunder_module._lc_cd
    for t in cd.transforms:
        if isinstance(t, TensorParallelTransform):
            t.merge(targets)
            t.transform_module(thunder_module)
            _clear_cache(thunder_module)
            return thunder_module
    return add_transform(thunder_module, transform=TensorParallelTransform(targets, process_group))


def _clear_cache(tm):
    cs = getattr(tm, "_lc_cs", None)
    if cs is not None and hasattr(cs, "interpreter_cache"):
        cs.interpreter_cache.clear()


def column_parallel(thunder_module, target_modules: Sequence[str], process_group=None, *, device=None):
    """Shard ``target_modules`` (Linear: output features / Embedding: vocabulary) over the group."""
    return _apply(thunder_module, {n: COLUMN for n in target_modules}, process_group)


def row_parallel(thunder_module, target_modules: Sequence[str], process_group=None, *, device=None):
    """Shard ``target_modules`` (Linear: input features / Embedding: embedding dim) over the group."""
    return _apply(thunder_module, {n: ROW for n in target_modules}, process_group)
