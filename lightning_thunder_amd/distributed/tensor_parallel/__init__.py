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
* Head-parallel attention (LitGPT convention: a module ``P`` with ``P.attn`` column-parallel, ``P.proj``
  row-parallel and a ``P.config`` carrying ``n_head`` / ``n_query_groups`` / ``head_size``): the fused
  qkv weight is sharded by *heads* (rank r keeps its n_head/W query heads and n_query_groups/W kv
  groups), ``P.config`` is localized to those counts, and both weights are traced with their local
  shapes.  The rank then runs qkv-split, RoPE and SDPA on its own heads and the row-parallel proj
  all-reduces once: no all-gather inside the block (Megatron attention).  The reference gathers the
  column output and runs attention on all heads on every rank (``column_wise.py:35-254``).
* A column-parallel (vocab-sharded) ``lm_head`` whose gathered logits only feed ``cross_entropy`` is
  rewritten to a vocab-parallel cross-entropy on the local logits (two small all-reduces per row in
  the forward, a purely local backward), so the [tokens, vocab] logits are never gathered.
* ``remove_redundant_comms`` then deletes all_gather -> slice pairs between a column-parallel and
  a row-parallel linear, *including through elementwise chains* (e.g. ``silu(fc_1) * fc_2`` between
  ``fc_1``/``fc_2`` column-parallel and ``proj`` row-parallel: the chain is recomputed on the
  local shards, which is the Megatron MLP with a single all-reduce per block — the reference only
  removes directly adjacent pairs).
"""
from __future__ import annotations

import dataclasses

from typing import Sequence

import torch
import torch.distributed as tdist

from ...core.proxies import TensorProxy, DistParallelType
from ...core.symbol import BoundSymbol
from ...core.trace import from_trace, tracectx, TraceProvenance
from ...core.transform_common import Transform, dce
from .. import prims as dist_prims
from ..prims import TPLayerType

__all__ = ["column_parallel", "row_parallel", "TensorParallelTransform", "remove_redundant_comms", "vocab_parallel_loss",
           "TPLayerType"]

COLUMN, ROW = "column", "row"


class TensorParallelTransform(Transform):
    """Shards ``target_modules`` (name -> 'column' | 'row') over ``process_group``."""

    def __init__(self, target_modules: dict[str, str], process_group=None, optimize_comms: bool = True,
                 head_parallel: bool = True, vocab_parallel_loss: bool = True):
        self.targets = dict(target_modules)
        self.process_group = process_group
        self.optimize_comms = optimize_comms
        self.head_parallel = head_parallel
        self.vocab_parallel_loss = vocab_parallel_loss
        self.head_info: dict[str, tuple] = {}  # "attn.attn.weight" -> (n_head, n_query_groups, head_size)
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
    def _head_groups(self, mods) -> list:
        """(parent, qkv name, proj name) of attention modules that can run head-parallel."""
        out = []
        for name, kind in self.targets.items():
            if kind != COLUMN or not name.endswith(".attn") and name != "attn":
                continue
            parent = name[: -len(".attn")] if name.endswith(".attn") else ""
            proj = f"{parent}.proj" if parent else "proj"
            pm = mods.get(parent)
            cfg = getattr(pm, "config", None)
            if self.targets.get(proj) != ROW or cfg is None:
                continue
            if not all(hasattr(cfg, a) for a in ("n_head", "n_query_groups", "head_size")):
                continue
            if not dataclasses.is_dataclass(cfg) or isinstance(cfg, type):
                continue  # the localized copy is made with dataclasses.replace
            if not isinstance(mods.get(name), torch.nn.Linear) or not isinstance(mods.get(proj), torch.nn.Linear):
                continue
            out.append((parent, name, proj))
        return out

    @staticmethod
    def _qkv_rows(nh, ng, hs, world, rank):
        """Row indices of rank ``rank``'s heads in a fused [q | k | v] weight (litgpt layout)."""
        nhl, ngl = nh // world, ng // world
        q = torch.arange(rank * nhl * hs, (rank + 1) * nhl * hs)
        k = nh * hs + torch.arange(rank * ngl * hs, (rank + 1) * ngl * hs)
        v = (nh + ng) * hs + torch.arange(rank * ngl * hs, (rank + 1) * ngl * hs)
        return torch.cat((q, k, v))

    def transform_module(self, model) -> None:
        from dataclasses import replace

        group = self._group()
        rank, world = tdist.get_rank(group), tdist.get_world_size(group)
        inner = model._model
        mods = dict(inner.named_modules())
        head_done = set()
        with torch.no_grad():
            if self.head_parallel:
                for parent, qkv_name, proj_name in self._head_groups(mods):
                    pm, qm, prm = mods[parent], mods[qkv_name], mods[proj_name]
                    qkind = getattr(qm.weight, "_lc_tp_kind", None)
                    if qkind == "head_qkv" or getattr(prm.weight, "_lc_tp_kind", None) is not None:
                        head_done.update((qkv_name, proj_name))
                        continue
                    cfg = pm.config
                    nh, ng, hs = cfg.n_head, cfg.n_query_groups, cfg.head_size
                    full_rows = getattr(qm.weight, "_lc_full_shape", tuple(qm.weight.shape))[0]
                    if nh % world or ng % world or full_rows != (nh + 2 * ng) * hs:
                        continue  # not shardable by heads: plain column/row handling below
                    rows = self._qkv_rows(nh, ng, hs, world, rank).to(qm.weight.device)
                    self.head_info[f"{qkv_name}.weight"] = (nh, ng, hs)
                    for pname in ("weight", "bias"):
                        t = getattr(qm, pname, None)
                        if t is None:
                            continue
                        if getattr(t, "_lc_tp_kind", None) in (COLUMN, "column_bias"):
                            # column_parallel() ran before row_parallel() named the proj: re-assemble
                            # the plain dim-0 shards (a collective every rank makes) and re-shard by heads
                            parts = [torch.empty_like(t) for _ in range(world)]
                            tdist.all_gather(parts, t.detach().contiguous(), group=group)
                            t_full = torch.cat(parts, 0)
                        else:
                            t_full = t
                        newp = torch.nn.Parameter(t_full.detach().index_select(0, rows).clone(), requires_grad=t.requires_grad)
                        newp._lc_tp_kind = "head_qkv"
                        newp.distparallel_type = DistParallelType.COLUMN_WISE
                        self.original_shapes[f"{qkv_name}.{pname}"] = t_full.shape
                        self.param_kinds[f"{qkv_name}.{pname}"] = ("head_qkv", type(qm))
                        self.head_info[f"{qkv_name}.{pname}"] = (nh, ng, hs)
                        qm._parameters[pname] = newp
                    w = prm.weight
                    n = w.shape[1] // world
                    newp = torch.nn.Parameter(w.detach().narrow(1, rank * n, n).clone(), requires_grad=w.requires_grad)
                    newp._lc_tp_kind = "head_proj"
                    newp.distparallel_type = DistParallelType.ROW_WISE
                    self.original_shapes[f"{proj_name}.weight"] = w.shape
                    self.param_kinds[f"{proj_name}.weight"] = (ROW, type(prm))
                    prm._parameters["weight"] = newp
                    # the attention code now sees this rank's heads only
                    pm.config = replace(cfg, n_head=nh // world, n_query_groups=ng // world)
                    kv = getattr(pm, "kv_cache", None)
                    if kv is not None and hasattr(kv, "k") and kv.k.shape[1] == ng:
                        # a cache allocated before sharding holds every kv group: keep this rank's
                        kv.k = kv.k[:, rank * (ng // world):(rank + 1) * (ng // world)].contiguous()
                        kv.v = kv.v[:, rank * (ng // world):(rank + 1) * (ng // world)].contiguous()
                    head_done.update((qkv_name, proj_name))
            for name, kind in self.targets.items():
                if name in head_done:
                    continue
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
            if "tp_head_qkv" in a.tags or "tp_head_proj" in a.tags:
                # traced with the local shape already (head-parallel attention)
                kinds[a.name] = "head_qkv" if "tp_head_qkv" in a.tags else "head_proj"
                local[a.name] = a
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
                    if name == "linear" and kind == "head_qkv":
                        # this rank's heads: the local qkv feeds the local attention, no gather
                        x2 = col_inputs.get(x.name)
                        if x2 is None:
                            x2 = dist_prims.synchronize_tensor_parallel_input(x, group, TPLayerType.COLUMN_LINEAR)
                            col_inputs[x.name] = x2
                        y = ltorch.linear(x2, wl, bias)
                    elif name == "linear" and kind == "head_proj":
                        # input already holds this rank's heads: no slice, one all-reduce
                        y = ltorch.linear(x, wl, None)
                        y = dist_prims.synchronize_tensor_parallel_output(y, group, TPLayerType.ROW_LINEAR)
                        if bias is not None:
                            y = ltorch.add(y, bias)
                    elif name == "linear" and kind == COLUMN:
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
        if self.vocab_parallel_loss:
            new = vocab_parallel_loss(new, group)
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
                if kind == "head_qkv":
                    nh, ng, hs = self.head_info[full]
                    out[k] = v.index_select(0, self._qkv_rows(nh, ng, hs, world, rank).to(v.device)).clone()
                    continue
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
                parts = [torch.empty_like(v) for _ in range(world)]
                tdist.all_gather(parts, v.contiguous(), group=group)
                if kind == "head_qkv":
                    nh, ng, hs = self.head_info[full]
                    full_t = torch.empty((self.original_shapes[full][0],) + tuple(v.shape[1:]), dtype=v.dtype,
                                         device=v.device)
                    for r, part in enumerate(parts):
                        full_t.index_copy_(0, self._qkv_rows(nh, ng, hs, world, r).to(v.device), part)
                    out[k] = full_t
                    continue
                dim = 0 if (kind == COLUMN or k.endswith("bias")) else 1
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
# Vocab-parallel loss
# ---------------------------------------------------------------------------------------------
_RESHAPES = ("reshape", "view", "flatten")


def vocab_parallel_loss(trace, group):
    """Rewrites ``cross_entropy(reshape*(all_gather_lastdim(linear(x, W_vocab_shard))), target)`` into
    a vocab-parallel cross-entropy on the local logits (weight None, no label smoothing, 2-D logits
    after the reshapes, mean / sum reduction)."""
    from ... import torch as ltorch

    consumers: dict[str, list] = {}
    producers: dict[str, BoundSymbol] = {}
    for b in trace.bound_symbols:
        for a in b.flat_proxy_args:
            consumers.setdefault(a.name, []).append(b)
        for o in b.flat_proxy_outs:
            producers[o.name] = b
    plans = {}
    for b in trace.bound_symbols:
        if b.sym.name != "cross_entropy":
            continue
        args = list(b.args)
        kw = dict(b.kwargs)
        inp = args[0]
        target = args[1] if len(args) > 1 else kw.get("target")
        weight = args[2] if len(args) > 2 else kw.get("weight")
        ignore_index = args[4] if len(args) > 4 else kw.get("ignore_index", -100)
        reduction = args[6] if len(args) > 6 else kw.get("reduction", "mean")
        smoothing = args[7] if len(args) > 7 else kw.get("label_smoothing", 0.0)
        size_average = args[3] if len(args) > 3 else kw.get("size_average")
        reduce_ = args[5] if len(args) > 5 else kw.get("reduce")
        if size_average is not None or reduce_ is not None:
            continue  # legacy reduction flags (reduce=False means 'none'): leave the call alone
        if weight is not None or smoothing or reduction not in ("mean", "sum") or not isinstance(inp, TensorProxy):
            continue
        if inp.ndim != 2 or target is None:
            continue
        chain = []
        p = inp
        ok = False
        while True:
            pb = producers.get(p.name)
            if pb is None:
                break
            if len(consumers.get(p.name, ())) != 1:
                break
            if _is_tp(pb, TPLayerType.COLUMN_LINEAR, out=True):
                ok = True
                break
            if pb.sym.name in _RESHAPES and isinstance(pb.args[0], TensorProxy):
                chain.append(pb)
                p = pb.args[0]
                continue
            break
        if not ok:
            continue
        sync = producers[p.name]
        local = sync.args[0]
        if tuple(local.shape[:-1]) != tuple(p.shape[:-1]) or inp.shape[-1] != p.shape[-1]:
            continue  # the reshapes must only flatten the token dims
        plans[b.output.name if isinstance(b.output, TensorProxy) else id(b)] = (b, local, target, ignore_index, reduction)
    if not plans:
        return trace
    rank, world = tdist.get_rank(group), tdist.get_world_size(group)
    new = from_trace(trace)
    new.bound_symbols = []
    new.scopes = [new.bound_symbols]
    swap: dict = {}
    targets = {id(v[0]): v for v in plans.values()}
    with tracectx(new):
        for b in trace.bound_symbols:
            if id(b) in targets:
                _, local, target, ignore_index, reduction = targets[id(b)]
                local = swap.get(local.name, local)
                target = swap.get(target.name, target) if isinstance(target, TensorProxy) else target
                vl = local.shape[-1]
                l2 = ltorch.reshape(local, (-1, vl))
                t2 = ltorch.reshape(target, (-1,))
                rows, _lse = dist_prims.vocab_parallel_cross_entropy_fwd(l2, t2, group, rank * vl, ignore_index)
                total = ltorch.sum(rows)
                if reduction == "mean":
                    cnt = ltorch.sum(ltorch.to(ltorch.ne(t2, ignore_index), rows.dtype))
                    total = ltorch.true_divide(total, cnt)
                loss = ltorch.to(total, b.output.dtype)
                swap[b.output.name] = loss
                continue
            new.bound_symbols.append(b.swap_proxies(swap))
    new = dce(new)
    new.set_provenance(TraceProvenance("Vocab-parallel cross-entropy"))
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
