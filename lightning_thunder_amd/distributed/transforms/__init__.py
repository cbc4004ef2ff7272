"""Data-parallel trace transforms (parity: reference ``thunder/distributed/transforms/{ddp_v2,fsdp_v2}.py``)."""
from __future__ import annotations

import math

import torch
import torch.distributed as tdist

from ...core.proxies import TensorProxy, DistParallelType, ProxyTag
from ...core.symbol import BoundSymbol
from ...core.trace import TraceCtx, from_trace, tracectx, TraceProvenance
from ...core.transform_common import Transform
from .. import prims as dist_prims


def _is_param(p) -> bool:
    return isinstance(p, TensorProxy) and "parameter" in p.tags


def _insert_after_inputs(comp: TraceCtx, make_new) -> TraceCtx:
    """Builds a new computation trace where ``make_new(p)`` (recorded at the top) replaces each param proxy."""
    new = from_trace(comp)
    new.bound_symbols = []
    new.scopes = [new.bound_symbols]
    swap = {}
    with tracectx(new):
        for p in comp.args:
            if _is_param(p):
                q = make_new(p)
                if q is not None and q is not p:
                    swap[p.name] = q
    for b in comp.bound_symbols:
        new.bound_symbols.append(b.swap_proxies(swap))
    return new


class DDPTransform(Transform):
    """Replicated parameters; bucketed async all-reduce(AVG) of gradients overlapped with the backward.

    Reference: ``thunder/distributed/transforms/ddp_v2.py:24-197``.
    """

    def __init__(self, process_group=None, bucket_size_in_mb: float = 256.0, broadcast_from: int | None = 0):
        self.process_group = process_group
        self.bucket_size_in_mb = bucket_size_in_mb
        self.broadcast_from = broadcast_from

    def _group(self):
        return self.process_group if self.process_group is not None else tdist.distributed_c10d._get_default_group()

    def transform_module(self, model) -> None:
        cd = getattr(model, "_lc_cd", None)
        if cd is not None:
            cd.compile_options.setdefault("lta_bucket_size_mb", self.bucket_size_in_mb)
        inner = model._model
        if self.broadcast_from is not None:
            with torch.no_grad():
                seen = set()
                tensors = []
                for t in list(inner.parameters()) + list(inner.buffers()):
                    if id(t) in seen:
                        continue
                    seen.add(id(t))
                    tensors.append(t)
                for t in tensors:
                    tdist.broadcast(t.data, self.broadcast_from, group=self._group())
        group = self._group()

        def sync_grads():
            grads = [p.grad for p in inner.parameters() if p.grad is not None]
            if not grads:
                return
            flat = torch._utils._flatten_dense_tensors(grads)
            tdist.all_reduce(flat, group=group)
            flat.div_(tdist.get_world_size(group))
            for g, s in zip(grads, torch._utils._unflatten_dense_tensors(flat, grads)):
                g.copy_(s)

        model._lc_sync_grads = sync_grads

    def transform_traces_pre_prologue(self, prologue_trace, computation_trace, epilogue_trace, **kwargs):
        group = self._group()

        def mk(p):
            if not p.requires_grad:
                return None
            p.distparallel_type = DistParallelType.REPLICATED
            return dist_prims.synchronize(p, group, DistParallelType.REPLICATED)

        comp = _insert_after_inputs(computation_trace, mk)
        comp.set_provenance(TraceProvenance("DDP: parameters marked REPLICATED"))
        return prologue_trace, comp, epilogue_trace


class FSDPType:
    ZERO2 = "zero2"
    ZERO3 = "zero3"


class FSDPBucketingStrategy:
    """Granularity of the FSDP forward parameter all-gathers (reference ``FSDPBucketingStrategy``,
    unwired there): per parameter, per module (LAYER) or per numbered block (BLOCK, ~400 MB per
    Llama-2-7B block: one grouped collective that loads all 7 xGMI links)."""

    NONE = "none"
    LAYER = "layer"
    BLOCK = "block"


def shard_tensor(t: torch.Tensor, rank: int, world: int, dim: int = 0):
    """Shard along ``dim`` with padding to a multiple of ``world`` (reference distributed/__init__.py:508-546)."""
    n = t.shape[dim]
    chunk = (n + world - 1) // world
    pad = chunk * world - n
    if pad:
        pad_shape = list(t.shape)
        pad_shape[dim] = pad
        t = torch.cat([t, torch.zeros(pad_shape, dtype=t.dtype, device=t.device)], dim)
    return t.narrow(dim, rank * chunk, chunk).clone(), pad


class FSDPTransform(Transform):
    """Fully-sharded data parallel: every parameter sharded along dim 0 (padded); forward all-gather
    (issued early, waited late); backward bucketed reduce-scatter(AVG).  ZeRO-3 re-gathers
    parameters in the backward instead of saving the gathered copies.

    Reference: ``thunder/distributed/transforms/fsdp_v2.py`` + ``thunder/distributed/__init__.py:324-460``.
    """

    def __init__(self, process_group=None, sharding_strategy=FSDPType.ZERO2, bucketing_strategy=FSDPBucketingStrategy.NONE,
                 bucket_size_in_mb: float = 256.0, broadcast_from: int | None = None, device=None,
                 replicate_process_group=None):
        self.process_group = process_group
        self.replicate_process_group = replicate_process_group  # hybrid (ddp x fsdp) mesh
        self.sharding_strategy = sharding_strategy
        self.bucketing_strategy = bucketing_strategy
        self.bucket_size_in_mb = bucket_size_in_mb
        self.broadcast_from = broadcast_from
        self.device = device
        self.original_shapes: dict[str, torch.Size] = {}

    def _group(self):
        return self.process_group if self.process_group is not None else tdist.distributed_c10d._get_default_group()

    def transform_module(self, model) -> None:
        cd = getattr(model, "_lc_cd", None)
        if cd is not None:
            cd.compile_options.setdefault("lta_bucket_size_mb", self.bucket_size_in_mb)
            # forward all-gathers: one coalesced RCCL launch per layer / block instead of one per
            # parameter (executors/passes.py -> distributed/bucketing.py:bucket_fsdp_all_gathers)
            cd.compile_options.setdefault("lta_fsdp_bucketing", self.bucketing_strategy)
            if self.sharding_strategy == FSDPType.ZERO3:
                # ZeRO-3 frees gathered parameters after use: bound the in-flight gathers to a
                # 2-bucket prefetch window (distributed/utils.py:schedule_allgathers)
                cd.compile_options.setdefault("lta_fsdp_allgather_window", 2)
        group = self._group()
        rank, world = tdist.get_rank(group), tdist.get_world_size(group)
        inner = model._model
        if self.device is not None:
            inner.to(self.device)
        with torch.no_grad():
            if self.broadcast_from is not None:
                for t in list(inner.parameters()) + list(inner.buffers()):
                    tdist.broadcast(t.data, self.broadcast_from, group=group)
            done: dict[int, torch.nn.Parameter] = {}
            for mname, m in inner.named_modules():
                for pname, p in list(m._parameters.items()):
                    if p is None:
                        continue
                    full = f"{mname}.{pname}" if mname else pname
                    if id(p) in done:
                        m._parameters[pname] = done[id(p)]
                        continue
                    if getattr(p, "_lc_full_shape", None) is not None:
                        continue  # already sharded (transform_module re-run by add_transform)
                    self.original_shapes[full] = p.shape
                    shard, pad = shard_tensor(p.data, rank, world)
                    newp = torch.nn.Parameter(shard, requires_grad=p.requires_grad)
                    newp.distparallel_type = DistParallelType.FULLY_SHARDED
                    newp.thunder_fsdp_padding_size = pad
                    newp._lc_full_shape = tuple(p.shape)
                    done[id(p)] = newp
                    m._parameters[pname] = newp
        model._lc_fsdp = self
        replicate = self.replicate_process_group

        def sync_grads():
            """Leaving ``no_sync``: reduce-scatter (AVG) every stashed unsharded gradient in one
            collective (interleaved pack: rank r's chunk holds its rows of every gradient) and add
            the shards to ``.grad`` (reference ``_sync_grads``, thunder/distributed/__init__.py:144-182)."""
            from .. import prims as dp

            params = [p for p in inner.parameters() if getattr(p, "_lc_unsharded_grad", None) is not None]
            if not params:
                return
            grads = [p._lc_unsharded_grad for p in params]
            for p in params:
                del p._lc_unsharded_grad
            buf = dp._pack_for_fsdp_impl(grads, world, "scatter")
            shards = dp._reduce_scatter_impl(buf, dp.DistributedReduceOps.AVG, group)
            if replicate is not None:
                shards = dp._all_reduce_impl(shards, dp.DistributedReduceOps.AVG, replicate, skip_clone=True)
            with torch.no_grad():
                for p, g in zip(params, dp._unpack_for_fsdp_impl(shards, grads, world, "scatter")):
                    g = g.to(p.dtype)
                    if p.grad is None or p.grad.stride() == (0,) * p.grad.dim():
                        p.grad = g.clone()
                    else:
                        p.grad.add_(g)

        model._lc_sync_grads = sync_grads

    def transform_traces_pre_prologue(self, prologue_trace, computation_trace, epilogue_trace, **kwargs):
        from ... import torch as ltorch

        group = self._group()
        world = tdist.get_world_size(group)
        zero3 = self.sharding_strategy == FSDPType.ZERO3
        new_args = {}

        def mk(p):
            if p.distparallel_type is not DistParallelType.FULLY_SHARDED:
                return None
            pad = p.thunder_fsdp_padding_size or 0
            n = p.shape[0]
            shard_shape = ((n + pad) // world,) + tuple(p.shape[1:])
            shard = TensorProxy(like=p, shape=shard_shape, name=computation_trace.make_unique_name(p.name + "_shard"))
            shard.tags = set(p.tags)
            new_args[p.name] = shard
            full = dist_prims.synchronize(shard, group, DistParallelType.FULLY_SHARDED, self.replicate_process_group)
            if pad:
                full = ltorch.narrow(full, 0, 0, n)
            return full

        comp = _insert_after_inputs(computation_trace, mk)
        comp.args = [new_args.get(a.name, a) for a in comp.args]
        if zero3:
            from ...core.symbol import BoundSymbolTag

            gathered = set()
            for b in comp.bound_symbols:
                if b.sym is dist_prims.synchronize:
                    b.tags.add(BoundSymbolTag.RECOMPUTE_IN_BACKWARD)
                    gathered.add(b.output.name)
                elif "narrow" in b.sym.name and b.args and getattr(b.args[0], "name", None) in gathered:
                    # the padding trim of a gathered parameter is re-done with the gather, so the
                    # backward saves the shard, not the full parameter
                    b.tags.add(BoundSymbolTag.RECOMPUTE_IN_BACKWARD)
        comp.set_provenance(TraceProvenance(f"FSDP ({self.sharding_strategy}): parameters all-gathered"))
        return prologue_trace, comp, epilogue_trace

    # --- state dict: shard on load, gather on save (reference fsdp_v2.py:249-294) ------------------
    def transform_state_dict_for_submodule(self, model, submodule_name, state_dict):
        group = self._group()
        rank, world = tdist.get_rank(group), tdist.get_world_size(group)
        out = {}
        for k, v in state_dict.items():
            full = f"{submodule_name}.{k}" if submodule_name else k
            if full in self.original_shapes and isinstance(v, torch.Tensor):
                out[k], _ = shard_tensor(v, rank, world)
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
                gathered = torch.empty((v.shape[0] * world,) + tuple(v.shape[1:]), dtype=v.dtype, device=v.device)
                tdist.all_gather_into_tensor(gathered, v.contiguous(), group=group)
                out[k] = gathered[: self.original_shapes[full][0]]
            else:
                out[k] = v
        return out
