"""Distributed checkpointing of (FSDP/TP-)sharded ThunderModules (reference
``thunder/distributed/checkpoint.py``: ``StateDictOptions``, ``get_model_state_dict``,
``load_model_state_dict``, ``save``, ``load``).

Sharded state dicts are ``torch.distributed.checkpoint`` (DCP) compatible: every FSDP parameter
becomes a ``DTensor`` with a ``Shard(0)`` placement (so DCP writes one file set per rank and can
re-shard on load); ``full_state_dict=True`` gathers full tensors instead (optionally only on
rank 0 and/or offloaded to CPU — with 288 GB of HBM per GPU the gather itself fits for any
model that trains on the node).
"""
from __future__ import annotations

from dataclasses import dataclass
from pathlib import Path
from typing import Any

import torch
import torch.distributed as tdist


@dataclass(frozen=True)
class StateDictOptions:
    full_state_dict: bool = False
    cpu_offload: bool = False
    strict: bool = True
    rank0_only: bool = False

    def __post_init__(self):
        if self.rank0_only and not self.full_state_dict:
            raise ValueError("rank0_only requires full_state_dict=True")


def _fsdp_transform(module):
    from .transforms import FSDPTransform

    cd = getattr(module, "_lc_cd", None)
    for t in (cd.transforms if cd is not None else []):
        if isinstance(t, FSDPTransform):
            return t
    return None


def has_fsdp_modules(module) -> bool:
    return _fsdp_transform(module) is not None


def get_model_state_dict(module, options: StateDictOptions = StateDictOptions(), rank: int | None = None) -> dict[str, Any]:
    rank = tdist.get_rank() if rank is None and tdist.is_initialized() else (rank or 0)
    fsdp = _fsdp_transform(module)
    if options.full_state_dict:
        sd = module.original_state_dict() if hasattr(module, "original_state_dict") else module.state_dict()
        if options.rank0_only and rank != 0:
            return {}
        if options.cpu_offload:
            sd = {k: (v.cpu() if isinstance(v, torch.Tensor) else v) for k, v in sd.items()}
        return sd
    sd = module.state_dict()
    if fsdp is None:
        return {k: (v.cpu() if options.cpu_offload and isinstance(v, torch.Tensor) else v) for k, v in sd.items()}
    from torch.distributed.tensor import DTensor, Shard
    from torch.distributed.device_mesh import DeviceMesh

    group = fsdp._group()
    ranks = tdist.get_process_group_ranks(group)
    dev = "cuda" if torch.cuda.is_available() and next(iter(sd.values())).is_cuda else "cpu"
    mesh = DeviceMesh.from_group(group, dev)
    out = {}
    for k, v in sd.items():
        if k in fsdp.original_shapes and isinstance(v, torch.Tensor):
            full = fsdp.original_shapes[k]
            # shard_tensor pads dim 0 to chunk * world (chunk = ceil(n / world)), so the padding can
            # cover several trailing ranks: rank r holds rows [r*chunk, min((r+1)*chunk, n)) of the
            # real tensor, possibly none (torch.chunk / Shard(0) placement semantics)
            chunk = v.shape[0]
            real = max(0, min(chunk, full[0] - tdist.get_rank(group) * chunk))
            local = v[:real]
            out[k] = DTensor.from_local(local.cpu() if options.cpu_offload else local, mesh, [Shard(0)],
                                        run_check=False, shape=torch.Size(full),
                                        stride=torch.empty(full, device="meta").stride())
        else:
            out[k] = v.cpu() if options.cpu_offload and isinstance(v, torch.Tensor) else v
    return out


def load_model_state_dict(state_dict: dict[str, Any], module, options: StateDictOptions = StateDictOptions(),
                          rank: int | None = None) -> None:
    fsdp = _fsdp_transform(module)
    if options.full_state_dict:
        if hasattr(module, "load_original_state_dict"):
            module.load_original_state_dict(state_dict, strict=options.strict)
        else:
            module.load_state_dict(state_dict, strict=options.strict)
        return
    local = {}
    for k, v in state_dict.items():
        if hasattr(v, "to_local"):
            v = v.to_local()
        local[k] = v
    if fsdp is not None:
        # a Shard(0) local holds this rank's real rows (none on fully padded ranks): re-pad to the
        # module's chunk-sized shard
        own = module.state_dict()
        for k, v in list(local.items()):
            if k in fsdp.original_shapes and k in own and isinstance(v, torch.Tensor) and v.shape != own[k].shape:
                pad = own[k].shape[0] - v.shape[0]
                if pad < 0 or tuple(v.shape[1:]) != tuple(own[k].shape[1:]):
                    raise ValueError(f"{k}: checkpoint shard {tuple(v.shape)} does not fit local shard {tuple(own[k].shape)}")
                local[k] = torch.cat([v.to(own[k].device), v.new_zeros((pad,) + tuple(v.shape[1:]), device=own[k].device)])
    module.load_state_dict(local, strict=options.strict)


def save(converted_state: dict[str, Any], path: Path | str, **kwargs) -> None:
    """Writes a (sharded) state dict with ``torch.distributed.checkpoint``."""
    import torch.distributed.checkpoint as dcp

    dcp.save(converted_state, checkpoint_id=str(path), **kwargs)


def load(module_state: dict[str, Any], path: Path | str, **kwargs) -> None:
    """Fills ``module_state`` (from :func:`get_model_state_dict`) in place from a DCP checkpoint."""
    import torch.distributed.checkpoint as dcp

    dcp.load(module_state, checkpoint_id=str(path), **kwargs)
