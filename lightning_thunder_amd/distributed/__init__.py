"""Distributed training over RCCL/xGMI (parity: reference ``thunder/distributed/__init__.py``).

* ``ddp(jitted_module)``: replicated parameters, bucketed async all-reduce of gradients
  overlapped with the backward (``DDPTransform``).
* ``fsdp(jitted_module, sharding_strategy=ZERO2|ZERO3)``: dim-0 sharded parameters,
  all-gathers issued early / waited late, bucketed async reduce-scatter of gradients
  (``FSDPTransform``).  The optimizer then steps on shards (sharded optimizer state).
* ``column_parallel`` / ``row_parallel``: Megatron-style tensor parallelism.
* ``no_sync()`` on the jitted module for gradient accumulation.

One process per GPU; backend ``"nccl"`` is RCCL on ROCm.
"""
from __future__ import annotations

import os
from contextvars import ContextVar

import torch
import torch.distributed as tdist

_skip_data_parallel_grad_sync = ContextVar("skip_data_parallel_grad_sync", default=False)


def set_skip_data_parallel_grad_sync(value: bool) -> bool:
    prev = _skip_data_parallel_grad_sync.get()
    _skip_data_parallel_grad_sync.set(value)
    return prev


def get_skip_data_parallel_grad_sync() -> bool:
    return _skip_data_parallel_grad_sync.get()


def _sync_grads(module) -> None:
    """Runs the gradient collectives skipped under ``no_sync`` (set up by the DDP transform)."""
    hook = getattr(module, "_lc_sync_grads", None)
    if hook is not None:
        hook()


def high_priority_pg_options():
    """RCCL process-group options with a high-priority internal stream.  On ROCm a high-priority
    stream is placed on a hardware queue of its own; a normal-priority collective stream can land on
    the compute stream's queue (``GPU_MAX_HW_QUEUES`` queues are shared round-robin) and then never
    overlaps compute (``profiles/llama2_7b_world1_rccl_fsdp_step_breakdown.txt``: 0.02 ms of overlap
    on a shared queue, 68 ms on separate ones).  ``LTA_NCCL_HIGH_PRIORITY=0`` turns it off."""
    if not hasattr(tdist, "ProcessGroupNCCL"):
        return None
    opts = tdist.ProcessGroupNCCL.Options()
    opts.is_high_priority_stream = os.environ.get("LTA_NCCL_HIGH_PRIORITY", "1") == "1"
    return opts


def copy_default_process_group():
    """A copy of the default group (reference :39-75): separate RCCL communicator for compiled
    collectives, on a high-priority stream (:func:`high_priority_pg_options`) when the backend is RCCL."""
    os.environ.setdefault("TORCH_NCCL_AVOID_RECORD_STREAMS", "1")
    if tdist.get_backend() == "nccl":
        return tdist.new_group(pg_options=high_priority_pg_options())
    return tdist.new_group()


def _add(model, transform):
    from ..core.transforms import add_transform
    from ..core.module import ThunderModule

    if not isinstance(model, ThunderModule):
        from .. import jit

        model = jit(model)
    return add_transform(model, transform=transform)


def ddp(model, *, broadcast_from: int | None = 0, bucket_size_in_mb: float = 256.0, process_group=None):
    """Distributed data parallel for a ``lightning_thunder_amd.jit`` module (reference :203-321)."""
    from .transforms import DDPTransform

    if not tdist.is_initialized():
        raise RuntimeError("ddp requires torch.distributed to be initialized")
    return _add(model, DDPTransform(process_group, bucket_size_in_mb, broadcast_from))


def fsdp(model, *, device=None, broadcast_from: int | None = None, sharding_strategy=None, bucketing_strategy=None,
         bucket_size_in_mb: float = 256.0, process_group=None):
    """Fully sharded data parallel (reference :382-458)."""
    from .transforms import FSDPTransform, FSDPType, FSDPBucketingStrategy

    if not tdist.is_initialized():
        raise RuntimeError("fsdp requires torch.distributed to be initialized")
    t = FSDPTransform(process_group, sharding_strategy or FSDPType.ZERO2, bucketing_strategy or FSDPBucketingStrategy.NONE,
                      bucket_size_in_mb, broadcast_from, device)
    return _add(model, t)


def column_parallel(model, target_modules, process_group=None):
    from .tensor_parallel import column_parallel as _cp

    return _cp(model, target_modules, process_group)


def row_parallel(model, target_modules, process_group=None):
    from .tensor_parallel import row_parallel as _rp

    return _rp(model, target_modules, process_group)


def __getattr__(name):
    if name in ("FSDPType", "FSDPBucketingStrategy", "DDPTransform", "FSDPTransform"):
        from . import transforms

        return getattr(transforms, name)
    raise AttributeError(name)


from . import prims  # noqa: E402,F401  (registers collectives with the torch executor)
from . import torch_ops  # noqa: E402,F401  (user-visible collectives: ltorch.all_reduce, torch.distributed.*)
