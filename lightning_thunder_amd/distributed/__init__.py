"""Distributed data/tensor parallelism over RCCL (parity: reference ``thunder/distributed/__init__.py``)."""
from __future__ import annotations

from contextvars import ContextVar

_skip_data_parallel_grad_sync = ContextVar("skip_data_parallel_grad_sync", default=False)


def set_skip_data_parallel_grad_sync(value: bool) -> bool:
    prev = _skip_data_parallel_grad_sync.get()
    _skip_data_parallel_grad_sync.set(value)
    return prev


def get_skip_data_parallel_grad_sync() -> bool:
    return _skip_data_parallel_grad_sync.get()


def _sync_grads(module) -> None:
    """Runs the gradient collectives skipped under ``no_sync`` (filled in by the DDP/FSDP transforms)."""
    hook = getattr(module, "_lc_sync_grads", None)
    if hook is not None:
        hook()
