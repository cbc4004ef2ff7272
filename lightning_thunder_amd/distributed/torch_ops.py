"""User-visible collectives inside compiled programs (parity: reference ``thunder/torch/__init__.py:6417-6672``:
``all_gather`` / ``all_reduce`` / ``broadcast`` / ``reduce_scatter`` / ``wait`` and the in-place
``torch.distributed.*`` forms).

* Functional forms (``ltorch.all_reduce(a, op, group, async_op)`` ...) return a new tensor, or a
  ``FutureTensorProxy`` for ``async_op=True`` that ``ltorch.wait`` materializes -- the wait-sorting
  pass then overlaps the collective with compute.
* ``torch.distributed.all_reduce(t)`` / ``broadcast(t, src)`` / ``all_gather_into_tensor(out, t)`` /
  ``reduce_scatter_tensor(out, t)`` called by user code are in-place in PyTorch; here they are the
  functional collective followed by ``copy_`` into the destination, which the acquisition
  functionalizes like any other in-place op (the destination's later readers see the result).
All of them lower to RCCL (``nccl`` backend) over xGMI, or gloo on CPU.
"""
from __future__ import annotations

import torch.distributed as tdist

from ..core import prims
from ..core.proxies import FutureTensorProxy
from ..core.prims import OpTags
from . import prims as dist_prims
from .prims import DistributedReduceOps

_REDUCE = {
    "sum": DistributedReduceOps.SUM, "avg": DistributedReduceOps.AVG, "max": DistributedReduceOps.MAX,
    "min": DistributedReduceOps.MIN, "product": DistributedReduceOps.PRODUCT,
}


def to_reduce_op(op) -> DistributedReduceOps:
    if op is None:
        return DistributedReduceOps.SUM
    if isinstance(op, DistributedReduceOps):
        return op
    if isinstance(op, str):
        return _REDUCE[op.lower()]
    for name in ("SUM", "AVG", "MAX", "MIN", "PRODUCT", "BAND", "BOR", "BXOR"):
        if op == getattr(tdist.ReduceOp, name):
            return getattr(DistributedReduceOps, name)
    raise ValueError(f"unsupported reduce op {op!r}")


def _group(group):
    if isinstance(group, str):
        from torch._C._distributed_c10d import _resolve_process_group

        return _resolve_process_group(group)
    return group if group is not None else tdist.distributed_c10d._get_default_group()


def _register():
    import lightning_thunder_amd.torch as ltorch
    from ..torch import torchsymbol

    @torchsymbol(id="functional_all_reduce")
    def all_reduce(a, op=None, group=None, async_op: bool = False):
        return dist_prims.all_reduce(a, to_reduce_op(op), _group(group), async_op)

    @torchsymbol(id="functional_all_gather")
    def all_gather(a, group=None, async_op: bool = False, dim: int = 0):
        return dist_prims.all_gather(a, _group(group), async_op, dim)

    @torchsymbol(id="functional_reduce_scatter")
    def reduce_scatter(a, op=None, group=None, async_op: bool = False, dim: int = 0):
        return dist_prims.reduce_scatter(a, to_reduce_op(op), _group(group), async_op, dim)

    @torchsymbol(id="functional_broadcast")
    def broadcast(a, root: int = 0, group=None, async_op: bool = False):
        return dist_prims.broadcast(a, root, _group(group), async_op)

    @torchsymbol(id="functional_wait")
    def wait(fut):
        return dist_prims.wait(fut) if isinstance(fut, FutureTensorProxy) else fut

    @torchsymbol(tdist.all_reduce, id="all_reduce_", tags=(OpTags.IN_PLACE,))
    def all_reduce_(tensor, op=tdist.ReduceOp.SUM, group=None, async_op: bool = False):
        out = dist_prims.all_reduce(tensor, to_reduce_op(op), _group(group), False)
        prims.copy_(out, tensor)

    @torchsymbol(tdist.broadcast, id="broadcast_", tags=(OpTags.IN_PLACE,))
    def broadcast_(tensor, src: int = 0, group=None, async_op: bool = False, group_src=None):
        out = dist_prims.broadcast(tensor, src if group_src is None else group_src, _group(group), False)
        prims.copy_(out, tensor)

    @torchsymbol(tdist.all_gather_into_tensor, id="all_gather_", tags=(OpTags.IN_PLACE,))
    def all_gather_(output_tensor, input_tensor, group=None, async_op: bool = False):
        out = dist_prims.all_gather(input_tensor, _group(group), False, 0)
        prims.copy_(prims.reshape(out, tuple(output_tensor.shape)), output_tensor)

    @torchsymbol(tdist.reduce_scatter_tensor, id="reduce_scatter_", tags=(OpTags.IN_PLACE,))
    def reduce_scatter_(output, input, op=tdist.ReduceOp.SUM, group=None, async_op: bool = False):
        out = dist_prims.reduce_scatter(input, to_reduce_op(op), _group(group), False, 0)
        prims.copy_(prims.reshape(out, tuple(output.shape)), output)

    for f in (all_reduce_, broadcast_, all_gather_, reduce_scatter_):
        f.written_args = (0,)  # the tensor / output_tensor argument; inputs are only read
    for f in (all_reduce, all_gather, reduce_scatter, broadcast, wait, all_reduce_, broadcast_, all_gather_,
              reduce_scatter_):
        setattr(ltorch, f.name, f)


if tdist.is_available():
    _register()
