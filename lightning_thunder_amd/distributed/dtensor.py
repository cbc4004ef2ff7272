"""DTensor support (parity: reference ``thunder/torch/experimental/dtensor_torch_and_prims.py``
:1-700, ``dtensor_proxy.py``, ``dtensor_utils.py``; tests ``thunder/tests/distributed/test_dtensor.py``).

The reference registers a dtensor twin for a list of prims (reshape, transpose, linear, exp,
``_grouped_mm`` ...) whose metas call DTensor's sharding propagation and whose executions
call ``torch`` on the real DTensors.  Here that pattern is generic: any torch callable reached
with a :class:`~lightning_thunder_amd.core.proxies.DTensorProxy` argument becomes a
``dtensor.<op>`` symbol that

* **meta**: rebuilds the arguments as DTensors over *meta* local tensors (same mesh, placements,
  global shape and stride) and runs the torch op on them — DTensor's propagation rules decide the
  output placements (a needed redistribution runs its functional collectives on meta tensors);
* **execution** (torch executor): the torch op on the real DTensors, so redistributions issue
  the real RCCL collectives (gloo on CPU);
* **gradient**: the generic ``torch.autograd`` rule for opaque ops re-runs the op on the saved
  DTensors in the backward, so cotangents are DTensors as well.

Mixing DTensors with plain tensors, or ops DTensor does not implement, fail during tracing (the
meta raises), like the reference's unsupported-op assertion.
"""
from __future__ import annotations

from typing import Callable

import torch

from ..core.proxies import DTensorProxy, TensorProxy, NumberProxy, Proxy, pyval
from ..core.pytree import tree_flatten, tree_unflatten, tree_map
from ..core.symbol import Symbol, register_symbol

_dtensor_symbols: dict[Callable, Symbol] = {}


def _meta_dtensor(p: DTensorProxy):
    from torch.distributed.tensor import DTensor

    local = torch.empty(p.local_shape, dtype=p.dtype, device="meta")
    return DTensor.from_local(local, p.mesh, p.placements, run_check=False, shape=torch.Size(p.shape),
                              stride=p.stride_)


def _to_meta(x):
    if isinstance(x, DTensorProxy):
        return _meta_dtensor(x)
    if isinstance(x, TensorProxy):
        return torch.empty(x.shape, dtype=x.dtype, device="meta")
    if isinstance(x, NumberProxy):
        return pyval(x)
    return x


def _from_meta(o, device):
    from torch.distributed.tensor import DTensor

    if isinstance(o, DTensor):
        return DTensorProxy(shape=tuple(o.shape), device=device, dtype=o.dtype, mesh=o.device_mesh,
                            placements=o.placements, local_shape=tuple(o.to_local().shape), stride=tuple(o.stride()))
    if isinstance(o, torch.Tensor):
        return TensorProxy(shape=tuple(o.shape), device=device, dtype=o.dtype)
    return o


def dtensor_symbol(fn: Callable, name: str | None = None) -> Symbol:
    """The DTensor-aware symbol for a torch callable (created on first use)."""
    sym = _dtensor_symbols.get(fn)
    if sym is not None:
        return sym
    from ..core.prims import OpTags

    qual = name or getattr(fn, "__qualname__", None) or getattr(fn, "__name__", "op")
    pname = "dtensor_" + "".join(c if c.isalnum() else "_" for c in qual)

    def meta(*args, **kwargs):
        flat, spec = tree_flatten((args, kwargs))
        device = next((x.device for x in flat if isinstance(x, TensorProxy)), torch.device("cpu"))
        margs, mkw = tree_unflatten([_to_meta(x) for x in flat], spec)
        if getattr(fn, "__name__", "") == "redistribute":
            mkw["async_op"] = False
        with torch.no_grad():
            out = fn(*margs, **mkw)
        return tree_map(lambda o: _from_meta(o, device), out)

    sym = Symbol(pname, meta, id=f"dtensor.{qual}", is_prim=True, tags=(OpTags.AUTO_REGISTERED,))
    sym.torch_fn = fn
    register_symbol(sym)
    _dtensor_symbols[fn] = sym
    from ..executors import torchex

    impl = fn
    if fn in (torch.nn.functional.linear, torch._grouped_mm):
        def impl(*a, _fn=fn, **k):
            out = _local_product(_fn, a, k)
            return _fn(*a, **k) if out is None else out
    if getattr(fn, "__name__", "") == "redistribute":
        # the trace orders every consumer after the collective: run it synchronously on the stream
        def impl(*a, _fn=fn, **k):
            k["async_op"] = False
            return _fn(*a, **k)

    torchex.register_opaque(sym, impl)
    return sym


def _local_product(fn, args, kwargs):
    """Column-parallel products whose placements need no communication, run on the local shards
    with the hand-written GEMM kernels (``ops/gemm.py``) and re-wrapped as DTensors:

    * ``linear(x, w, b)``: x replicated, w (and b) sharded on the output features (``Shard(0)``) or
      replicated on each mesh dim -> y sharded on its last dim where w is sharded;
    * ``torch._grouped_mm(x, w, offs)`` (MoE experts): x and offs replicated, w ``[G, K, N]`` sharded
      on N (``Shard(2)``) or replicated -> y sharded on its last dim.

    Returns None when the pattern does not apply (the DTensor op then runs as is).  Only the forward
    uses this path: the backward re-runs the DTensor op under torch autograd."""
    try:
        from torch.distributed.tensor import DTensor, Replicate, Shard
    except ImportError:  # pragma: no cover
        return None
    if fn is torch.nn.functional.linear:
        x, w = args[0], args[1]
        b = args[2] if len(args) > 2 else kwargs.get("bias")
        wdim = 0
    else:
        if len(args) < 3 or kwargs:
            return None
        x, w, b = args[0], args[1], None
        offs = args[2]
        if isinstance(offs, DTensor):
            if any(not p.is_replicate() for p in offs.placements):
                return None
            offs = offs.to_local()
        wdim = 2
    if not (isinstance(x, DTensor) and isinstance(w, DTensor)) or x.device_mesh != w.device_mesh:
        return None
    if not x.to_local().is_cuda or any(not p.is_replicate() for p in x.placements):
        return None
    out_pl = []
    for p in w.placements:
        if p.is_replicate():
            out_pl.append(Replicate())
        elif p.is_shard() and p.dim % w.ndim == wdim:
            out_pl.append(Shard(x.ndim - 1))
        else:
            return None
    bl = None
    if b is not None:
        if not isinstance(b, DTensor) or len(b.placements) != len(w.placements):
            return None
        for pb, pw in zip(b.placements, w.placements):
            if not ((pb.is_replicate() and pw.is_replicate()) or (pb.is_shard() and pw.is_shard() and pb.dim % b.ndim == 0)):
                return None
        bl = b.to_local()
    from ..ops import gemm

    xl, wl = x.to_local(), w.to_local()
    if fn is torch.nn.functional.linear:
        yl = gemm.linear(xl, wl, bl)
        shape = tuple(x.shape[:-1]) + (w.shape[0],)
    else:
        if xl.ndim != 2 or wl.ndim != 3:
            return None
        yl = gemm.grouped_mm(xl, wl, offs)
        shape = (x.shape[0], w.shape[2])
    stride = []
    acc = 1
    for n in reversed(shape):
        stride.append(acc)
        acc *= n
    return DTensor.from_local(yl, x.device_mesh, out_pl, run_check=False, shape=torch.Size(shape),
                              stride=tuple(reversed(stride)))


def has_dtensor(flat) -> bool:
    return any(isinstance(x, DTensorProxy) for x in flat)


def is_dtensor(t) -> bool:
    try:
        from torch.distributed.tensor import DTensor
    except ImportError:  # pragma: no cover
        return False
    return isinstance(t, DTensor)


# --- frontend lookasides -------------------------------------------------------------------------
def _from_local_impl(local, mesh, placements, run_check, shape, stride):
    from torch.distributed.tensor import DTensor

    return DTensor.from_local(local, mesh, placements, run_check=run_check, shape=shape, stride=stride)


_from_local_impl.__qualname__ = "DTensor.from_local"


def python_lookasides() -> list:
    """``(owner, attribute, replacement)`` patched while a program is acquired: DTensor construction
    from a traced local tensor becomes a ``dtensor.DTensor.from_local`` symbol."""
    try:
        from torch.distributed.tensor import DTensor, Replicate
    except ImportError:  # pragma: no cover
        return []
    orig = DTensor.from_local

    def from_local(local_tensor, device_mesh=None, placements=None, *, run_check=False, shape=None, stride=None):
        if isinstance(local_tensor, DTensorProxy):
            # already a DTensor: native torch code (parallel styles) cannot see that through
            # isinstance on the proxy and would wrap it again; torch skips from_local for DTensors
            return local_tensor
        if not isinstance(local_tensor, TensorProxy):
            return orig(local_tensor, device_mesh, placements, run_check=run_check, shape=shape, stride=stride)
        if device_mesh is None:
            from torch.distributed.device_mesh import _mesh_resources

            device_mesh = _mesh_resources.get_current_mesh()
        if placements is None:
            placements = [Replicate() for _ in range(device_mesh.ndim)]
        shape = tuple(shape) if shape is not None else None
        stride = tuple(stride) if stride is not None else None
        return dtensor_symbol(_from_local_impl)(local_tensor, device_mesh, tuple(placements), run_check, shape, stride)

    return [(DTensor, "from_local", from_local)]
