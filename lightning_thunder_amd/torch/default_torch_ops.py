"""Auto-registration of long-tail torch ops as opaque symbols (parity: reference
``thunder/torch/default_torch_ops.py:3-691`` and registration ``thunder/torch/__init__.py:6800-6885``).

Any torch callable reached while tracing that has no hand-written ``@torchsymbol``
becomes an opaque prim tagged ``AUTO_REGISTERED``:

* meta: the torch callable run on ``meta`` tensors (output shapes/dtypes exactly torch's),
* execution: the torch executor calls the original callable,
* gradient: ``torch.autograd`` re-runs the callable on saved inputs in the backward
  (see ``transforms/autodiff.py``).

Unlike the reference (a fixed list of 670 names) registration happens on first
use, so every torch op a model touches is covered; the list below is what is
pre-registered and reported by ``get_auto_registered_torch_op_names``.
"""
from __future__ import annotations

import math
from typing import Callable

import torch

from ..core import dtypes, prims
from ..core.proxies import TensorProxy, NumberProxy, Proxy, pyval
from ..core.pytree import tree_flatten, tree_unflatten, tree_map
from ..core.symbol import Symbol, register_symbol

_opaque_symbols: dict[Callable, Symbol] = {}
_auto_registered_names: set[str] = set()

# Pre-registered long tail (names resolved against torch at import time)
DEFAULT_OPS = [
    "torch.nn.functional.conv1d", "torch.nn.functional.conv2d", "torch.nn.functional.conv3d",
    "torch.nn.functional.conv_transpose1d", "torch.nn.functional.conv_transpose2d",
    "torch.nn.functional.max_pool1d", "torch.nn.functional.max_pool2d", "torch.nn.functional.avg_pool1d",
    "torch.nn.functional.avg_pool2d", "torch.nn.functional.adaptive_avg_pool2d", "torch.nn.functional.batch_norm",
    "torch.nn.functional.instance_norm", "torch.nn.functional.interpolate", "torch.nn.functional.unfold",
    "torch.nn.functional.fold", "torch.nn.functional.pixel_shuffle", "torch.nn.functional.glu",
    "torch.nn.functional.selu", "torch.nn.functional.celu", "torch.nn.functional.softsign",
    "torch.nn.functional.tanhshrink", "torch.nn.functional.hardsigmoid", "torch.nn.functional.smooth_l1_loss",
    "torch.nn.functional.huber_loss", "torch.nn.functional.kl_div", "torch.nn.functional.cosine_similarity",
    "torch.nn.functional.pairwise_distance", "torch.nn.functional.embedding_bag",
    "torch.cumprod", "torch.cummax", "torch.cummin", "torch.diag", "torch.diagonal", "torch.diag_embed",
    "torch.trace", "torch.kron", "torch.cross", "torch.linalg.norm", "torch.linalg.vector_norm",
    "torch.linalg.matrix_norm", "torch.linalg.inv", "torch.linalg.solve", "torch.linalg.cholesky",
    "torch.linalg.qr", "torch.linalg.svd", "torch.linalg.eigh", "torch.linalg.det", "torch.norm",
    "torch.fft.fft", "torch.fft.ifft", "torch.fft.rfft", "torch.fft.irfft", "torch.fft.fft2", "torch.fft.ifft2",
    "torch.special.gammaln", "torch.special.i0", "torch.special.ndtr", "torch.special.log_ndtr",
    "torch.special.xlogy", "torch.special.entr", "torch.hypot", "torch.logaddexp", "torch.logaddexp2",
    "torch.heaviside", "torch.frac", "torch.deg2rad", "torch.rad2deg", "torch.sinc", "torch.logit",
    "torch.count_nonzero", "torch.bincount", "torch.histc", "torch.bucketize", "torch.searchsorted",
    "torch.meshgrid", "torch.cartesian_prod", "torch.block_diag", "torch.tile", "torch.rot90",
    "torch.diff", "torch.trapezoid", "torch.vander", "torch.tensordot", "torch.inner", "torch.dot",
    "torch.vdot", "torch.mv", "torch.addmv", "torch.addr", "torch.chain_matmul", "torch.cdist",
    "torch.median", "torch.nanmedian", "torch.mode", "torch.kthvalue", "torch.quantile", "torch.nansum",
    "torch.nanmean", "torch.std", "torch.logcumsumexp", "torch.unique_consecutive", "torch.take",
    "torch.masked_select", "torch.nonzero", "torch.unique", "torch.view_as_real", "torch.view_as_complex",
    "torch.complex", "torch.angle", "torch.conj", "torch.conj_physical", "torch.as_strided",
]


def _resolve(name: str):
    obj = None
    parts = name.split(".")
    try:
        obj = __import__(parts[0])
        for p in parts[1:]:
            obj = getattr(obj, p)
    except (ImportError, AttributeError):
        return None
    return obj


def _to_meta(x):
    if isinstance(x, TensorProxy):
        return torch.empty(x.shape, dtype=x.dtype, device="meta", requires_grad=False)
    if isinstance(x, NumberProxy):
        return x.value
    if isinstance(x, torch.Tensor):
        return x.to("meta") if x.device.type != "meta" else x
    return x


def _first_device(flat):
    for x in flat:
        if isinstance(x, TensorProxy):
            return x.device
    return torch.device("cpu")


def _make_meta(fn: Callable):
    def meta(*args, **kwargs):
        flat, spec = tree_flatten((args, kwargs))
        device = kwargs.get("device", None)
        device = torch.device(device) if device is not None else _first_device(flat)
        margs, mkwargs = tree_unflatten([_to_meta(x) for x in flat], spec)
        if "device" in mkwargs:
            mkwargs["device"] = "meta"
        with torch.no_grad():
            out = fn(*margs, **mkwargs)

        def back(o):
            if isinstance(o, torch.Tensor):
                return TensorProxy(shape=tuple(o.shape), device=device, dtype=o.dtype)
            return o

        return tree_map(back, out)

    return meta


def opaque_symbol(fn: Callable, name: str | None = None) -> Symbol:
    """Returns (creating on first use) the opaque symbol for a torch callable."""
    sym = _opaque_symbols.get(fn)
    if sym is not None:
        return sym
    from ..core.prims import OpTags

    qual = name or getattr(fn, "__qualname__", None) or getattr(fn, "__name__", "op")
    mod = getattr(fn, "__module__", None) or "torch"
    full = f"{mod}.{qual}".replace("torch._C._nn.", "torch.nn.functional.").replace("torch._C._VariableFunctions.", "torch.")
    pname = "".join(c if c.isalnum() else "_" for c in full)
    sym = Symbol(pname, _make_meta(fn), id=f"auto.{full}", is_prim=True, tags=(OpTags.AUTO_REGISTERED,))
    sym.torch_fn = fn
    register_symbol(sym)
    _opaque_symbols[fn] = sym
    _auto_registered_names.add(full)
    _register_torch_impl(sym, fn)
    return sym


def _register_torch_impl(sym, fn):
    from ..executors import torchex

    torchex.register_opaque(sym, fn)


def get_auto_registered_torch_op_names() -> set[str]:
    return set(_auto_registered_names)


# --- helpers used by ltorch ------------------------------------------------------------
def _setitem_impl(a, key, value):
    out = a.clone()
    out[key] = value
    return out


_setitem_impl.__qualname__ = "functional_setitem"
_setitem_impl.__module__ = "thunder"


def functional_setitem(a, key, value):
    return opaque_symbol(_setitem_impl, "functional_setitem")(a, key, value)


def _index_impl(a, key):
    return a[key]


_index_impl.__qualname__ = "advanced_getitem"
_index_impl.__module__ = "thunder"


def _opaque_index(a, key):
    return opaque_symbol(_index_impl, "advanced_getitem")(a, key)


def opaque_einsum(equation, *operands):
    return opaque_symbol(torch.einsum)(equation, *operands)


def opaque_polar(a, b):
    return opaque_symbol(torch.polar)(a, b)


def _install():
    from .. import torch as ltorch

    ltorch._opaque_index = _opaque_index
    for name in DEFAULT_OPS:
        fn = _resolve(name)
        if fn is not None and fn not in ltorch._torch_to_thunder_function_map:
            _auto_registered_names.add(name)


_install()
