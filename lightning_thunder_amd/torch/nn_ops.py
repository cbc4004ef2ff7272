"""More ltorch decompositions: activations, shape utilities, convolution, pooling, normalization and
interpolation (parity: reference ``thunder/torch/__init__.py`` — ``celu``/``selu``/… activations,
``atleast_*``, ``diagonal``, ``unfold``, ``index_copy``, ``multi_dot``, ``batch_norm`` /
``instance_norm`` / ``local_response_norm``, ``convolution`` + ``conv{1,2,3}d``, ``avg_pool*`` /
``max_pool*`` / ``adaptive_avg_pool2d``, ``interpolate``, ``softmin``, ``embedding_backward``).

Every op here is a decomposition into existing ltorch / clang / prims symbols, so it gets an
analytic VJP (through its parts) and can be fused by hipfuse; the torch executor still runs the
whole op as one ATen call when nothing better claims it.  Options a decomposition does not cover
(e.g. ``return_indices`` of max pooling, bicubic interpolation) route to the opaque ATen op.

Convolution is the prim ``convolution`` with an explicit backward prim (``convolution_backward``
-> ``aten.convolution_backward``), so its VJP no longer re-runs torch.autograd.
"""
from __future__ import annotations

import builtins
import math

import torch

from ..core import dtypes, prims
from ..core.baseutils import check
from ..core.proxies import TensorProxy, pyval
from .. import clang
from . import (torchsymbol, _tfn, _this, add, sub, mul, true_divide, where, gt, ge, lt, abs, neg, exp, expm1, tanh,
               sigmoid, relu, leaky_relu, clamp, softmax, reshape, movedim, unsqueeze, squeeze, index_select,
               index_put, arange, pad, sum, mean, var_mean, maximum, square, pow, rsqrt, matmul, full_like, cat,
               flatten, expand, copy_, log_softmax)


def _export(sym):
    setattr(_this, sym.name, sym)
    return sym


def _opaque(fn, name=None):
    from .default_torch_ops import opaque_symbol

    return opaque_symbol(fn, name)


def _tuple(v, n):
    v = pyval(v) if not isinstance(v, (tuple, list)) else tuple(pyval(x) for x in v)
    if isinstance(v, (tuple, list)):
        check(len(v) in (1, n), f"expected {n} values, got {v}")
        return tuple(v) * (n if len(v) == 1 else 1)
    return (v,) * n


# =========================================================================================
# Activations
# =========================================================================================
@_export
@torchsymbol(*_tfn("celu", "nn.functional.celu"), id="torch.celu")
def celu(a, alpha: float = 1.0, inplace: bool = False):
    return where(gt(a, 0), a, mul(expm1(true_divide(a, alpha)), alpha))


_SELU_ALPHA = 1.6732632423543772848170429916717
_SELU_SCALE = 1.0507009873554804934193349852946


@_export
@torchsymbol(*_tfn("selu", "nn.functional.selu"), id="torch.selu")
def selu(a, inplace: bool = False):
    return mul(where(gt(a, 0), a, mul(expm1(a), _SELU_ALPHA)), _SELU_SCALE)


@_export
@torchsymbol(*_tfn("nn.functional.hardshrink", "Tensor.hardshrink"), id="torch.nn.functional.hardshrink")
def hardshrink(a, lambd: float = 0.5):
    return where(gt(abs(a), lambd), a, 0.0)


@_export
@torchsymbol(*_tfn("nn.functional.softshrink"), id="torch.nn.functional.softshrink")
def softshrink(a, lambd: float = 0.5):
    return where(gt(a, lambd), sub(a, lambd), where(lt(a, -lambd), add(a, lambd), 0.0))


@_export
@torchsymbol(*_tfn("nn.functional.hardsigmoid"), id="torch.nn.functional.hardsigmoid")
def hardsigmoid(a, inplace: bool = False):
    return true_divide(clamp(add(a, 3.0), 0.0, 6.0), 6.0)


@_export
@torchsymbol(*_tfn("nn.functional.softsign"), id="torch.nn.functional.softsign")
def softsign(a):
    return true_divide(a, add(abs(a), 1.0))


@_export
@torchsymbol(*_tfn("nn.functional.tanhshrink"), id="torch.nn.functional.tanhshrink")
def tanhshrink(a):
    return sub(a, tanh(a))


@_export
@torchsymbol(*_tfn("threshold", "nn.functional.threshold"), id="torch.threshold")
def threshold(a, threshold, value, inplace: bool = False):
    return where(gt(a, threshold), a, value)


@_export
@torchsymbol(*_tfn("nn.functional.glu"), id="torch.nn.functional.glu")
def glu(a, dim: int = -1):
    d = clang.canonicalize_dim(a.ndim, dim)
    n = a.shape[d]
    check(n % 2 == 0, f"glu: dim {dim} of size {n} is not even")
    x = clang.slice_in_dim(a, 0, n // 2, 1, d)
    g = clang.slice_in_dim(a, n // 2, n, 1, d)
    return mul(x, sigmoid(g))


@_export
@torchsymbol(*_tfn("nn.functional.prelu", "prelu", "Tensor.prelu"), id="torch.nn.functional.prelu")
def prelu(a, weight):
    w = weight
    if a.ndim >= 2 and weight.numel > 1:
        w = reshape(weight, (1, weight.shape[0]) + (1,) * (a.ndim - 2))
    return where(ge(a, 0), a, mul(a, w))


@_export
@torchsymbol(*_tfn("nn.functional.rrelu", "rrelu"), id="torch.nn.functional.rrelu")
def rrelu(a, lower: float = 1.0 / 8.0, upper: float = 1.0 / 3.0, training: bool = False, inplace: bool = False):
    if not training:
        return leaky_relu(a, (lower + upper) / 2.0)
    slope = prims.uniform(a.shape, lower, upper, device=a.device, dtype=clang.compute_dtype(a.dtype))
    return where(ge(a, 0), a, clang.maybe_convert_to_dtype(mul(a, slope), a.dtype))


@_export
@torchsymbol(*_tfn("nn.functional.softmin"), id="torch.nn.functional.softmin")
def softmin(a, dim=None, _stacklevel: int = 3, dtype=None):
    check(dim is not None, "softmin: pass dim explicitly")
    return softmax(neg(a), dim, dtype)


@_export
@torchsymbol(*_tfn("ldexp", "Tensor.ldexp"), is_method=True, id="torch.ldexp")
def ldexp(a, other):
    return mul(a, pow(2.0, other))


# =========================================================================================
# Shape utilities
# =========================================================================================
@_export
@torchsymbol(*_tfn("atleast_1d"), id="torch.atleast_1d")
def atleast_1d(*tensors):
    ts = tensors[0] if len(tensors) == 1 and isinstance(tensors[0], (tuple, list)) else tensors
    out = [reshape(t, (1,)) if t.ndim == 0 else t for t in ts]
    return out[0] if len(out) == 1 and not (len(tensors) == 1 and isinstance(tensors[0], (tuple, list))) else tuple(out)


@_export
@torchsymbol(*_tfn("atleast_2d"), id="torch.atleast_2d")
def atleast_2d(*tensors):
    ts = tensors[0] if len(tensors) == 1 and isinstance(tensors[0], (tuple, list)) else tensors
    out = []
    for t in ts:
        out.append(reshape(t, (1, 1)) if t.ndim == 0 else (unsqueeze(t, 0) if t.ndim == 1 else t))
    return out[0] if len(out) == 1 and not (len(tensors) == 1 and isinstance(tensors[0], (tuple, list))) else tuple(out)


@_export
@torchsymbol(*_tfn("atleast_3d"), id="torch.atleast_3d")
def atleast_3d(*tensors):
    ts = tensors[0] if len(tensors) == 1 and isinstance(tensors[0], (tuple, list)) else tensors
    out = []
    for t in ts:
        if t.ndim == 0:
            t = reshape(t, (1, 1, 1))
        elif t.ndim == 1:
            t = reshape(t, (1, t.shape[0], 1))
        elif t.ndim == 2:
            t = unsqueeze(t, 2)
        out.append(t)
    return out[0] if len(out) == 1 and not (len(tensors) == 1 and isinstance(tensors[0], (tuple, list))) else tuple(out)


@_export
@torchsymbol(*_tfn("diagonal", "Tensor.diagonal"), is_method=True, id="torch.diagonal")
def diagonal(a, offset: int = 0, dim1: int = 0, dim2: int = 1):
    d1, d2 = clang.canonicalize_dim(a.ndim, dim1), clang.canonicalize_dim(a.ndim, dim2)
    check(d1 != d2, "diagonal: dims must differ")
    x = movedim(a, (d1, d2), (-2, -1))
    n1, n2 = x.shape[-2], x.shape[-1]
    if offset >= 0:
        length = builtins.max(builtins.min(n1, n2 - offset), 0)
        start = offset
    else:
        length = builtins.max(builtins.min(n1 + offset, n2), 0)
        start = -offset * n2
    flat = reshape(x, tuple(x.shape[:-2]) + (n1 * n2,))
    idx = arange(start, start + length * (n2 + 1), n2 + 1, device=a.device) if length else \
        arange(0, 0, device=a.device)
    return index_select(flat, flat.ndim - 1, idx)


@_export
@torchsymbol(torch.Tensor.unfold, is_method=True, id="torch.Tensor.unfold")
def unfold(a, dimension: int, size: int, step: int):
    d = clang.canonicalize_dim(a.ndim, dimension) if a.ndim else 0
    n = a.shape[d] if a.ndim else 1
    nw = (n - size) // step + 1
    check(nw >= 1, f"unfold: size {size} exceeds dimension {n}")
    # window w, element j -> source index w*step + j
    starts = arange(0, nw * step, step, device=a.device)
    offs = arange(0, size, device=a.device)
    idx = reshape(add(unsqueeze(starts, 1), unsqueeze(offs, 0)), (nw * size,))
    g = index_select(a, d, idx)  # [..., nw*size, ...]
    g = reshape(g, tuple(a.shape[:d]) + (nw, size) + tuple(a.shape[d + 1:]))
    return movedim(g, d + 1, -1)


@_export
@torchsymbol(*_tfn("index_copy", "Tensor.index_copy"), is_method=True, id="torch.index_copy")
def index_copy(a, dim: int, index, source):
    d = clang.canonicalize_dim(a.ndim, dim)
    x = movedim(a, d, 0)
    s = movedim(source, d, 0) if source.ndim == a.ndim else source
    y = index_put(x, (index,), s, False)
    return movedim(y, 0, d)


@_export
@torchsymbol(*_tfn("linalg.multi_dot"), id="torch.linalg.multi_dot")
def multi_dot(tensors, *, out=None):
    check(len(tensors) >= 2, "multi_dot needs at least two tensors")
    y = tensors[0]
    for t in tensors[1:]:
        y = matmul(y, t)
    return y


@_export
@torchsymbol(torch.ops.aten.embedding_backward.default if hasattr(torch.ops.aten, "embedding_backward") else None,
             id="torch.ops.aten.embedding_backward")
def embedding_backward(grad, indices, num_weights, padding_idx, scale_grad_by_freq, sparse):
    return prims.embedding_backward(grad, indices, num_weights, padding_idx, scale_grad_by_freq, sparse)


# =========================================================================================
# Convolution (prim + explicit backward prim)
# =========================================================================================
def _convolution_backward_meta(grad, a, weight, bias_sizes, stride, padding, dilation, transposed, output_padding,
                               groups, output_mask):
    gi = TensorProxy(like=a) if output_mask[0] else None
    gw = TensorProxy(like=weight) if output_mask[1] else None
    gb = TensorProxy(like=weight, shape=(weight.shape[1 if transposed else 0] * (groups if transposed else 1),)) \
        if output_mask[2] else None
    return gi, gw, gb


convolution_backward = prims.make_prim("lta.convolution_backward", "convolution_backward",
                                       meta=_convolution_backward_meta)


def _register_conv_impls():
    from ..executors import torchex
    from ..core.transforms import register_vjp

    def impl(grad, a, weight, bias_sizes, stride, padding, dilation, transposed, output_padding, groups, output_mask):
        return tuple(torch.ops.aten.convolution_backward(grad, a, weight, bias_sizes, list(stride), list(padding),
                                                         list(dilation), transposed, list(output_padding), groups,
                                                         list(output_mask)))

    op = torchex.ex.register_operator("convolution_backward", like=convolution_backward, fn=impl)
    torchex.ex.register_implementation(convolution_backward, op)

    @register_vjp(prims.PrimIDs.CONVOLUTION)
    def _conv_vjp(a, weight, bias, stride, padding, dilation, transposed, output_padding, groups):
        out = prims.convolution(a, weight, bias, stride, padding, dilation, transposed, output_padding, groups)

        def bwd(g):
            mask = (a.requires_grad, weight.requires_grad, bias is not None and bias.requires_grad)
            bias_sizes = None if bias is None else list(bias.shape)
            gi, gw, gb = convolution_backward(g, a, weight, bias_sizes, tuple(stride), tuple(padding), tuple(dilation),
                                              transposed, tuple(output_padding), groups, mask)
            return gi, gw, gb

        return out, bwd


_register_conv_impls()


@_export
@torchsymbol(*_tfn("convolution"), id="torch.convolution")
def convolution(a, weight, bias, stride, padding, dilation, transposed, output_padding, groups):
    return prims.convolution(a, weight, bias, tuple(pyval(s) for s in stride), tuple(pyval(p) for p in padding),
                             tuple(pyval(d) for d in dilation), bool(transposed),
                             tuple(pyval(p) for p in output_padding), pyval(groups))


def _conv_nd(n, a, weight, bias, stride, padding, dilation, groups):
    stride, dilation = _tuple(stride, n), _tuple(dilation, n)
    k = tuple(weight.shape[2:])
    if isinstance(padding, str):
        if padding == "valid":
            padding = (0,) * n
        else:
            check(padding == "same", f"conv{n}d: unknown padding {padding!r}")
            check(builtins.all(s == 1 for s in stride), "conv: padding='same' needs stride 1")
            tot = [dilation[i] * (k[i] - 1) for i in range(n)]
            lo = [t // 2 for t in tot]
            hi = [t - l for t, l in zip(tot, lo)]
            if lo != hi:  # asymmetric: pad explicitly (torch pads the extra element on the right)
                p = []
                for i in reversed(range(n)):
                    p += [lo[i], hi[i]]
                a = pad(a, tuple(p))
                padding = (0,) * n
            else:
                padding = tuple(lo)
    padding = _tuple(padding, n)
    return convolution(a, weight, bias, stride, padding, dilation, False, (0,) * n, pyval(groups))


@_export
@torchsymbol(*_tfn("conv1d", "nn.functional.conv1d"), id="torch.nn.functional.conv1d")
def conv1d(a, weight, bias=None, stride=1, padding=0, dilation=1, groups: int = 1):
    return _conv_nd(1, a, weight, bias, stride, padding, dilation, groups)


@_export
@torchsymbol(*_tfn("conv2d", "nn.functional.conv2d"), id="torch.nn.functional.conv2d")
def conv2d(a, weight, bias=None, stride=1, padding=0, dilation=1, groups: int = 1):
    return _conv_nd(2, a, weight, bias, stride, padding, dilation, groups)


@_export
@torchsymbol(*_tfn("conv3d", "nn.functional.conv3d"), id="torch.nn.functional.conv3d")
def conv3d(a, weight, bias=None, stride=1, padding=0, dilation=1, groups: int = 1):
    return _conv_nd(3, a, weight, bias, stride, padding, dilation, groups)


# =========================================================================================
# Pooling
# =========================================================================================
def _pool_out(n_in, k, s, p, d, ceil_mode):
    eff = d * (k - 1) + 1
    num = n_in + 2 * p - eff
    o = (num + (s - 1 if ceil_mode else 0)) // s + 1
    if ceil_mode and (o - 1) * s >= n_in + p:  # the last window must start inside the input (+ left pad)
        o -= 1
    return o


def _window_slices(x, n, k, s, p, d, outs, fill):
    """Padded input and the list of strided slices, one per kernel offset (spatial dims = last n)."""
    lead = x.ndim - n
    # pad: left p, right enough to cover the last window
    cfg = []
    for i in reversed(range(n)):
        size = x.shape[lead + i]
        need = (outs[i] - 1) * s[i] + d[i] * (k[i] - 1) + 1
        right = builtins.max(need - size - p[i], 0)
        cfg += [p[i], right]
    xp = pad(x, tuple(cfg), value=fill) if builtins.any(cfg) else x
    import itertools

    slices = []
    for offs in itertools.product(*[range(k[i]) for i in range(n)]):
        y = xp
        for i, o in enumerate(offs):
            st = o * d[i]
            y = clang.slice_in_dim(y, st, st + (outs[i] - 1) * s[i] + 1, s[i], lead + i)
        slices.append(y)
    return slices


def _max_pool(n, a, kernel_size, stride, padding, dilation, ceil_mode, return_indices, torch_fn):
    if return_indices:
        return _opaque(torch_fn)(a, kernel_size, stride, padding, dilation, ceil_mode=ceil_mode,
                                 return_indices=return_indices)
    k = _tuple(kernel_size, n)
    s = _tuple(stride if stride not in (None, ()) and stride != [] else k, n)
    p, d = _tuple(padding, n), _tuple(dilation, n)
    lead = a.ndim - n
    outs = [_pool_out(a.shape[lead + i], k[i], s[i], p[i], d[i], ceil_mode) for i in range(n)]
    fill = -math.inf if dtypes.is_float_dtype(a.dtype) else (torch.iinfo(a.dtype).min if a.dtype != torch.bool else False)
    sl = _window_slices(a, n, k, s, p, d, outs, fill)
    y = sl[0]
    for t in sl[1:]:
        y = maximum(y, t)
    return y


@_export
@torchsymbol(*_tfn("max_pool1d", "nn.functional.max_pool1d"), id="torch.nn.functional.max_pool1d")
def max_pool1d(a, kernel_size, stride=None, padding=0, dilation=1, ceil_mode=False, return_indices=False):
    return _max_pool(1, a, kernel_size, stride, padding, dilation, ceil_mode, return_indices,
                     torch.nn.functional.max_pool1d)


@_export
@torchsymbol(*_tfn("max_pool2d", "nn.functional.max_pool2d"), id="torch.nn.functional.max_pool2d")
def max_pool2d(a, kernel_size, stride=None, padding=0, dilation=1, ceil_mode=False, return_indices=False):
    return _max_pool(2, a, kernel_size, stride, padding, dilation, ceil_mode, return_indices,
                     torch.nn.functional.max_pool2d)


@_export
@torchsymbol(*_tfn("max_pool3d", "nn.functional.max_pool3d"), id="torch.nn.functional.max_pool3d")
def max_pool3d(a, kernel_size, stride=None, padding=0, dilation=1, ceil_mode=False, return_indices=False):
    return _max_pool(3, a, kernel_size, stride, padding, dilation, ceil_mode, return_indices,
                     torch.nn.functional.max_pool3d)


def _avg_pool(n, a, kernel_size, stride, padding, ceil_mode, count_include_pad, divisor_override, torch_fn):
    k = _tuple(kernel_size, n)
    s = _tuple(stride if stride not in (None, ()) and stride != [] else k, n)
    p = _tuple(padding, n)
    if ceil_mode:  # windows hanging over the right edge are divided by their clipped size: ATen
        kw = {} if n == 1 else {"divisor_override": divisor_override}
        return _opaque(torch_fn)(a, kernel_size, stride, padding, ceil_mode, count_include_pad, **kw)
    d = (1,) * n
    lead = a.ndim - n
    outs = [_pool_out(a.shape[lead + i], k[i], s[i], p[i], 1, False) for i in range(n)]
    compute = clang.compute_dtype(a.dtype)
    x = clang.maybe_convert_to_dtype(a, compute)
    sl = _window_slices(x, n, k, s, p, d, outs, 0.0)
    tot = sl[0]
    for t in sl[1:]:
        tot = add(tot, t)
    if divisor_override:
        y = true_divide(tot, float(divisor_override))
    elif count_include_pad or not builtins.any(p):
        y = true_divide(tot, float(math.prod(k)))
    else:
        ones = full_like(x, 1.0)
        cnt = _window_slices(ones, n, k, s, p, d, outs, 0.0)
        c = cnt[0]
        for t in cnt[1:]:
            c = add(c, t)
        y = true_divide(tot, c)
    return clang.maybe_convert_to_dtype(y, a.dtype)


@_export
@torchsymbol(*_tfn("avg_pool1d", "nn.functional.avg_pool1d"), id="torch.nn.functional.avg_pool1d")
def avg_pool1d(a, kernel_size, stride=None, padding=0, ceil_mode=False, count_include_pad=True):
    return _avg_pool(1, a, kernel_size, stride, padding, ceil_mode, count_include_pad, None,
                     torch.nn.functional.avg_pool1d)


@_export
@torchsymbol(*_tfn("nn.functional.avg_pool2d"), id="torch.nn.functional.avg_pool2d")
def avg_pool2d(a, kernel_size, stride=None, padding=0, ceil_mode=False, count_include_pad=True, divisor_override=None):
    return _avg_pool(2, a, kernel_size, stride, padding, ceil_mode, count_include_pad, divisor_override,
                     torch.nn.functional.avg_pool2d)


@_export
@torchsymbol(*_tfn("nn.functional.avg_pool3d"), id="torch.nn.functional.avg_pool3d")
def avg_pool3d(a, kernel_size, stride=None, padding=0, ceil_mode=False, count_include_pad=True, divisor_override=None):
    return _avg_pool(3, a, kernel_size, stride, padding, ceil_mode, count_include_pad, divisor_override,
                     torch.nn.functional.avg_pool3d)


@_export
@torchsymbol(*_tfn("nn.functional.adaptive_avg_pool2d"), id="torch.nn.functional.adaptive_avg_pool2d")
def adaptive_avg_pool2d(a, output_size):
    osz = _tuple(output_size, 2)
    h, w = a.shape[-2], a.shape[-1]
    osz = tuple(h if o is None else o for o in osz[:1]) + tuple(w if o is None else o for o in osz[1:])
    if h % osz[0] == 0 and w % osz[1] == 0:
        kh, kw = h // osz[0], w // osz[1]
        return avg_pool2d(a, (kh, kw), (kh, kw))
    return _opaque(torch.nn.functional.adaptive_avg_pool2d)(a, osz)


# =========================================================================================
# Normalization
# =========================================================================================
def _bn_shape(a):
    return (1, a.shape[1]) + (1,) * (a.ndim - 2)


@_export
@torchsymbol(*_tfn("nn.functional.batch_norm"), id="torch.nn.functional.batch_norm")
def batch_norm(a, running_mean, running_var, weight=None, bias=None, training: bool = False, momentum: float = 0.1,
               eps: float = 1e-5):
    compute = clang.compute_dtype(a.dtype)
    x = clang.maybe_convert_to_dtype(a, compute)
    dims = (0,) + tuple(range(2, a.ndim))
    shape = _bn_shape(a)
    if training:
        var, m = var_mean(x, dims, correction=0)
        n = a.numel // a.shape[1]
        if running_mean is not None:
            nm = add(mul(running_mean, 1.0 - momentum), mul(clang.maybe_convert_to_dtype(m, running_mean.dtype), momentum))
            copy_(running_mean, nm)
        if running_var is not None:
            unbiased = mul(var, n / builtins.max(n - 1, 1))
            nv = add(mul(running_var, 1.0 - momentum),
                     mul(clang.maybe_convert_to_dtype(unbiased, running_var.dtype), momentum))
            copy_(running_var, nv)
        mean_, var_ = m, var
    else:
        check(running_mean is not None and running_var is not None, "batch_norm: eval needs running statistics")
        mean_ = clang.maybe_convert_to_dtype(running_mean, compute)
        var_ = clang.maybe_convert_to_dtype(running_var, compute)
    y = mul(sub(x, reshape(mean_, shape)), reshape(rsqrt(add(var_, eps)), shape))
    if weight is not None:
        y = mul(y, reshape(clang.maybe_convert_to_dtype(weight, compute), shape))
    if bias is not None:
        y = add(y, reshape(clang.maybe_convert_to_dtype(bias, compute), shape))
    return clang.maybe_convert_to_dtype(y, a.dtype)


@_export
@torchsymbol(*_tfn("nn.functional.instance_norm"), id="torch.nn.functional.instance_norm")
def instance_norm(a, running_mean=None, running_var=None, weight=None, bias=None, use_input_stats: bool = True,
                  momentum: float = 0.1, eps: float = 1e-5):
    check(use_input_stats or (running_mean is not None and running_var is not None),
          "instance_norm: use_input_stats=False needs running statistics")
    if not use_input_stats:
        return batch_norm(a, running_mean, running_var, weight, bias, False, momentum, eps)
    check(running_mean is None and running_var is None,
          "instance_norm: tracking running statistics is routed to ATen")
    compute = clang.compute_dtype(a.dtype)
    x = clang.maybe_convert_to_dtype(a, compute)
    dims = tuple(range(2, a.ndim))
    var, m = var_mean(x, dims, correction=0, keepdim=True)
    y = mul(sub(x, m), rsqrt(add(var, eps)))
    shape = _bn_shape(a)
    if weight is not None:
        y = mul(y, reshape(clang.maybe_convert_to_dtype(weight, compute), shape))
    if bias is not None:
        y = add(y, reshape(clang.maybe_convert_to_dtype(bias, compute), shape))
    return clang.maybe_convert_to_dtype(y, a.dtype)


@_export
@torchsymbol(*_tfn("nn.functional.local_response_norm"), id="torch.nn.functional.local_response_norm")
def local_response_norm(a, size: int, alpha: float = 1e-4, beta: float = 0.75, k: float = 1.0):
    check(a.ndim >= 3, "local_response_norm: expected 3-D or higher input")
    compute = clang.compute_dtype(a.dtype)
    x = clang.maybe_convert_to_dtype(a, compute)
    sq = square(x)
    C = a.shape[1]
    # zero-padded channel window [c - size//2, c + (size-1)//2], averaged over `size`
    lo, hi = size // 2, (size - 1) // 2
    cfg = [(0, 0, 0)] * a.ndim
    cfg[1] = (lo, hi, 0)
    sp = prims.pad(sq, 0.0, cfg)
    acc = clang.slice_in_dim(sp, 0, C, 1, 1)
    for j in range(1, size):
        acc = add(acc, clang.slice_in_dim(sp, j, j + C, 1, 1))
    div = pow(add(mul(acc, alpha / size), k), beta)
    return clang.maybe_convert_to_dtype(true_divide(x, div), a.dtype)


# =========================================================================================
# Interpolation (nearest, linear / bilinear / trilinear)
# =========================================================================================
def _src_index(out_n, in_n, scale, align_corners, mode, device):
    o = clang.maybe_convert_to_dtype(arange(0, out_n, device=device), dtypes.float32)
    if mode == "nearest":
        r = in_n / out_n if scale is None else 1.0 / scale
        i = clang.maybe_convert_to_dtype(clang.floor(mul(o, r)), dtypes.int64)
        return clamp(i, 0, in_n - 1), None, None
    if align_corners:
        r = (in_n - 1) / (out_n - 1) if out_n > 1 else 0.0
        src = mul(o, r)
    else:
        r = in_n / out_n if scale is None else 1.0 / scale
        src = clamp(sub(mul(add(o, 0.5), r), 0.5), 0.0, None)
    i0f = clang.floor(src)
    i0 = clamp(clang.maybe_convert_to_dtype(i0f, dtypes.int64), 0, in_n - 1)
    i1 = clamp(add(i0, 1), 0, in_n - 1)
    w1 = sub(src, i0f)
    return i0, i1, w1


@_export
@torchsymbol(*_tfn("nn.functional.interpolate"), id="torch.nn.functional.interpolate")
def interpolate(a, size=None, scale_factor=None, mode: str = "nearest", align_corners=None, recompute_scale_factor=None,
                antialias: bool = False):
    n = a.ndim - 2
    linear_modes = {"linear": 1, "bilinear": 2, "trilinear": 3}
    if antialias or (mode not in ("nearest",) and mode not in linear_modes) or (mode in linear_modes
                                                                                 and linear_modes[mode] != n):
        return _opaque(torch.nn.functional.interpolate)(a, size, scale_factor, mode, align_corners,
                                                        recompute_scale_factor, antialias)
    if size is not None:
        outs = _tuple(size, n)
        scales = (None,) * n
    else:
        sf = _tuple(scale_factor, n)
        outs = tuple(int(math.floor(a.shape[2 + i] * sf[i])) for i in range(n))
        scales = (None,) * n if recompute_scale_factor else sf
    compute = clang.compute_dtype(a.dtype)
    y = clang.maybe_convert_to_dtype(a, compute) if mode != "nearest" else a
    for i in range(n):
        d = 2 + i
        i0, i1, w1 = _src_index(outs[i], a.shape[d], scales[i], bool(align_corners), mode, a.device)
        if mode == "nearest":
            y = index_select(y, d, i0)
            continue
        y0 = index_select(y, d, i0)
        y1 = index_select(y, d, i1)
        wshape = [1] * y.ndim
        wshape[d] = outs[i]
        w = reshape(clang.maybe_convert_to_dtype(w1, compute), tuple(wshape))
        y = add(y0, mul(sub(y1, y0), w))
    return clang.maybe_convert_to_dtype(y, a.dtype)
