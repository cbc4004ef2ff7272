"""Hugging Face attention prologue -> fused projections + RoPE kernels (MI355X-native counterpart
of the reference HF recipe's trace rewrites, ``thunder/recipes/hf_transformers.py:26-345``).

HF Llama-family attention computes ``q/k/v = proj(x).view(B, T, -1, D).transpose(1, 2)`` with three
separate linears and applies ``rotate_half`` RoPE as ``x * cos + cat(-x2, x1) * sin`` (slices, neg,
cat, two muls, add: five to seven launches per tensor).  This pass rewrites, on the computation
trace, each layer's

    q, k, v (3 projections of one x) -> q_rot, k_rot (rotate-half RoPE with the same cos / sin)

into ``qkv = cat(linear(x, Wq), linear(x, Wk), linear(x, Wv), dim=-1)`` followed by the fused
split + RoPE kernel (``hip_qkv_rope``; [all q | all k | all v] per token is exactly its input
layout).  The executor passes then turn the concatenated decode projections into one grouped
weight-streaming GEMV writing the packed qkv row, and the static-cache ``index_copy`` writes into
the RoPE kernel's epilogue (``hip_qkv_rope_cache``).
"""
from __future__ import annotations

import torch

from ..core.proxies import TensorProxy
from ..core.trace import from_trace, tracectx, TraceProvenance
from ..core.transform_common import Transform, dce


def _name(x):
    return getattr(x, "name", None)


def _is_slice(s, start, stop):
    return isinstance(s, slice) and s.start == start and s.stop == stop and s.step is None


class _Matcher:
    def __init__(self, trace):
        self.producer = {}
        self.uses: dict[str, list[int]] = {}
        self.index = {}
        for i, b in enumerate(trace.bound_symbols):
            self.index[id(b)] = i
            for o in b.flat_proxy_outs:
                self.producer[o.name] = b
            for a in b.flat_proxy_args:
                self.uses.setdefault(a.name, []).append(i)

    def prod(self, x, *names):
        b = self.producer.get(_name(x))
        return b if b is not None and b.sym.name in names else None

    def head_proj(self, x):
        """``transpose(view(linear(h, W, None), (B, T, -1, D)), 1, 2)`` -> (h, W, linear output)."""
        tb = self.prod(x, "transpose")
        if tb is None or tuple(tb.args[1:3]) not in ((1, 2), (2, 1)):
            return None
        vb = self.prod(tb.args[0], "view", "reshape")
        if vb is None:
            return None
        lb = self.prod(vb.args[0], "linear")
        if lb is None:
            return None
        bias = lb.args[2] if len(lb.args) > 2 else lb.kwargs.get("bias")
        if bias is not None:
            return None
        return lb.args[0], lb.args[1], lb.output

    def rope(self, add_b):
        """``add(mul(X, C), mul(cat((neg(X[..., h:]), X[..., :h]), -1), S))`` -> (X, C, S)."""
        if add_b.sym.name != "add" or len(add_b.args) < 2 or add_b.kwargs.get("alpha") not in (None, 1):
            return None
        for m1, m2 in (add_b.args[:2], add_b.args[1::-1]):
            mb1, mb2 = self.prod(m1, "mul"), self.prod(m2, "mul")
            if mb1 is None or mb2 is None:
                continue
            for X, C in (mb1.args[:2], mb1.args[1::-1]):
                for R, S in (mb2.args[:2], mb2.args[1::-1]):
                    cb = self.prod(R, "cat")
                    if not isinstance(X, TensorProxy) or cb is None:
                        continue
                    parts = cb.args[0] if cb.args else None
                    dim = cb.args[1] if len(cb.args) > 1 else cb.kwargs.get("dim", 0)
                    if not isinstance(parts, (list, tuple)) or len(parts) != 2 or dim not in (-1, X.ndim - 1):
                        continue
                    nb = self.prod(parts[0], "neg")
                    g1 = self.prod(parts[1], "_getitem_sym", "getitem")
                    g2 = self.prod(nb.args[0], "_getitem_sym", "getitem") if nb is not None else None
                    if g1 is None or g2 is None or _name(g1.args[0]) != X.name or _name(g2.args[0]) != X.name:
                        continue
                    h = X.shape[-1] // 2
                    i1, i2 = g1.args[1], g2.args[1]
                    ok1 = isinstance(i1, tuple) and len(i1) == 2 and i1[0] is Ellipsis and _is_slice(i1[1], None, h)
                    ok2 = isinstance(i2, tuple) and len(i2) == 2 and i2[0] is Ellipsis and _is_slice(i2[1], h, None)
                    if ok1 and ok2:
                        return X, C, S
        return None


class HFRoPETransform(Transform):
    def __init__(self, require_gpu: bool = True):
        self.require_gpu = require_gpu  # False: rewrite CPU traces too (trace-structure tests)

    def transform_traces_pre_prologue(self, prologue_trace, computation_trace, epilogue_trace, **kwargs):
        trc = computation_trace
        m = _Matcher(trc)
        ropes = []
        for b in trc.bound_symbols:
            r = m.rope(b)
            if r is None:
                continue
            X, C, S = r
            if (self.require_gpu and X.device.type != "cuda") or X.ndim != 4:
                continue
            if self.require_gpu and X.dtype not in (torch.bfloat16, torch.float16):
                continue
            ropes.append((b, X, C, S))
        # pair q / k ropes sharing (projection input, cos, sin); v = the third projection of that input
        plans = []
        used = set()
        for i, (bq, Xq, Cq, Sq) in enumerate(ropes):
            if i in used:
                continue
            pq = m.head_proj(Xq)
            if pq is None:
                continue
            for j in range(i + 1, len(ropes)):
                bk, Xk, Ck, Sk = ropes[j]
                if j in used or _name(Ck) != _name(Cq) or _name(Sk) != _name(Sq):
                    continue
                pk = m.head_proj(Xk)
                if pk is None or _name(pk[0]) != _name(pq[0]):
                    continue
                # v: another head projection of the same input consumed by neither rope
                v = None
                for cand in trc.bound_symbols:
                    if cand.sym.name == "transpose":
                        out = cand.output
                        pv = m.head_proj(out)
                        if pv is not None and _name(pv[0]) == _name(pq[0]) and out.name not in (Xq.name, Xk.name):
                            v = (out, pv)
                            break
                if v is None:
                    continue
                plans.append((bq, bk, Xq, Xk, Cq, Sq, pq, pk, v))
                used.update((i, j))
                break
        plans = [p for p in plans if self._valid(p)]
        if not plans:
            return prologue_trace, computation_trace, epilogue_trace
        from .. import torch as ltorch
        from ..executors.hipex import hip_qkv_rope

        emit_at = {}
        for p in plans:
            bq, bk = p[0], p[1]
            later = bq if m.index[id(bq)] > m.index[id(bk)] else bk
            emit_at[id(later)] = p
        new = from_trace(trc)
        new.bound_symbols = []
        new.scopes = [new.bound_symbols]
        swap = {}
        with tracectx(new):
            for b in trc.bound_symbols:
                nb = b.swap_proxies(swap, skip_output=True) if swap else b
                new.bound_symbols.append(nb)
                p = emit_at.get(id(b))
                if p is None:
                    continue
                bq, bk, Xq, Xk, C, S, pq, pk, (vt, pv) = p
                T, D = Xq.shape[2], Xq.shape[3]
                qkv = ltorch.cat((pq[2], pk[2], pv[2]), -1)
                c2 = ltorch.reshape(self._base(C, m), (T, D))
                s2 = ltorch.reshape(self._base(S, m), (T, D))
                qn, kn, vn = hip_qkv_rope(qkv, c2, s2, Xq.shape[1], Xk.shape[1], D, D)
                swap[bq.output.name] = qn
                swap[bk.output.name] = kn
                swap[vt.name] = vn
        new = dce(new)
        new.set_provenance(TraceProvenance(f"HF attention prologue -> fused qkv RoPE ({len(plans)} layer(s))"))
        return prologue_trace, new, epilogue_trace

    @staticmethod
    def _base(c, m):
        ub = m.prod(c, "unsqueeze")
        return ub.args[0] if ub is not None else c

    def _valid(self, p):
        bq, bk, Xq, Xk, C, S, pq, pk, (vt, pv) = p
        B, nh, T, D = Xq.shape
        if B != 1 or D % 16 or Xk.shape[0] != 1 or Xk.shape[2:] != (T, D) or tuple(vt.shape) != tuple(Xk.shape):
            return False
        if nh % Xk.shape[1]:
            return False
        for c in (C, S):
            if tuple(c.shape[-2:]) != (T, D) or c.numel() != T * D or c.dtype not in (torch.float32, Xq.dtype):
                return False
        return True
