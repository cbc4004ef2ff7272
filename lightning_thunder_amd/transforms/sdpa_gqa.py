"""SDPA on grouped KV heads without materialising ``repeat_kv`` (MI355X-native counterpart of the
reference HF recipe's attention rewrites, ``thunder/recipes/hf_transformers.py:99-345``).

Hugging Face attention expands a [B, Hkv, S, D] KV cache to [B, Hq, S, D] before SDPA
(``repeat_kv``: ``x[:, :, None, :, :].expand(B, Hkv, n_rep, S, D).reshape(B, Hkv*n_rep, S, D)``);
the reshape of the expanded view copies the whole cache, twice per layer per token, and the
attention then reads n_rep times the bytes.  The HIP attention kernels handle grouped heads
natively, so SDPA is given the cache itself with ``enable_gqa=True`` and dead-code elimination
drops the expansion.
"""
from __future__ import annotations

from ..core.proxies import TensorProxy
from ..core.trace import from_trace, TraceProvenance
from ..core.transform_common import Transform, dce


def _is_none_slice(s) -> bool:
    return isinstance(s, slice) and s.start is None and s.stop is None and s.step is None


def _repeat_kv_source(p, producer):
    """``x`` if ``p = reshape(expand(x[:, :, None, :, :], (B, Hkv, r, S, D)), (B, Hkv*r, S, D))``."""
    rb = producer.get(p.name)
    if rb is None or rb.sym.name != "reshape":
        return None
    e = rb.args[0]
    eb = producer.get(getattr(e, "name", None))
    if eb is None or eb.sym.name != "expand":
        return None
    g = eb.args[0]
    gb = producer.get(getattr(g, "name", None))
    if gb is None or gb.sym.name not in ("_getitem_sym", "getitem"):
        return None
    x, idx = gb.args[0], gb.args[1] if len(gb.args) > 1 else None
    if not isinstance(x, TensorProxy) or x.ndim != 4 or not isinstance(idx, tuple) or len(idx) != 5:
        return None
    if not (idx[2] is None and all(_is_none_slice(s) for i, s in enumerate(idx) if i != 2)):
        return None
    B, Hkv, S, D = x.shape
    if tuple(e.shape) != (B, Hkv, e.shape[2], S, D) or tuple(p.shape) != (B, Hkv * e.shape[2], S, D):
        return None
    return x


class SDPAGQATransform(Transform):
    def transform_traces_pre_prologue(self, prologue_trace, computation_trace, epilogue_trace, **kwargs):
        producer = {}
        for b in computation_trace.bound_symbols:
            for o in b.flat_proxy_outs:
                producer[o.name] = b
        new_bsyms = []
        n = 0
        for b in computation_trace.bound_symbols:
            if b.sym.name == "scaled_dot_product_attention" and len(b.args) >= 3:
                q, k, v = b.args[:3]
                xk, xv = _repeat_kv_source(k, producer), _repeat_kv_source(v, producer)
                if xk is not None and xv is not None and q.shape[1] % xk.shape[1] == 0:
                    kw = dict(b.kwargs)
                    kw["enable_gqa"] = True
                    b = b.from_bsym(args=(q, xk, xv) + tuple(b.args[3:]), kwargs=kw)
                    n += 1
            new_bsyms.append(b)
        if not n:
            return prologue_trace, computation_trace, epilogue_trace
        new = from_trace(computation_trace)
        new.bound_symbols = new_bsyms
        new.scopes = [new.bound_symbols]
        new = dce(new)
        new.set_provenance(TraceProvenance(f"SDPA on grouped KV heads ({n} repeat_kv expansion(s) removed)"))
        return prologue_trace, new, epilogue_trace
