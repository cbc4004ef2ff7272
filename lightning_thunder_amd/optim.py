"""Optimizers backed by fused CDNA4 kernels (K15).

``AdamW`` updates every parameter of a group with ONE multi-tensor HIP launch
(``ops/csrc/adamw.hip``), streaming params/grads/moments once at HBM speed.  Semantics
match ``torch.optim.AdamW`` (decoupled weight decay, bias correction); moments are kept
in the parameter dtype by default (like torch's fused AdamW) or in fp32 with
``state_dtype=torch.float32``.  Falls back to torch's implementation for CPU tensors.
"""
from __future__ import annotations

import math

import torch


class AdamW(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2, state_dtype=None):
        defaults = dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay)
        super().__init__(params, defaults)
        self.state_dtype = state_dtype
        self._chunk_cache: dict = {}

    def _state(self, p):
        st = self.state[p]
        if not st:
            dt = self.state_dtype or p.dtype
            st["step"] = 0
            st["exp_avg"] = torch.zeros_like(p, dtype=dt, memory_format=torch.contiguous_format)
            st["exp_avg_sq"] = torch.zeros_like(p, dtype=dt, memory_format=torch.contiguous_format)
        return st

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for group in self.param_groups:
            lr, (b1, b2), eps, wd = group["lr"], group["betas"], group["eps"], group["weight_decay"]
            buckets: dict = {}
            for p in group["params"]:
                if p.grad is None:
                    continue
                st = self._state(p)
                st["step"] += 1
                if p.device.type != "cuda":
                    self._torch_step(p, st, lr, b1, b2, eps, wd)
                    continue
                key = (p.dtype, st["exp_avg"].dtype, p.device, st["step"])
                buckets.setdefault(key, []).append(p)
            for (pdt, sdt, dev, step), ps in buckets.items():
                self._fused(ps, pdt, sdt, dev, step, lr, b1, b2, eps, wd)
        return loss

    def _torch_step(self, p, st, lr, b1, b2, eps, wd):
        g = p.grad
        p.mul_(1 - lr * wd)
        st["exp_avg"].lerp_(g.to(st["exp_avg"].dtype), 1 - b1)
        st["exp_avg_sq"].mul_(b2).addcmul_(g, g, value=1 - b2)
        bc1 = 1 - b1 ** st["step"]
        bc2 = 1 - b2 ** st["step"]
        denom = (st["exp_avg_sq"].sqrt() / math.sqrt(bc2)).add_(eps)
        p.addcdiv_(st["exp_avg"].to(p.dtype), denom.to(p.dtype), value=-lr / bc1)

    def _fused(self, ps, pdt, sdt, dev, step, lr, b1, b2, eps, wd):
        from .ops._lib import require, DTYPE_CODE, stream_ptr, check, register_signature, c_int, c_void_p, c_float

        lib = require()
        register_signature("lta_adamw", [c_int, c_int, c_void_p, c_void_p, c_int, c_float, c_float, c_float, c_float,
                                         c_float, c_float, c_float, c_float, c_void_p])
        metas = []
        for p in ps:
            st = self.state[p]
            g = p.grad if p.grad.is_contiguous() else p.grad.contiguous()
            if g.dtype != p.dtype:
                g = g.to(p.dtype)
            metas += [p.data_ptr(), g.data_ptr(), st["exp_avg"].data_ptr(), st["exp_avg_sq"].data_ptr(), p.numel()]
        meta_t = torch.tensor(metas, dtype=torch.int64).pin_memory().to(dev, non_blocking=True)
        key = (dev, tuple(p.numel() for p in ps))
        chunks = self._chunk_cache.get(key)
        if chunks is None:
            C = lib.lta_adamw_chunk_size()
            rows = []
            for i, p in enumerate(ps):
                n = (p.numel() + C - 1) // C
                t = torch.empty((n, 2), dtype=torch.int32)
                t[:, 0] = i
                t[:, 1] = torch.arange(n, dtype=torch.int32)
                rows.append(t)
            chunks = torch.cat(rows).to(dev)
            self._chunk_cache[key] = chunks
        bc1 = 1 - b1 ** step
        bc2_sqrt = math.sqrt(1 - b2 ** step)
        rc = lib.lta_adamw(DTYPE_CODE[pdt], DTYPE_CODE[sdt], meta_t.data_ptr(), chunks.data_ptr(), chunks.shape[0], lr, b1,
                           b2, eps, wd, bc1, bc2_sqrt, 1.0, stream_ptr(dev))
        check(rc, "lta_adamw")
        # keep the metadata alive until the kernel has consumed it
        self._last_meta = meta_t
