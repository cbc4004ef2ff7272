"""Optimizers backed by fused CDNA4 kernels (K15).

``AdamW`` updates every parameter of a group with ONE multi-tensor HIP launch
(``ops/csrc/adamw.hip``), streaming params/grads/moments once at HBM speed.  Semantics
match ``torch.optim.AdamW`` (decoupled weight decay, bias correction); moments are kept
in the parameter dtype by default (like torch's fused AdamW) or in fp32 with
``state_dtype=torch.float32``.  Falls back to torch's implementation for CPU tensors.

``overlap_with_backward(jitted_model)`` moves the update into the compiled backward: each bucket
of parameters is updated on a side stream as soon as its gradients are final and the backward no
longer reads the parameters (``transforms/optimizer_overlap.py``); ``step()`` then joins that
stream and updates only what the backward did not.
"""
from __future__ import annotations

import math
import struct

import torch


class AdamW(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2, state_dtype=None):
        defaults = dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay)
        super().__init__(params, defaults)
        self.state_dtype = state_dtype
        self._chunk_cache: dict = {}
        self._managed: dict = {}  # id(param) -> param group (overlap mode)
        self._side: dict = {}  # device -> side stream of the overlapped updates
        self._inflight: list = []  # metadata tensors read by queued side-stream launches
        self._handled: set = set()  # id(param) updated inside a backward since the last step()

    # --- update overlapped with the backward (transforms/optimizer_overlap.py) ----------------------
    def overlap_with_backward(self, jitted, bucket_mb: int = 128) -> None:
        """Update parameters inside ``jitted``'s compiled backward (call before its first forward).
        Every backward must then be followed by ``step()`` (no gradient accumulation / clipping)."""
        from .transforms.optimizer_overlap import overlap_with_backward

        self._managed = {id(p): g for g in self.param_groups for p in g["params"]}
        overlap_with_backward(jitted, self, bucket_mb)

    def manages(self, t) -> bool:
        return isinstance(t, torch.Tensor) and t.is_cuda and id(t) in self._managed

    def _mark_handled(self, params) -> None:
        """Records that ``params`` were updated inside a backward of this iteration; a second update
        before ``step()`` is an error.  It would come from a second backward node (the jitted function
        called twice before one backward, or a weight shared between jitted calls), each holding only
        a partial gradient, and would apply a second AdamW step."""
        for p in params:
            if id(p) in self._handled:
                raise RuntimeError("overlapped optimizer: parameter of shape "
                                   f"{tuple(p.shape)} updated twice in one iteration; call step() after every "
                                   "backward, or do not use overlap_with_backward for this model")
        self._handled.update(id(p) for p in params)

    @torch.no_grad()
    def overlapped_update(self, params, grads) -> None:
        """Called from the backward: update ``params`` with ``grads`` on the side stream, ordered
        after everything the compute stream has queued so far."""
        self._mark_handled(params)
        dev = params[0].device
        side = self._side.get(dev)
        if side is None:
            # high priority: a stream of its own priority class gets its own hardware queue (a
            # normal-priority side stream can share the compute stream's queue and never overlap)
            side = self._side[dev] = torch.cuda.Stream(device=dev, priority=-1)
        side.wait_stream(torch.cuda.current_stream(dev))
        buckets: dict = {}
        with torch.cuda.stream(side):
            for p, g in zip(params, grads):
                group = self._managed[id(p)]
                st = self._state(p)
                st["step"] += 1
                key = (id(group), p.dtype, st["exp_avg"].dtype, st["step"])
                buckets.setdefault(key, (group, []))[1].append((p, g))
            for (_, pdt, sdt, step), (group, pg) in buckets.items():
                lr, (b1, b2), eps, wd = group["lr"], group["betas"], group["eps"], group["weight_decay"]
                self._fused([p for p, _ in pg], pdt, sdt, dev, step, lr, b1, b2, eps, wd,
                            grads=[g for _, g in pg], lean=True)
        for g in grads:
            g.record_stream(side)  # the compute stream may free the gradient before the update ran

    def _join(self):
        for dev, side in self._side.items():
            torch.cuda.current_stream(dev).wait_stream(side)
        self._inflight.clear()

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
        self._join()
        handled = self._handled
        # validate every parameter before any state changes, so a failed step() leaves the
        # optimizer exactly as it was (no partial step counts, no second update on a retry)
        for group in self.param_groups:
            for p in group["params"]:
                if p.grad is not None and id(p) in handled:
                    # p was already updated inside the backward; a gradient accumulated into p.grad by
                    # another autograd path would otherwise get a second step this iteration
                    raise RuntimeError(f"overlapped optimizer: parameter of shape {tuple(p.shape)} was updated "
                                       "in the backward and also has p.grad set")
        self._handled = set()
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

    def _fused(self, ps, pdt, sdt, dev, step, lr, b1, b2, eps, wd, grads=None, lean=False):
        from .ops._lib import require, DTYPE_CODE, stream_ptr, check, register_signature, c_int, c_void_p, c_float

        lib = require()
        register_signature("lta_adamw_ex2", [c_int, c_int, c_void_p, c_void_p, c_int, c_float, c_float, c_float,
                                             c_float, c_float, c_float, c_float, c_float, c_int, c_int, c_void_p])
        from .ops import fp8 as _fp8

        metas = []
        keep = []
        shadow = False
        zero: dict = {}
        for i, p in enumerate(ps):
            st = self.state[p]
            g = p.grad if grads is None else grads[i]
            g = g if g.is_contiguous() else g.contiguous()
            if g.dtype != p.dtype:
                g = g.to(p.dtype)
            keep.append(g)
            metas += [p.data_ptr(), g.data_ptr(), st["exp_avg"].data_ptr(), st["exp_avg_sq"].data_ptr(), p.numel()]
            # fp8 weight shadow (ops/fp8.py): refreshed by this launch; not beside a running backward,
            # which may still read the old e4m3 copy (the overlapped update drops it instead)
            sh = _fp8.weight_shadow(p) if _fp8._SHADOWS else None
            if sh is not None and lean:
                _fp8.invalidate_weight_shadow(p)
                sh = None
            if sh is not None:
                q, src, scale, dst, slot, fmax = sh
                shadow = True
                zero.setdefault(id(dst), (dst, []))[1].append(slot)
                metas += [q.data_ptr(), src.data_ptr(), scale.data_ptr(), dst.shadow_amax[slot].data_ptr(),
                          int.from_bytes(struct.pack("<f", fmax), "little")]
            else:
                metas += [0, 0, 0, 0, 0]
        for dst, slots in zero.values():  # the kernel max-folds each refreshed weight's max |w| into these
            dst.shadow_amax.index_fill_(0, torch.tensor(slots, dtype=torch.int64).to(dev, non_blocking=True), 0.0)
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
        rc = lib.lta_adamw_ex2(DTYPE_CODE[pdt], DTYPE_CODE[sdt], meta_t.data_ptr(), chunks.data_ptr(), chunks.shape[0],
                               lr, b1, b2, eps, wd, bc1, bc2_sqrt, 1.0, int(lean), int(shadow), stream_ptr(dev))
        check(rc, "lta_adamw")
        # keep the metadata (and converted gradients) alive until the kernel has consumed them
        self._last_meta = meta_t
        if lean:
            self._inflight.append((meta_t, keep))
