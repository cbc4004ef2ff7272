"""MaterializationTransform: allocate and initialise meta-device parameters after sharding.

Reference parity: ``thunder/transforms/materialization.py`` (init from the original module's
``reset_parameters``, from the original state dict, or from the transformed state dict).

With 288 GB of HBM per MI355X a 7B model fits unsharded, but 70B-class models do not: build
the model under ``torch.device("meta")``, apply FSDP/TP (which shard the *meta* tensors, costing
nothing) and let this transform allocate only the local shards on the GPU.  Initialisation
from module code materialises one submodule at a time at full size, runs its
``reset_parameters()`` and keeps the local shard, so every rank produces exactly the values an
unsharded init would (given the same RNG seed).
"""
from __future__ import annotations

import torch

from ..core.transform_common import Transform


class MaterializationTransform(Transform):
    def __init__(self, sharding_transform=None, device=None, init=None):
        self.sharding_transform = sharding_transform
        self.device = torch.device(device) if device is not None else None
        self.init = init if init is not None else MaterializationTransform.init_from_original_module_init()

    # --- init strategies -----------------------------------------------------------------------
    @staticmethod
    def init_from_original_state_dict(state_dict):
        def _init(transform, tm):
            tm.load_original_state_dict(state_dict)

        return _init

    @staticmethod
    def init_from_transformed_state_dict(state_dict):
        def _init(transform, tm):
            tm.load_state_dict(state_dict)

        return _init

    @staticmethod
    def init_from_original_module_init():
        def _init(transform, tm):
            transform._init_from_module(tm)

        return _init

    # --- transform hooks -------------------------------------------------------------------------
    def transform_module(self, tm) -> None:
        inner = tm._model
        has_meta = any(t.is_meta for t in list(inner.parameters()) + list(inner.buffers()))
        if not has_meta:
            return
        device = self.device
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu")
        self._device = device
        self._meta_names = set()
        for mname, m in inner.named_modules():
            for pname, p in list(m._parameters.items()):
                if p is not None and p.is_meta:
                    newp = torch.nn.Parameter(torch.empty(p.shape, dtype=p.dtype, device=device),
                                              requires_grad=p.requires_grad)
                    for attr in ("_lc_full_shape", "_lc_tp_kind", "distparallel_type", "thunder_fsdp_padding_size"):
                        if hasattr(p, attr):
                            setattr(newp, attr, getattr(p, attr))
                    m._parameters[pname] = newp
                    self._meta_names.add(f"{mname}.{pname}" if mname else pname)
            for bname, b in list(m._buffers.items()):
                if b is not None and b.is_meta:
                    m._buffers[bname] = torch.empty(b.shape, dtype=b.dtype, device=device)
                    self._meta_names.add(f"{mname}.{bname}" if mname else bname)
        self.init(self, tm)

    def _init_from_module(self, tm):
        """Run each submodule's ``reset_parameters`` on full-size tensors and keep the local shard."""
        inner = tm._model
        transforms = tm._transforms() if hasattr(tm, "_transforms") else []
        for mname, m in inner.named_modules():
            if not hasattr(m, "reset_parameters"):
                continue
            local = {n: t for n, t in list(m._parameters.items()) + list(m._buffers.items()) if t is not None}
            names = {n for n in local if (f"{mname}.{n}" if mname else n) in self._meta_names}
            if not names:
                continue
            # full-size stand-ins for the (possibly sharded) tensors
            full = {}
            for n in names:
                t = local[n]
                shape = getattr(t, "_lc_full_shape", None) or tuple(t.shape)
                full[n] = torch.empty(shape, dtype=t.dtype, device=self._device)
            saved = {}
            for n, t in full.items():
                if n in m._parameters:
                    saved[n] = m._parameters[n]
                    m._parameters[n] = torch.nn.Parameter(t, requires_grad=False)
                else:
                    saved[n] = m._buffers[n]
                    m._buffers[n] = t
            with torch.no_grad():
                m.reset_parameters()
            sd = {n: (m._parameters[n] if n in m._parameters else m._buffers[n]).detach() for n in full}
            for n, t in saved.items():
                if n in m._parameters:
                    m._parameters[n] = t
                else:
                    m._buffers[n] = t
            for t in transforms:
                if t is self:
                    continue
                sd = t.transform_state_dict_for_submodule(tm, mname, sd)
            with torch.no_grad():
                for n, v in sd.items():
                    dst = m._parameters[n] if n in m._parameters else m._buffers[n]
                    dst.copy_(v.to(dst.device, dst.dtype).reshape(dst.shape))
