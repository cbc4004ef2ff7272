"""ThunderModule: the compiled wrapper around an ``nn.Module`` (parity: reference ``thunder/core/module.py``
state-dict hooks :137-338, ``no_sync`` :340-382).
"""
from __future__ import annotations

import contextlib
from typing import Any, Iterator

import torch


# attributes a transform sets on the parameters it rewrites (sharding metadata): they must survive a
# load_state_dict(assign=True) that swaps the Parameter objects
_PARAM_META = ("_lc_full_shape", "_lc_tp_kind", "distparallel_type", "thunder_fsdp_padding_size")


class ThunderModule(torch.nn.Module):
    """Transforms rewrite the wrapped module's parameters IN PLACE (FSDP / TP shards, quantized
    weights, LoRA adapters live in ``_model``), so unlike the reference there is no separate
    ``_overrides_parameters`` table: ``state_dict()`` is the *transformed* state (the reference's
    semantics), ``original_state_dict()`` runs every transform's reverse hook, and
    ``load_original_state_dict`` runs the forward hooks."""

    def __init__(self, model: torch.nn.Module, compiled_fn):
        super().__init__()
        self._model = model
        self._forward_fn = compiled_fn
        self._null_ctx = contextlib.nullcontext()
        self._is_no_sync = False

    def forward(self, *args, **kwargs):
        return self._forward_fn(*args, **kwargs)

    # --- parameter access (shard-aware through the underlying module) -------------------------
    def get_parameter(self, name: str) -> torch.nn.Parameter:
        return self._model.get_parameter(name)

    def get_buffer(self, name: str) -> torch.Tensor:
        return self._model.get_buffer(name)

    def named_parameters(self, prefix: str = "", recurse: bool = True, remove_duplicate: bool = True) -> Iterator:
        return self._model.named_parameters(prefix=prefix, recurse=recurse, remove_duplicate=remove_duplicate)

    def named_buffers(self, prefix: str = "", recurse: bool = True, remove_duplicate: bool = True) -> Iterator:
        return self._model.named_buffers(prefix=prefix, recurse=recurse, remove_duplicate=remove_duplicate)

    # --- state dict with transform hooks ------------------------------------------------------
    def _transforms(self):
        cd = getattr(self._forward_fn, "_lc_cd", None)
        return [] if cd is None else cd.transforms

    def original_state_dict(self, *args, **kwargs) -> dict:
        sd = self._model.state_dict(*args, **kwargs)
        for t in reversed(self._transforms()):
            sd = t.reverse_transform_state_dict_for_submodule(self, "", sd)
        return sd

    def state_dict(self, *args, **kwargs) -> dict:
        """State of the TRANSFORMED module (e.g. this rank's FSDP / TP shards)."""
        return self._model.state_dict(*args, **kwargs)

    def load_original_state_dict(self, state_dict: dict, strict: bool = True, assign: bool = False):
        """Loads an untransformed (e.g. full, unsharded) state dict through every transform's
        ``transform_state_dict_for_submodule`` hook (shard / quantize on load)."""
        sd = dict(state_dict)
        for t in self._transforms():
            sd = t.transform_state_dict_for_submodule(self, "", sd)
        return self.load_state_dict(sd, strict=strict, assign=assign)

    def load_state_dict(self, state_dict: dict, strict: bool = True, assign: bool = False):
        """Loads a TRANSFORMED state dict (reference ``ThunderModule.load_state_dict``): shapes are
        checked against the transformed parameters; with ``assign`` the new tensors replace the
        parameters and inherit their sharding metadata, so the compiled program keeps working."""
        params = dict(self._model.named_parameters(remove_duplicate=False))
        errors = []
        for k, v in state_dict.items():
            cur = params.get(k)
            if cur is not None and isinstance(v, torch.Tensor) and tuple(v.shape) != tuple(cur.shape):
                errors.append(f"size mismatch for {k}: copying a param with shape {tuple(v.shape)} from checkpoint, "
                              f"the shape in the transformed model is {tuple(cur.shape)}.")
        if errors:
            raise RuntimeError("Error(s) in loading state_dict:\n\t" + "\n\t".join(errors))
        meta = {k: {a: getattr(p, a) for a in _PARAM_META if hasattr(p, a)} for k, p in params.items()}
        res = self._model.load_state_dict(state_dict, strict=strict, assign=assign)
        if assign:
            for k, p in self._model.named_parameters(remove_duplicate=False):
                for a, val in meta.get(k, {}).items():
                    if not hasattr(p, a):
                        setattr(p, a, val)
        return res

    # --- gradient sync control ------------------------------------------------------------------
    @contextlib.contextmanager
    def no_sync(self):
        """Skip gradient collectives (DDP all-reduce / FSDP reduce-scatter) for accumulation steps."""
        from ..distributed import set_skip_data_parallel_grad_sync, _sync_grads

        prev = set_skip_data_parallel_grad_sync(True)
        self._is_no_sync = True
        try:
            yield
        finally:
            set_skip_data_parallel_grad_sync(prev)
            self._is_no_sync = False
        _sync_grads(self)

    def __getattr__(self, name: str):
        try:
            return super().__getattr__(name)
        except AttributeError:
            return getattr(self._modules["_model"], name)
