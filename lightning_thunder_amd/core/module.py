"""ThunderModule: the compiled wrapper around an ``nn.Module`` (parity: reference ``thunder/core/module.py``
state-dict hooks :137-338, ``no_sync`` :340-382).
"""
from __future__ import annotations

import contextlib
from typing import Any, Iterator

import torch


class ThunderModule(torch.nn.Module):
    def __init__(self, model: torch.nn.Module, compiled_fn):
        super().__init__()
        self._model = model
        self._forward_fn = compiled_fn
        self._overrides_parameters: dict[str, torch.nn.Parameter] = {}
        self._overrides_buffers: dict[str, torch.Tensor] = {}
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
        return self._model.state_dict(*args, **kwargs)

    def load_original_state_dict(self, state_dict: dict, strict: bool = True, assign: bool = False):
        sd = dict(state_dict)
        for t in self._transforms():
            sd = t.transform_state_dict_for_submodule(self, "", sd)
        return self._model.load_state_dict(sd, strict=strict, assign=assign)

    def load_state_dict(self, state_dict: dict, strict: bool = True, assign: bool = False):
        return self._model.load_state_dict(state_dict, strict=strict, assign=assign)

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
