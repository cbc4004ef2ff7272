"""LoRA adapters on ``nn.Linear`` (reference ``thunder/transforms/qlora.py:15-238``: ``LORATransform``
with ``r``, ``lora_alpha``, ``lora_dropout``, ``weights``, ``merged``).

Design: instead of editing the prologue/computation traces proxy by proxy (the reference),
``transform_module`` freezes each target weight, registers ``lora_a`` [r, in] and ``lora_b``
[out, r] on the Linear and gives the module a LoRA forward.  The program is acquired *through*
that forward, so the trace holds ``linear(x, W) + s * linear(linear(drop(x), A), B)`` and the
executors see it like any other computation (the small rank-r GEMMs run on hipBLASLt; with NF4
base weights (``NF4LinearQuant4bit``) this is QLoRA).  ``merged=True`` folds ``s * B @ A`` into the
weight inside the trace (inference).
"""
from __future__ import annotations

import math

import torch

from ..core.transform_common import Transform


class _LoRAForward:
    def __init__(self, mod, scaling: float, dropout: float, merged: bool, base_forward):
        self.mod = mod
        self.scaling = scaling
        self.dropout = dropout
        self.merged = merged
        self.base_forward = base_forward

    def __call__(self, x):
        m = self.mod
        if self.merged and hasattr(m, "weight"):
            w = m.weight + (m.lora_b @ m.lora_a) * self.scaling
            return torch.nn.functional.linear(x, w, m.bias)
        y = self.base_forward(x)
        h = torch.nn.functional.dropout(x, self.dropout, m.training) if self.dropout > 0 else x
        return y + torch.nn.functional.linear(torch.nn.functional.linear(h, m.lora_a), m.lora_b) * self.scaling


class LORATransform(Transform):
    def __init__(self, *, r: int = 8, lora_alpha: int = 16, lora_dropout: float = 0.0, weights: list[str] | None = None,
                 merged: bool = False):
        if r <= 0:
            raise ValueError("LoRA rank r must be positive")
        self.r = r
        self.lora_alpha = lora_alpha
        self.lora_dropout = lora_dropout
        self.scaling = lora_alpha / r
        self.weights = weights
        self.merged = merged
        self.lora_linear_names: set[str] = set()

    @staticmethod
    def init_lora_linear(lora_a, lora_b):
        torch.nn.init.kaiming_uniform_(lora_a, a=math.sqrt(5))
        torch.nn.init.zeros_(lora_b)

    def _selected(self, name: str) -> bool:
        if self.weights is None:
            return True
        return any(name == w or name.endswith("." + w) or w in name.split(".") for w in self.weights)

    def transform_module(self, model) -> None:
        for name, m in model._model.named_modules():
            if not isinstance(m, torch.nn.Linear) or hasattr(m, "lora_a") or not self._selected(name):
                continue
            ref = m.weight if hasattr(m, "weight") else m.qweight
            dtype = m.weight.dtype if hasattr(m, "weight") else torch.bfloat16
            if hasattr(m, "weight"):
                m.weight.requires_grad_(False)
            if m.bias is not None:
                m.bias.requires_grad_(False)
            a = torch.nn.Parameter(torch.empty(self.r, m.in_features, dtype=dtype, device=ref.device))
            b = torch.nn.Parameter(torch.empty(m.out_features, self.r, dtype=dtype, device=ref.device))
            self.init_lora_linear(a, b)
            m.register_parameter("lora_a", a)
            m.register_parameter("lora_b", b)
            base = m.forward if "forward" in m.__dict__ else type(m).forward.__get__(m)
            m.forward = _LoRAForward(m, self.scaling, self.lora_dropout, self.merged, base)
            self.lora_linear_names.add(name)

    def transform_state_dict_for_submodule(self, model, submodule_name, state_dict):
        if submodule_name not in self.lora_linear_names or "lora_a" in state_dict:
            return state_dict
        sd = dict(state_dict)
        m = model._model.get_submodule(submodule_name)
        sd["lora_a"] = m.lora_a.detach().clone()
        sd["lora_b"] = m.lora_b.detach().clone()
        return sd
