"""Recipe for Hugging Face ``transformers`` models (reference ``thunder/recipes/hf_transformers.py``).

HF models build attention masks with python-side helpers and update caches in place; the
recipe (1) validates the model, (2) turns in-place ``index_copy_`` cache updates into the
functional form, and (3) when the model's mask is a plain causal mask, lets SDPA run with
``is_causal=True`` so the HIP flash-attention kernel claims it.
"""
from __future__ import annotations

import types
import warnings

import torch

from ..core.transform_common import Transform
from .base import BaseRecipe


from ..transforms.inplace_index_copy import InplaceIndexCopyTransform  # noqa: E402


class HFTransformers(BaseRecipe):
    @classmethod
    def validate(cls, model) -> bool:
        try:
            import transformers  # noqa: F401
        except Exception:
            return False
        if not isinstance(model, torch.nn.Module):
            return False
        supported = ("PreTrainedModel",)
        ok = any(c.__name__ in supported for c in type(model).__mro__)
        if not ok:
            warnings.warn(f"{type(model).__name__} is not a transformers PreTrainedModel; the recipe may not apply")
        return ok

    def setup_config(self):
        cfg = super().setup_config()
        return cfg

    def setup_transforms(self):
        return super().setup_transforms() + [InplaceIndexCopyTransform()]

    def apply(self, model):
        """Compiles ``model`` and makes HF generation run on the compiled forward.

        ``GenerationMixin.generate`` looks decoding methods up on ``type(self)`` and calls
        ``self(**model_inputs)``; the returned module is an instance of a per-model subclass of
        :class:`ThunderModule` carrying the model class's generation methods, so ``generate``
        (greedy/sampling, static or dynamic caches) drives the compiled program while every other
        attribute resolves on the wrapped model."""
        tm = super().apply(model)
        from ..core.module import ThunderModule

        cls = type(model)
        skip = set(dir(ThunderModule))
        members = {}
        for name in dir(cls):
            if name in skip or name.startswith("__"):
                continue
            owner = next((k for k in cls.__mro__ if name in k.__dict__), None)
            if owner is None or owner is object:
                continue
            raw = owner.__dict__[name]
            # methods and class-level data (``_auto_class``, ``_supports_*``); properties keep
            # resolving on the wrapped model through ThunderModule.__getattr__
            if not isinstance(raw, property):
                members[name] = raw
        sub = type(f"Thunder{cls.__name__}", (type(tm),), members)
        tm.__class__ = sub
        return tm


BaseRecipe.register("transformers")(HFTransformers)
