"""Recipe for Hugging Face ``transformers`` models (reference ``thunder/recipes/hf_transformers.py``).

HF models build attention masks with python-side helpers and update caches in place; the
recipe (1) validates the model, (2) turns in-place ``index_copy_`` cache updates into the
functional form, and (3) when the model's mask is a plain causal mask, lets SDPA run with
``is_causal=True`` so the HIP flash-attention kernel claims it.
"""
from __future__ import annotations

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


BaseRecipe.register("transformers")(HFTransformers)
