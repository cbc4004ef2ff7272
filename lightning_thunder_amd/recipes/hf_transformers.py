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
from ..transforms.sdpa_gqa import SDPAGQATransform  # noqa: E402
from ..transforms.hf_rope import HFRoPETransform  # noqa: E402


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
        return super().setup_transforms() + [HFRoPETransform(), SDPAGQATransform(), InplaceIndexCopyTransform()]

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
        members["forward"] = _forward_with_static_cache_init
        sub = type(f"Thunder{cls.__name__}", (type(tm),), members)
        tm.__class__ = sub
        gc = getattr(model, "generation_config", None)
        if gc is not None and hasattr(gc, "disable_compile"):
            # HF auto-wraps the forward in torch.compile for static caches: the compiled program
            # must run as it is (no second compiler tracing through its kernels)
            gc.disable_compile = True
        return tm


def _init_static_cache(cache, model, args, kwargs):
    """Allocates a fresh HF static cache's storage before the compiled program runs.

    HF creates a new ``StaticCache`` per ``generate`` call whose layers allocate their tensors on the
    first ``update`` (``is_initialized`` False).  Initialising them here, with the shapes the model
    will write, means every call sees an initialised cache, so the prefill program traced once is
    reused by later ``generate`` calls instead of being retraced for the ``is_initialized`` flip."""
    layers = getattr(cache, "layers", None)
    if not layers:
        return None
    todo = [l for l in layers if "Static" in type(l).__name__ and hasattr(l, "lazy_initialization")
            and not getattr(l, "is_initialized", True)]
    if not todo:
        return None
    ids = kwargs.get("input_ids", args[0] if args else None)
    emb = kwargs.get("inputs_embeds")
    ref = ids if ids is not None else emb
    cfg = getattr(model, "config", None)
    if ref is None or cfg is None:
        return None
    n_kv = getattr(cfg, "num_key_value_heads", None) or cfg.num_attention_heads
    hd = getattr(cfg, "head_dim", None) or cfg.hidden_size // cfg.num_attention_heads
    dtype = next(model.parameters()).dtype
    kv = torch.empty((ref.shape[0], n_kv, 1, hd), dtype=dtype, device=ref.device)
    for layer in todo:
        layer.lazy_initialization(kv, kv)
        layer.is_initialized = False  # the storage exists; the flag flips after this call (see below)
    return todo


def _forward_with_static_cache_init(self, *args, **kwargs):
    from ..core import interpreter

    cache = kwargs.get("past_key_values")
    fresh = _init_static_cache(cache, self._model, args, kwargs) if cache is not None else None
    if not fresh:
        return self._forward_fn(*args, **kwargs)
    # the compiled prefill sees `is_initialized == False` (get_seq_length() == 0, as in eager) on
    # storage allocated above, so one prefill program serves every generate() call
    prev = interpreter.STATIC_CACHE_PREALLOCATED[0]
    interpreter.STATIC_CACHE_PREALLOCATED[0] = True
    try:
        out = self._forward_fn(*args, **kwargs)
    finally:
        interpreter.STATIC_CACHE_PREALLOCATED[0] = prev
    for layer in fresh:
        layer.is_initialized = True
    return out


BaseRecipe.register("transformers")(HFTransformers)
