"""Recipe registry (reference ``thunder/recipes/__init__.py``)."""
from __future__ import annotations

from .base import BaseRecipe
from .hf_transformers import HFTransformers

_names: dict[str, type] = {"default": BaseRecipe, "base": BaseRecipe, "hf-transformers": HFTransformers}


def get_recipe_class(name: str):
    if name not in _names:
        raise ValueError(f"unknown recipe {name!r}; known: {sorted(_names)}")
    return _names[name]


def get_recipes() -> list[str]:
    return list(_names)


def register_recipe(name: str, cls) -> None:
    if name == "auto":
        raise ValueError("'auto' is reserved (model-based recipe selection)")
    _names[name] = cls


__all__ = ["BaseRecipe", "HFTransformers", "get_recipe_class", "get_recipes", "register_recipe"]
