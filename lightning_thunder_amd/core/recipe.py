"""Recipes and plugins: bundles of executors, transforms and lookasides applied by
``lightning_thunder_amd.compile`` (reference ``thunder/core/recipe.py``: ``Recipe``, ``Plugin``,
``PluginPolicy``, ``Lookaside``, ``Interpreter``, registry keyed by model class path).
"""
from __future__ import annotations

import warnings
from contextlib import contextmanager
from enum import Enum, auto
from typing import Any

import torch

from .transform_common import Transform

_RECIPES: dict[str, type] = {}


class Lookaside:
    """Replace ``fn`` by ``replace_with`` while the program is acquired."""

    def __init__(self, fn, replace_with):
        self._fn = fn
        self._replace_with = replace_with


class PluginPolicy(Enum):
    PRE = auto()   # contributes before the recipe's own transforms/executors
    POST = auto()  # after (e.g. hipGraphs, profiling: they must see the final trace)


class Plugin:
    policy: PluginPolicy = PluginPolicy.PRE

    def setup_lookasides(self) -> list[Lookaside] | None:
        return None

    def setup_transforms(self) -> list[Transform] | None:
        return None

    def setup_executors(self) -> list | None:
        return None


class Interpreter(Enum):
    THUNDER_JIT = auto()
    THUNDER_FX = auto()


@contextmanager
def _reported_warnings():
    with warnings.catch_warnings(record=True) as caught:
        warnings.simplefilter("always", UserWarning)
        yield
    for w in caught:
        print(f"{w.category.__name__}: {w.message}")


class Recipe:
    def __init__(self, plugins: list | None = None, interpreter: Interpreter | str = Interpreter.THUNDER_JIT):
        if isinstance(interpreter, str):
            table = {"thunder.jit": Interpreter.THUNDER_JIT, "thunder.fx": Interpreter.THUNDER_FX,
                     "jit": Interpreter.THUNDER_JIT, "fx": Interpreter.THUNDER_FX}
            if interpreter not in table:
                raise ValueError(f"unknown interpreter {interpreter!r}; expected one of {sorted(table)}")
            interpreter = table[interpreter]
        self.interpreter = interpreter
        self.plugins = list(plugins or [])
        self.lookasides: list[Lookaside] = []
        self.transforms: list = []
        self.executors: list = []
        self.config: dict = {}
        self._lookaside_executor = None

    def add_plugins(self, plugins):
        self.plugins.extend(plugins)

    @classmethod
    def validate(cls, model) -> bool:
        return True

    def setup_lookasides(self):
        return None

    def setup_transforms(self):
        return None

    def setup_executors(self):
        return []

    def setup_config(self) -> dict[str, Any]:
        return {}

    @classmethod
    def register(cls, key: str):
        def deco(sub):
            _RECIPES[key] = sub
            return sub

        return deco

    @classmethod
    def get_for_model(cls, model) -> "Recipe":
        path = f"{type(model).__module__}.{type(model).__name__}".split(".")
        for i in range(len(path), 0, -1):
            sub = _RECIPES.get(".".join(path[:i]))
            if sub is not None and sub.validate(model):
                return sub()
        default = _RECIPES.get("")
        if default is None:
            raise RuntimeError("no recipe applies to this model and no default recipe is registered")
        return default()

    def _collect(self, attr):
        pre = [p for p in self.plugins if p.policy is PluginPolicy.PRE]
        post = [p for p in self.plugins if p.policy is PluginPolicy.POST]
        out = []
        for p in pre:
            out.extend(getattr(p, attr)() or [])
        out.extend(getattr(self, attr)() or [])
        for p in post:
            out.extend(getattr(p, attr)() or [])
        return out

    def apply(self, model):
        from ..extend import TemporaryExecutor

        with _reported_warnings():
            self.validate(model)
        self.config = self.setup_config()
        self.lookasides = self._collect("setup_lookasides")
        if self.lookasides:
            self._lookaside_executor = TemporaryExecutor()
            for lk in self.lookasides:
                self._lookaside_executor._lookasides[lk._fn] = lk._replace_with
        self.transforms = self._collect("setup_transforms")
        self.executors = ([self._lookaside_executor] if self._lookaside_executor is not None else []) + self._collect(
            "setup_executors")
        if self.interpreter is Interpreter.THUNDER_JIT:
            from .. import jit

            return jit(model, transforms=self.transforms, executors=self.executors or None, **self.config)
        from ..dynamo import ThunderCompiler

        backend = ThunderCompiler(transforms=self.transforms, executors=self.executors or None, **self.config)
        return torch.compile(model, backend=backend)
