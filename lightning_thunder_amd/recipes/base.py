"""BaseRecipe: the framework defaults (reference ``thunder/recipes/base.py:51-165``).

The reference picks a fuser ("nvfuser" or "torch.compile"); here the fusion backend is
``hipfuse`` (HIP codegen) or ``None`` (hand-written HIP kernels + ATen only).  The default
executor list is the MI355X one: ``hipex`` (hand-written CDNA4 kernels) → [``hipfuse``] →
``torch`` (+ ``python``), and ``PrunePrologueChecks`` drops parameter metadata guards.
"""
from __future__ import annotations

from typing import Any

from ..core.recipe import Recipe
from ..common import DebugOptions


@Recipe.register("")
class BaseRecipe(Recipe):
    def __init__(self, show_progress: bool = False, fuser: str | None = "hipfuse", interpreter="thunder.jit",
                 plugins=None):
        super().__init__(plugins=plugins, interpreter=interpreter)
        if fuser not in ("hipfuse", None, "none"):
            raise ValueError(f"unknown fuser {fuser!r}; MI355X fusers: 'hipfuse' or None")
        self.fuser = None if fuser == "none" else fuser
        self.show_progress = show_progress
        self.executor_names = ["hipex"] + (["hipfuse"] if self.fuser else []) + ["torch"]

    def setup_config(self) -> dict[str, Any]:
        if not self.show_progress:
            return {}
        return dict(debug_options=DebugOptions(show_interpreter_progress=True))

    def setup_transforms(self):
        from ..transforms.prune_prologue_checks import PrunePrologueChecks

        return [PrunePrologueChecks()]

    def setup_executors(self):
        from ..extend import get_executor

        return [get_executor(n) for n in self.executor_names]
