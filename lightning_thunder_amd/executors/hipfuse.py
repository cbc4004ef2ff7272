"""hipfuse: HIP fusion code generator (placeholder until codegen is wired)."""
from __future__ import annotations

from ..extend import FusionExecutor, register_executor

ex = FusionExecutor("hipfuse")
register_executor(ex)
