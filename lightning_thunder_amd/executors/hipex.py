"""hipex: hand-written CDNA4 HIP kernels (placeholder until kernels are wired)."""
from __future__ import annotations

from ..extend import OperatorExecutor, register_executor, add_default_executor

ex = OperatorExecutor("hipex")
register_executor(ex)
