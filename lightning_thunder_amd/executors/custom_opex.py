"""``custom_op`` executor: runs ``torch.library.custom_op`` operators (parity: reference
``thunder/executors/custom_op_ex.py:15``).  The symbols themselves, their metas and their
autograd rules come from :mod:`lightning_thunder_amd.torch.custom_op`; this executor only binds
each symbol to the operator's dispatcher overload (and the backward symbol to the op's registered
backward function).  It sits below the HIP executors and above the torch fallback.
"""
from __future__ import annotations

from ..extend import OperatorExecutor, register_executor, add_default_executor

ex = OperatorExecutor("custom_op", version="0.1")
register_executor(ex)
add_default_executor(ex, last=True)

custom_op_ex = ex


def register(sym, fn) -> None:
    op = ex.register_operator(f"custom_op_impl_{sym.name}", like=sym, fn=fn)
    ex.register_implementation(sym, op)
