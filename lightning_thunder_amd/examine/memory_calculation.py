"""Static memory estimate of a trace under the reference's module path
(``thunder/examine/memory_calculation.py:151``); implemented in ``examine/__init__.py``."""
from . import get_alloc_memory

__all__ = ["get_alloc_memory"]
