"""Profiling annotations (reference ``thunder/core/profile.py:10-71``).

``THUNDER_ANNOTATE_TRACES=1`` (or ``LTA_ANNOTATE_TRACES=1``) turns on named ranges around
the framework's host-side phases and around every HIP fusion launch.  On ROCm the ranges are
roctx ranges (``torch.cuda.nvtx`` is backed by roctx), so ``rocprofv3 --marker-trace`` shows
them next to the kernels, and ``torch.profiler`` sees the same names through
``record_function``.  Disabled, ``annotate_for_profile`` is a no-op decorator / context and
``add_markers`` costs one boolean check.
"""
from __future__ import annotations

import contextlib
import functools
import os

import torch

_ENABLED = any(os.getenv(v) in ("1", "y", "Y") for v in ("THUNDER_ANNOTATE_TRACES", "LTA_ANNOTATE_TRACES"))


def profiling_enabled() -> bool:
    return _ENABLED


def set_profiling_enabled(value: bool) -> bool:
    """Turns annotations on or off at run time; returns the previous setting."""
    global _ENABLED
    prev, _ENABLED = _ENABLED, bool(value)
    return prev


def _push(msg: str) -> None:
    if torch.cuda.is_available():
        torch.cuda.nvtx.range_push(msg)


def _pop() -> None:
    if torch.cuda.is_available():
        torch.cuda.nvtx.range_pop()


@contextlib.contextmanager
def add_markers(msg: str):
    """A roctx range plus a ``torch.profiler`` record_function named ``msg`` (when enabled)."""
    if not _ENABLED:
        yield
        return
    # the reference asserts the same: roctx/JSON consumers reject these characters
    assert "\n" not in msg and '"' not in msg, msg
    with torch.profiler.record_function(msg):
        _push(msg)
        try:
            yield
        finally:
            _pop()


class annotate_for_profile(contextlib.ContextDecorator):
    """``@annotate_for_profile("name")`` decorator or ``with annotate_for_profile("name"):``.

    The enabled check happens per call, so a function decorated at import time follows
    ``set_profiling_enabled`` later on.
    """

    def __init__(self, name: str):
        self.name = name
        self._cm = None

    def __enter__(self):
        self._cm = add_markers(self.name)
        return self._cm.__enter__()

    def __exit__(self, *exc):
        cm, self._cm = self._cm, None
        return cm.__exit__(*exc)

    def __call__(self, fn):
        @functools.wraps(fn)
        def wrapper(*args, **kwargs):
            if not _ENABLED:
                return fn(*args, **kwargs)
            with add_markers(self.name):
                return fn(*args, **kwargs)

        return wrapper
