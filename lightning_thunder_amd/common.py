"""Compile data and statistics (parity: reference ``thunder/common.py`` ``CompileData``/``CompileStats`` :65-175,
and ``thunder/core/compile_data.py`` / ``thunder/core/options.py``).
"""
from __future__ import annotations

import time
from contextvars import ContextVar
from enum import Enum
from typing import Any, Callable

import torch


class CACHE_OPTIONS(Enum):
    NO_CACHING = "no caching"
    SAME_INPUT = "same input"
    CONSTANT_VALUES = "constant values"
    SYMBOLIC_VALUES = "symbolic values"


class SHARP_EDGES_OPTIONS(Enum):
    ALLOW = "allow"
    WARN = "warn"
    ERROR = "error"


def resolve_cache_option(x) -> CACHE_OPTIONS:
    if x is None:
        return CACHE_OPTIONS.CONSTANT_VALUES
    if isinstance(x, CACHE_OPTIONS):
        return x
    for o in CACHE_OPTIONS:
        if o.value == x:
            return o
    raise ValueError(f"Unknown cache option {x}")


def resolve_sharp_edges_option(x) -> SHARP_EDGES_OPTIONS:
    if x is None:
        return SHARP_EDGES_OPTIONS.ALLOW
    if isinstance(x, SHARP_EDGES_OPTIONS):
        return x
    for o in SHARP_EDGES_OPTIONS:
        if o.value == x:
            return o
    raise ValueError(f"Unknown sharp edges option {x}")


class DebugOptions:
    """Registrable, type-checked debug options (reference options.py:144-211)."""

    _registry: dict[str, tuple[type, Any, str]] = {}

    @classmethod
    def register_option(cls, name: str, typ: type, default: Any, doc: str = "") -> None:
        cls._registry[name] = (typ, default, doc)

    def __init__(self, **kwargs):
        for name, (typ, default, _) in self._registry.items():
            setattr(self, name, default)
        for k, v in kwargs.items():
            if k not in self._registry:
                raise ValueError(f"Unknown debug option {k}; known: {list(self._registry)}")
            typ = self._registry[k][0]
            if not isinstance(v, typ):
                raise TypeError(f"Debug option {k} expects {typ}, got {type(v)}")
            setattr(self, k, v)

    def __repr__(self):
        return "DebugOptions(" + ", ".join(f"{k}={getattr(self, k)!r}" for k in self._registry) + ")"


DebugOptions.register_option("check_traces", bool, False, "Validate every trace appended during compilation")
DebugOptions.register_option("show_interpreter_progress", bool, False, "Print acquisition progress")
DebugOptions.register_option("record_interpreter_history", bool, False, "Record the acquisition log")
DebugOptions.register_option("sync_after_each_kernel", bool, False, "Synchronize after each HIP kernel (debug numerics)")


class CompileStats:
    def __init__(self):
        self.calls = 0
        self.cache_hits = 0
        self.cache_misses = 0
        self.last_trace_cache_start = 0
        self.last_trace_cache_stop = 0
        self.last_trace_tracing_start = 0
        self.last_trace_tracing_stop = 0
        self.last_trace_host_start = 0
        self.last_trace_host_stop = 0
        self.last_trace_host_execution_start = 0
        self.last_trace_host_execution_stop = 0
        self.last_traces = None
        self.last_backward_traces = None
        self.last_prologue_traces = None
        self.last_compile_reasons: list[str] = []
        self.interpreter_cache: list = []
        self.last_interpreter_log = None
        self.last_executed = None

    @property
    def last_cache_lookup_time(self):
        return (self.last_trace_cache_stop - self.last_trace_cache_start) / 1e6

    @property
    def last_tracing_time(self):
        return (self.last_trace_tracing_stop - self.last_trace_tracing_start) / 1e6

    @property
    def last_host_time(self):
        return (self.last_trace_host_stop - self.last_trace_host_start) / 1e6


class CompileData:
    def __init__(self, *, fn, executors_list, cache_option, sharp_edges, disable_torch_autograd, transforms, debug_options,
                 compile_options, is_module):
        self.fn = fn
        self.executors_list = tuple(executors_list)
        self.cache_option = cache_option
        self.sharp_edges = sharp_edges
        self.disable_torch_autograd = disable_torch_autograd
        self.transforms = list(transforms)
        self.debug_options = debug_options or DebugOptions()
        self.compile_options = dict(compile_options)
        self.is_module = is_module
        self.process_group_for_ddp = None
        self.no_grad_sync = False
        self._compile_options_used: set[str] = set()

    def get_compile_option(self, name: str, description: str = "", default=None):
        self._compile_options_used.add(name)
        return self.compile_options.get(name, default)


_compile_data_ctx: ContextVar = ContextVar("compile_data", default=None)


def get_compile_data() -> CompileData | None:
    return _compile_data_ctx.get()


def get_compile_option(name: str, description: str = "", default=None):
    cd = get_compile_data()
    if cd is None:
        return default
    return cd.get_compile_option(name, description, default)


def compile_data_of(fn) -> CompileData | None:
    return getattr(fn, "_lc_cd", None)


def compile_stats_of(fn) -> CompileStats | None:
    return getattr(fn, "_lc_cs", None)
