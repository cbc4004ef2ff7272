"""Graph-by-graph benchmarking of the ThunderFX splits (parity: reference
``thunder/dynamo/compiler_graph_benchmark.py:1-170``, ``ThunderCompilerGraphBenchmarking``).

A ``torch.compile`` backend that splits each dynamo graph exactly as :class:`ThunderCompiler` does,
then times every Thunder-supported split module under several executors (any ``GraphModule ->
callable`` compile function; ``None`` runs the module eagerly) on random inputs built from the
placeholders' example values.  The split program itself still runs through Thunder.

Timing backend:
* a ``pytest-benchmark`` fixture (the reference's contract: ``bench(fn, *args)``, the stats name is
  suffixed ``-GraphID[i]-SplitModuleName[name]-executor[ex]`` for ``--benchmark-group-by``), or
* when no fixture is given (pytest-benchmark is not part of this image), the built-in timer:
  device-synchronized wall time, median over ``iters`` calls after ``warmup``; the peak allocated
  device memory of each run is recorded too (reference ``record_peak_allocated_memory``).

``results`` holds one row per (graph, split module, executor); :meth:`report` formats them with
each executor's speedup over the first one.
"""
from __future__ import annotations

import statistics
import time
from typing import Callable

import torch

from . import ThunderCompiler

GRAPH_BY_GRAPH_BENCHMARK_PARAMS_KEYS = ("GraphID", "SplitModuleName", "executor")
MAX_ALLOCATED_MEMORY_KEYWORD = "max_allocated_memory_MB"


def _example_input(node: torch.fx.Node, gen: torch.Generator):
    """A random tensor shaped like the placeholder's example value (fake tensor) — or the value itself."""
    ev = node.meta.get("example_value", node.meta.get("val"))
    if isinstance(ev, torch.SymInt):
        return int(ev.node.hint) if ev.node.has_hint() else 1
    if not isinstance(ev, torch.Tensor):
        return ev
    shape = tuple(int(s) for s in ev.shape)
    dev = ev.device
    if ev.dtype.is_floating_point or ev.dtype.is_complex:
        t = torch.randn(shape, generator=gen, dtype=torch.float32).to(device=dev, dtype=ev.dtype)
    elif ev.dtype == torch.bool:
        t = (torch.rand(shape, generator=gen) > 0.5).to(dev)
    else:
        t = torch.randint(0, 8, shape, generator=gen, dtype=torch.int64).to(device=dev, dtype=ev.dtype)
    return t.requires_grad_(ev.requires_grad) if ev.dtype.is_floating_point else t


def _sync():
    if torch.cuda.is_available():
        torch.cuda.synchronize()


class _Timer:
    """Built-in stand-in for the pytest-benchmark fixture."""

    def __init__(self, warmup: int, iters: int):
        self.warmup, self.iters = warmup, iters

    def __call__(self, fn, *args) -> dict:
        for _ in range(self.warmup):
            fn(*args)
        _sync()
        if torch.cuda.is_available():
            torch.cuda.reset_peak_memory_stats()
        ts = []
        for _ in range(self.iters):
            t0 = time.perf_counter()
            fn(*args)
            _sync()
            ts.append((time.perf_counter() - t0) * 1e3)
        mem = torch.cuda.max_memory_allocated() / 2**20 if torch.cuda.is_available() else None
        return {"median_ms": statistics.median(ts), "min_ms": min(ts), MAX_ALLOCATED_MEMORY_KEYWORD: mem}


class ThunderCompilerGraphBenchmarking(ThunderCompiler):
    _executors = ("eager", "thunder")

    def __init__(self, bench=None, executors: dict[str, Callable | None] | None = None, *, warmup: int = 3,
                 iters: int = 20, post_graph: Callable | None = None, **thunder_options):
        """``bench``: a pytest-benchmark fixture, or None for the built-in timer.  ``executors``: name ->
        compile function applied to each split ``GraphModule`` (None: eager); default eager vs
        ``lightning_thunder_amd.jit``.  ``post_graph(compiled_fn, sample_args)`` may wrap each compiled
        function (e.g. to time forward + backward)."""
        super().__init__(**thunder_options)
        if executors is None:
            from .. import jit

            executors = {"eager": None, "thunder": jit}
        if not isinstance(executors, dict) or not executors:
            raise ValueError("'executors' must be a non-empty dictionary")
        if any("-" in k for k in executors):
            raise ValueError("executor names cannot contain '-' (it separates the benchmark-group-by fields)")
        self.executors = executors
        self.bench = bench
        self.timer = _Timer(warmup, iters)
        self.post_graph = post_graph
        self.graph_idx = 0
        self.results: list[dict] = []

    def run_bench(self, gm: torch.fx.GraphModule, name: str, *sample_args) -> None:
        for ex_name, ex in self.executors.items():
            try:
                fn = gm if ex is None else ex(gm)
            except Exception as e:
                raise RuntimeError(f"the executor {ex_name} failed to compile {name}") from e
            if self.post_graph is not None:
                fn = self.post_graph(fn, sample_args)
            row = {GRAPH_BY_GRAPH_BENCHMARK_PARAMS_KEYS[0]: self.graph_idx,
                   GRAPH_BY_GRAPH_BENCHMARK_PARAMS_KEYS[1]: name,
                   GRAPH_BY_GRAPH_BENCHMARK_PARAMS_KEYS[2]: ex_name}
            if self.bench is None:
                row.update(self.timer(fn, *sample_args))
            else:
                self.bench(fn, *sample_args)
                gid, mod, exk = GRAPH_BY_GRAPH_BENCHMARK_PARAMS_KEYS
                stats = getattr(self.bench, "stats", None)
                if stats is not None and hasattr(stats, "name"):
                    stats.name += f"-{gid}[{self.graph_idx}]-{mod}[{name}]-{exk}[{ex_name}]"
                # a fixture may only be used once per test: reset its mode for the next split / executor
                if hasattr(self.bench, "_mode"):
                    self.bench._mode = None
            self.results.append(row)

    def __call__(self, gm: torch.fx.GraphModule, sample_args):
        originals = {}
        # the split modules as dynamo produced them, before ThunderCompiler swaps in their jitted forms
        out = super().__call__(gm, sample_args)
        info = self.subgraph_infos[-1]
        gen = torch.Generator().manual_seed(self.graph_idx)
        if info.split_graph_module is None:
            originals = {"whole": gm}
        else:
            originals = dict(getattr(info, "original_split_modules", {}) or {})
        for name, sub in originals.items():
            args = [_example_input(n, gen) for n in sub.graph.nodes if n.op == "placeholder"]
            self.run_bench(sub, name, *args)
        self.graph_idx += 1
        return out

    def report(self) -> str:
        """One line per split module: each executor's median time and speedup over the first executor."""
        lines = []
        keys = []
        for r in self.results:
            k = (r["GraphID"], r["SplitModuleName"])
            if k not in keys:
                keys.append(k)
        for k in keys:
            rows = [r for r in self.results if (r["GraphID"], r["SplitModuleName"]) == k]
            base = rows[0].get("median_ms")
            parts = []
            for r in rows:
                ms = r.get("median_ms")
                if ms is None:
                    parts.append(f"{r['executor']}: (pytest-benchmark)")
                    continue
                sp = f" ({base / ms:.2f}x)" if base and ms else ""
                parts.append(f"{r['executor']} {ms:.3f} ms{sp}")
            lines.append(f"GraphID[{k[0]}] SplitModuleName[{k[1]}]: " + ", ".join(parts))
        return "\n".join(lines)
