"""Timing helpers (reference ``thunder/dev_utils/benchmark.py``): median device time of a callable
measured with HIP events, interleavable A/B comparisons."""
from __future__ import annotations

import statistics
from typing import Callable

import torch


def benchmark_n(n: int, fn: Callable, *args, warmup: int = 3, **kwargs) -> float:
    """Median milliseconds of ``fn(*args, **kwargs)`` over ``n`` runs (device events on GPU)."""
    for _ in range(warmup):
        fn(*args, **kwargs)
    times = []
    if torch.cuda.is_available():
        torch.cuda.synchronize()
        for _ in range(n):
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            fn(*args, **kwargs)
            e.record()
            torch.cuda.synchronize()
            times.append(s.elapsed_time(e))
    else:
        import time

        for _ in range(n):
            t0 = time.perf_counter()
            fn(*args, **kwargs)
            times.append((time.perf_counter() - t0) * 1e3)
    return statistics.median(times)


def interleaved(n: int, fns: dict[str, Callable], warmup: int = 3) -> dict[str, float]:
    """A/B(/C...) timing with the candidates interleaved run by run (removes clock drift bias)."""
    for f in fns.values():
        for _ in range(warmup):
            f()
    res = {k: [] for k in fns}
    for _ in range(n):
        for k, f in fns.items():
            res[k].append(benchmark_n(1, f, warmup=0))
    return {k: statistics.median(v) for k, v in res.items()}
