"""``core/profile.py`` (reference ``thunder/core/profile.py:10-71``): with annotations on,
the jitted call, the cache lookup and every HIP fusion run inside named ranges that
``torch.profiler`` (and, on ROCm, roctx / rocprofv3 marker traces) record."""
import torch

import lightning_thunder_amd as thunder
from lightning_thunder_amd.core import profile


def test_annotations_recorded_by_torch_profiler():
    def f(x):
        return (x.sin() * 2 + 1).relu()

    jf = thunder.jit(f)
    x = torch.randn(16)
    jf(x)
    prev = profile.set_profiling_enabled(True)
    try:
        with torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CPU]) as prof:
            out = jf(x)
    finally:
        profile.set_profiling_enabled(prev)
    names = {e.name for e in prof.events()}
    assert {"fn_", "get_computation_and_inputs"} <= names, names
    torch.testing.assert_close(out, f(x))


def test_annotations_off_is_noop():
    assert not profile.profiling_enabled()

    @profile.annotate_for_profile("x")
    def g(a):
        return a + 1

    with profile.annotate_for_profile("block"):
        assert g(1) == 2
    with profile.add_markers("m"):
        pass
