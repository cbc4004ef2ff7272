"""ThunderFX reports, reproducers and per-subgraph backend selection (reference: ``thunder/tests/test_dynamo.py``
report/repro tests)."""
import os
import subprocess
import sys

import pytest
import torch

from lightning_thunder_amd.dynamo.report import fx_report, thunder_optimize, thunder_profile


def _fn(x, w):
    y = torch.nn.functional.gelu(x @ w)
    if y.sum() > 0:  # graph break: data-dependent branch
        y = y * 2
    return torch.softmax(y, -1)


def test_fx_report_and_repro(tmp_path):
    x, w = torch.randn(4, 8), torch.randn(8, 8)
    rep = fx_report(_fn, x, w)
    assert len(rep.graphs) >= 2 and rep.graph_breaks >= 1
    assert "graph0" in str(rep)
    paths = rep.write_repros(str(tmp_path))
    assert all(os.path.exists(p) for p in paths)
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, paths[0]], capture_output=True, text=True, timeout=300,
                       env={**os.environ, "PYTHONPATH": root})
    assert r.returncode == 0, r.stderr[-3000:]
    assert "outputs match" in r.stdout and "eager" in r.stdout


def test_thunder_optimize_selects_a_backend():
    m = torch.nn.Sequential(torch.nn.Linear(16, 16), torch.nn.GELU(), torch.nn.Linear(16, 4))
    x = torch.randn(8, 16)
    opt = thunder_profile(m, trials=2)
    ref = m(x)
    for _ in range(8):
        out = opt(x)
    torch.testing.assert_close(out, ref)
    assert opt.selection_log and opt.selection_log[0]["choice"] in ("compiled", "eager")
    assert "->" in opt.report()
    torch._dynamo.reset()
    o2 = thunder_optimize(lambda a: torch.tanh(a) * 2, trials=1)
    torch.testing.assert_close(o2(x), torch.tanh(x) * 2)


def _fusing_fn(x, w):
    y = torch.nn.functional.gelu(x @ w) * 2 + 1
    z = torch.sin(y).sum(-1)
    return (y.exp() * z.unsqueeze(-1)).tanh()


@pytest.fixture
def cpu_fusion():
    from lightning_thunder_amd.executors import hipfuse

    old = hipfuse.ex.allow_cpu
    hipfuse.ex.allow_cpu = True
    yield
    hipfuse.ex.allow_cpu = old


def test_fusion_level_reports_cpu(tmp_path, cpu_fusion):
    """ThunderFX split subgraphs -> their hipfuse regions: each re-runs against its prims, is timed
    alone, and dumps a standalone repro script (generated HIP source + data file)."""
    import py_compile

    from lightning_thunder_amd.dynamo.report import (analyze_thunder_splits, get_thunder_split_reports,
                                                     save_failing_repros)

    x = torch.randn(8, 16, requires_grad=True)
    w = torch.randn(16, 32, requires_grad=True)
    reps = get_thunder_split_reports(_fusing_fn, x, w)
    assert reps
    fus = reps[0].create_fusion_reports()
    assert any("_fwd_" in f.name for f in fus) and any("_bwd_" in f.name for f in fus), [str(f) for f in fus]
    for f in fus:
        assert f.run_repro()["ok"]
        bench = f.run_benchmark(2)
        assert bench["fusion_ms"] > 0 and bench["bytes"] > 0
        path = f.write_repro(str(tmp_path))
        py_compile.compile(path, doraise=True)
        src = open(path).read()
        assert "__global__" in src and "hipfuse.launch" in src
        data = torch.load(path.replace("_repro.py", "_data.pt"), weights_only=True)
        assert "in0" in data and "out0" in data
    summary = analyze_thunder_splits(_fusing_fn, x, w)
    assert summary["subgraphs"] and summary["subgraphs"][0]["fusions"]
    assert save_failing_repros(reps, str(tmp_path / "failing")) == []  # nothing fails


@pytest.mark.gpu
def test_fusion_repro_runs_standalone_gpu(tmp_path):
    """The dumped repro of a generated kernel compiles, launches and matches on the GPU by itself, and
    the benchmark report times every fusion region (bytes / GB/s)."""
    import subprocess
    import sys

    from lightning_thunder_amd.dynamo.report import get_thunder_split_reports, thunderfx_benchmark_report

    x = torch.randn(256, 512, device="cuda", requires_grad=True)
    w = torch.randn(512, 1024, device="cuda", requires_grad=True)
    reps = get_thunder_split_reports(_fusing_fn, x, w)
    fus = reps[0].create_fusion_reports()
    assert fus
    path = fus[0].write_repro(str(tmp_path))
    env = dict(os.environ, PYTHONPATH=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    r = subprocess.run([sys.executable, path], capture_output=True, text=True, timeout=240, env=env)
    assert r.returncode == 0 and "matches" in r.stdout, r.stderr[-2000:]
    assert "GB/s" in r.stdout
    rows = thunderfx_benchmark_report(_fusing_fn, x, w, folder=str(tmp_path / "bench"))
    assert rows and all("fusion_ms" in row and row["fusion_gbps"] > 0 for row in rows), rows


def test_compiler_graph_benchmarking_times_every_split_under_every_executor():
    """Reference thunder/dynamo/compiler_graph_benchmark.py: each Thunder split module of each dynamo
    graph is timed under every executor (built-in timer here: pytest-benchmark is not in the image)."""
    import torch._dynamo

    from lightning_thunder_amd import jit
    from lightning_thunder_amd.dynamo.compiler_graph_benchmark import ThunderCompilerGraphBenchmarking

    def func(x):
        x = torch.sin(x)
        if x.sum() > 0:  # graph break: two dynamo graphs
            return torch.cos(x) + 1
        return x - 1

    torch._dynamo.reset()
    backend = ThunderCompilerGraphBenchmarking(executors={"eager": None, "thunder": jit}, warmup=1, iters=3)
    compiled = torch.compile(func, backend=backend, dynamic=False)
    x = torch.ones(64, 32, requires_grad=True)
    out = compiled(x)
    torch.testing.assert_close(out, func(x))
    assert backend.graph_idx >= 2
    names = {(r["GraphID"], r["SplitModuleName"], r["executor"]) for r in backend.results}
    for g in range(backend.graph_idx):
        assert any(k[0] == g and k[2] == "eager" for k in names), names
        assert any(k[0] == g and k[2] == "thunder" for k in names), names
    assert all(r["median_ms"] > 0 for r in backend.results)
    rep = backend.report()
    assert "GraphID[0]" in rep and "thunder" in rep, rep
    with pytest.raises(ValueError):
        ThunderCompilerGraphBenchmarking(executors={"bad-name": None})
    torch._dynamo.reset()
