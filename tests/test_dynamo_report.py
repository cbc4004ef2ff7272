"""ThunderFX reports, reproducers and per-subgraph backend selection (reference: ``thunder/tests/test_dynamo.py``
report/repro tests)."""
import os
import subprocess
import sys

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
