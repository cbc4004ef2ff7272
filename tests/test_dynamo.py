"""ThunderFX (torch.compile backend) tests (reference: thunder/tests/test_dynamo.py)."""
import torch

from lightning_thunder_amd.dynamo import thunderfx, ThunderCompiler, split_report


def test_thunderfx_module_matches_eager():
    torch.manual_seed(0)
    m = torch.nn.Sequential(torch.nn.Linear(4, 8), torch.nn.GELU(), torch.nn.Linear(8, 2))
    cm = thunderfx(m)
    x = torch.randn(3, 4, requires_grad=True)
    out = cm(x)
    torch.testing.assert_close(out, m(x))
    out.sum().backward()
    assert x.grad is not None
    assert sum(len(i.thunder_compiled_fns) for i in cm.subgraph_infos) >= 1


def test_graph_break_and_split():
    def f(x, y):
        z = torch.sin(x) + y
        idx = torch.nonzero(z > 0)  # data-dependent: stays eager, splits the graph
        return z * 2 + idx.numel(), torch.tanh(z)

    backend = ThunderCompiler()
    cf = torch.compile(f, backend=backend, dynamic=False)
    x, y = torch.randn(6), torch.randn(6)
    out = cf(x, y)
    ref = f(x, y)
    for o, r in zip(out, ref):
        torch.testing.assert_close(o, r)
    report = split_report(backend.subgraph_infos)
    assert "graph 0" in report


def test_recipe_fx_interpreter():
    import lightning_thunder_amd as thunder
    from lightning_thunder_amd.recipes import BaseRecipe

    m = torch.nn.Sequential(torch.nn.Linear(4, 4), torch.nn.ReLU())
    cm = thunder.compile(m, recipe=BaseRecipe(fuser=None, interpreter="thunder.fx"))
    x = torch.randn(2, 4)
    torch.testing.assert_close(cm(x), m(x))
