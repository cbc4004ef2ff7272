"""ThunderFX battery (reference model: ``thunder/tests/test_dynamo.py``): programs handed to
``torch.compile(backend=ThunderCompiler())`` with graph breaks, Python side effects, buffers,
no-grad / autocast regions, activation checkpointing and dynamic sizes; forward values and input
gradients must match eager PyTorch, and each program must compile at least one subgraph through
thunder.
"""
import pytest
import torch
import torch.utils.checkpoint

from lightning_thunder_amd.dynamo import ThunderCompiler


class _Buffers(torch.nn.Module):
    def __init__(self):
        super().__init__()
        self.lin = torch.nn.Linear(6, 6)
        self.register_buffer("scale", torch.full((6,), 0.5))

    def forward(self, x):
        return torch.relu(self.lin(x)) * self.scale + x


class _GraphBreak(torch.nn.Module):
    def __init__(self):
        super().__init__()
        self.a = torch.nn.Linear(6, 6)
        self.b = torch.nn.Linear(6, 6)

    def forward(self, x):
        y = self.a(x).tanh()
        if y.sum().item() > 1e9:  # data-dependent Python: dynamo breaks the graph here
            y = y * 2
        return self.b(y).sigmoid()


class _NoGradInside(torch.nn.Module):
    def __init__(self):
        super().__init__()
        self.lin = torch.nn.Linear(6, 6)

    def forward(self, x):
        with torch.no_grad():
            stats = x.abs().mean(0)
        return self.lin(x) * (1 + stats)


class _Checkpointed(torch.nn.Module):
    def __init__(self):
        super().__init__()
        self.blk = torch.nn.Sequential(torch.nn.Linear(6, 12), torch.nn.GELU(), torch.nn.Linear(12, 6))

    def forward(self, x):
        return torch.utils.checkpoint.checkpoint(self.blk, x, use_reentrant=False) + x


class _MultiOutput(torch.nn.Module):
    def __init__(self):
        super().__init__()
        self.lin = torch.nn.Linear(6, 4)

    def forward(self, x):
        h = self.lin(x)
        return {"logits": h, "probs": h.softmax(-1), "pair": (h.max(-1).values, h.argmax(-1))}


class _Attention(torch.nn.Module):
    def __init__(self):
        super().__init__()
        self.qkv = torch.nn.Linear(6, 18)

    def forward(self, x):
        q, k, v = self.qkv(x).unsqueeze(1).chunk(3, dim=-1)
        return torch.nn.functional.scaled_dot_product_attention(q, k, v, is_causal=True).squeeze(1)


class _Autocast(torch.nn.Module):
    def __init__(self):
        super().__init__()
        self.lin = torch.nn.Linear(6, 6)

    def forward(self, x):
        with torch.autocast("cpu", dtype=torch.bfloat16):
            y = self.lin(x)
        return y.float().tanh()


def _fn_side_effects(x):
    log = []
    y = x.sin()
    log.append(y.shape[0])  # a Python side effect dynamo replays
    return y * len(log) + x.cos()


def _fn_inplace(x):
    y = x.clone()
    y.mul_(3).add_(1)
    y[:, 0] = 0
    return y.exp().sum(-1)


PROGRAMS = {
    "buffers": _Buffers, "graph_break": _GraphBreak, "no_grad_inside": _NoGradInside, "checkpoint": _Checkpointed,
    "multi_output": _MultiOutput, "sdpa": _Attention, "autocast": _Autocast,
    "side_effects": lambda: _fn_side_effects, "inplace": lambda: _fn_inplace,
}


def _flat(o):
    if isinstance(o, dict):
        return [t for v in o.values() for t in _flat(v)]
    if isinstance(o, (tuple, list)):
        return [t for v in o for t in _flat(v)]
    return [o]


@pytest.mark.parametrize("name", sorted(PROGRAMS))
@pytest.mark.parametrize("dynamic", [False, True])
def test_thunderfx_program(name, dynamic):
    torch._dynamo.reset()
    torch.manual_seed(0)
    prog = PROGRAMS[name]()
    backend = ThunderCompiler()
    compiled = torch.compile(prog, backend=backend, dynamic=dynamic)
    for rows in (5, 7):
        x = torch.randn(rows, 6, requires_grad=True)
        x2 = x.detach().clone().requires_grad_(True)
        out = compiled(x)
        ref = prog(x2)
        for a, b in zip(_flat(out), _flat(ref)):
            if a.dtype.is_floating_point and b.dtype.is_floating_point and a.dtype == torch.bfloat16:
                torch.testing.assert_close(a.float(), b.float(), atol=2e-2, rtol=2e-2)
            else:
                torch.testing.assert_close(a, b)
        loss = sum(t.float().sum() for t in _flat(out) if t.dtype.is_floating_point and t.requires_grad)
        rloss = sum(t.float().sum() for t in _flat(ref) if t.dtype.is_floating_point and t.requires_grad)
        if isinstance(loss, torch.Tensor):
            loss.backward()
            rloss.backward()
            torch.testing.assert_close(x.grad, x2.grad, atol=2e-2, rtol=2e-2)
    compiled_fns = sum(len(i.thunder_compiled_fns) for i in backend.subgraph_infos)
    assert compiled_fns >= 1, [i.split_reasons for i in backend.subgraph_infos]
