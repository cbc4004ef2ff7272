"""Optimizer step overlapped with the backward (transforms/optimizer_overlap.py).

CPU: the grad-ready hooks sit after each parameter's last read in the backward, and a model trained
with updates issued from inside the backward equals the usual backward-then-step run.
GPU: the fused AdamW on the side stream (lean kernel) equals the post-backward fused AdamW.
"""
import pytest
import torch

import lightning_thunder_amd as thunder
from lightning_thunder_amd.optim import AdamW
from lightning_thunder_amd.transforms.optimizer_overlap import _is_view, may_alias_bsym


class _CPUOverlapAdamW(AdamW):
    """AdamW whose in-backward updates run immediately with torch ops (CPU tensors)."""

    def manages(self, t):
        return isinstance(t, torch.Tensor) and id(t) in self._managed

    @torch.no_grad()
    def overlapped_update(self, params, grads):
        self._mark_handled(params)
        self.calls = getattr(self, "calls", 0) + 1
        for p, g in zip(params, grads):
            group = self._managed[id(p)]
            st = self._state(p)
            st["step"] += 1
            p.grad = g
            self._torch_step(p, st, group["lr"], *group["betas"], group["eps"], group["weight_decay"])
            p.grad = None


def _mlp():
    torch.manual_seed(0)
    return torch.nn.Sequential(torch.nn.Linear(32, 64), torch.nn.GELU(), torch.nn.Linear(64, 64), torch.nn.GELU(),
                               torch.nn.Linear(64, 16))


def _train(model, opt, steps=3, overlap=False):
    jm = thunder.jit(model)
    if overlap:
        opt.overlap_with_backward(jm, bucket_mb=0)  # every ready point its own bucket
    torch.manual_seed(1)
    xs = [torch.randn(8, 32) for _ in range(steps)]
    for x in xs:
        loss = jm(x).square().mean()
        loss.backward()
        opt.step()
        opt.zero_grad(set_to_none=True)
    return jm


def test_updates_inside_backward_match_post_backward_step():
    ref = _mlp()
    o_ref = torch.optim.AdamW(ref.parameters(), lr=1e-2, betas=(0.9, 0.95), weight_decay=0.1)
    _train(ref, o_ref)
    m = _mlp()
    opt = _CPUOverlapAdamW(m.parameters(), lr=1e-2, betas=(0.9, 0.95), weight_decay=0.1)
    jm = _train(m, opt, overlap=True)
    assert opt.calls >= 3 * 3, opt.calls  # several buckets per backward
    for p, q in zip(m.parameters(), ref.parameters()):
        torch.testing.assert_close(p, q, rtol=1e-5, atol=1e-6)
    bw = thunder.last_backward_traces(jm)[-1]
    hooks = [b for b in bw.bound_symbols if str(b.sym.name).startswith("optim_grad_ready")]
    assert hooks
    # every hook comes after the last read of each parameter whose gradient it hands over
    names = [str(b.sym.name) for b in bw.bound_symbols]
    for h in hooks:
        hi = names.index(str(h.sym.name))
        for g in h.args[1:]:
            for j, b in enumerate(bw.bound_symbols):
                if any(o.name == g.name for o in b.flat_proxy_outs):
                    assert j < hi


def test_hooks_wait_for_the_last_parameter_read():
    """The weight of the first linear is read by no backward op (its input needs no gradient), but the
    second layer's weight is read by the dgrad that feeds the first layer: its hook must follow it."""
    from lightning_thunder_amd.transforms.optimizer_overlap import insert_grad_ready_hooks

    m = _mlp()
    jm = thunder.jit(m)
    jm(torch.randn(8, 32)).sum().backward()
    bw = thunder.last_backward_traces(jm)[0]  # pre-execution backward: plain prims / torch symbols
    comp = thunder.last_traces(jm)[0]
    names = [a.name for a in comp.args if hasattr(a, "requires_grad") and a.requires_grad]
    new = insert_grad_ready_hooks(bw, names, bucket_bytes=0)
    bs = new.bound_symbols
    pos = {}
    for i, b in enumerate(bs):
        if str(b.sym.name).startswith("optim_grad_ready"):
            for k in b.args[0]:
                pos[k] = i
    assert pos
    for k, i in pos.items():
        pname = names[k]
        alias = {pname}
        for j, b in enumerate(bs):
            if _is_view(b) and any(a.name in alias for a in b.flat_proxy_args):
                alias |= {o.name for o in b.flat_proxy_outs}
            if j > i and any(a.name in alias for a in b.flat_proxy_args) and not str(b.sym.name).startswith("optim_"):
                if b.sym.name not in ("python_return", "python_del"):
                    raise AssertionError(f"{pname} read by {b.sym.name} after its update hook")


def test_second_backward_update_in_one_iteration_raises():
    """Two calls of the jitted model before one backward: two backward nodes would each hand over a
    partial gradient and the parameter would get two AdamW steps; the optimizer refuses."""
    m = _mlp()
    opt = _CPUOverlapAdamW(m.parameters(), lr=1e-2)
    jm = thunder.jit(m)
    opt.overlap_with_backward(jm, bucket_mb=0)
    x1, x2 = torch.randn(8, 32), torch.randn(8, 32)
    with pytest.raises(RuntimeError, match="updated twice"):
        (jm(x1).sum() + jm(x2).sum()).backward()
    # one call per backward keeps working after a step() clears the iteration's record
    opt._handled.clear()
    opt.zero_grad(set_to_none=True)
    jm(x1).sum().backward()
    opt.step()
    jm(x2).sum().backward()
    opt.step()


def test_updated_param_with_grad_from_another_path_raises():
    m = _mlp()
    opt = _CPUOverlapAdamW(m.parameters(), lr=1e-2)
    jm = thunder.jit(m)
    opt.overlap_with_backward(jm, bucket_mb=0)
    w = m[0].weight
    (jm(torch.randn(8, 32)).sum() + w.square().sum()).backward()  # eager use of w outside the program
    assert w.grad is not None
    with pytest.raises(RuntimeError, match="also has p.grad"):
        opt.step()


class _ContiguousWeight(torch.nn.Module):
    def __init__(self):
        super().__init__()
        torch.manual_seed(0)
        self.w = torch.nn.Parameter(torch.randn(32, 32))
        self.v = torch.nn.Parameter(torch.randn(32, 32))

    def forward(self, x):
        wc = self.w.contiguous()  # may return w itself at run time: an alias saved for the backward
        h = torch.tanh(x @ wc.t())
        h = torch.tanh(h @ self.v.t())
        return (h @ wc).sum()  # wc read again late in the backward (dgrad of the last product)


def test_hook_waits_for_reads_through_identity_ops():
    """``contiguous(w)`` saved in the forward is read late in the backward: the update hook of w must
    follow that read (an early hook would let the side-stream AdamW write w while it is still read)."""
    from lightning_thunder_amd.transforms.optimizer_overlap import insert_grad_ready_hooks

    m = _ContiguousWeight()
    jm = thunder.jit(m)
    jm(torch.randn(8, 32)).backward()
    bw = thunder.last_backward_traces(jm)[0]
    fw = thunder.last_traces(jm)[0]
    comp = thunder.last_traces(jm)[0]
    names = [a.name for a in comp.args if hasattr(a, "requires_grad") and a.requires_grad]
    new = insert_grad_ready_hooks(bw, names, bucket_bytes=0, fw=fw)
    alias = {}
    for tr in (fw, new):
        for b in tr.bound_symbols:
            if may_alias_bsym(b):
                srcs = [a.name for a in b.flat_proxy_args if hasattr(a, "shape")]
                if srcs:
                    for o in b.flat_proxy_outs:
                        alias[o.name] = alias.get(srcs[0], srcs[0])
    bs = new.bound_symbols
    checked = 0
    for i, b in enumerate(bs):
        if not str(b.sym.name).startswith("optim_grad_ready"):
            continue
        for k in b.args[0]:
            pname = names[k]
            for j in range(i + 1, len(bs)):
                bj = bs[j]
                if str(bj.sym.name) in ("python_return", "python_del") or str(bj.sym.name).startswith("optim_"):
                    continue
                for a in bj.flat_proxy_args:
                    assert alias.get(a.name, a.name) != pname, f"{pname} read through {a.name} after its hook"
            checked += 1
    assert checked >= 1


def test_may_alias_bsym_identity_ops():
    def f(x):
        a = x.contiguous()
        b = x.to(torch.float32)
        c = x.to(torch.float64)
        return a, b, c

    jf = thunder.jit(f)
    jf(torch.randn(4, 4))
    tr = thunder.last_traces(jf)[0]
    flags = {str(b.sym.name): may_alias_bsym(b) for b in tr.bound_symbols if b.flat_proxy_args}
    assert flags.get("contiguous") is True
    conv = [may_alias_bsym(b) for b in tr.bound_symbols if str(b.sym.name) in ("to", "convert_element_type")]
    assert conv == [False], flags  # x.to(float32) of a float32 x is x itself in the trace; float64 allocates


@pytest.mark.gpu
def test_fused_adamw_overlapped_with_backward_gpu():
    torch.manual_seed(0)
    dims = [(512, 1024), (1024, 1024), (1024, 512)]

    def make():
        torch.manual_seed(0)
        layers = []
        for i, (a, b) in enumerate(dims):
            layers += [torch.nn.Linear(a, b)] + ([torch.nn.GELU()] if i < len(dims) - 1 else [])
        return torch.nn.Sequential(*layers).to("cuda", torch.bfloat16)

    m1, m2 = make(), make()
    o1 = AdamW(m1.parameters(), lr=1e-3, betas=(0.9, 0.95), weight_decay=0.1)
    o2 = AdamW(m2.parameters(), lr=1e-3, betas=(0.9, 0.95), weight_decay=0.1)
    j1, j2 = thunder.jit(m1), thunder.jit(m2)
    o2.overlap_with_backward(j2, bucket_mb=1)
    for s in range(4):
        x = torch.randn(256, 512, device="cuda", dtype=torch.bfloat16)
        for j, o in ((j1, o1), (j2, o2)):
            j(x).float().square().mean().backward()
            o.step()
            o.zero_grad(set_to_none=True)
        if s == 0:
            assert all(p.grad is None for p in m2.parameters())  # handled inside the backward
    torch.cuda.synchronize()
    for p, q in zip(m1.parameters(), m2.parameters()):
        torch.testing.assert_close(p, q, rtol=0, atol=0)
    assert o2._side, "no update ran on the side stream"


def test_failed_step_leaves_state_untouched():
    """A step() that rejects a parameter updated in the backward AND carrying p.grad raises before
    any state changes: no step counts move and the handled set survives for a consistent retry."""
    from lightning_thunder_amd.optim import AdamW

    a = torch.nn.Parameter(torch.randn(4))
    b = torch.nn.Parameter(torch.randn(4))
    opt = AdamW([a, b], lr=1e-2)
    a.grad = torch.randn(4)
    b.grad = torch.randn(4)
    opt._handled.add(id(b))
    a0 = a.detach().clone()
    with pytest.raises(RuntimeError, match="updated in the backward"):
        opt.step()
    assert not opt.state[a] or opt.state[a]["step"] == 0
    assert torch.equal(a.detach(), a0)
    assert id(b) in opt._handled
