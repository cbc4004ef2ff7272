"""HipGraphTransform tests (reference: ``thunder/tests/test_transforms.py`` CUDAGraph tests)."""
import os

import pytest
import torch

import lightning_thunder_amd as thunder
from lightning_thunder_amd.transforms.hipgraph import HipGraphRunner, HipGraphTransform, default_capturable


def test_region_structure_cpu():
    """Regions are formed (with a permissive capturability predicate on CPU) and run eagerly."""
    from lightning_thunder_amd.transforms import hipgraph as hg

    t = HipGraphTransform(is_capturable=lambda b: b.sym.id not in hg._NOT_CAPTURABLE_IDS and not hg._is_unpack(b))
    m = torch.nn.Sequential(torch.nn.Linear(8, 16), torch.nn.ReLU(), torch.nn.Linear(16, 4))
    jm = thunder.jit(m, transforms=[t])
    x = torch.randn(3, 8)
    y = jm(x)
    torch.testing.assert_close(y, m(x))
    y.sum().backward()
    fw = thunder.last_traces(jm)[-1]
    bw = thunder.last_backward_traces(jm)[-1]
    assert any(b.sym.name.startswith("HipGraph") for b in fw.bound_symbols)
    assert any(b.sym.name.startswith("HipGraph") for b in bw.bound_symbols)


def test_cpu_ops_not_capturable():
    m = torch.nn.Linear(4, 4)
    jm = thunder.jit(m, transforms=[HipGraphTransform()])
    jm(torch.randn(2, 4))
    assert not any(b.sym.name.startswith("HipGraph") for b in thunder.last_traces(jm)[-1].bound_symbols)


@pytest.mark.gpu
def test_hipgraph_training_matches_eager_gpu():
    torch.manual_seed(0)

    def make():
        torch.manual_seed(0)
        return torch.nn.Sequential(torch.nn.Linear(64, 256), torch.nn.GELU(), torch.nn.Linear(256, 64)).cuda()

    m_ref, m_g = make(), make()
    t = HipGraphTransform()
    jm = thunder.jit(m_g, transforms=[t])
    opt_r = torch.optim.SGD(m_ref.parameters(), lr=0.1)
    opt_g = torch.optim.SGD(m_g.parameters(), lr=0.1)
    for step in range(5):
        x = torch.randn(32, 64, device="cuda")
        lr = m_ref(x).square().mean()
        lg = jm(x).square().mean()
        lr.backward()
        lg.backward()
        opt_r.step(); opt_r.zero_grad(set_to_none=True)
        opt_g.step(); opt_g.zero_grad(set_to_none=True)
        torch.testing.assert_close(lg, lr, rtol=1e-4, atol=1e-5)
    for pr, pg in zip(m_ref.parameters(), m_g.parameters()):
        torch.testing.assert_close(pg, pr, rtol=1e-4, atol=1e-5)
    assert sum(r.replays for r in t.runners) >= 4
    assert sum(r.captures for r in t.runners) >= 2


@pytest.mark.gpu
def test_hipgraph_with_hip_kernels_gpu():
    """A LitGPT block step (HIP attention / RMSNorm / RoPE / SwiGLU kernels) replays correctly."""
    from lightning_thunder_amd.models.litgpt import GPT, Config

    torch.manual_seed(0)
    cfg = Config.from_name("llama2-like", n_layer=2)
    m = GPT(cfg).cuda().to(torch.bfloat16)
    m.set_rope_cache(128, device="cuda")
    t = HipGraphTransform()
    jm = thunder.jit(m, transforms=[t])
    jplain = thunder.jit(m)
    for _ in range(3):
        x = torch.randint(0, cfg.vocab_size, (2, 128), device="cuda")
        out = jm(x)
        ref = jplain(x)
        torch.testing.assert_close(out, ref)
        out.float().sum().backward()
    assert sum(r.replays for r in t.runners) >= 1


def test_region_marks_only_written_inputs_cpu():
    """Only the destination of an in-place op is a written input: the index and source of a cache
    update stay read-only (private clones, no write-back)."""
    from lightning_thunder_amd.transforms import hipgraph as hg

    t = HipGraphTransform(is_capturable=lambda b: b.sym.id not in hg._NOT_CAPTURABLE_IDS and not hg._is_unpack(b))

    def f(cache, pos, val):
        cache.index_copy_(0, pos, val)
        return cache * 2

    jf = thunder.jit(f, transforms=[t])
    cache, pos, val = torch.zeros(6, 3), torch.tensor([1, 4]), torch.ones(2, 3)
    out = jf(cache, pos, val)
    torch.testing.assert_close(out, f(torch.zeros(6, 3), pos, val))
    trace = str(thunder.last_traces(jf)[-1])
    assert "index_copy_inplace" in trace or "copy_" in trace, trace
    (r,) = [r for r in t.runners]
    region = [b for b in thunder.last_traces(jf)[-1].bound_symbols if b.sym.name == r.name][0]
    names = [a.name for a in region.args]
    written = {n for n, m in zip(names, r.mutated_inputs) if m}
    caller = {n for n, p in zip(names, r.private_inputs) if p}
    assert len(written) == 1 and written <= caller, (names, r.mutated_inputs)
    assert len(caller) == 3


def test_written_args_table():
    from lightning_thunder_amd.core import prims
    from lightning_thunder_amd.core.proxies import TensorProxy
    from lightning_thunder_amd.core.trace import TraceCtx, tracectx
    from lightning_thunder_amd.transforms.inplace_index_copy import index_copy_inplace
    from lightning_thunder_amd.executors.hipex import hip_qkv_rope_cache

    with tracectx(TraceCtx()):
        a = TensorProxy(shape=(4, 4), device="cpu", dtype=torch.float32)
        b = TensorProxy(shape=(4, 4), device="cpu", dtype=torch.float32)
        i = TensorProxy(shape=(2,), device="cpu", dtype=torch.int64)
        s = TensorProxy(shape=(2, 4), device="cpu", dtype=torch.float32)
        cp = prims.copy_.bind(a, b, output=b)
        ic = index_copy_inplace.bind(a, 0, i, s, output=a)
        assert [p.name for p in prims.written_args(cp)] == [b.name]
        assert [p.name for p in prims.written_args(ic)] == [a.name]
        assert hip_qkv_rope_cache.written_args == (7, 8)
        # not in place: writes nothing
        assert prims.written_args(prims.python_return.bind(a, output=None)) == []


@pytest.mark.gpu
def test_runner_never_writes_other_callers_storage_gpu():
    """A graph captured on caller A's cache is not replayed for caller B's cache; B runs on private
    buffers with copy-in/back; read-only caller inputs are private clones; A stays intact."""
    def f(cache, pos, val):
        cache.index_copy_(0, pos, val)
        return (cache.sum(0),)

    t = HipGraphTransform()
    r = HipGraphRunner(f, "t", t, private_inputs=(True, True, True), mutated_inputs=(True, False, False))

    def run(cache, start, n, scale):
        ref = cache.clone()
        for p in range(start, start + n):
            pos = torch.tensor([p], device="cuda")
            val = torch.full((1, 4), float(p + 1) * scale, device="cuda")
            (s,) = r(cache, pos, val)
            ref[p] = val[0]
            torch.testing.assert_close(s, ref.sum(0))
            assert pos.item() == p  # caller's read-only input untouched
        torch.testing.assert_close(cache, ref)

    A = torch.zeros(16, 4, device="cuda")
    B = torch.zeros(16, 4, device="cuda")
    run(A, 0, 4, 1.0)
    snap_a = A.clone()
    run(B, 0, 6, -2.0)            # other storage: private graph, copied in and back
    torch.testing.assert_close(A, snap_a)
    B.zero_()                     # caller modifies its cache between calls: copy-in must not be skipped
    run(B, 6, 2, 3.0)
    run(A, 4, 3, 1.0)             # back on A: zero-copy bound graph
    assert r.captures == 2
    (ins_bound, _, _), = [e for k, e in r.entries.items() if not k[1]]
    assert ins_bound[0] is A and ins_bound[1] is not None


@pytest.mark.gpu
def test_capture_with_tuned_gemm_table_active():
    """The shipped TunableOp table is active for the GEMM selector; a hipGraph capture that runs a
    library GEMM first on the capture stream must still work (TunableOp off while capturing).
    Fresh process: the capture stream must not have a BLAS handle from earlier tests."""
    import subprocess
    import sys

    code = (
        "import torch, lightning_thunder_amd as thunder\n"
        "from lightning_thunder_amd.ops.gemm import enable_tuned_gemms\n"
        "from lightning_thunder_amd.transforms.hipgraph import HipGraphTransform\n"
        "assert enable_tuned_gemms() or True\n"
        "f = lambda a, b: (a @ b).sin() + 1\n"
        "jf = thunder.jit(f, transforms=[HipGraphTransform()])\n"
        "a = torch.randn(64, 32, device='cuda'); b = torch.randn(32, 48, device='cuda')\n"
        "for _ in range(3):\n"
        "    torch.testing.assert_close(jf(a, b), f(a, b), atol=1e-4, rtol=1e-4)\n"
        "print('OK')\n"
    )
    env = dict(os.environ)
    env["PYTHONPATH"] = os.path.dirname(os.path.dirname(os.path.abspath(__file__))) + os.pathsep + env.get("PYTHONPATH", "")
    env["LTA_TUNED_GEMMS"] = "1"  # opt-in
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=240, env=env)
    assert r.returncode == 0 and "OK" in r.stdout, r.stderr[-3000:]


class _FakeGraph:
    """CPU stand-in for a captured graph: replay re-runs the region on the captured inputs and writes
    the results into the captured outputs (the semantics of a hipGraph replay)."""

    def __init__(self, fn, ins, outs):
        self.fn, self.ins, self.outs = fn, ins, outs

    def replay(self):
        # .data aliases the storage with its own version counter: like a real replay, no version bump
        new = self.fn(*[a.data if isinstance(a, torch.Tensor) else a for a in self.ins])
        new = new if isinstance(new, tuple) else (new,)
        outs = self.outs() if callable(self.outs) else self.outs
        for o, n in zip(outs, new):
            o.copy_(n)


class _CpuRunner(HipGraphRunner):
    """HipGraphRunner whose capture builds a _FakeGraph (capture itself runs nothing on the inputs)."""

    def _capture(self, key, args, private):
        clone = set(self._clone) | (set(self._bound) if private else set())
        ins = tuple(a.clone() if i in clone and isinstance(a, torch.Tensor) else a for i, a in enumerate(args))
        outs = self.fn(*[a.clone() if isinstance(a, torch.Tensor) else a for a in ins])
        outs = tuple(outs) if isinstance(outs, (tuple, list)) else (outs,)
        if self.donate_outputs:  # a real graph holds no tensor objects: write through the stored storage
            from lightning_thunder_amd.transforms.hipgraph import _view_of

            g = _FakeGraph(self.fn, ins, lambda: [_view_of(m) for m in self.entries[key][2]])
        else:
            g = _FakeGraph(self.fn, ins, outs)
        return self._store(key, ins, g, outs)


def _write_rows(cache, x, pos):
    cache.index_copy_(0, pos, x)
    return cache.sum(0)


def _runner(owner):
    # inputs: cache (written in place), x and pos (caller-owned, read-only)
    return _CpuRunner(_write_rows, "HipGraphT", owner, private_inputs=(True, True, True),
                      mutated_inputs=(True, False, False))


def test_runner_epoch_invalidates_stale_writeback_cpu():
    """A bound replay of one signature writes cache B in-graph (no version bump); another signature's
    private graph must then copy B in again instead of trusting its last write-back."""
    owner = HipGraphTransform()
    r = _runner(owner)
    D = 4
    A, B = torch.zeros(8, D), torch.zeros(8, D)
    ref_B = torch.zeros(8, D)
    dec = lambda c, v, p: r(c, torch.full((1, D), float(v)), torch.tensor([p]))
    pre = lambda c, v: r(c, torch.full((4, D), float(v)), torch.arange(4))
    for v in range(3):  # decode signature: warm-up, then bound to A
        dec(A, v, 7)
    for v in range(2):  # prefill signature first seen with B: warm-up, then a graph bound to B
        pre(B, 10 + v)
    dec(B, 5, 6)  # decode on B: private graph, write-back recorded
    pre(B, 20)  # bound replay writes B's rows 0..3 in-graph: no version bump
    dec(B, 6, 5)  # private decode on B again: must copy B in, or it writes stale rows 0..3 back
    ref_B[:4] = 20
    ref_B[6] = 5
    ref_B[5] = 6
    torch.testing.assert_close(B, ref_B)
    assert r.replays >= 5


def test_runner_inference_mode_cpu():
    """Inference tensors carry no version counter: a private replay must copy them in."""
    owner = HipGraphTransform()
    r = _runner(owner)
    D = 4
    with torch.inference_mode():
        for gen in range(2):  # two "generate" calls, each with a fresh cache
            A = torch.zeros(8, D)
            for step in range(4):
                r(A, torch.full((1, D), float(gen * 10 + step)), torch.tensor([step]))
            torch.testing.assert_close(A[:4, 0], torch.tensor([gen * 10 + s for s in range(4)], dtype=A.dtype))


def test_donated_outputs_are_adopted_and_guarded_cpu():
    """donate_grads: a replay hands out fresh tensor objects over the graph's output storage (so
    AccumulateGrad can adopt them without a clone) and refuses to overwrite an output that is still
    referenced from the previous replay."""
    owner = HipGraphTransform(donate_grads=True)
    r = _CpuRunner(lambda x: (x * 2.0,), "HipGraphD", owner, private_inputs=(True,), donate_outputs=True)
    x = torch.ones(4)
    r(x)  # warm-up (eager)
    a = r(x)[0]  # capture
    torch.testing.assert_close(a, x * 2)
    ptr = a.data_ptr()
    del a
    b = r(x + 1)[0]  # replay: same storage, fresh tensor object
    assert b.data_ptr() == ptr
    torch.testing.assert_close(b, (x + 1) * 2)
    with pytest.raises(RuntimeError, match="still referenced"):
        r(x)  # b is alive: the replay would overwrite it
    del b
    torch.testing.assert_close(r(x)[0], x * 2)


def test_graph_rng_draws_and_torch_philox_cpu():
    """Graph-safe RNG (core/rng.py): inside a runner's context the draws are GraphRngInt seeds / offsets
    relative to the region's base; the torch Philox reads seed and base from the device state and gives
    exactly the uncaptured values; a warm-up context draws the same counter ranges as plain draws."""
    from lightning_thunder_amd.core import rng

    rng._state["seed"] = None
    torch.manual_seed(7)
    plain = [rng.next_seed_offset(n) for n in (100, 40, 12)]
    rng._state["seed"] = None
    state = torch.zeros(2, dtype=torch.int64)
    written = []

    def first_draw(st):
        seed, base = rng.peek_seed_offset()
        st[0], st[1] = seed, base
        written.append((seed, base))

    ctx = rng.GraphRngContext(state, on_first_draw=first_draw)
    rng.set_graph_context(ctx)
    try:
        draws = [rng.seed_offset_for(n) for n in (100, 40, 12)]
    finally:
        rng.set_graph_context(None)
    rng.advance_offset(ctx.total)
    assert rng.peek_seed_offset()[1] == plain[-1][1] + 12  # the counter ends where plain draws end
    assert len(written) == 1 and ctx.total == 152
    for (s_ref, o_ref), (s, o) in zip(plain, draws):
        assert type(s) is rng.GraphRngInt and type(o) is rng.GraphRngInt and o.state is state
        assert int(state[1]) + int(o) == o_ref and int(state[0]) == s_ref
        got = rng.philox_uniform_torch((5, 7), s, o, "cpu")
        want = rng.philox_uniform_torch((5, 7), s_ref, o_ref, "cpu")
        assert torch.equal(got, want)
    # runner keys tell graph draws of different regions apart
    other = torch.zeros(2, dtype=torch.int64)
    k1 = HipGraphRunner._key((rng.GraphRngInt(0, state, "offset"),))
    k2 = HipGraphRunner._key((rng.GraphRngInt(0, other, "offset"),))
    assert k1 != k2


def test_graph_rng_codegen_reads_device_state_cpu():
    """A hipfuse region whose Philox seed / offset are graph draws reads them from the state pointers
    appended after the numbers (seed and base from the state, offset relative)."""
    from lightning_thunder_amd.executors import hipfuse
    from lightning_thunder_amd.executors import hipfuse_codegen as cg
    from lightning_thunder_amd.core.proxies import TensorProxy

    old = hipfuse.ex.allow_cpu
    hipfuse.ex.allow_cpu = True
    try:
        def f(x):
            return torch.nn.functional.dropout(x * 2.0, p=0.3, training=True)

        jf = thunder.jit(f, executors=["hipfuse", "torch"])
        jf(torch.randn(64, 128, requires_grad=True))
        fus = [fb for fb in hipfuse.fusions(thunder.last_traces(jf)[-1])
               if "uniform_philox" in str(fb.subsymbols)]
        assert fus
        h = fus[0]._call_ctx[fus[0].sym.name]
        nums = [h.inputs[i] for i in h.number_pos]
        assert len(nums) >= 2
        targs = {p.name: cg.TensorArg(tuple(p.shape), tuple(torch.empty(tuple(p.shape)).stride()), p.dtype, True)
                 for p in h.inputs if isinstance(p, TensorProxy)}
        plain = cg.generate(h.plan, h.inputs, h.outputs, targs)
        rngmap = {nums[0].name: (0, "seed"), nums[1].name: (0, "offset")}
        g = cg.generate(h.plan, h.inputs, h.outputs, targs, rng=rngmap)
        assert "A.rng[" not in plain.src and "const long long* rng[1];" in g.src
        assert "rng_seed0 = A.rng[0][0], rng_base0 = A.rng[0][1]" in g.src and "rng_base0 +" in g.src
        hipfuse.compile_source(g)  # hiprtc compiles it (no GPU needed)
    finally:
        hipfuse.ex.allow_cpu = old


@pytest.mark.gpu
def test_hipgraph_dropout_training_matches_uncaptured_gpu():
    """A dropout model (NanoGPT blocks, dropout 0.1: hipfuse Philox regions and attention dropout) under
    HipGraphTransform: the RNG draws no longer split the trace into per-dropout regions, replays draw
    fresh masks, and every step's loss and gradients equal the uncaptured compiled run's (same counter
    ranges in the same order)."""
    from lightning_thunder_amd.core import rng
    from lightning_thunder_amd.models.nanogpt import NanoGPT, NanoGPTConfig

    cfg = NanoGPTConfig(n_layer=2, n_head=4, n_embd=256, seq_len=128, block_size=128, vocab_size=512, dropout=0.1)

    def run(graphs):
        torch.manual_seed(0)
        m = NanoGPT(cfg).to(device="cuda", dtype=torch.bfloat16)
        t = HipGraphTransform()
        jm = thunder.jit(m, transforms=[t] if graphs else [])
        rng._state["seed"] = None
        torch.manual_seed(11)
        out = []
        for step in range(5):
            g = torch.Generator(device="cuda").manual_seed(step)
            x = torch.randint(0, 512, (4, 128), device="cuda", generator=g)
            y = torch.randint(0, 512, (4, 128), device="cuda", generator=g)
            _, loss = jm(x, y)
            loss.backward()
            out.append((loss.detach().clone(), [p.grad.clone() for p in m.parameters()]))
            for p in m.parameters():
                p.grad = None
        return out, t, jm

    ref, _, _ = run(False)
    got, t, jm = run(True)
    for (lr, gr), (lg, gg) in zip(ref, got):
        torch.testing.assert_close(lg, lr, rtol=0, atol=0)
        for a, b in zip(gg, gr):
            torch.testing.assert_close(a, b, rtol=0, atol=0)
    fw = thunder.last_traces(jm)[-1]
    assert sum(b.sym.name.startswith("HipGraph") for b in fw.bound_symbols) <= 2, \
        [b.sym.name for b in fw.bound_symbols]
    assert sum(r.replays for r in t.runners) >= 3 and any(r._rng for r in t.runners)
