"""hipfuse (K1 fusion codegen) tests.

CPU: partitioning (regions, inputs/outputs) checked by running each region's prims through
the torch reference path, and every generated kernel is compiled with hiprtc for gfx950.
GPU: generated kernels vs a PyTorch fp32 reference of the same function.
(Reference test model: ``thunder/tests/test_nvfuser.py`` fusion-structure + numerics tests.)
"""
import os

import pytest
import torch

import lightning_thunder_amd as thunder
from lightning_thunder_amd.core.prims import PrimIDs
from lightning_thunder_amd.core.proxies import TensorProxy
from lightning_thunder_amd.executors import hipfuse
from lightning_thunder_amd.executors import hipfuse_codegen as cg

LIB = os.path.join(os.path.dirname(thunder.__file__), "ops", "_lta_kernels.so")


def _layer_norm_gelu_softmax(x, w, b):
    y = torch.nn.functional.layer_norm(x, (x.shape[-1],), w, b)
    z = torch.nn.functional.gelu(y, approximate="tanh") * 2.0 + x
    s = torch.softmax(z, -1)
    return s.sum(-1), z


def _rms(x, w):
    xf = x.float()
    r = torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + 1e-6)
    return (xf * r).to(x.dtype) * w


def _pointwise_bcast(a, b, c):
    return torch.where(a > 0, a * b + c, torch.exp(a) - 1.0), torch.sigmoid(a) * b


def _silu_mul(a, b):
    return torch.nn.functional.silu(a) * b


def _log_softmax_nll(x):
    return torch.log_softmax(x, -1).amax(-1)


def _bias_grad(dy):
    return (dy * 0.5).sum(0)


def _ln_dgamma_dbeta(dy, x, mean, rstd):
    xhat = (x - mean) * rstd
    return (dy * xhat).sum(0), dy.sum(0)


def _col_amax_epilogue(x):
    return x.abs().amax(dim=(0, 1)) * 0.5 + 1.0


def _full_and_col(a, b):
    y = torch.tanh(a) * b
    return y, y.sum(0)


def _split_grad_pad(dq, dk, dv):
    # the backward of a qkv split: the q / k / v gradients padded into d(qkv) and summed (one kernel)
    n = dq.shape[-1]
    g = torch.nn.functional.pad(dq, (0, 2 * n)) + torch.nn.functional.pad(dk, (n, n))
    return (g + torch.nn.functional.pad(dv, (2 * n, 0))) * 0.5


def _transpose_mix(x, y):
    # a transposed input and a transposed intermediate inside one region
    z = torch.tanh(x.t()) * 2.0 + y
    return z, (z * z).t() + x


CASES = {
    "ln_gelu_softmax": (_layer_norm_gelu_softmax, lambda dt, d: (torch.randn(4, 8, 256, device=d, dtype=dt),
                                                                  torch.randn(256, device=d, dtype=dt),
                                                                  torch.randn(256, device=d, dtype=dt))),
    "rmsnorm": (_rms, lambda dt, d: (torch.randn(2, 64, 4096, device=d, dtype=dt), torch.randn(4096, device=d, dtype=dt))),
    "pointwise_bcast": (_pointwise_bcast, lambda dt, d: (torch.randn(16, 32, 40, device=d, dtype=dt),
                                                         torch.randn(32, 1, device=d, dtype=dt),
                                                         torch.randn(40, device=d, dtype=dt))),
    "silu_mul": (_silu_mul, lambda dt, d: (torch.randn(3, 1000, device=d, dtype=dt), torch.randn(3, 1000, device=d, dtype=dt))),
    "log_softmax_amax": (_log_softmax_nll, lambda dt, d: (torch.randn(512, 1000, device=d, dtype=dt),)),
    # column (leading-dim) reductions: bias-grad and LayerNorm dgamma/dbeta shapes
    "bias_grad": (_bias_grad, lambda dt, d: (torch.randn(2048, 384, device=d, dtype=dt),)),
    "ln_dgamma_dbeta": (_ln_dgamma_dbeta, lambda dt, d: (torch.randn(1024, 768, device=d, dtype=dt),
                                                          torch.randn(1024, 768, device=d, dtype=dt),
                                                          torch.randn(1024, 1, device=d, dtype=dt),
                                                          torch.rand(1024, 1, device=d, dtype=dt) + 0.5)),
    "col_amax_epilogue": (_col_amax_epilogue, lambda dt, d: (torch.randn(8, 64, 96, device=d, dtype=dt),)),
    "full_and_col": (_full_and_col, lambda dt, d: (torch.randn(300, 200, device=d, dtype=dt),
                                                    torch.randn(300, 200, device=d, dtype=dt))),
}
CASES["pad_sum"] = (_split_grad_pad, lambda dt, d: tuple(torch.randn(4, 16, 64, device=d, dtype=dt) for _ in range(3)))
CASES["transpose_mix"] = (_transpose_mix, lambda dt, d: (torch.randn(96, 160, device=d, dtype=dt),
                                                          torch.randn(160, 96, device=d, dtype=dt)))


# shape / index ops on region inputs: affine (slice, viewable reshape), piecewise (cat) and
# indirect (index_select / gather / embedding) loads
def _slice_mix(x):
    n = x.shape[-1] // 3
    q, k, v = x[..., :n], x[..., n:2 * n], x[..., 2 * n:]
    return q * torch.sigmoid(k) + v[..., ::1] * x[..., ::3]


def _cat_mix(a, b, c):
    # last-dim cat with VEC-aligned pieces, a misaligned (5 + 11) last-dim cat, a leading-dim cat
    y = torch.cat([a, b], dim=-1) * 2.0 + c
    z = torch.cat([c[..., :5], c[..., 5:16]], -1)
    w = torch.cat([a, b, a], dim=0)
    return y, z.tanh() + 1.0, w * 3.0


def _gather_mix(w, idx, x, gidx):
    e = torch.index_select(w, 0, idx) + 1.0
    g = torch.gather(x, 1, gidx) * 2.0
    h = torch.index_select(w, 0, torch.minimum(idx + 1, torch.full_like(idx, 99))) * 0.5  # an in-region index
    return e.sin(), g.tanh(), h.cos()


def _embed_add(ids, wte, wpe):
    pos = torch.arange(ids.shape[1], device=ids.device)
    return (torch.nn.functional.embedding(ids, wte) + torch.nn.functional.embedding(pos, wpe)) * 0.5


def _reshape_ext(x, yt):
    # a viewable (contiguous) reshape and a copy-requiring one (``yt`` is a transposed input) of inputs
    return x.reshape(8, 4, 24) * yt.reshape(8, 4, 24) + 1.0, (x.reshape(16, 48) - yt.reshape(16, 48)).abs()


def _cat_inputs(dt, d):
    return (torch.randn(6, 32, 64, device=d, dtype=dt), torch.randn(6, 32, 64, device=d, dtype=dt),
            torch.randn(6, 32, 128, device=d, dtype=dt))


def _gather_inputs(dt, d):
    return (torch.randn(100, 48, device=d, dtype=dt), torch.randint(0, 100, (37,), device=d),
            torch.randn(16, 40, device=d, dtype=dt), torch.randint(0, 40, (16, 24), device=d))


def _two_reductions(x):
    # a column reduction and a row softmax-sum of the same elementwise value: two regions; the
    # second recomputes tanh(x) * 3 from x instead of reading a materialised copy
    a = torch.tanh(x) * 3.0
    return a.sum(0), (a - a.amax(1, keepdim=True)).exp().sum(1)


def _scatter_region(a, idx, src, b, pidx, vals):
    # a region closed by scatter (source computed in it) and one closed by index_put
    s = torch.scatter(a, 1, idx, torch.tanh(src) * 2.0)
    t = b.index_put((pidx,), vals.sin() + 1.0)
    return s, t


def _scatter_inputs(dt, d):
    g = torch.Generator(device="cpu").manual_seed(3)
    idx = torch.stack([torch.randperm(96, generator=g)[:40] for _ in range(24)]).to(d)  # unique per row
    pidx = torch.randperm(300, generator=g)[:77].to(d)
    return (torch.randn(24, 96, device=d, dtype=dt), idx, torch.randn(24, 40, device=d, dtype=dt),
            torch.randn(300, 64, device=d, dtype=dt), pidx, torch.randn(77, 64, device=d, dtype=dt))


CASES["scatter_region"] = (_scatter_region, _scatter_inputs)
CASES["remat_regions"] = (_two_reductions, lambda dt, d: (torch.randn(256, 512, device=d, dtype=dt),))
CASES["slice_mix"] = (_slice_mix, lambda dt, d: (torch.randn(4, 32, 3 * 96, device=d, dtype=dt),))
CASES["cat_mix"] = (_cat_mix, _cat_inputs)
CASES["gather_mix"] = (_gather_mix, _gather_inputs)
CASES["embed_add"] = (_embed_add, lambda dt, d: (torch.randint(0, 500, (4, 64), device=d),
                                                 torch.randn(500, 128, device=d, dtype=dt),
                                                 torch.randn(64, 128, device=d, dtype=dt)))
CASES["reshape_ext"] = (_reshape_ext, lambda dt, d: (torch.randn(32, 24, device=d, dtype=dt),
                                                      torch.randn(24, 32, device=d, dtype=dt).t()))
_COLUMN_CASES = ("bias_grad", "ln_dgamma_dbeta", "col_amax_epilogue", "full_and_col")
_SHAPE_CASES = ("slice_mix", "cat_mix", "gather_mix", "embed_add", "reshape_ext", "scatter_region")


@pytest.fixture
def cpu_fusion():
    old = hipfuse.ex.allow_cpu
    hipfuse.ex.allow_cpu = True
    yield
    hipfuse.ex.allow_cpu = old


@pytest.mark.parametrize("case", sorted(CASES))
def test_partition_cpu(case, cpu_fusion):
    fn, mk = CASES[case]
    args = mk(torch.float32, "cpu")
    jf = thunder.jit(fn, executors=["hipfuse", "torch"])
    out = jf(*args)
    ref = fn(*args)
    out = out if isinstance(out, tuple) else (out,)
    ref = ref if isinstance(ref, tuple) else (ref,)
    for o, r in zip(out, ref):
        torch.testing.assert_close(o, r, rtol=1e-5, atol=1e-5)
    fus = hipfuse.fusions(thunder.last_traces(jf)[-1])
    assert fus, "expected at least one hipFusion region"


@pytest.mark.parametrize("case", _COLUMN_CASES)
def test_column_reductions_fused_cpu(case, cpu_fusion):
    """Reductions over the leading dims (bias-grad, LayerNorm dgamma/dbeta) are claimed by ONE
    column-mode region, not left to ATen."""
    fn, mk = CASES[case]
    jf = thunder.jit(fn, executors=["hipfuse", "torch"])
    jf(*mk(torch.float32, "cpu"))
    fus = hipfuse.fusions(thunder.last_traces(jf)[-1])
    assert len(fus) == 1, fus
    f = fus[0]._call_ctx[fus[0].sym.name]
    assert f.plan.colred > 0
    ks = cg.generate(f.plan, f.inputs, f.outputs, {
        p.name: cg.TensorArg(tuple(p.shape), tuple(torch.empty(tuple(p.shape)).stride()), p.dtype, True)
        for p in f.inputs if isinstance(p, TensorProxy)})
    # one launch: the split partials are combined by the last workgroup of each column group
    assert not ks.extra and ks.ws_bytes > 0 and ks.counters > 0 and ks.mode.startswith("col")
    if ks.grid[1] > 1:  # row splits: arrival counter, reset by the last workgroup
        assert "atomicAdd(A.cnt" in ks.src and "__hip_atomic_store(A.cnt + blockIdx.x, 0u" in ks.src
    else:
        assert "atomicAdd" not in ks.src


@pytest.mark.parametrize("case", _SHAPE_CASES)
def test_shape_ops_fused_cpu(case, cpu_fusion):
    """Slices, concatenations, index_select / gather / embedding lookups and reshapes of region
    inputs are index maps of the fused kernel (affine, piecewise or indirect loads): none of them
    is left to ATen as a separate gather / copy kernel."""
    fn, mk = CASES[case]
    jf = thunder.jit(fn, executors=["hipfuse", "torch"])
    jf(*mk(torch.float32, "cpu"))
    tr = thunder.last_traces(jf)[-1]
    fus = hipfuse.fusions(tr)
    assert fus
    left = [b.sym.name for b in tr.bound_symbols if not b.sym.is_fusion]
    for name in ("cat", "take", "take_along_axis", "embedding", "embedding_prim", "reshape", "scatter", "index_put"):
        assert name not in left and name + "_prim" not in left, (case, left)
    kinds = set()
    for fb in fus:
        f = fb._call_ctx[fb.sym.name]
        for am in f.plan.arg_maps:
            kinds |= {cg._kind(m) for m in am.values()}
    want = {"slice_mix": "slice", "cat_mix": "cat", "gather_mix": "gather", "embed_add": "gather",
            "reshape_ext": "reshape", "scatter_region": "scatter_dst"}[case]
    assert want in kinds, kinds


def test_region_rematerialization_cpu(cpu_fusion):
    """Fusion-region rematerialisation (reference core/rematerialization.py:239-407): the value two
    regions share is recomputed by the consumer from the cheaper producer input, never written."""
    fn, mk = CASES["remat_regions"]
    (x,) = mk(torch.float32, "cpu")
    jf = thunder.jit(fn, executors=["hipfuse", "torch"])
    for o, r in zip(jf(x), fn(x)):
        torch.testing.assert_close(o, r)
    fus = hipfuse.fusions(thunder.last_traces(jf)[-1])
    assert len(fus) == 2
    for fb in fus:
        assert [a.name for a in fb.args] == [fus[0].args[0].name]  # both read only x
        assert len(fb.output) == 1  # nothing intermediate is materialised


def test_single_region_for_norm_chain(cpu_fusion):
    fn, mk = CASES["ln_gelu_softmax"]
    jf = thunder.jit(fn, executors=["hipfuse", "torch"])
    jf(*mk(torch.float32, "cpu"))
    tr = thunder.last_traces(jf)[-1]
    fus = hipfuse.fusions(tr)
    assert len(fus) == 1
    compute = [b for b in tr.bound_symbols if not b.sym.is_fusion and b.sym.id not in ("python_return", "python_del")]
    # nothing but the fusion, unpacking and bookkeeping remains
    assert all(b.sym.name in ("python_return", "python_del", "unpack_trivial") for b in compute), [b.sym.name for b in compute]


def test_fusion_type_consecutive_vs_dataflow(cpu_fusion):
    """``fusion_type`` compile option (reference data_dependent_partition.py): 'consecutive' only
    extends a region with the next bound symbol in program order, so two independent chains that
    the program interleaves are not fused at all, while 'dataflow' fuses each chain."""
    def f(a, b):
        x = a.exp()
        y = b.sin()  # interleaved, independent of x (different shape: cannot share x's region)
        x = x * 2.0
        y = y + 1.0
        x = x.tanh()
        y = y.cos()
        return x, y

    a, b = torch.randn(64, 32), torch.randn(16, 8)
    counts = {}
    for ft in ("dataflow", "consecutive"):
        jf = thunder.jit(f, executors=["hipfuse", "torch"], fusion_type=ft)
        out = jf(a, b)
        for o, r in zip(out, f(a, b)):
            torch.testing.assert_close(o, r)
        counts[ft] = len(hipfuse.fusions(thunder.last_traces(jf)[-1]))
    assert counts == {"dataflow": 2, "consecutive": 0}, counts

    def g(a):
        return a.exp().mul(2.0).tanh()

    for ft in ("dataflow", "consecutive"):
        jg = thunder.jit(g, executors=["hipfuse", "torch"], fusion_type=ft)
        torch.testing.assert_close(jg(a), g(a))
        assert len(hipfuse.fusions(thunder.last_traces(jg)[-1])) == 1
    with pytest.raises(ValueError):
        thunder.jit(f, executors=["hipfuse", "torch"], fusion_type="bogus")(a, b)


@pytest.mark.skipif(not os.path.exists(LIB), reason="native library not built")
@pytest.mark.parametrize("case", sorted(CASES))
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_codegen_compiles(case, dtype, cpu_fusion):
    fn, mk = CASES[case]
    args = mk(dtype, "cpu")
    jf = thunder.jit(fn, executors=["hipfuse", "torch"])
    jf(*args)
    for fb in hipfuse.fusions(thunder.last_traces(jf)[-1]):
        f = fb._call_ctx[fb.sym.name]
        targs = {}
        for p in f.inputs:
            if isinstance(p, TensorProxy):
                st = torch.empty(tuple(p.shape)).stride()
                targs[p.name] = cg.TensorArg(tuple(p.shape), tuple(st), p.dtype, True)
        ks = cg.generate(f.plan, f.inputs, f.outputs, targs)
        code = hipfuse.compile_source(ks)
        assert len(code) > 1000


# ------------------------------------------------------------------------------------------
# GPU numerics
# ------------------------------------------------------------------------------------------
def _to64(x):
    return x.double() if isinstance(x, torch.Tensor) and x.is_floating_point() else x


@pytest.mark.gpu
@pytest.mark.parametrize("case", sorted(CASES))
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_fused_numerics_gpu(case, dtype):
    torch.manual_seed(0)
    fn, mk = CASES[case]
    args = mk(dtype, "cuda")
    jf = thunder.jit(fn, executors=["hipfuse", "torch"])
    out = jf(*args)
    assert hipfuse.fusions(thunder.last_traces(jf)[-1])
    ref = fn(*[_to64(a) for a in args])
    eager = fn(*args)
    out = out if isinstance(out, tuple) else (out,)
    ref = ref if isinstance(ref, tuple) else (ref,)
    eager = eager if isinstance(eager, tuple) else (eager,)
    for o, r, e in zip(out, ref, eager):
        assert o.dtype == e.dtype and o.shape == e.shape
        err = (o.double() - r).abs().max().item()
        err_e = (e.double() - r).abs().max().item()
        assert err <= 2 * err_e + 1e-5, (case, err, err_e)


def _colsum_bf16(x):
    return x.float().sum(0).to(torch.bfloat16)


def _colamax_scaled(x):
    return x.float().abs().amax(0) * 0.5


@pytest.mark.gpu
@pytest.mark.parametrize("fn,shape", [(_colsum_bf16, (8192, 1024)), (_colsum_bf16, (4096, 1002)),
                                      (_colamax_scaled, (6000, 768)), (_colsum_bf16, (4096, 11008))])
def test_column_mode_split_handoff_gpu(fn, shape):
    """Column mode with row splits, one launch: every split's fp32 partial is handed to the last
    workgroup of its column group through agent-coherent memory operations and an arrival counter
    that workgroup resets.  vs fp64; bit-identical over repeated calls (fixed combine order, counters
    back at zero after every launch) and under a HIP graph replay."""
    torch.manual_seed(0)
    x = torch.randn(*shape, device="cuda", dtype=torch.bfloat16)
    jf = thunder.jit(fn, executors=["hipfuse", "torch"])
    out = jf(x)
    fus = hipfuse.fusions(thunder.last_traces(jf)[-1])
    assert len(fus) == 1
    hf = fus[0]._call_ctx[fus[0].sym.name]
    _, ks = hf._variant([x])
    assert ks.mode.startswith("col") and ks.grid[1] > 1 and not ks.extra, ks.mode
    ref = fn(x.double())
    eager = fn(x)
    err_e = (eager.double() - ref).abs().max().item()
    # the fp32 sums differ from ATen's in order: allow one unit in the last place of the output dtype
    ulp = 2.0 ** (torch.floor(torch.log2(ref.abs().clamp_min(1e-30))) - (7 if out.dtype == torch.bfloat16 else 23))
    excess = ((out.double() - ref).abs() - ulp).max().item()
    assert excess <= 2 * err_e + 1e-5, (excess, err_e)
    for _ in range(3):
        assert torch.equal(jf(x), out)
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        jf(x)  # counters / kernels of the capture stream exist before the capture
        with torch.cuda.graph(g, stream=s):
            gout = jf(x)
    torch.cuda.current_stream().wait_stream(s)
    for _ in range(2):
        g.replay()
        torch.cuda.synchronize()
        assert torch.equal(gout, out)


@pytest.mark.gpu
def test_fused_noncontiguous_and_backward_gpu():
    torch.manual_seed(0)

    def f(a, b):
        return torch.tanh(a.t() * b) + a.t()

    a = torch.randn(64, 96, device="cuda", requires_grad=True)
    b = torch.randn(96, 64, device="cuda", requires_grad=True)
    jf = thunder.jit(f, executors=["hipfuse", "torch"])
    out = jf(a, b)
    ref = f(a, b)
    torch.testing.assert_close(out, ref)
    g = torch.randn_like(out)
    ga, gb = torch.autograd.grad(out, (a, b), g)
    ra, rb = torch.autograd.grad(ref, (a, b), g)
    torch.testing.assert_close(ga, ra)
    torch.testing.assert_close(gb, rb)
    assert hipfuse.fusions(thunder.last_backward_traces(jf)[-1])


@pytest.mark.parametrize("name", ["llama2-like", "llama3-like", "gpt-neox-like"])
def test_litgpt_partition_cpu(name, cpu_fusion):
    """Whole-model fwd+bwd through the fusion partitioner (reference path on CPU): catches
    scheduling / region-output bugs without a GPU."""
    from lightning_thunder_amd.models.litgpt import GPT, Config

    torch.manual_seed(0)
    cfg = Config.from_name(name, n_layer=2)
    m = GPT(cfg)
    m.set_rope_cache(32)
    x = torch.randint(0, cfg.vocab_size, (2, 32))
    jm = thunder.jit(m)
    out = jm(x)
    ref = m(x)
    torch.testing.assert_close(out, ref, rtol=1e-4, atol=1e-4)
    g = torch.randn_like(out)
    gj = torch.autograd.grad(out, list(m.parameters()), g, allow_unused=True)
    gr = torch.autograd.grad(ref, list(m.parameters()), g, allow_unused=True)
    for a, b in zip(gj, gr):
        if b is not None:
            torch.testing.assert_close(a, b, rtol=1e-3, atol=1e-4)
    bw = thunder.last_backward_traces(jm)[-1]
    assert hipfuse.fusions(bw)
    if os.path.exists(LIB):  # every generated kernel must compile for gfx950
        for tr in (thunder.last_traces(jm)[-1], bw):
            for fb in hipfuse.fusions(tr):
                f = fb._call_ctx[fb.sym.name]
                targs = {p.name: cg.TensorArg(tuple(p.shape), tuple(torch.empty(tuple(p.shape)).stride()), p.dtype, True)
                         for p in f.inputs if isinstance(p, TensorProxy)}
                hipfuse.compile_source(cg.generate(f.plan, f.inputs, f.outputs, targs))


def test_philox_dropout_mask_recomputed(cpu_fusion):
    """Dropout masks come from the counter-based RNG and are regenerated in the backward."""
    torch.manual_seed(0)

    def f(x):
        return torch.nn.functional.dropout(x * 2.0, p=0.3, training=True)

    x = torch.randn(64, 128, requires_grad=True)
    jf = thunder.jit(f)
    y = jf(x)
    keep = y != 0
    frac = keep.float().mean().item()
    assert 0.65 < frac < 0.75
    torch.testing.assert_close(y[keep], (x * 2.0 / 0.7)[keep])
    g = torch.randn_like(y)
    (gx,) = torch.autograd.grad(y, (x,), g)
    torch.testing.assert_close(gx, torch.where(keep, g * 2.0 / 0.7, torch.zeros_like(g)))
    bw = thunder.last_backward_traces(jf)[-1]
    # nothing tensor-valued is saved for the mask: the backward regenerates it
    assert "uniform_philox" in str(bw)
    # a second call draws a fresh mask
    y2 = jf(x)
    assert not torch.equal(y2 != 0, keep)


def test_philox_torch_matches_reference_vectors():
    from lightning_thunder_amd.core.rng import philox_uniform_torch, philox4x32

    # Random123 known-answer vectors for philox4x32_R(10)
    kat = [((0, 0, 0, 0), (0, 0), (0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8)),
           ((0xffffffff,) * 4, (0xffffffff,) * 2, (0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd)),
           ((0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344), (0xa4093822, 0x299f31d0),
            (0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1))]
    for ctr, key, want in kat:
        got = philox4x32(*[torch.tensor([c], dtype=torch.int64) for c in ctr], *key)
        assert tuple(int(g) for g in got) == want
    # element e = word e % 4 of block e // 4
    u4 = philox_uniform_torch((8,), 77, 5, "cpu")
    for blk in range(2):
        words = philox4x32(torch.tensor([blk]), torch.tensor([0]), torch.tensor([5]), torch.tensor([0]), 77, 0)
        for i, w in enumerate(words):
            assert u4[4 * blk + i].item() == (int(w) >> 8) / 16777216.0

    u = philox_uniform_torch((8,), 1234, 0, "cpu")
    assert ((u >= 0) & (u < 1)).all()
    v = philox_uniform_torch((8,), 1234, 0, "cpu")
    assert torch.equal(u, v)
    w = philox_uniform_torch((8,), 1234, 8, "cpu")
    assert not torch.equal(u, w)


@pytest.mark.gpu
@pytest.mark.parametrize("shape", [(256, 384), (33, 7)])  # whole-block vector draws / per-element draws
def test_philox_dropout_gpu_matches_torch_philox(shape):
    from lightning_thunder_amd.core import rng
    from lightning_thunder_amd.core.rng import philox_uniform_torch

    def f(x):
        return torch.nn.functional.dropout(torch.tanh(x), p=0.25, training=True)

    x = torch.randn(*shape, device="cuda", requires_grad=True)
    jf = thunder.jit(f)
    torch.manual_seed(123)
    rng._state["seed"] = None  # restart the counter for this seed
    y = jf(x)
    assert any("uniform_philox" in str(b.subsymbols) for b in hipfuse.fusions(thunder.last_traces(jf)[-1]))
    keep_ref = philox_uniform_torch(x.shape, 123, 0, "cuda") < 0.75
    assert torch.equal(y != 0, keep_ref)
    g = torch.randn_like(y)
    (gx,) = torch.autograd.grad(y, (x,), g)
    ref = torch.where(keep_ref, g / 0.75 * (1 - torch.tanh(x) ** 2), torch.zeros_like(g))
    torch.testing.assert_close(gx, ref, rtol=1e-4, atol=1e-5)


@pytest.mark.gpu
@pytest.mark.parametrize("shape", [(4, 512, 1024), (64, 36), (33, 7)])  # 4-word vector draws / scalar draws
def test_philox_dropout_column_region_gpu(shape):
    """Dropout on a biased activation: the backward's mask regeneration and the bias-gradient column
    sum share one column-mode kernel (Philox words drawn whole blocks at a time where the columns
    allow); mask and both gradients match the torch Philox reference."""
    from lightning_thunder_amd.core import rng
    from lightning_thunder_amd.core.rng import philox_uniform_torch

    def f(x, b):
        return torch.nn.functional.dropout(x + b, p=0.25, training=True)

    x = torch.randn(*shape, device="cuda", requires_grad=True)
    b = torch.randn(shape[-1], device="cuda", requires_grad=True)
    jf = thunder.jit(f, executors=["hipfuse", "torch"])
    torch.manual_seed(321)
    rng._state["seed"] = None
    y = jf(x, b)
    keep = philox_uniform_torch(x.shape, 321, 0, "cuda") < 0.75
    assert torch.equal(y != 0, keep)
    g = torch.randn_like(y)
    gx, gb = torch.autograd.grad(y, (x, b), g)
    bw = thunder.last_backward_traces(jf)[-1]
    assert any("uniform_philox" in s and "sum" in s for s in (str(fb.subsymbols) for fb in hipfuse.fusions(bw))), bw
    ref = torch.where(keep, g / 0.75, torch.zeros_like(g))
    torch.testing.assert_close(gx, ref, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(gb, ref.reshape(-1, shape[-1]).sum(0), rtol=1e-4, atol=1e-4)


def test_moe_model_cpu():
    """Mixtral-style MoE (top-k routing, sorted tokens, grouped GEMMs) fwd+bwd vs eager."""
    from lightning_thunder_amd.models.litgpt import GPT, Config

    torch.manual_seed(0)
    cfg = Config.from_name("mixtral-like")
    m = GPT(cfg)
    m.set_rope_cache(32)
    x = torch.randint(0, cfg.vocab_size, (2, 32))
    jm = thunder.jit(m)
    out = jm(x)
    torch.testing.assert_close(out, m(x), rtol=1e-4, atol=1e-4)
    g = torch.randn_like(out)
    gj = torch.autograd.grad(out, list(m.parameters()), g)
    gr = torch.autograd.grad(m(x), list(m.parameters()), g)
    for a, b in zip(gj, gr):
        torch.testing.assert_close(a, b, rtol=1e-3, atol=1e-4)


def test_repeated_fusions_share_one_kernel(cpu_fusion):
    """Structurally identical regions (the same block in every layer) generate the same source
    (value names are canonicalised), so they hash to one kernel and compile once."""
    from lightning_thunder_amd.models.nanogpt import NanoGPT, NanoGPTConfig

    torch.manual_seed(0)
    m = NanoGPT(NanoGPTConfig(n_layer=3, n_head=2, n_embd=64, block_size=32, vocab_size=128))
    jm = thunder.jit(m, executors=["hipfuse", "torch"])
    x = torch.randint(0, 128, (2, 32))
    jm(x, x)
    names = []
    for fb in hipfuse.fusions(thunder.last_traces(jm)[-1]):
        fu = fb._call_ctx[fb.sym.name]
        targs = {p.name: cg.TensorArg(tuple(p.shape), tuple(torch.empty(tuple(p.shape)).stride()), p.dtype, True)
                 for p in fu.inputs if isinstance(p, TensorProxy)}
        names.append(cg.generate(fu.plan, fu.inputs, fu.outputs, targs).name)
    assert len(names) >= 6 and len(set(names)) < len(names), names  # per-layer regions dedupe
    src = cg._canonical_names("float v_t12[8]; v_t12[j] = r_t3 + v_t12[j]; v8_float q; r_t3 = 1;")
    assert src == "float v_n0[8]; v_n0[j] = r_n1 + v_n0[j]; v8_float q; r_n1 = 1;"


def _compile_fusions_of(jf):
    """Every region's kernel source, compiled with hiprtc on the CPU (hipfuse.precompile)."""
    return hipfuse.precompile(thunder.last_traces(jf)[-1])


_SOURCE_CASES = {
    # ops whose decompositions put a constant (full) into several regions: the consumer region
    # recomputes the producer cones (fusion-region rematerialisation) without defining a value twice
    "heaviside": (lambda a, b: torch.heaviside(a, b), lambda: (torch.randn(2, 3, 8, 8), torch.randn(2, 3, 8, 8))),
    "bce": (lambda a, b: torch.nn.functional.binary_cross_entropy(torch.sigmoid(a), torch.sigmoid(b)),
            lambda: (torch.randn(4, 33), torch.randn(4, 33))),
    "gaussian_nll": (lambda a, b, v: torch.nn.functional.gaussian_nll_loss(a, b, v.abs() + 0.1),
                     lambda: (torch.randn(8, 12), torch.randn(8, 12), torch.randn(8, 12))),
    "interp": (lambda a: torch.nn.functional.interpolate(a, scale_factor=1.6, mode="linear"),
               lambda: (torch.randn(2, 3, 5),)),
}


@pytest.mark.skipif(not os.path.exists("/opt/rocm/lib/libhiprtc.so"), reason="needs ROCm hiprtc")
@pytest.mark.parametrize("case", sorted(_SOURCE_CASES) + ["slice_mix", "cat_mix", "gather_mix", "remat_regions",
                                                          "pad_sum", "ln_gelu_softmax"])
def test_generated_sources_compile_cpu(case, cpu_fusion):
    if case in _SOURCE_CASES:
        fn, mk = _SOURCE_CASES[case]
        args = mk()
    else:
        fn, mk = CASES[case]
        args = mk(torch.float32, "cpu")
    jf = thunder.jit(fn, executors=["hipfuse", "torch"])
    out = jf(*args)
    ref = fn(*args)
    for o, r in zip(out if isinstance(out, tuple) else (out,), ref if isinstance(ref, tuple) else (ref,)):
        torch.testing.assert_close(o, r, rtol=1e-5, atol=1e-5)
    assert _compile_fusions_of(jf) >= 1


def test_trailing_transpose_left_as_view_cpu(cpu_fusion):
    """A region value consumed transposed by a GEMM (autodiff's wgrad operand dY^T) is stored once,
    untransposed; the reshape/transpose chain runs after the region as zero-copy views instead of
    the region storing a transposed copy (Gemma's GeGLU backward stored two [24576, 4096] copies)."""
    def f(a, b, w):
        d = torch.nn.functional.gelu(a, approximate="tanh") * b
        g = d.reshape(-1, d.shape[-1])
        return d, g.t() @ w

    a, b, w = torch.randn(1, 8, 16), torch.randn(1, 8, 16), torch.randn(8, 4)
    jf = thunder.jit(f, executors=["hipfuse", "torch"])
    for o, r in zip(jf(a, b, w), f(a, b, w)):
        torch.testing.assert_close(o, r, rtol=1e-5, atol=1e-5)
    tr = thunder.last_traces(jf)[-1]
    fus = hipfuse.fusions(tr)
    assert fus
    for fb in fus:
        assert all(tuple(o.shape) != (16, 8) for o in fb.flat_proxy_outs), fb
        assert all(s.sym.id != PrimIDs.TRANSPOSE for s in fb.subsymbols)
