"""Transforms, recipes/plugins and dev utilities on CPU (reference: thunder/tests/test_transforms.py,
test_recipes.py, test_check_trace.py)."""
import pytest
import torch

import lightning_thunder_amd as thunder
from lightning_thunder_amd.common import DebugOptions


def _mlp():
    torch.manual_seed(0)
    return torch.nn.Sequential(torch.nn.Linear(4, 8), torch.nn.ReLU(), torch.nn.Linear(8, 2))


def test_constant_folding():
    from lightning_thunder_amd.transforms.constant_folding import ConstantFolding

    def f(x):
        mask = torch.ones(4, 4).tril() * 2 + 1
        return x * mask + torch.arange(4).float()

    x = torch.randn(4, 4)
    jf = thunder.jit(f, transforms=[ConstantFolding()])
    torch.testing.assert_close(jf(x), f(x))
    names = [b.sym.name for b in thunder.last_traces(jf)[-1].bound_symbols]
    assert sum(n.startswith("folded_constant") for n in names) == 2
    assert not any(n in ("torch.ones", "torch_ones", "tril", "arange") for n in names)


def test_prune_prologue_checks():
    from lightning_thunder_amd.transforms.prune_prologue_checks import PrunePrologueChecks, ExtractionOnlyPrologueTransform

    m = _mlp()
    jm = thunder.jit(m, transforms=[ExtractionOnlyPrologueTransform()], prune_prologue_checks=False)
    x = torch.randn(3, 4)
    torch.testing.assert_close(jm(x), m(x))
    pro = thunder.last_prologue_traces(jm)[-1]
    assert not any(b.sym.name.startswith("check_") for b in pro.bound_symbols)
    jm2 = thunder.jit(m, transforms=[PrunePrologueChecks()], prune_prologue_checks=False)
    jm2(x)
    pro2 = thunder.last_prologue_traces(jm2)[-1]
    checks = [b for b in pro2.bound_symbols if b.sym.name.startswith("check_tensor")]
    assert len(checks) == 1  # only the user input remains guarded


def test_check_traces_and_debug_transform():
    from lightning_thunder_amd.dev_utils.debug_transform import DebugTransform
    from lightning_thunder_amd.dev_utils.profile_transform import RoctxProfileTransform, ProfileTransform

    seen = []
    m = _mlp()
    jm = thunder.jit(m, transforms=[DebugTransform(pre_callback=lambda b, *a: seen.append(b.sym.name)),
                                    RoctxProfileTransform(), ProfileTransform(warmup_runs=0)],
                     debug_options=DebugOptions(check_traces=True))
    x = torch.randn(3, 4)
    y = jm(x)
    y.sum().backward()
    torch.testing.assert_close(y, m(x))
    assert "torch_linear" in seen or "linear" in " ".join(seen)


def test_check_trace_detects_use_before_def():
    from lightning_thunder_amd.dev_utils.check_trace import check_trace, TraceCheckError

    jf = thunder.jit(lambda a: a * 2 + 1)
    jf(torch.randn(2))
    tr = thunder.last_traces(jf)[-1]
    check_trace(tr)
    bad = thunder.core.trace.from_trace(tr)
    bad.bound_symbols = list(reversed(tr.bound_symbols[:-1])) + [tr.bound_symbols[-1]]
    with pytest.raises(TraceCheckError):
        check_trace(bad)


def test_compile_with_recipe_and_plugins():
    from lightning_thunder_amd.core.recipe import Recipe, Plugin, PluginPolicy
    from lightning_thunder_amd.recipes import BaseRecipe, get_recipes
    from lightning_thunder_amd.plugins import get_plugin_names, ReduceOverhead

    assert "base" in get_recipes() and "reduce-overhead" in get_plugin_names()
    m = _mlp()
    tm = thunder.compile(m, recipe=BaseRecipe(fuser=None))
    x = torch.randn(3, 4)
    torch.testing.assert_close(tm(x), m(x))
    assert isinstance(Recipe.get_for_model(m), BaseRecipe)

    class Marker(Plugin):
        policy = PluginPolicy.POST

        def setup_transforms(self):
            from lightning_thunder_amd.transforms.constant_folding import ConstantFolding

            return [ConstantFolding()]

    tm2 = thunder.compile(m, plugins=[Marker()])
    torch.testing.assert_close(tm2(x), m(x))
    assert type(ReduceOverhead().setup_transforms()[0]).__name__ == "HipGraphTransform"


def test_materialization_from_module_init():
    from lightning_thunder_amd.transforms.materialization import MaterializationTransform

    torch.manual_seed(0)
    ref = _mlp()
    with torch.device("meta"):
        m = torch.nn.Sequential(torch.nn.Linear(4, 8), torch.nn.ReLU(), torch.nn.Linear(8, 2))
    torch.manual_seed(0)
    tm = thunder.jit(m, transforms=[MaterializationTransform(device="cpu")])
    assert not any(p.is_meta for p in tm.parameters())
    for p, q in zip(tm.parameters(), ref.parameters()):
        torch.testing.assert_close(p, q)
    x = torch.randn(3, 4)
    torch.testing.assert_close(tm(x), ref(x))


def test_lora_transform_trains_only_adapters():
    from lightning_thunder_amd.transforms.qlora import LORATransform

    torch.manual_seed(0)
    m = _mlp()
    ref = _mlp()
    t = LORATransform(r=2, lora_alpha=4)
    jm = thunder.jit(m, transforms=[t])
    x = torch.randn(3, 4)
    # lora_b starts at zero: identical to the base model
    torch.testing.assert_close(jm(x), ref(x))
    with torch.no_grad():
        m[0].lora_b.normal_()
    y = jm(x)
    expect = ref(x) * 0
    h = torch.nn.functional.linear(x, ref[0].weight, ref[0].bias) + (x @ m[0].lora_a.t() @ m[0].lora_b.t()) * 2.0
    expect = torch.nn.functional.linear(torch.relu(h), ref[2].weight, ref[2].bias) + \
        (torch.relu(h) @ m[2].lora_a.t() @ m[2].lora_b.t()) * 2.0
    torch.testing.assert_close(y, expect)
    y.sum().backward()
    assert m[0].weight.grad is None and m[0].lora_a.grad is not None and m[2].lora_b.grad is not None
    assert {"0", "2"} == t.lora_linear_names


def test_nf4_quantization_cpu():
    from lightning_thunder_amd.transforms.quantization import NF4LinearQuant4bit, quantize_nf4, dequantize_nf4

    torch.manual_seed(0)
    w = torch.randn(64, 128)
    q, a = quantize_nf4(w)
    assert q.dtype == torch.uint8 and q.numel() == w.numel() // 2 and a.numel() == w.numel() // 64
    wd = dequantize_nf4(q, a, w.shape, torch.float32)
    assert (wd - w).abs().max() / w.abs().max() < 0.2
    m = torch.nn.Sequential(torch.nn.Linear(128, 64), torch.nn.ReLU(), torch.nn.Linear(64, 32))
    ref = [torch.nn.functional.linear, ]
    x = torch.randn(4, 128, requires_grad=True)
    ref_out = m(x)
    jm = thunder.jit(m, transforms=[NF4LinearQuant4bit(skip=())])
    out = jm(x)
    assert (out - ref_out).abs().max() / ref_out.abs().max() < 0.2
    out.sum().backward()
    assert x.grad is not None
    assert any("nf4" in b.sym.name for b in thunder.last_traces(jm)[-1].bound_symbols)


def test_custom_op_traced_with_autograd():
    @torch.library.custom_op("lta_test::scaled_sin", mutates_args=())
    def scaled_sin(x: torch.Tensor, k: float) -> torch.Tensor:
        return torch.sin(x) * k

    @scaled_sin.register_fake
    def _(x, k):
        return torch.empty_like(x)

    def setup(ctx, inputs, output):
        ctx.save_for_backward(inputs[0])
        ctx.k = inputs[1]

    def bwd(ctx, g):
        (x,) = ctx.saved_tensors
        return g * torch.cos(x) * ctx.k, None

    scaled_sin.register_autograd(bwd, setup_context=setup)

    def f(x):
        return scaled_sin(x * 2, 3.0).sum()

    x = torch.randn(5, requires_grad=True)
    jf = thunder.jit(f)
    jf(x).backward()
    g = x.grad.clone()
    x.grad = None
    f(x).backward()
    torch.testing.assert_close(g, x.grad)
    # the op is its own symbol (custom_op executor), and the backward calls the registered
    # backward on exactly what setup_context saved -- the forward is not re-run
    fw = str(thunder.last_traces(jf)[-1])
    bw = str(thunder.last_backward_traces(jf)[-1])
    assert "custom_op_lta_test_scaled_sin" in fw, fw
    assert "custom_op_bwd_lta_test_scaled_sin" in bw and "custom_op_lta_test_scaled_sin(" not in bw, bw


def test_custom_op_saves_output_and_computed_attrs():
    """setup_context saving the OUTPUT and a computed non-tensor attribute (reference
    thunder/tests/test_torch_library_custom_op.py)."""
    calls = {"fwd": 0}

    @torch.library.custom_op("lta_test::exp_cast", mutates_args=())
    def exp_cast(x: torch.Tensor) -> torch.Tensor:
        calls["fwd"] += 1
        return torch.exp(x)

    @exp_cast.register_fake
    def _(x):
        return torch.empty_like(x)

    def setup(ctx, inputs, output):
        ctx.save_for_backward(output)
        ctx.in_dtype = inputs[0].dtype
        ctx.scale = inputs[0].shape[-1] * 0 + 2.0

    def bwd(ctx, g):
        (y,) = ctx.saved_tensors
        return (g * y * (ctx.scale / 2.0)).to(ctx.in_dtype)

    exp_cast.register_autograd(bwd, setup_context=setup)

    x = torch.randn(3, 4, requires_grad=True)
    jf = thunder.jit(lambda x: exp_cast(x * 0.5).sum())
    jf(x).backward()
    assert calls["fwd"] == 1  # executed once: the backward does not re-run the forward
    g = x.grad.clone()
    x.grad = None
    exp_cast(x * 0.5).sum().backward()
    torch.testing.assert_close(g, x.grad)


def test_custom_op_mutating_args_is_refused():
    """A custom op with non-empty ``mutates_args`` is refused (reference
    thunder/torch/custom_op.py:347-350), never traced as a pure symbol whose write DCE could drop."""
    @torch.library.custom_op("lta_test::add_into", mutates_args=("out",))
    def add_into(x: torch.Tensor, out: torch.Tensor) -> None:
        out.add_(x)

    @add_into.register_fake
    def _(x, out):
        return None

    def f(x, out):
        add_into(x, out)
        return x * 2

    x, buf = torch.randn(4), torch.zeros(4)
    with pytest.raises(NotImplementedError, match="mutates"):
        thunder.jit(f)(x, buf)
    # eager still works, and the write is observable
    f(x, buf)
    torch.testing.assert_close(buf, x)


def test_custom_op_backward_state_is_trace_owned():
    """The backward symbol's per-call state rides in the bound symbol (freed with the trace), not
    in a process-global dict that grows with every retrace."""
    import lightning_thunder_amd.torch.custom_op as co

    assert not hasattr(co, "_bwd_state") and not hasattr(co, "_bwd_inputs")

    @torch.library.custom_op("lta_test::cube", mutates_args=())
    def cube(x: torch.Tensor) -> torch.Tensor:
        return x * x * x

    @cube.register_fake
    def _(x):
        return torch.empty_like(x)

    def setup(ctx, inputs, output):
        ctx.save_for_backward(inputs[0])

    def bwd(ctx, g):
        (x,) = ctx.saved_tensors
        return 3 * g * x * x

    cube.register_autograd(bwd, setup_context=setup)
    jf = thunder.jit(lambda x: cube(x).sum())
    x = torch.randn(6, requires_grad=True)
    jf(x).backward()
    torch.testing.assert_close(x.grad, 3 * x.detach() ** 2)
    bw = thunder.last_backward_traces(jf)[-1]
    def walk(bsyms):
        for b in bsyms:
            yield b
            yield from walk(b.subsymbols)

    states = [v for b in walk(bw.bound_symbols) for v in b.kwargs.values() if isinstance(v, co._BwdState)]
    assert len(states) == 1, str(bw)


def test_examine_patterns_and_memory(capsys):
    from lightning_thunder_amd.examine import examine, make_trace_dot, get_alloc_memory
    from lightning_thunder_amd.core.patterns import Pattern

    def f(x):
        return torch.nn.functional.gelu(torch.special.erfcx(x) + x.sum())

    assert examine(f, torch.randn(4)) is not None
    assert "opaque" in capsys.readouterr().out
    jf = thunder.jit(lambda x, w, b: torch.relu(torch.nn.functional.linear(x, w) + b))
    jf(torch.randn(2, 3), torch.randn(4, 3), torch.randn(4))
    tr = thunder.last_traces(jf)[-1]
    p = Pattern().match(lambda b: "linear" in b.sym.name).match(lambda b: "add" in b.sym.name).match(
        lambda b: "relu" in b.sym.name)
    m = p(tr)
    assert len(m) == 1 and len(m[0]) == 3
    peak, _ = get_alloc_memory(tr)
    assert peak > 0
    assert make_trace_dot(tr).startswith("digraph")


def test_numpy_language_and_langctx():
    from lightning_thunder_amd.core.langctxs import langctx, Languages, resolve_method
    from lightning_thunder_amd import numpy as lnp
    from lightning_thunder_amd.core.trace import TraceCtx, tracectx
    from lightning_thunder_amd.core.proxies import TensorProxy

    with tracectx(TraceCtx()):
        t = TensorProxy(shape=(3, 4), device="cpu", dtype=torch.float32)
        assert lnp.size(t) == 12 and lnp.compute_len(t) == 3
        s = lnp.add(t, 1.0)
        assert tuple(s.shape) == (3, 4)
    with langctx(Languages.NUMPY):
        assert resolve_method("size") is lnp.size
    assert resolve_method("sum") is not None


def test_fp8_inference_transform_cpu():
    from lightning_thunder_amd.transforms.fp8_inference import FP8InferenceTransform, quantize_weight_e4m3, dequantize_e4m3

    torch.manual_seed(0)
    w = torch.randn(64, 128)
    q, s = quantize_weight_e4m3(w)
    assert q.dtype == torch.uint8 and s.shape == ()
    assert (dequantize_e4m3(q, s, torch.float32) - w).abs().max() / w.abs().max() < 0.07
    m = torch.nn.Sequential(torch.nn.Linear(128, 64), torch.nn.GELU(), torch.nn.Linear(64, 32))
    x = torch.randn(4, 128, requires_grad=True)
    ref = m(x)
    jm = thunder.jit(m, transforms=[FP8InferenceTransform(skip=())])
    out = jm(x)
    assert (out - ref).abs().max() / ref.abs().max() < 0.1
    out.sum().backward()
    assert x.grad is not None
    assert any("fp8_linear_inference" in b.sym.name for b in thunder.last_traces(jm)[-1].bound_symbols)


def test_fp8_inference_transform_moe_experts_cpu():
    """Grouped experts are quantized per expert (te_groupedmm_fp8 counterpart) and traced as the
    grouped fp8 custom op; the CPU path matches the model within fp8 error."""
    from lightning_thunder_amd.models.llama4_moe import Llama4MoE, MoEConfig
    from lightning_thunder_amd.transforms.fp8_inference import FP8InferenceTransform, quantize_experts_e4m3

    torch.manual_seed(0)
    w = torch.randn(4, 32, 16)
    w[2] *= 100.0  # one expert with a far larger range: per-expert scales keep the others precise
    q, s = quantize_experts_e4m3(w)
    assert q.shape == w.shape and s.shape == (4,)
    deq = q.view(torch.float8_e4m3fn).float() / s[:, None, None]
    assert ((deq - w).abs().amax(dim=(1, 2)) / w.abs().amax(dim=(1, 2))).max() < 0.07
    m = Llama4MoE(MoEConfig(hidden_size=64, intermediate_size=128, num_routed_experts=4))
    x = torch.randn(2, 8, 64)
    ref = m(x)
    t = FP8InferenceTransform(skip=())
    jm = thunder.jit(m, transforms=[t])
    out = jm(x)
    assert any(n.endswith("routed_experts.gate_proj") for n in t.quantized)
    assert (out - ref).abs().max() / ref.abs().max() < 0.15
    names = [b.sym.name for b in thunder.last_traces(jm)[-1].bound_symbols]
    assert any("fp8_grouped_mm_inference" in n for n in names), names


def test_numerics_check_transform_cpu():
    import lightning_thunder_amd as thunder
    from lightning_thunder_amd.dev_utils.numerics_check import NumericsCheckTransform

    def f(x, y):
        return torch.log(x) * y + torch.exp(y).sum(-1, keepdim=True)

    t = NumericsCheckTransform(sync=False)
    jf = thunder.jit(f, transforms=[t])
    x, y = torch.rand(4, 8) + 0.1, torch.randn(4, 8)
    torch.testing.assert_close(jf(x, y), f(x, y))
    assert t.checked > 0 and not t.findings
    jf(-x, y)  # log of negatives -> nan from finite inputs: reported
    assert any("non-finite" in m for m in t.findings)
    jd = thunder.jit(f, debug_options=thunder.DebugOptions(sync_after_each_kernel=True))
    torch.testing.assert_close(jd(x, y), f(x, y))


def test_reference_module_paths():
    import torch

    import lightning_thunder_amd as thunder
    from lightning_thunder_amd.dev_utils.nvtx_profile_transform import NvtxProfileTransform
    from lightning_thunder_amd.examine.memory_calculation import get_alloc_memory

    jf = thunder.jit(lambda x: (x * 2).sin(), transforms=[NvtxProfileTransform(include_shapes=True)])
    jf(torch.ones(4))
    peak, _ = get_alloc_memory(thunder.last_traces(jf)[-1])
    assert peak > 0
    # views share their source's storage; a freed intermediate is not counted twice
    jg = thunder.jit(lambda x: x.reshape(-1).t().sin(), executors=["torch"])
    jg(torch.ones(64, 32))
    peak, live, tl = get_alloc_memory(thunder.last_traces(jg)[-1], timeline=True)
    assert peak == 2 * 64 * 32 * 4, (peak, tl)
    assert tl and all(isinstance(n, str) and m >= 0 for n, m in tl)


def test_fp8_training_recipes_parse():
    """Recipe names of ``FP8LinearTransform`` / the ``fp8`` plugin (TE DelayedScaling,
    MXFP8BlockScaling, and MXFP4BlockScaling as the counterpart of NVFP4BlockScaling); CPU
    programs keep their linears (the fp8 GEMMs need a gfx950 device)."""
    from lightning_thunder_amd.ops.fp8 import DelayedScaling, MXFP8BlockScaling, MXFP4BlockScaling
    from lightning_thunder_amd.transforms.fp8 import FP8LinearTransform

    assert FP8LinearTransform("current").recipe == "current"
    assert isinstance(FP8LinearTransform("delayed").recipe, DelayedScaling)
    assert isinstance(FP8LinearTransform("mxfp8").recipe, MXFP8BlockScaling)
    assert isinstance(FP8LinearTransform("mxfp4").recipe, MXFP4BlockScaling)
    with pytest.raises(ValueError):
        FP8LinearTransform("nvfp4")
    m = torch.nn.Linear(256, 256)
    t = FP8LinearTransform("mxfp4")
    jm = thunder.jit(m, transforms=[t])
    x = torch.randn(256, 256)
    torch.testing.assert_close(jm(x), m(x))
    assert t.n_converted == 0


def test_jit_inner_autocast_context():
    """``with torch.autocast(...)`` inside jitted code applies the autocast rules to the region only."""
    import lightning_thunder_amd as lta

    def f(x, w):
        with torch.autocast("cpu", dtype=torch.bfloat16):
            y = x @ w
        return y, x @ w

    torch.manual_seed(0)
    x = torch.randn(8, 8, requires_grad=True)
    w = torch.randn(8, 8, requires_grad=True)
    jf = lta.jit(f)
    y, z = jf(x, w)
    ry, rz = f(x, w)
    assert y.dtype == torch.bfloat16 and z.dtype == torch.float32
    torch.testing.assert_close(y, ry)
    torch.testing.assert_close(z, rz)
    (y.float().sum() + z.sum()).backward()
    gx = x.grad.clone()
    x.grad = None
    (ry.float().sum() + rz.sum()).backward()
    torch.testing.assert_close(gx, x.grad, atol=5e-2, rtol=2e-2)


def test_fp8_delayed_state_resize_sizes_every_per_slot_list():
    """The FP8 transform sizes the delayed-scaling state after rewriting the trace: every per-slot
    list (scaling source, first-use and per-step flags) must follow the new slot count."""
    from lightning_thunder_amd.ops.fp8 import DelayedScaling, new_delayed_state, delayed_state

    st = delayed_state(new_delayed_state(DelayedScaling(), 0))
    st.resize(7)
    assert st.n == 7 and len(st.step_src) == len(st.seen) == len(st.step_seen) == 7
