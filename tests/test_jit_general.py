"""General ``jit`` behaviour (reference: ``thunder/tests/test_jit_general.py``, ``test_einops.py``,
``test_autocast.py``, ``test_randomness.py``, ``test_extend.py``, ``test_auto_register_torchops.py``)."""
import pytest
import torch

import lightning_thunder_amd as thunder


def test_kwargs_nested_containers_and_python_values():
    def f(x, *, scale=2.0, d=None, flag=True):
        out = x * scale
        if flag:
            out = out + d["b"][1]
        return {"out": out, "pair": (out.sum(), [x.shape[0], "tag"])}

    x = torch.randn(3, 4)
    d = {"a": 1, "b": [torch.zeros(4), torch.ones(4)]}
    jf = thunder.jit(f)
    r, e = jf(x, scale=3.0, d=d), f(x, scale=3.0, d=d)
    torch.testing.assert_close(r["out"], e["out"])
    assert r["pair"][1] == [3, "tag"]
    jf(x, scale=3.0, d=d)
    assert thunder.cache_hits(jf) == 1
    jf(x, scale=4.0, d=d)  # a different Python number: a new specialization
    assert thunder.cache_misses(jf) == 2


def test_cache_options():
    def f(x, k):
        return x * k

    x = torch.randn(4)
    same = thunder.jit(f, cache="same input")
    same(x, 2)
    torch.testing.assert_close(same(x, 2), x * 2)
    assert thunder.cache_hits(same) == 1
    none = thunder.jit(f, cache="no caching")
    none(x, 2)
    none(x, 2)
    assert thunder.cache_misses(none) == 2 and thunder.cache_hits(none) == 0
    assert thunder.cache_option(none) == thunder.CACHE_OPTIONS.NO_CACHING if hasattr(thunder, "CACHE_OPTIONS") else True


def test_shape_change_recompiles():
    jf = thunder.jit(lambda x: x.relu() + 1)
    jf(torch.randn(2, 3))
    jf(torch.randn(4, 3))
    jf(torch.randn(2, 3))
    assert thunder.cache_misses(jf) == 2 and thunder.cache_hits(jf) == 1


class _Counter(torch.nn.Module):
    def __init__(self):
        super().__init__()
        self.lin = torch.nn.Linear(4, 4)
        self.register_buffer("running", torch.zeros(4))

    def forward(self, x):
        y = self.lin(x)
        self.running = self.running * 0.9 + y.mean(0).detach() * 0.1  # attribute write -> epilogue
        return y


def test_module_buffer_rebinding_epilogue():
    m = _Counter()
    ref = _Counter()
    ref.load_state_dict(m.state_dict())
    jm = thunder.jit(m)
    x = torch.randn(8, 4)
    for _ in range(3):
        torch.testing.assert_close(jm(x), ref(x))
    torch.testing.assert_close(m.running, ref.running)


def test_no_grad_and_grad_enabled_entries():
    m = torch.nn.Linear(4, 2)
    jm = thunder.jit(m)
    x = torch.randn(3, 4)
    with torch.no_grad():
        y = jm(x)
    assert not y.requires_grad
    y2 = jm(x)
    assert y2.requires_grad
    assert thunder.cache_misses(jm) == 2


def test_nested_modules_shared_weights_and_containers():
    class M(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.layers = torch.nn.ModuleList(torch.nn.Linear(4, 4) for _ in range(3))
            self.heads = torch.nn.ModuleDict({"a": torch.nn.Linear(4, 2), "b": torch.nn.Linear(4, 2)})
            self.heads["b"].weight = self.heads["a"].weight  # tied

        def forward(self, x, which: str):
            for i, l in enumerate(self.layers):
                x = torch.tanh(l(x)) if i % 2 == 0 else l(x)
            return self.heads[which](x)

    m = M()
    jm = thunder.jit(m)
    x = torch.randn(5, 4)
    for w in ("a", "b"):
        torch.testing.assert_close(jm(x, w), m(x, w))
    out = jm(x, "b").sum()
    out.backward()
    assert m.heads["a"].weight.grad is not None


def test_einops_rearrange_reduce_repeat():
    einops = pytest.importorskip("einops")

    def f(x):
        y = einops.rearrange(x, "b (h d) t -> b h t d", h=2)
        z = einops.reduce(y, "b h t d -> b t", "mean")
        return einops.repeat(z, "b t -> b t k", k=3)

    x = torch.randn(2, 8, 5, requires_grad=True)
    jf = thunder.jit(f)
    out = jf(x)
    torch.testing.assert_close(out, f(x))
    out.sum().backward()
    g = x.grad.clone()
    x.grad = None
    f(x).sum().backward()
    torch.testing.assert_close(g, x.grad)


def test_autocast_bf16_matmul():
    def f(a, b):
        return (a @ b).sum(-1)

    a, b = torch.randn(8, 16), torch.randn(16, 4)
    jf = thunder.jit(f)
    with torch.autocast("cpu", dtype=torch.bfloat16):
        out = jf(a, b)
        ref = f(a, b)
    assert out.dtype == ref.dtype == torch.bfloat16
    torch.testing.assert_close(out, ref, atol=1e-1, rtol=2e-2)
    out2 = jf(a, b)  # outside autocast: another cache entry, fp32
    assert out2.dtype == torch.float32


def test_randomness_follows_torch_seed():
    def f(x):
        return torch.nn.functional.dropout(x, 0.5, training=True) + torch.rand_like(x)

    jf = thunder.jit(f)
    x = torch.ones(64, 64)
    torch.manual_seed(7)
    a = jf(x)
    torch.manual_seed(7)
    b = jf(x)
    torch.testing.assert_close(a, b)
    c = jf(x)
    assert not torch.equal(a, c)
    kept = (a >= 1.0).float().mean().item()
    assert 0.35 < kept < 0.65  # dropout keeps ~half


def test_custom_executor_register_operator_and_claim():
    from lightning_thunder_amd.extend import OperatorExecutor, register_executor
    from lightning_thunder_amd import torch as ltorch

    ex = OperatorExecutor("test_relu_ex")
    register_executor(ex)
    calls = []

    def relu_impl(a):
        calls.append(1)
        return torch.clamp_min(a, 0)

    op = ex.register_operator("my_relu", like=ltorch.relu, fn=relu_impl)
    ex.register_implementation(ltorch.relu, op, checker=lambda a, *r, **k: True)
    jf = thunder.jit(lambda x: torch.relu(x) * 2, executors=[ex])
    x = torch.randn(10)
    torch.testing.assert_close(jf(x), torch.relu(x) * 2)
    assert calls and "my_relu" in str(thunder.last_traces(jf)[-1])


def test_auto_registered_torch_op_fwd_bwd():
    def f(x):
        return torch.special.i0(x).sum() + torch.cummax(x, 0).values.sum()

    x = torch.randn(6, requires_grad=True)
    jf = thunder.jit(f)
    out = jf(x)
    torch.testing.assert_close(out, f(x))
    out.backward()
    g = x.grad.clone()
    x.grad = None
    f(x).backward()
    torch.testing.assert_close(g, x.grad)
    names = thunder.get_auto_registered_torch_op_names()
    assert any("i0" in n for n in names)


class _Box:
    def __init__(self, t):
        self.t = t
        self.n = torch.zeros((), dtype=torch.int64)


def _forward_through(*args, **kwargs):  # a forwarding decorator-style wrapper (drops nothing, hides provenance)
    return _use_box(*args, **kwargs)


def _use_box(x, box):
    box.n.add_(1)
    return {"y": x + box.t, "box": box}


def test_returned_input_objects_and_forwarded_provenance():
    jf = thunder.jit(lambda x, box: _forward_through(x, box=box))
    x = torch.randn(3)
    b1, b2 = _Box(torch.ones(3)), _Box(torch.full((3,), 2.0))
    o1 = jf(x, b1)
    o2 = jf(x, b2)  # same program (cache hit) on another object
    assert thunder.cache_hits(jf) == 1
    assert o1["box"] is b1 and o2["box"] is b2  # the caller's objects of each call come back
    torch.testing.assert_close(o2["y"], x + 2)
    assert int(b1.n) == 1 and int(b2.n) == 1  # in-place updates land on each call's own tensor


# ---- cache="symbolic values" (reference CACHE_OPTIONS.SYMBOLIC_VALUES, thunder/core/options.py:45-88) ----
def test_symbolic_values_reuse_program_across_numbers():
    def f(x, a, b):
        return x * a + b

    jf = thunder.jit(f, cache="symbolic values")
    x = torch.randn(4)
    for a, b in [(2.0, 1), (3.5, 2), (-1.0, 7)]:
        torch.testing.assert_close(jf(x, a, b), f(x, a, b))
    assert thunder.cache_misses(jf) == 1 and thunder.cache_hits(jf) == 2
    pro = str(thunder.last_prologue_traces(jf)[-1])
    assert "check_number_type(" in pro and "check_number_type_and_value" not in pro
    comp = str(thunder.last_traces(jf)[-1])
    assert "2.0" not in comp  # the number is an input of the program, not a baked constant
    # a different Python type is a different program
    jf(x, 2, 1)
    assert thunder.cache_misses(jf) == 2


def test_symbolic_values_specialize_when_value_is_read():
    def g(x, n):
        if n > 2:  # branching on a size-like int records the guard n > 2 (core/symbolic.py)
            return x * n
        return x - n

    jg = thunder.jit(g, cache="symbolic values")
    x = torch.randn(6)
    for n in (3, 5, 1, 3):
        torch.testing.assert_close(jg(x, n), g(x, n))
    # 3 and 5 take the same branch: one program (guard s0 > 2); 1 (< 2, a static value) is another
    assert thunder.cache_misses(jg) == 2 and thunder.cache_hits(jg) == 2
    guards = thunder.compile_stats(jg).interpreter_cache[0].shape_guards.source
    assert "s1 > 2" in guards, guards  # s0 is x.shape[0], s1 the int argument n

    def h(x, n):
        return x * float(n)  # float() needs the bare value: this input is specialized

    jh = thunder.jit(h, cache="symbolic values")
    for n in (3, 5, 3):
        torch.testing.assert_close(jh(x, n), h(x, n))
    assert thunder.cache_misses(jh) == 2 and thunder.cache_hits(jh) == 1

    def h(x, n):  # used as a shape
        return x.reshape(n, -1).sum(0) * n

    jh = thunder.jit(h, cache="symbolic values")
    for n in (2, 3, 2):
        torch.testing.assert_close(jh(x, n), h(x, n))
    # a size argument is a dim symbol: reshape(n, -1) prints as reshape(s1, s0 // s1), one program
    # (guarded by s1 * (s0 // s1) == s0) serves n = 2 and n = 3
    assert thunder.cache_misses(jh) == 1


def test_symbolic_values_backward():
    def f(x, a):
        return (x * a).sin().sum()

    jf = thunder.jit(f, cache="symbolic values")
    for a in (2.0, 3.0, -0.5):
        x = torch.randn(5, requires_grad=True)
        jf(x, a).backward()
        x2 = x.detach().requires_grad_()
        f(x2, a).backward()
        torch.testing.assert_close(x.grad, x2.grad)
    assert thunder.cache_misses(jf) == 1


# ---- grad mode, default dtype / device, layout, trace I/O (reference test_core.py parity) --------
def test_no_grad_region_inside_jitted_function():
    def f(a):
        with torch.no_grad():
            b = a * 2
        return a * b

    a = torch.randn(3, requires_grad=True)
    thunder.jit(f)(a).sum().backward()
    a2 = a.detach().clone().requires_grad_(True)
    f(a2).sum().backward()
    torch.testing.assert_close(a.grad, a2.grad)
    assert torch.is_grad_enabled()


def test_set_grad_enabled_inside_jitted_function():
    def f(a):
        torch.set_grad_enabled(False)
        b = a.exp()
        torch.set_grad_enabled(True)
        return (a * b).sum()

    a = torch.randn(4, requires_grad=True)
    thunder.jit(f)(a).backward()
    torch.testing.assert_close(a.grad, a.detach().exp())  # b is a constant for autograd


def test_change_default_dtype_in_jitted_fn_raises():
    def fn(x):
        torch.set_default_dtype(torch.float16)
        return torch.ones(x.shape)

    with pytest.raises(RuntimeError, match="Default dtype is changed during the execution of jitted function"):
        thunder.jit(fn)(torch.randn(3, 3))
    assert torch.get_default_dtype() == torch.float32


def test_factory_dtype_resolved_at_trace_time():
    def fn():
        torch.set_default_dtype(torch.float64)
        r = torch.ones(2)
        torch.set_default_dtype(torch.float32)
        return r

    jf = thunder.jit(fn)
    assert jf().dtype == torch.float64 and jf().dtype == torch.float64
    assert "dtype=torch.float64" in str(thunder.last_traces(jf)[-1])


def test_to_memory_format():
    def fn(a):
        return a.to(memory_format=torch.channels_last)

    a = torch.randn(2, 3, 4, 5)
    out = thunder.jit(fn)(a)
    assert out.is_contiguous(memory_format=torch.channels_last)
    torch.testing.assert_close(out, a)


def _serialize_fn(a, b, arr):
    res = a + b
    for t in arr:
        res = res + t
    return res


def test_serialize_and_save_trace(tmp_path):
    import dill

    from lightning_thunder_amd.core.transforms import eval_trace

    tm = thunder.jit(_serialize_fn)
    a, b = torch.randn(2, 5)
    tm(a, b, [a, b])
    trace = thunder.last_traces(tm)[0]
    assert str(dill.loads(dill.dumps(trace))) == str(trace)
    pro = thunder.last_prologue_traces(tm)[0]
    assert str(dill.loads(dill.dumps(pro))) == str(pro)
    assert dill.loads(dill.dumps(thunder.dtypes.float32)) is thunder.dtypes.float32
    p = tmp_path / "trace.py"
    trace.save_trace(p)
    assert p.read_text() == trace.python()
    final = thunder.last_traces(tm)[-1]
    out = eval_trace(final, *[a, b, a, b][: len(final.args)])  # the computation takes flattened inputs
    torch.testing.assert_close(out if isinstance(out, torch.Tensor) else out[0], _serialize_fn(a, b, [a, b]))


def test_dataclass_outputs_hold_tensors():
    import dataclasses

    @dataclasses.dataclass
    class Out:
        a: torch.Tensor
        d: dict

    def f(x):
        return Out(x * 2, {"k": x + 1})

    r = thunder.jit(f)(torch.ones(2))
    assert isinstance(r, Out) and type(r.a) is torch.Tensor and type(r.d["k"]) is torch.Tensor
    torch.testing.assert_close(r.d["k"], torch.full((2,), 2.0))


def test_dataclass_dict_output():
    import dataclasses

    @dataclasses.dataclass
    class Foo(dict):  # diffusers-style output
        musthave: int

    def fn():
        return Foo(musthave=1)

    assert fn() == thunder.jit(fn)()
    assert thunder.jit(fn)().musthave == 1


def test_isinstance_parameter():
    class Model(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.fc = torch.nn.Linear(1, 1)

        def forward(self, x):
            return x + 1 if isinstance(self.fc.weight, torch.nn.Parameter) else x

    m = Model()
    x = torch.ones(1)
    torch.testing.assert_close(thunder.jit(m)(x), m(x))
    # a parameter reached through a closure
    w = torch.nn.Parameter(torch.ones(1))
    torch.testing.assert_close(thunder.jit(lambda x: x * 2 if isinstance(w, torch.nn.Parameter) else x)(x), x * 2)


def test_compile_within_jit():
    def model(a, b, c):
        return a @ b + c

    def jit_me(a, b, c):
        return torch.compile(model)(a, b, c)

    with pytest.raises(NotImplementedError, match="Using torch.compile within a function"):
        thunder.jit(jit_me)(torch.randn(2, 2), torch.randn(2, 2), torch.randn(2, 2))


def test_jitted_callable_inlined_in_jit():
    g = thunder.jit(lambda x: x * 2)
    lin = thunder.jit(torch.nn.Linear(2, 2))

    def f(x):
        return g(x) + lin(x).sum()

    x = torch.randn(3, 2)
    jf = thunder.jit(f)
    torch.testing.assert_close(jf(x), x * 2 + lin._model(x).sum())
    assert len(thunder.last_traces(jf)) > 0


def test_isinstance_tensor_and_is_tensor_in_user_code():
    def f(x, m):
        y = x * 2 if isinstance(x, torch.Tensor) else x
        if torch.is_tensor(m):
            y = y + m
        return y

    x = torch.ones(2)
    torch.testing.assert_close(thunder.jit(f)(x, x), f(x, x))
    torch.testing.assert_close(thunder.jit(f)(x, None), f(x, None))


@pytest.mark.parametrize("k", range(4))
def test_complex_gradients(k):
    fns = [lambda x: (x * x.conj()).real.sum(), lambda x: (x * 3).imag.sum(), lambda x: (x.real * x.imag).sum(),
           lambda x: torch.view_as_real(x * 2).sum()]
    f = fns[k]
    x = torch.randn(3, dtype=torch.complex64, requires_grad=True)
    y = x.detach().clone().requires_grad_(True)
    thunder.jit(f)(x).backward()
    f(y).backward()
    torch.testing.assert_close(x.grad, y.grad)


def test_backward_retain_graph():
    x = torch.randn(3, requires_grad=True)
    out = thunder.jit(lambda x: (x ** 2).sum())(x)
    out.backward(retain_graph=True)
    out.backward()
    torch.testing.assert_close(x.grad, 4 * x.detach())
    with pytest.raises(RuntimeError, match="second time"):
        out.backward()


def test_train_eval_switch_retraces():
    m = torch.nn.Sequential(torch.nn.Linear(4, 4), torch.nn.Dropout(0.5))
    jm = thunder.jit(m)
    x = torch.ones(8, 4)
    m.eval()
    torch.testing.assert_close(jm(x), m(x))
    m.train()
    torch.manual_seed(0)
    out = jm(x)
    assert (out == 0).any()  # dropout active again
    assert thunder.cache_misses(jm) == 2
