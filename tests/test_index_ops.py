"""K11 / K12 index kernels (csrc/index_ops.hip) against PyTorch references: stable sort / argsort,
top-k, cumsum, deterministic index_add and embedding backward, and their claiming by the HIP
executor (reference coverage: nvFuser embedding / index_put / topk / argsort / cumsum,
thunder/executors/nvfuserex_impl.py:3162-3302)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _x(shape, dtype, ties=False, seed=0):
    g = torch.Generator(device="cuda").manual_seed(seed)
    if dtype == torch.int32:
        return torch.randint(-50, 50, shape, device="cuda", dtype=dtype, generator=g)
    x = torch.randn(shape, device="cuda", generator=g)
    if ties:
        x = (x * 4).round() / 4  # many equal values
    return x.to(dtype)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16, torch.int32])
@pytest.mark.parametrize("shape,dim", [((4, 1000), -1), ((3, 7, 33), 1), ((2, 16384), -1), ((5, 1), -1)])
@pytest.mark.parametrize("descending", [False, True])
def test_sort_matches_stable_torch(dtype, shape, dim, descending):
    from lightning_thunder_amd.ops import index_ops

    x = _x(shape, dtype, ties=True)
    v, i = index_ops.sort(x, dim, descending)
    rv, ri = torch.sort(x, dim=dim, descending=descending, stable=True)
    assert torch.equal(v, rv)
    assert torch.equal(i, ri)


def test_sort_nan_and_signed_zero():
    from lightning_thunder_amd.ops import index_ops

    x = torch.tensor([[1.0, float("nan"), -0.0, 0.0, -float("inf"), 2.0, float("nan")]], device="cuda")
    v, i = index_ops.sort(x, -1, False)
    rv, ri = torch.sort(x, stable=True)
    assert torch.equal(i, ri)
    assert torch.equal(v.isnan(), rv.isnan())


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("N,k", [(8, 2), (64, 8), (256, 8), (160, 6), (2048, 64), (5000, 10)])
@pytest.mark.parametrize("largest", [True, False])
def test_topk(dtype, N, k, largest):
    from lightning_thunder_amd.ops import index_ops

    x = _x((300, N), dtype)
    v, i = index_ops.topk(x, k, -1, largest)
    rv, ri = torch.topk(x.float(), k, -1, largest)
    assert torch.equal(v.float(), rv)
    assert torch.equal(torch.gather(x, -1, i), v)
    if dtype == torch.float32:
        assert torch.equal(i, ri)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.int64, torch.int32])
@pytest.mark.parametrize("shape,dim", [((8, 5000), -1), ((3, 100, 4), 1), ((1, 1), 0)])
def test_cumsum(dtype, shape, dim):
    from lightning_thunder_amd.ops import index_ops

    x = _x(shape, torch.int32 if dtype in (torch.int32, torch.int64) else dtype).to(dtype)
    y = index_ops.cumsum(x, dim)
    if dtype in (torch.int32, torch.int64):
        assert y.dtype == torch.int64
        assert torch.equal(y, torch.cumsum(x, dim, dtype=torch.int64))
        y32 = index_ops.cumsum(x, dim, torch.int32)  # MoE routing offsets are int32
        assert y32.dtype == torch.int32 and torch.equal(y32, torch.cumsum(x, dim, dtype=torch.int32))
    else:
        ref = torch.cumsum(x.double(), dim)
        assert y.dtype == dtype
        tol = 1e-4 if dtype == torch.float32 else 2e-2
        torch.testing.assert_close(y.double(), ref, rtol=tol, atol=tol * ref.abs().max().item())


@pytest.mark.parametrize("T", [4096, 20000])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_embedding_backward(T, dtype):
    from lightning_thunder_amd.ops import index_ops

    V, D = 3000, 256
    g = torch.Generator(device="cuda").manual_seed(1)
    idx = torch.randint(0, V, (T,), device="cuda", generator=g)
    idx[::7] = 5  # a heavily repeated token
    grad = torch.randn(T, D, device="cuda", generator=g).to(dtype)
    out = index_ops.embedding_backward(grad, idx, V, padding_idx=-1)
    ref = torch.zeros(V, D, device="cuda", dtype=torch.float64).index_add_(0, idx, grad.double())
    torch.testing.assert_close(out.double(), ref, rtol=1e-2, atol=1e-2 if dtype == torch.bfloat16 else 1e-4)
    assert torch.equal(out, index_ops.embedding_backward(grad, idx, V))  # bitwise reproducible

    out_p = index_ops.embedding_backward(grad, idx, V, padding_idx=5, scale_grad_by_freq=True)
    ref_p = torch.ops.aten.embedding_backward(grad.float(), idx, V, 5, True, False)
    assert (out_p[5] == 0).all()
    torch.testing.assert_close(out_p.float(), ref_p, rtol=1e-2, atol=1e-2)


def test_index_add():
    from lightning_thunder_amd.ops import index_ops

    a = torch.randn(100, 4, 16, device="cuda")
    idx = torch.randint(0, 100, (700,), device="cuda")
    src = torch.randn(700, 4, 16, device="cuda")
    out = index_ops.index_add(a, idx, src, alpha=0.5)
    torch.testing.assert_close(out, torch.index_add(a, 0, idx, src, alpha=0.5), rtol=1e-5, atol=1e-5)


def test_claimed_by_hipex_in_training():
    import lightning_thunder_amd as thunder

    emb = torch.nn.Embedding(512, 128, device="cuda", dtype=torch.bfloat16)
    router = torch.randn(128, 16, device="cuda", dtype=torch.bfloat16)

    def f(tok):
        h = emb(tok)  # [T, 128]
        scores = h @ router  # [T, 16]
        w, e = torch.topk(scores, 2, dim=-1)
        order = torch.argsort(e.reshape(-1), stable=True)
        counts = torch.cumsum(e.reshape(-1) % 3, 0)  # int64 scan (routing offsets)
        return (w.float().sum() + h.float().pow(2).mean()), order, counts, e

    tok = torch.randint(0, 512, (4, 256), device="cuda")
    jf = thunder.jit(f)
    loss, order, counts, e = jf(tok)
    rl, _, _, _ = f(tok)
    # bf16 scores tie often and torch.topk breaks ties in its own order: check the routing ops
    # against torch applied to the SAME expert choice, and the choice itself by gathered values
    assert torch.equal(order, torch.argsort(e.reshape(-1), stable=True))
    assert torch.equal(counts, torch.cumsum(e.reshape(-1) % 3, 0))
    torch.testing.assert_close(loss, rl, rtol=1e-3, atol=1e-3)
    loss.backward()
    gw = emb.weight.grad.clone()
    emb.weight.grad = None
    rl.backward()
    torch.testing.assert_close(gw.float(), emb.weight.grad.float(), rtol=2e-2, atol=2e-3)
    fw = str(thunder.last_traces(jf)[-1])
    bw = str(thunder.last_backward_traces(jf)[-1])
    assert "hip_topk" in fw and "hip_sort" in fw and "hip_cumsum" in fw, fw
    assert "hip_embedding_backward" in bw, bw
