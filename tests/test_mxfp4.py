"""MXFP4 (OCP e2m1 elements, E8M0 scale per 32): operand layout of the block-scaled MFMA, the
quantiser and the GEMM.  Numerics are checked against a pure-torch fp32 dequantise-and-matmul."""
import pytest
import torch

E2M1 = [0.0, 0.5, 1.0, 1.5, 2.0, 3.0, 4.0, 6.0]


def e2m1_value(codes: torch.Tensor) -> torch.Tensor:
    mag = torch.tensor(E2M1, dtype=torch.float64)[(codes & 7).long()]
    return torch.where((codes & 8) != 0, -mag, mag)


# candidate k orders for lane l, byte j, nibble n of a 16x16x128 fp4 operand
HYPOTHESES = {
    "lane-block, low nibble first": lambda l, j, n: 32 * (l >> 4) + 2 * j + n,
    "lane-block, high nibble first": lambda l, j, n: 32 * (l >> 4) + 2 * j + 1 - n,
    "split halves": lambda l, j, n: (16 * (l >> 4) + 2 * j + n) if j < 8 else (64 + 16 * (l >> 4) + 2 * (j - 8) + n),
    "split halves, high nibble first": lambda l, j, n: ((16 * (l >> 4) + 2 * j + 1 - n) if j < 8
                                                         else (64 + 16 * (l >> 4) + 2 * (j - 8) + 1 - n)),
}
FP4_ORDER = "lane-block, low nibble first"


def _pack_fp4(codes: torch.Tensor, order) -> torch.Tensor:
    """codes [16 rows, 128 k] -> per-lane registers [64, 32] bytes (upper 16 bytes zero)."""
    regs = torch.zeros(64, 32, dtype=torch.int32)
    for l in range(64):
        for j in range(16):
            lo = codes[l & 15, order(l, j, 0)]
            hi = codes[l & 15, order(l, j, 1)]
            regs[l, j] = int(lo) | (int(hi) << 4)
    return regs.to(torch.uint8)


def _unpack_acc(c: torch.Tensor) -> torch.Tensor:
    got = torch.zeros(16, 16, dtype=torch.float64)
    for l in range(64):
        for r in range(4):
            got[(l >> 4) * 4 + r, l & 15] = float(c[l, r])
    return got


def _fp8_lanes(x: torch.Tensor) -> torch.Tensor:
    """e4m3 operand [16, 128] -> per-lane registers (the measured fp8 map of gemm.hip: lane group g
    holds k = 16g..16g+15 in bytes 0-15 and k = 64+16g..+15 in bytes 16-31)."""
    q = x.float().to(torch.float8_e4m3fn).view(torch.uint8)
    a = torch.zeros(64, 32, dtype=torch.uint8)
    for l in range(64):
        g = l >> 4
        a[l, :16] = q[l & 15, 16 * g: 16 * g + 16]
        a[l, 16:] = q[l & 15, 64 + 16 * g: 64 + 16 * g + 16]
    return a


def _matching_orders(fp4_is_a: bool, seed: int):
    """Which candidate order reproduces A . B^T exactly when one operand is e2m1 (in that order) and
    the other e4m3 in its known map (a same-order pair of fp4 operands cannot tell orders apart:
    the sum over k is invariant under any common permutation)."""
    from lightning_thunder_amd.ops.fp8 import mfma_probe

    g = torch.Generator().manual_seed(seed)
    x8 = torch.randint(-8, 9, (16, 128), generator=g).double() / 4  # exact in e4m3
    c4 = torch.randint(0, 16, (16, 128), generator=g)
    found = []
    for name, order in HYPOTHESES.items():
        if fp4_is_a:
            c = mfma_probe(_pack_fp4(c4, order).cuda(), _fp8_lanes(x8).cuda(), 4, 0)
            ref = e2m1_value(c4) @ x8.T
        else:
            c = mfma_probe(_fp8_lanes(x8).cuda(), _pack_fp4(c4, order).cuda(), 0, 4)
            ref = x8 @ e2m1_value(c4).T
        if torch.equal(_unpack_acc(c.cpu()), ref):
            found.append(name)
    return found


@pytest.mark.gpu
@pytest.mark.parametrize("fp4_is_a", [True, False])
def test_mfma_fp4_operand_k_order(fp4_is_a):
    """Pins the e2m1 operand map of v_mfma_scale_f32_16x16x128_f8f6f4 (A and B side) with exact
    data against an e4m3 partner: exactly one candidate order must reproduce the product."""
    found = _matching_orders(fp4_is_a, seed=int(fp4_is_a))
    print("fp4 k order:", found)
    assert found == [FP4_ORDER], found


@pytest.mark.gpu
def test_mfma_fp4_pair_ignores_upper_registers():
    from lightning_thunder_amd.ops.fp8 import mfma_probe

    g = torch.Generator().manual_seed(2)
    ca = torch.randint(0, 16, (16, 128), generator=g)
    cb = torch.randint(0, 16, (16, 128), generator=g)
    order = HYPOTHESES[FP4_ORDER]
    a, b = _pack_fp4(ca, order), _pack_fp4(cb, order)
    a[:, 16:] = torch.randint(0, 256, (64, 16), generator=g).to(torch.uint8)
    b[:, 16:] = torch.randint(0, 256, (64, 16), generator=g).to(torch.uint8)
    got = _unpack_acc(mfma_probe(a.cuda(), b.cuda(), 4, 4).cpu())
    torch.testing.assert_close(got, e2m1_value(ca) @ e2m1_value(cb).T, rtol=0, atol=0)


# ---- quantiser ---------------------------------------------------------------------------------
def test_reference_quantiser_properties():
    from lightning_thunder_amd.ops import mxfp4

    torch.manual_seed(0)
    x = torch.randn(64, 256) * torch.logspace(-3, 3, 64).unsqueeze(1)
    x[3, 32:64] = 0.0  # an all-zero block
    q, s = mxfp4.quantize_reference(x)
    assert q.shape == (64, 128) and s.shape == (64, 8) and q.dtype == s.dtype == torch.uint8
    assert int(s[3, 1]) == 0 and int(q[3, 16:32].abs().sum()) == 0
    d = mxfp4.dequantize(q, s)
    xb, db = x.reshape(64, 8, 32), d.reshape(64, 8, 32)
    # no element saturates (the scale exponent rounds up) and the block max is represented to
    # within half an e2m1 step at the top of the range
    amax = xb.abs().amax(-1)
    scale = torch.exp2(s.float() - 127.0)
    assert torch.all(amax / torch.where(amax > 0, scale, torch.ones_like(scale)) <= 6.0)
    err = (db - xb).abs().amax(-1)
    assert torch.all(err <= scale * 1.0 + 1e-30)
    # grid values are exact
    g = torch.tensor([[0.5, -1.5, 3.0, -6.0] * 8])
    qg, sg = mxfp4.quantize_reference(g)
    assert torch.equal(mxfp4.dequantize(qg, sg), g)


def test_round_half_even_ties():
    from lightning_thunder_amd.ops import mxfp4

    # block max 6 -> scale 1: ties land on the even code
    v = torch.tensor([0.25, 0.75, 1.25, 1.75, 2.5, 3.5, 5.0, 6.0] * 4)
    q, s = mxfp4.quantize_reference(v.reshape(1, 32))
    assert int(s[0, 0]) == 127
    d = mxfp4.dequantize(q, s)[0, :8]
    assert d.tolist() == [0.0, 1.0, 1.0, 2.0, 2.0, 4.0, 4.0, 6.0]


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_quantise_kernel_matches_reference(dtype):
    from lightning_thunder_amd.ops import mxfp4

    torch.manual_seed(1)
    x = (torch.randn(256, 512) * torch.logspace(-4, 4, 256).unsqueeze(1)).to(dtype)
    x[7, :64] = 0
    q, s = mxfp4.quantize(x.cuda())
    rq, rs = mxfp4.quantize_reference(x)
    assert torch.equal(s.cpu(), rs)
    assert torch.equal(q.cpu(), rq)


@pytest.mark.gpu
@pytest.mark.parametrize("M,N,K,bias", [(256, 256, 256, False), (512, 768, 1024, True), (1024, 512, 4096, False)])
def test_gemm_nt_mxfp4(M, N, K, bias):
    """The MXFP4 GEMM equals an fp32 matmul of the dequantised operands (exact products; fp32
    accumulation order and the bf16 output rounding are the only differences)."""
    from lightning_thunder_amd.ops import mxfp4

    torch.manual_seed(2)
    a = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    b = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.05
    bi = torch.randn(N, device="cuda", dtype=torch.bfloat16) if bias else None
    qa, sa = mxfp4.quantize(a)
    qb, sb = mxfp4.quantize(b)
    out = mxfp4.gemm_nt(qa, sa, qb, sb, bi).float()
    ref = mxfp4.dequantize(qa, sa) @ mxfp4.dequantize(qb, sb).T
    if bias:
        ref = ref + bi.float()
    torch.testing.assert_close(out, ref, atol=2e-2 * ref.abs().max().item() / 8, rtol=1e-2)
    # and approximates the bf16 product at 4-bit accuracy
    full = a.float() @ b.float().T + (bi.float() if bias else 0)
    rel = ((out - full).norm() / full.norm()).item()
    assert rel < 0.2, rel


@pytest.mark.gpu
@pytest.mark.parametrize("M,N,K", [(1, 2048, 2048), (3, 8192, 2048), (8, 2048, 8192), (1, 130, 96)])
def test_gemv_mxfp4(M, N, K):
    """Weight-only decode GEMV (bf16 activations x 4-bit weights) against fp32 x . dequant(W)^T."""
    from lightning_thunder_amd.ops import mxfp4

    torch.manual_seed(3)
    w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    bias = torch.randn(N, device="cuda", dtype=torch.bfloat16)
    q, s = mxfp4.quantize(w)
    y = mxfp4.gemv(x, q, s, bias).float()
    ref = x.float() @ mxfp4.dequantize(q, s).T + bias.float()
    torch.testing.assert_close(y, ref, atol=3e-2, rtol=1e-2)


# ---- inference transform -----------------------------------------------------------------------
def _mlp(device, dtype):
    torch.manual_seed(4)
    return torch.nn.Sequential(torch.nn.Linear(256, 512), torch.nn.SiLU(), torch.nn.Linear(512, 256)).to(device, dtype)


def _dequant_reference(m, x):
    from lightning_thunder_amd.ops import mxfp4

    h = x.float()
    for layer in m:
        if isinstance(layer, torch.nn.Linear):
            q, s = mxfp4.quantize_reference(layer.weight.detach().float())
            h = h @ mxfp4.dequantize(q, s).T + layer.bias.float()
        else:
            h = layer(h)
    return h


def test_mxfp4_inference_transform_cpu():
    import lightning_thunder_amd as thunder
    from lightning_thunder_amd.transforms.mxfp4_inference import MXFP4InferenceTransform

    m = _mlp("cpu", torch.float32)
    x = torch.randn(4, 256)
    ref = _dequant_reference(m, x)
    t = MXFP4InferenceTransform()
    jm = thunder.jit(m, transforms=[t])
    out = jm(x)
    assert t.quantized == ["0", "2"]
    assert any("mxfp4" in str(b.sym.name) for b in thunder.last_traces(jm)[-1].bound_symbols)
    torch.testing.assert_close(out, ref, atol=1e-4, rtol=1e-4)
    # gradients reach the activations through the dequantized weights
    x.requires_grad_(True)
    jm(x).sum().backward()
    assert x.grad is not None and x.grad.abs().sum() > 0


@pytest.mark.gpu
@pytest.mark.parametrize("rows,activations", [(1, "bf16"), (6, "bf16"), (512, "bf16"), (300, "mxfp4")])
def test_mxfp4_inference_transform_gpu(rows, activations):
    import lightning_thunder_amd as thunder
    from lightning_thunder_amd.transforms.mxfp4_inference import MXFP4InferenceTransform

    m = _mlp("cuda", torch.bfloat16)
    x = torch.randn(rows, 256, device="cuda", dtype=torch.bfloat16)
    ref = _dequant_reference(m, x)
    jm = thunder.jit(m, transforms=[MXFP4InferenceTransform(activations=activations)])
    out = jm(x).float()
    rel = ((out - ref).norm() / ref.norm()).item()
    # W4A16 matches the dequantized model to bf16 rounding; W4A4 also quantizes the activations
    assert rel < (0.02 if activations == "bf16" else 0.25), rel
