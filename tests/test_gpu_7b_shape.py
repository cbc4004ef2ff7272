"""Llama-2-7B-shaped end-to-end numerics on the hand-written kernels.

``llama2-7b-shape-2l`` is two layers of the exact Llama-2-7B block (d 4096, 32 heads of 128,
SwiGLU 11008, vocab 32000) at sequence 2048, so every linear takes the hand-written MFMA GEMM
(forward NT, dgrad NN, wgrad TN), attention takes the flash kernels at a real length and the loss
takes the fused cross-entropy.  The compiled bf16 model is compared against an fp32 eager copy with
the rule of test_gpu_models.py: loss, logits and every parameter gradient within 3x the error of
bf16 eager (plus a small floor).  The traces must show the hand kernels were used.
"""
import pytest
import torch

import lightning_thunder_amd as thunder
from lightning_thunder_amd.models.litgpt import GPT, init_weights

pytestmark = pytest.mark.gpu

SEQ = 2048


def _rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


@pytest.mark.parametrize("gemm_mode", ["default", "hip", "fused_swiglu"])
def test_llama2_7b_shape_bf16_vs_fp32(gemm_mode, monkeypatch):
    if gemm_mode == "hip":
        monkeypatch.setenv("LTA_GEMM", "hip")
    if gemm_mode == "fused_swiglu":
        monkeypatch.setenv("LTA_FUSED_SWIGLU", "1")
    from lightning_thunder_amd.ops import gemm as G

    G.last_gemm_backend_counts(reset=True)  # counts are per process: earlier tests may have used torch
    torch.manual_seed(0)
    dev = torch.device("cuda")
    m32 = GPT.from_name("llama2-7b-shape-2l").to(device=dev)
    init_weights(m32)
    m32.set_rope_cache(SEQ, device=dev)
    m = GPT.from_name("llama2-7b-shape-2l").to(device=dev)
    m.load_state_dict(m32.state_dict())
    m = m.to(torch.bfloat16)
    m.set_rope_cache(SEQ, device=dev)
    V = m.config.padded_vocab_size
    idx = torch.randint(0, V, (1, SEQ), device=dev)
    tgt = torch.randint(0, V, (1, SEQ), device=dev)

    class TrainStep(torch.nn.Module):
        def __init__(self, mm):
            super().__init__()
            self.m = mm

        def forward(self, x, y):
            logits = self.m(x)
            return torch.nn.functional.cross_entropy(logits.reshape(-1, V), y.reshape(-1)), logits

    tm = thunder.jit(TrainStep(m))
    loss, logits = tm(idx, tgt)
    loss.backward()
    got = {n: p.grad.float() for n, p in m.named_parameters()}
    for p in m.parameters():
        p.grad = None
    eloss, elogits = TrainStep(m)(idx, tgt)
    eloss.backward()
    eg = {n: p.grad.float() for n, p in m.named_parameters()}
    rloss, rlogits = TrainStep(m32)(idx, tgt)
    rloss.backward()

    base = max(abs(eloss.item() - rloss.item()) / abs(rloss.item()), 1e-4)
    assert abs(loss.item() - rloss.item()) / abs(rloss.item()) <= 3 * base, (loss.item(), eloss.item(), rloss.item())
    base = max(_rel(elogits, rlogits), 1e-5)
    assert _rel(logits, rlogits) <= 3 * base + 1e-4, (_rel(logits, rlogits), base)
    for n, p in m32.named_parameters():
        b = max(_rel(eg[n], p.grad), 1e-5)
        e = _rel(got[n], p.grad)
        assert e <= 3 * b + 1e-4, (n, e, b)

    fw = str(thunder.last_traces(tm)[-1])
    bw = str(thunder.last_backward_traces(tm)[-1])
    assert "hip_linear" in fw and "hip_flash_attn_fwd" in fw and "hip_cross_entropy_fwd" in fw, fw
    assert "hip_matmul" in bw and "hip_flash_attn_bwd" in bw, bw
    # the MLP's SwiGLU runs in the GEMM epilogues (gate-up forward, down-projection dgrad backward)
    if gemm_mode == "fused_swiglu":
        assert "hip_gate_up" in fw and "hip_swiglu(" not in fw, fw
        assert "hip_matmul_swiglu_bwd" in bw and "hip_swiglu_bwd(" not in bw, bw
    assert "hip_linear_qkv_rope" in fw and "hip_qkv_rope(" not in fw, fw
    # ... and its backward in the attention backward's dQ / dK epilogues
    assert "hip_flash_attn_bwd_rope" in bw and "hip_qkv_rope_bwd(" not in bw, bw
    from lightning_thunder_amd.ops import gemm as G

    # every GEMM of the step ran on the hand-written kernel (no library fallback)
    assert G.last_gemm_backend_counts().get("torch", 0) == 0, G.last_gemm_backend_counts()


@pytest.mark.parametrize("tp", [2, 8])
def test_llama3_8b_tensor_parallel_shard_shapes_on_hand_gemms(tp):
    """BASELINE config 4 (Llama-3-8B, TP=8, seq 8192): one rank's GEMMs are the shard shapes — the
    head-parallel qkv (4 query heads + 1 kv group at TP=8), the row-parallel proj (K = 512), the
    column-parallel SwiGLU pair (N = 1792) and its down projection (K = 1792), the vocab-parallel LM head
    (N = 16032).  One rank's block runs here as a plain model with those local sizes (the collectives
    are identity at world 1); every forward and backward GEMM must take the hand-written kernel (no
    library fallback), and the step must match fp32 eager."""
    from lightning_thunder_amd.ops import gemm as G

    seq = 8192
    cfg = dict(n_layer=1, n_head=32 // tp, n_query_groups=8 // tp, intermediate_size=14336 // tp,
               padded_vocab_size=128256 // tp, vocab_size=128256 // tp)
    torch.manual_seed(0)
    dev = torch.device("cuda")
    m = GPT.from_name("Llama-3-8B", **cfg).to(device=dev)
    init_weights(m)
    m = m.to(torch.bfloat16)
    m.set_rope_cache(seq, device=dev)
    idx = torch.randint(0, cfg["vocab_size"], (1, seq), device=dev)
    tgt = torch.randint(0, cfg["vocab_size"], (1, seq), device=dev)

    class TrainStep(torch.nn.Module):
        def __init__(self, mm):
            super().__init__()
            self.m = mm

        def forward(self, x, y):
            logits = self.m(x)
            return torch.nn.functional.cross_entropy(logits.reshape(-1, logits.shape[-1]), y.reshape(-1))

    tm = thunder.jit(TrainStep(m))
    G.last_gemm_backend_counts(reset=True)
    loss = tm(idx, tgt)
    loss.backward()
    torch.cuda.synchronize()
    counts = G.last_gemm_backend_counts(reset=True)
    assert counts.get("torch", 0) == 0 and counts.get("gemm4", 0) > 0, counts
    with torch.no_grad():
        ref = TrainStep(m)(idx, tgt).float()
    assert abs(loss.item() - ref.item()) / abs(ref.item()) < 2e-2, (loss.item(), ref.item())
    assert all(p.grad is not None and torch.isfinite(p.grad).all() for p in m.parameters())


def _loss_curve(step_module, params, opt, data, steps):
    curve = []
    for i in range(steps):
        x, y = data[i % len(data)]
        loss = step_module(x, y)
        loss.backward()
        opt.step()
        opt.zero_grad(set_to_none=True)
        curve.append(loss.detach().float().clone())  # a graphed loss is overwritten by the next replay
    return [float(v) for v in torch.stack(curve).cpu()]


def test_llama2_7b_shape_training_trajectory_vs_eager():
    """10 optimizer steps of the 2-layer Llama-2-7B-shape model: thunder (HIP kernels + the fused HIP
    AdamW, as bench.py runs it) vs bf16 eager (torch fused AdamW) vs an fp32 eager reference, from one
    init and the same 4 cycling batches (reference: benchmark_litgpt.py:842-846 logs every iteration's
    loss).  Thunder's distance from the fp32 curve must stay within the band bf16 eager itself keeps."""
    from lightning_thunder_amd.optim import AdamW as HipAdamW

    torch.manual_seed(0)
    dev = torch.device("cuda")
    m32 = GPT.from_name("llama2-7b-shape-2l").to(device=dev)
    init_weights(m32)
    m32.set_rope_cache(SEQ, device=dev)
    V = m32.config.padded_vocab_size
    state = {k: v.clone() for k, v in m32.state_dict().items()}
    gen = torch.Generator(device=dev)
    gen.manual_seed(7)
    data = []
    for _ in range(4):
        t = torch.randint(0, m32.config.vocab_size, (1, SEQ + 1), device=dev, generator=gen)
        data.append((t[:, :-1].contiguous(), t[:, 1:].contiguous()))

    class TrainStep(torch.nn.Module):
        def __init__(self, mm):
            super().__init__()
            self.m = mm

        def forward(self, x, y):
            return torch.nn.functional.cross_entropy(self.m(x).reshape(-1, V).float(), y.reshape(-1))

    kw = dict(lr=1e-4, betas=(0.9, 0.95), weight_decay=0.1)
    steps = 10
    c32 = _loss_curve(TrainStep(m32), None, torch.optim.AdamW(m32.parameters(), **kw), data, steps)

    def bf16_model():
        m = GPT.from_name("llama2-7b-shape-2l").to(device=dev)
        m.load_state_dict(state)
        m = m.to(torch.bfloat16)
        m.set_rope_cache(SEQ, device=dev)
        return m

    me = bf16_model()
    ce = _loss_curve(TrainStep(me), None, torch.optim.AdamW(me.parameters(), fused=True, **kw), data, steps)
    del me
    mt = bf16_model()
    tm = thunder.jit(TrainStep(mt))
    ct = _loss_curve(tm, None, HipAdamW([p for p in mt.parameters()], **kw), data, steps)

    band = max(abs(a - b) for a, b in zip(ce, c32))
    gap = max(abs(a - b) for a, b in zip(ct, c32))
    assert c32[-1] < 0.5 * c32[0], c32  # the run trains (memorizes the 4 batches)
    assert gap <= 2 * band + 0.05, {"fp32": c32, "eager_bf16": ce, "thunder": ct, "band": band, "gap": gap}
    for k in range(steps):
        assert abs(ct[k] - ce[k]) <= 2 * band + 0.05, (k, ct, ce, band)


def test_llama2_7b_shape_training_under_hipgraph():
    """The 2-layer 7B-shape model trains under HipGraphTransform(donate_grads=True) (forward and
    backward replayed as hipGraphs, gradients adopted by autograd without a clone, the HIP AdamW
    outside the graphs) with the same loss trajectory band as the uncaptured program, and the graphs
    really replay (reference thunder/tests/test_networks.py:95-160)."""
    from lightning_thunder_amd.optim import AdamW as HipAdamW
    from lightning_thunder_amd.transforms.hipgraph import HipGraphTransform

    torch.manual_seed(0)
    dev = torch.device("cuda")
    m32 = GPT.from_name("llama2-7b-shape-2l").to(device=dev)
    init_weights(m32)
    m32.set_rope_cache(SEQ, device=dev)
    V = m32.config.padded_vocab_size
    state = {k: v.clone() for k, v in m32.state_dict().items()}
    gen = torch.Generator(device=dev)
    gen.manual_seed(7)
    data = []
    for _ in range(4):
        t = torch.randint(0, m32.config.vocab_size, (1, SEQ + 1), device=dev, generator=gen)
        data.append((t[:, :-1].contiguous(), t[:, 1:].contiguous()))

    class TrainStep(torch.nn.Module):
        def __init__(self, mm):
            super().__init__()
            self.m = mm

        def forward(self, x, y):
            return torch.nn.functional.cross_entropy(self.m(x).reshape(-1, V).float(), y.reshape(-1))

    kw = dict(lr=1e-4, betas=(0.9, 0.95), weight_decay=0.1)
    steps = 8
    c32 = _loss_curve(TrainStep(m32), None, torch.optim.AdamW(m32.parameters(), **kw), data, steps)
    curves = {}
    for mode in ("plain", "hipgraph"):
        m = GPT.from_name("llama2-7b-shape-2l").to(device=dev)
        m.load_state_dict(state)
        m = m.to(torch.bfloat16)
        m.set_rope_cache(SEQ, device=dev)
        t = HipGraphTransform(donate_grads=True) if mode == "hipgraph" else None
        tm = thunder.jit(TrainStep(m), transforms=[t] if t else [])
        curves[mode] = _loss_curve(tm, None, HipAdamW(list(m.parameters()), **kw), data, steps)
        if t is not None:
            assert sum(r.replays for r in t.runners) >= 2 * (steps - 2), [(r.name, r.replays) for r in t.runners]
        del tm, m
    band = max(abs(a - b) for a, b in zip(curves["plain"], c32))
    gap = max(abs(a - b) for a, b in zip(curves["hipgraph"], c32))
    assert gap <= 2 * band + 0.05, {"fp32": c32, **curves, "band": band}


def test_llama2_7b_shape_fp8_delayed_training_fusions():
    """The FP8 (delayed scaling) path of BASELINE config 5 on the 7B block: the attention input
    projection runs the fp8 GEMM with the RoPE split in its epilogue (no qkv tensor, no rope pass),
    the fused AdamW refreshes the e4m3 weight shadows (later forwards launch no weight casts), and
    three training steps track the bf16 compiled model's losses to fp8 accuracy."""
    from lightning_thunder_amd.ops import fp8
    from lightning_thunder_amd.optim import AdamW
    from lightning_thunder_amd.transforms.fp8 import FP8LinearTransform

    dev = torch.device("cuda")
    losses = {}
    for mode in ("fp8", "bf16"):
        torch.manual_seed(0)
        m = GPT.from_name("llama2-7b-shape-2l").to(device=dev, dtype=torch.bfloat16)
        init_weights(m)
        m.set_rope_cache(SEQ, device=dev)
        V = m.config.padded_vocab_size

        class TrainStep(torch.nn.Module):
            def __init__(self, mm):
                super().__init__()
                self.m = mm

            def forward(self, x, y):
                return torch.nn.functional.cross_entropy(self.m(x).reshape(-1, V), y.reshape(-1))

        tm = thunder.jit(TrainStep(m), transforms=[FP8LinearTransform("delayed")] if mode == "fp8" else [])
        opt = AdamW(m.parameters(), lr=1e-4)
        n0 = fp8.SHADOW_STATS["reused"]
        out = []
        for step in range(3):
            g = torch.Generator(device=dev).manual_seed(step)
            idx = torch.randint(0, V, (1, SEQ), device=dev, generator=g)
            loss = tm(idx, torch.roll(idx, -1, 1))
            loss.backward()
            opt.step()
            opt.zero_grad(set_to_none=True)
            out.append(loss.item())
        losses[mode] = out
        if mode == "fp8":
            fw = str(thunder.last_traces(tm)[-1])
            assert "hip_fp8_gemm_qkv_rope" in fw and "hip_qkv_rope(" not in fw, fw
            assert "hip_flash_attn_fwd_fp8" in fw, fw  # the o-projection's e4m3 input from the attention epilogue
            bw = str(thunder.last_backward_traces(tm)[-1])
            assert "hip_rms_norm_bwd_fp8" in bw, bw  # residual-stream e5m2 gradients from the norm backward
            # 2 layers x 5 linears (qkv, proj, fc_1, fc_2, mlp.proj) + lm head, forwards 2 and 3
            assert fp8.SHADOW_STATS["reused"] - n0 >= 2 * 11, fp8.SHADOW_STATS
        fp8._SHADOWS.clear()
    for a, b in zip(losses["fp8"], losses["bf16"]):
        assert abs(a - b) <= 0.02 * abs(b), losses


def test_llama2_7b_shape_fp8_producer_fusions_bit_identical(monkeypatch):
    """Every FP8 producer fusion of the 7B block (RMSNorm / SwiGLU forwards, the attention epilogue's e4m3
    output, the SwiGLU and RMSNorm backwards' e5m2 gradients) against the same program with the casts as
    separate launches: losses and all parameter gradients of two delayed-scaling steps are bit-identical."""
    from lightning_thunder_amd.transforms.fp8 import FP8LinearTransform

    dev = torch.device("cuda")
    res = {}
    for fuse in ("1", "0"):
        monkeypatch.setenv("LTA_FP8_FUSE_PRODUCERS", fuse)
        torch.manual_seed(0)
        m = GPT.from_name("llama2-7b-shape-2l").to(device=dev, dtype=torch.bfloat16)
        init_weights(m)
        m.set_rope_cache(SEQ, device=dev)
        V = m.config.padded_vocab_size
        tm = thunder.jit(m, transforms=[FP8LinearTransform("delayed")])
        outs = []
        for step in range(2):
            g = torch.Generator(device=dev).manual_seed(step)
            idx = torch.randint(0, V, (1, SEQ), device=dev, generator=g)
            loss = torch.nn.functional.cross_entropy(tm(idx).reshape(-1, V).float(), torch.roll(idx, -1, 1).reshape(-1))
            grads = torch.autograd.grad(loss, [p for p in m.parameters() if p.requires_grad])
            outs.append((loss.detach(),) + tuple(grads))
        fw = str(thunder.last_traces(tm)[-1])
        assert ("hip_flash_attn_fwd_fp8" in fw) == (fuse == "1"), fw
        res[fuse] = outs
        del tm, m
    for a, b in zip(res["1"], res["0"]):
        for u, v in zip(a, b):
            torch.testing.assert_close(u, v, rtol=0, atol=0)
