"""Component benchmarks, forward and backward timed separately (parity: reference
``thunder/benchmarks/targets.py`` + ``thunder/benchmarks/__init__.py`` benchmark classes, run with
pytest-benchmark there; ``docs/source/intermediate/benchmarking.rst:90-101`` quotes
``test_nanogpt_gpt2``: forward torch 5.107 ms / Thunder 7.688 ms, backward 11.279 / 11.619 ms).

``python -m lightning_thunder_amd.benchmarks.targets [-k nanogpt_gpt2] [--executors eager,thunder]``
prints one JSON line per (benchmark, executor, phase) with the mean over ``--iters`` timed runs
(``torch.cuda.synchronize`` around each).  "forward" runs with ``requires_grad`` inputs (saving
for backward, the reference's TRAINING_FORWARD); "backward" times only ``loss.backward()``.
"""
from __future__ import annotations

import argparse
import json
import statistics
import time
from dataclasses import dataclass
from typing import Callable

import torch
import torch.nn.functional as F


@dataclass
class Bench:
    name: str
    make: Callable  # device -> (module_or_fn, args, to_loss)
    description: str = ""


def _nanogpt(config: str, batch: int = 16):
    def make(device):
        from ..models.nanogpt import NanoGPT

        torch.manual_seed(0)
        m = NanoGPT.from_name(config).to(device=device, dtype=torch.bfloat16)
        cfg = m.config
        x = torch.randint(0, 255, (batch, cfg.seq_len), device=device)
        y = torch.randint(0, 255, (batch, cfg.seq_len), device=device)
        return m, (x, y), lambda out: out[1]

    return make


def _litgpt_qkv_split_rope(device):
    from ..models.litgpt import Config, build_rope_cache, qkv_split_rope

    c = Config.from_name("Llama-2-7b-hf")
    T = 4096
    qkv = torch.randn(1, T, c.qkv_size, device=device, dtype=torch.bfloat16, requires_grad=True)
    cos, sin = build_rope_cache(T, c.rope_n_elem, device=device)

    def fn(qkv, cos, sin):
        return qkv_split_rope(qkv, cos, sin, c.n_head, c.n_query_groups, c.head_size, c.rope_n_elem)

    return fn, (qkv, cos, sin), lambda out: sum(o.float().sum() for o in out)


def _rmsnorm(device):
    x = torch.randn(4096, 4096, device=device, dtype=torch.bfloat16, requires_grad=True)
    w = torch.ones(4096, device=device, dtype=torch.bfloat16, requires_grad=True)
    return (lambda x, w: F.rms_norm(x, (4096,), w, 1e-5)), (x, w), lambda out: out.float().sum()


def _sdpa(device):
    q, k, v = (torch.randn(1, 32, 4096, 128, device=device, dtype=torch.bfloat16, requires_grad=True) for _ in range(3))
    return (lambda q, k, v: F.scaled_dot_product_attention(q, k, v, is_causal=True)), (q, k, v), lambda o: o.float().sum()


def _cross_entropy(device):
    logits = torch.randn(4096, 32000, device=device, dtype=torch.bfloat16, requires_grad=True)
    tgt = torch.randint(0, 32000, (4096,), device=device)
    return (lambda a, t: F.cross_entropy(a, t)), (logits, tgt), lambda o: o


def _llama_mlp(device):
    from ..models.litgpt import Config, LLaMAMLP

    m = LLaMAMLP(Config.from_name("Llama-2-7b-hf")).to(device=device, dtype=torch.bfloat16)
    x = torch.randn(1, 4096, 4096, device=device, dtype=torch.bfloat16, requires_grad=True)
    return m, (x,), lambda o: o.float().sum()


BENCHMARKS = {
    "nanogpt_gpt2": Bench("nanogpt_gpt2", _nanogpt("gpt2"), "NanoGPT GPT-2 124M, batch 16 x seq 128, bf16, dropout 0.1"),
    "nanogpt_gpt2xl": Bench("nanogpt_gpt2xl", _nanogpt("gpt2-xl"), "NanoGPT GPT-2 XL, batch 16 x seq 128, bf16"),
    "litgpt_qkv_split_rope": Bench("litgpt_qkv_split_rope", _litgpt_qkv_split_rope, "Llama-2-7B qkv split + RoPE, T=4096"),
    "rmsnorm": Bench("rmsnorm", _rmsnorm, "RMSNorm [4096, 4096] bf16"),
    "sdpa_causal": Bench("sdpa_causal", _sdpa, "causal SDPA B=1 H=32 S=4096 D=128 bf16"),
    "cross_entropy": Bench("cross_entropy", _cross_entropy, "cross-entropy [4096, 32000] bf16"),
    "llama_mlp": Bench("llama_mlp", _llama_mlp, "Llama-2-7B SwiGLU MLP, 4096 tokens, bf16"),
}


def _time(fn, iters, warmup):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(iters):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t0) * 1000)
    return statistics.mean(ts), statistics.median(ts)


def run_one(bench: Bench, executor: str, iters: int, warmup: int, device="cuda") -> list[dict]:
    import lightning_thunder_amd as thunder

    fn, args, to_loss = bench.make(device)
    if executor == "thunder":
        fn = thunder.jit(fn)
    elif executor == "thunder+hipgraph":
        from ..transforms.hipgraph import HipGraphTransform

        # gradients donated to autograd (the timed backward drops p.grad after every call)
        fn = thunder.jit(fn, transforms=[HipGraphTransform(donate_grads=True)])
    elif executor != "eager":
        raise ValueError(executor)
    params = [p for p in (fn.parameters() if hasattr(fn, "parameters") else [])]

    def fwd():
        return fn(*args)

    fwd_mean, fwd_med = _time(fwd, iters, warmup)
    state = {}

    def setup_bwd():
        out = fwd()
        state["loss"] = to_loss(out)

    def bwd():
        state["loss"].backward()
        for p in params:
            p.grad = None

    ts = []
    for i in range(warmup + iters):
        setup_bwd()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        bwd()
        torch.cuda.synchronize()
        if i >= warmup:
            ts.append((time.perf_counter() - t0) * 1000)
    base = {"benchmark": bench.name, "executor": executor, "unit": "ms", "description": bench.description}
    return [dict(base, phase="forward", mean=round(fwd_mean, 4), median=round(fwd_med, 4)),
            dict(base, phase="backward", mean=round(statistics.mean(ts), 4), median=round(statistics.median(ts), 4))]


def main(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("-k", default=None, help="substring filter on benchmark names")
    p.add_argument("--executors", default="eager,thunder")
    p.add_argument("--iters", type=int, default=20)
    p.add_argument("--warmup", type=int, default=5)
    args = p.parse_args(argv)
    for name, b in BENCHMARKS.items():
        if args.k and args.k not in name:
            continue
        for ex in args.executors.split(","):
            for r in run_one(b, ex, args.iters, args.warmup):
                print(json.dumps(r), flush=True)
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
