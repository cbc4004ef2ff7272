"""Prefill / decode inference benchmark (parity: reference ``thunder/benchmarks/benchmark_inference.py``:
throughput and latency of the prefill and decode phases — TTFT, TBOT, tokens/s — with batch size,
input/output lengths, warmup and iteration counts).

The reference drives an HF ``AutoModelForCausalLM`` with a ``HybridChunkedCache``; here the model
is the LitGPT-architecture model of this package (``--model``, random-init bf16 weights, no
checkpoints offline) with its static KV cache, so every mode runs the same model code:

* ``eager``    — PyTorch eager (ROCm);
* ``thunder``  — ``jit(model)``: prefill and decode are two cached programs on the HIP executors;
* ``hipgraph`` — ``jit`` + ``HipGraphTransform``: the decode step replays as a hipGraph.

Per iteration: one prefill of ``--input-length`` tokens for ``--batch-size`` sequences (TTFT =
its latency, including the first sampled token), then ``--output-length - 1`` decode steps
(TBOT = mean latency of one decode step).  Every phase is bracketed by device synchronisation.
Prints one JSON line per mode with mean / median / p90 over ``--num-iterations`` iterations
after ``--warmup-iterations`` untimed ones.
"""
from __future__ import annotations

import argparse
import json
import statistics
import time

import torch


def _percentile(xs, q):
    s = sorted(xs)
    return s[min(len(s) - 1, int(round(q * (len(s) - 1))))]


def _build(args, device):
    from ..models.litgpt import GPT, Config, init_weights

    kw = {} if args.n_layer is None else {"n_layer": args.n_layer}
    cfg = Config.from_name(args.model, **kw)
    with torch.device("meta"):
        model = GPT(cfg)
    model = model.to_empty(device=device).to(torch.bfloat16)
    torch.manual_seed(0)
    init_weights(model)
    model.requires_grad_(False)
    model.eval()
    model.set_kv_cache(args.batch_size, args.input_length + args.output_length + 8, device=device,
                       dtype=torch.bfloat16)
    return model, cfg


def _forward_for(mode, model):
    import lightning_thunder_amd as thunder

    if mode == "eager":
        return model
    if mode == "thunder":
        return thunder.jit(model)
    if mode == "hipgraph":
        from ..transforms.hipgraph import HipGraphTransform

        return thunder.jit(model, transforms=[HipGraphTransform()])
    raise ValueError(f"unknown mode {mode!r}")


def run(mode: str, args) -> dict:
    from ..ops.sampling import argmax_last

    device = torch.device("cuda", 0)
    model, cfg = _build(args, device)
    fwd = _forward_for(mode, model)
    gen = torch.Generator(device).manual_seed(1)
    prompt = torch.randint(0, cfg.vocab_size, (args.batch_size, args.input_length), device=device, generator=gen)
    prefill_pos = torch.arange(args.input_length, device=device)
    pos = torch.empty(1, dtype=torch.int64, device=device)

    def iteration():
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        logits = fwd(prompt, prefill_pos)
        tok = argmax_last(logits[:, -1], keepdim=True)
        torch.cuda.synchronize()
        ttft = time.perf_counter() - t0
        pos.fill_(args.input_length)
        steps = []
        for _ in range(args.output_length - 1):
            t1 = time.perf_counter()
            logits = fwd(tok, pos)
            tok = argmax_last(logits[:, -1], keepdim=True)
            pos.add_(1)
            torch.cuda.synchronize()
            steps.append(time.perf_counter() - t1)
        return ttft, steps

    t0 = time.perf_counter()
    iteration()
    first = time.perf_counter() - t0
    for _ in range(args.warmup_iterations):
        iteration()
    ttfts, tbots, totals = [], [], []
    for _ in range(args.num_iterations):
        ttft, steps = iteration()
        ttfts.append(ttft)
        tbots.extend(steps)
        totals.append(ttft + sum(steps))
    B, n_out = args.batch_size, args.output_length
    decode_s = sum(tbots)
    return {
        "metric": f"{args.model} prefill/decode inference (batch {B}, {args.input_length} in, {n_out} out)",
        "mode": mode,
        "ttft_ms": {"mean": round(1e3 * statistics.mean(ttfts), 3), "median": round(1e3 * statistics.median(ttfts), 3),
                    "p90": round(1e3 * _percentile(ttfts, 0.9), 3)},
        "tbot_ms": ({"mean": round(1e3 * statistics.mean(tbots), 3), "median": round(1e3 * statistics.median(tbots), 3),
                     "p90": round(1e3 * _percentile(tbots, 0.9), 3)} if tbots else None),
        "prefill_tokens_per_s": round(B * args.input_length / statistics.mean(ttfts), 1),
        "decode_tokens_per_s": round(B * len(tbots) / decode_s, 1) if tbots else None,
        "total_tokens_per_s": round(B * n_out * len(totals) / sum(totals), 1),
        "latency_ms_per_request": round(1e3 * statistics.mean(totals), 2),
        "first_call_s": round(first, 2),
        "batch_size": B, "input_length": args.input_length, "output_length": n_out,
        "dtype": "bf16", "data": "synthetic prompt, random-init weights", "n_gpus": 1,
    }


def main(argv=None):
    p = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    p.add_argument("--model", default="Llama-3.2-1B")
    p.add_argument("--batch-size", type=int, default=1)
    p.add_argument("--input-length", type=int, default=2048)
    p.add_argument("--output-length", type=int, default=128)
    p.add_argument("--num-iterations", type=int, default=5)
    p.add_argument("--warmup-iterations", type=int, default=2)
    p.add_argument("--modes", default="eager,thunder,hipgraph")
    p.add_argument("--n-layer", type=int, default=None, help="debug only")
    args = p.parse_args(argv)
    if args.output_length < 1:
        p.error("--output-length must be >= 1")
    for mode in args.modes.split(","):
        print(json.dumps(run(mode, args)), flush=True)
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
