#!/usr/bin/env python
"""Headline benchmark: LitGPT Llama-2-7B pretraining step (seq 4096, micro-batch 1, bf16, AdamW) on MI355X.

Mirrors the reference's ``thunder/benchmarks/benchmark_litgpt.py`` headline run
(``docs/source/intermediate/benchmarking.rst:36-54``: 10,690 tokens/s/GPU on 1×H100).

    python bench.py --gpus 1 --steps 10 --warmup 3
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 bench.py --gpus 8

Synthetic token ids and random-init weights of the exact Llama-2-7B architecture
(no network for datasets/checkpoints).  One JSON line is printed by rank 0;
``value`` is the whole-job aggregate tokens/s (sum over ranks), timing is the max
over ranks of K steps bracketed by barrier + device synchronize.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import torch

BASELINE_TOKENS_PER_SEC_PER_GPU_1 = 10690.01  # 1x H100, Thunder default executors (benchmarking.rst:36-54)
BASELINE_TOKENS_PER_SEC_PER_GPU_FSDP = 11750.0  # 8x H100 ZeRO-2 Thunder (chart, normalized_training_throughput_zero2.png)
METRIC = "tokens/sec/GPU Llama-2-7B pretrain (LitGPT) + speedup vs eager at 1/2/4/8 MI355X"


def parse_args():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--model", default="Llama-2-7b-hf")
    p.add_argument("--seq", type=int, default=4096)
    p.add_argument("--mbs", type=int, default=None,
                   help="micro-batch per GPU; default 1 on one GPU (BASELINE config 1: MBS 1) and 2 for data-parallel "
                        "N>1 (the reference's ZeRO-2 chart is at batch 2 per GPU, BASELINE.md)")
    p.add_argument("--mode", default="thunder", choices=["thunder", "eager"])
    p.add_argument("--parallel", default="auto", choices=["auto", "fsdp", "ddp", "tp", "none"],
                   help="auto: fsdp for N>1; tp: Megatron tensor parallel over all ranks (BASELINE config 4, "
                        "e.g. --model Llama-3-8B --parallel tp; strong scaling)")
    p.add_argument("--fsdp-bucketing", default="block", choices=["none", "layer", "block"],
                   help="FSDP forward all-gather granularity: per parameter, per module or per transformer block "
                        "(one coalesced RCCL launch per ~400 MB block of Llama-2-7B)")
    p.add_argument("--executors", default=None, help="comma separated executor names (default: framework defaults)")
    p.add_argument("--fp8", action="store_true")
    p.add_argument("--fp8-recipe", default="current", choices=["current", "delayed", "mxfp8", "mxfp4"],
                   help="FP8 scaling: per-tensor current, delayed (amax history, TE DelayedScaling), MXFP8 blocks, "
                        "or mxfp4 (MXFP4 forward GEMMs, MXFP8 backward)")
    p.add_argument("--hipgraph", action="store_true")
    p.add_argument("--optim-overlap", default="off", choices=["auto", "on", "off"],
                   help="issue the fused AdamW update of each parameter bucket on a side stream inside the "
                        "backward (auto: on for 1-process thunder runs without hipGraphs).  Off by default: "
                        "measured no faster on 1x MI355X (profiles/optim_overlap_ab.txt)")
    p.add_argument("--lora", type=int, default=0, metavar="R",
                   help="LoRA fine-tuning of every transformer linear at rank R (base weights frozen; reference "
                        "benchmark_peft.py); not the pretraining headline")
    p.add_argument("--checkpoint-activations", action="store_true",
                   help="recompute every transformer block in the backward (memory for longer sequences)")
    p.add_argument("--n-layer", type=int, default=None, help="override layer count (debug only; invalid for the headline)")
    p.add_argument("--eager-baseline", default="auto", choices=["auto", "on", "off"],
                   help="also time PyTorch eager on the same config for speedup_vs_eager (auto: on for the 1-GPU "
                        "thunder run; --eager-warmup + --eager-steps from the same init and data, outside "
                        "thunder's timed region; both per-step loss curves go into the JSON line)")
    p.add_argument("--eager-steps", type=int, default=None, help="default: --steps (same loss-curve length)")
    p.add_argument("--eager-warmup", type=int, default=None, help="default: --warmup")
    p.add_argument("--lr", type=float, default=1e-4,
                   help="AdamW learning rate (1e-4: on the 4 cycling synthetic batches thunder and eager both descend "
                        "smoothly and their per-step losses can be compared; a constant 3e-4 oscillates in bf16 for "
                        "both, profiles/loss_curves_r6.txt)")
    p.add_argument("--lr-warmup", type=int, default=0,
                   help="linear learning-rate warmup over this many optimizer steps (0: constant --lr)")
    p.add_argument("--profile-dir", default=None)
    return p.parse_args()


def log(rank, *a):
    if rank == 0:
        print(*a, file=sys.stderr, flush=True)


def build_model(args, device):
    from lightning_thunder_amd.models.litgpt import GPT, Config, init_weights

    kw = {}
    if args.n_layer is not None:
        kw["n_layer"] = args.n_layer
    cfg = Config.from_name(args.model, **kw)
    with torch.device("meta"):
        model = GPT(cfg)
    model = model.to_empty(device=device).to(torch.bfloat16)
    torch.manual_seed(1234)
    init_weights(model)
    model.set_rope_cache(args.seq, device=device)
    model.activation_checkpointing = args.checkpoint_activations
    return model, cfg


def make_optimizer(params, mode="eager", lr=3e-4):
    if mode == "thunder" and os.environ.get("LTA_TORCH_ADAMW") != "1":
        from lightning_thunder_amd.optim import AdamW

        return AdamW(params, lr=lr, betas=(0.9, 0.95), weight_decay=0.1)  # fused multi-tensor HIP kernel
    try:
        return torch.optim.AdamW(params, lr=lr, betas=(0.9, 0.95), weight_decay=0.1, fused=True)
    except (RuntimeError, TypeError):
        return torch.optim.AdamW(params, lr=lr, betas=(0.9, 0.95), weight_decay=0.1, foreach=True)


def _rccl_record(world):
    if world == 1 and not _force_dist():
        return None
    from lightning_thunder_amd.distributed import rccl_policy

    return {k: v for k, v in rccl_policy.describe().items() if v is not None}


def _force_dist() -> bool:
    return os.environ.get("LTA_BENCH_FORCE_DIST") == "1"


def run(args, rank, world, device, mode, steps=None, warmup=None):
    import lightning_thunder_amd as thunder

    steps = args.steps if steps is None else steps
    warmup = args.warmup if warmup is None else warmup

    model, cfg = build_model(args, device)
    parallel = args.parallel
    if parallel == "auto":
        parallel = "fsdp" if world > 1 else "none"
    V = cfg.padded_vocab_size
    if mode == "thunder":
        kwargs = {}
        if args.executors:
            kwargs["executors"] = args.executors.split(",")
        transforms = []
        if args.hipgraph:
            from lightning_thunder_amd.transforms.hipgraph import HipGraphTransform

            # backward-graph gradients handed to autograd without a clone (the loop below zeroes them
            # with set_to_none every step, which donation requires)
            transforms.append(HipGraphTransform(donate_grads=True))
        if args.fp8:
            from lightning_thunder_amd.transforms.fp8 import FP8LinearTransform

            transforms.append(FP8LinearTransform(recipe=args.fp8_recipe))

        class TrainStep(torch.nn.Module):
            """Model + loss in one compiled program so the fused cross-entropy kernel is used."""

            def __init__(self, m):
                super().__init__()
                self.m = m

            def forward(self, x, y):
                logits = self.m(x)
                return torch.nn.functional.cross_entropy(logits.reshape(-1, V), y.reshape(-1))

        if args.lora:
            from lightning_thunder_amd.transforms.qlora import LORATransform

            model.requires_grad_(False)  # only the adapters train
            transforms.insert(0, LORATransform(r=args.lora, lora_alpha=2 * args.lora,
                                               weights=["attn", "proj", "fc_1", "fc_2"]))
        jm = thunder.jit(TrainStep(model), transforms=transforms, **kwargs)
        if (world > 1 or _force_dist()) and parallel == "fsdp":
            from lightning_thunder_amd.distributed import fsdp

            jm = fsdp(jm, bucketing_strategy=args.fsdp_bucketing)
        elif (world > 1 or _force_dist()) and parallel == "ddp":
            from lightning_thunder_amd.distributed import ddp

            jm = ddp(jm)
        elif (world > 1 or _force_dist()) and parallel == "tp":
            from lightning_thunder_amd.distributed import column_parallel, row_parallel

            # Megatron layout: head-parallel attention (qkv by heads, proj by rows), column fc_1/fc_2 +
            # row proj MLP, vocab-parallel embedding and lm_head with a vocab-parallel cross-entropy
            n = cfg.n_layer
            cols = [f"m.transformer.h.{i}.{s}" for i in range(n) for s in ("attn.attn", "mlp.fc_1", "mlp.fc_2")]
            cols += ["m.lm_head"] + ([] if cfg.tie_embeddings else ["m.transformer.wte"])
            rows = [f"m.transformer.h.{i}.{s}" for i in range(n) for s in ("attn.proj", "mlp.proj")]
            jm = row_parallel(column_parallel(jm, cols), rows)
        fwd = jm
        params = [p for p in jm.parameters() if p.requires_grad]
    else:
        fwd = model
        if world > 1:
            from torch.nn.parallel import DistributedDataParallel

            fwd = DistributedDataParallel(model, device_ids=[device.index])
        params = list(model.parameters())
    opt = make_optimizer(params, mode, args.lr)
    overlap = args.optim_overlap == "on" or (args.optim_overlap == "auto" and world == 1 and not _force_dist())
    if mode == "thunder" and overlap and not args.hipgraph and hasattr(opt, "overlap_with_backward"):
        # the update still runs inside the timed step: in the backward's shadow, joined by opt.step()
        opt.overlap_with_backward(fwd)
        args.overlap_used = True
    gen = torch.Generator(device=device)
    gen.manual_seed(1000 + rank)

    if parallel == "tp":
        gen.manual_seed(1000)  # tensor parallel: every rank sees the same tokens

    def batch():
        x = torch.randint(0, cfg.vocab_size, (args.mbs, args.seq + 1), device=device, generator=gen)
        return x[:, :-1].contiguous(), x[:, 1:].contiguous()

    n_step = [0]

    def step(x, y):
        if args.lr_warmup:
            # host-side only (the fused AdamW kernels take lr as an argument): same schedule both modes
            for g in opt.param_groups:
                g["lr"] = args.lr * min(1.0, (n_step[0] + 1) / args.lr_warmup)
            n_step[0] += 1
        if mode == "thunder":
            loss = fwd(x, y)
        else:
            logits = fwd(x)
            loss = torch.nn.functional.cross_entropy(logits.reshape(-1, V), y.reshape(-1))
        loss.backward()
        opt.step()
        opt.zero_grad(set_to_none=True)
        return loss

    data = [batch() for _ in range(4)]
    # every step's loss stays on the device; .item() only after the timed region (no added syncs)
    losses = []
    t_first = time.perf_counter()
    for i in range(warmup):
        loss = step(*data[i % 4])
        # a graphed forward's loss is a static tensor the next replay overwrites: keep a copy
        losses.append(loss.detach().clone() if args.hipgraph else loss.detach())
        if i == 0:
            torch.cuda.synchronize()
            log(rank, f"[{mode}] first step (incl. compile) {time.perf_counter() - t_first:.1f}s loss={loss.item():.4f}")
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        loss = step(*data[(warmup + i) % 4])
        losses.append(loss.detach().clone() if args.hipgraph else loss.detach())
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], device=device, dtype=torch.float64)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        dt = t.item()
    mem = torch.cuda.max_memory_allocated(device) / 1e9
    log(rank, f"[{mode}] {steps} steps in {dt:.3f}s, loss={loss.item():.4f}, peak mem {mem:.1f} GB")
    if mode == "thunder":
        from lightning_thunder_amd.ops import gemm as _g

        log(rank, f"[gemm] calls per backend since start (gemm4 = hand MFMA kernel, torch = library): "
                  f"{_g.last_gemm_backend_counts()}")
    curve = [round(v, 4) for v in torch.stack([l.float() for l in losses]).cpu().tolist()]
    del model, opt, fwd, params, losses, loss
    return dt, cfg, mem, parallel, curve


def main():
    args = parse_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if args.mbs is None:
        args.mbs = 2 if world > 1 and args.parallel in ("auto", "fsdp", "ddp") else 1
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
    # Rehearsal knobs (never used for reported numbers): several ranks on one GPU over gloo.
    dev_index = 0 if os.environ.get("LTA_BENCH_SAME_DEVICE") == "1" else local_rank
    backend = os.environ.get("LTA_DIST_BACKEND", "nccl")
    torch.cuda.set_device(dev_index)
    device = torch.device("cuda", dev_index)
    # LTA_BENCH_FORCE_DIST=1: run the data/tensor-parallel path even at world size 1 (a one-GPU
    # rehearsal of the RCCL program: bucketed / coalesced collectives at full model size)
    force = os.environ.get("LTA_BENCH_FORCE_DIST") == "1"
    if world > 1 or force:
        from datetime import timedelta

        # as the reference's benchmark_litgpt.py:64-69: no record_stream allocator thrash, async
        # error handling, and a bounded rendezvous / collective timeout instead of an endless hang;
        # the RCCL policy (distributed/rccl_policy.py) is applied before the communicator exists
        from lightning_thunder_amd.distributed import rccl_policy

        rccl_policy.apply()
        os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
        if rank == 0:
            print(f"[rccl] policy {rccl_policy.describe()}", file=sys.stderr, flush=True)
        timeout = timedelta(minutes=int(os.environ.get("LTA_DIST_TIMEOUT_MIN", "10")))
        if backend == "nccl":
            # a high-priority RCCL stream gets a hardware queue of its own: on the normal-priority
            # pool the collectives' stream can share the compute stream's queue (GPU_MAX_HW_QUEUES)
            # and then never run concurrently with compute (measured: one queue, zero overlap)
            from lightning_thunder_amd.distributed import high_priority_pg_options

            torch.distributed.init_process_group("nccl", device_id=device, pg_options=high_priority_pg_options(),
                                                 timeout=timeout)
        else:
            torch.distributed.init_process_group(backend, timeout=timeout)

    dt, cfg, mem, parallel, curve = run(args, rank, world, device, args.mode)
    data_parallel = parallel != "tp"
    tokens = args.steps * args.mbs * args.seq * (world if data_parallel else 1)
    value = tokens / dt
    per_gpu = value / world
    from lightning_thunder_amd.models.litgpt import flops_per_token

    tflops = flops_per_token(cfg, args.seq) * per_gpu / 1e12
    speedup = eager_ms = curve_eager = None
    want_eager = args.eager_baseline == "on" or (args.eager_baseline == "auto" and world == 1 and not _force_dist()
                                                 and not args.lora)
    if want_eager and args.mode == "thunder":
        # PyTorch eager on the same model / batch / optimizer semantics (torch fused AdamW), after
        # thunder's timed region; thunder's model and optimizer state are freed first
        torch.cuda.empty_cache()
        torch.cuda.reset_peak_memory_stats()
        esteps = args.steps if args.eager_steps is None else args.eager_steps
        ewarm = args.warmup if args.eager_warmup is None else args.eager_warmup
        dte, _, _, _, curve_eager = run(args, rank, world, device, "eager", steps=esteps, warmup=ewarm)
        eager_ms = dte / esteps * 1000
        speedup = eager_ms / (dt / args.steps * 1000)
    base = BASELINE_TOKENS_PER_SEC_PER_GPU_1 if world == 1 else BASELINE_TOKENS_PER_SEC_PER_GPU_FSDP
    if rank == 0:
        out = {
            "metric": METRIC if not args.lora else f"tokens/sec/GPU {args.model} LoRA r={args.lora} fine-tuning (LitGPT)",
            "value": round(value, 2),
            "unit": "tokens/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(dt / args.steps * 1000, 3),
            "higher_is_better": True,
            "scaling": "weak" if data_parallel else "strong",
            # no published TP or LoRA number to compare with
            "vs_baseline": round(per_gpu / base, 4) if data_parallel and not args.lora else None,
            "dtype": (("mxfp4 forward / mxfp8 backward linears, bf16 elsewhere" if args.fp8_recipe == "mxfp4" else
                       f"fp8 ({args.fp8_recipe} scaling) linears, bf16 elsewhere") if args.fp8 else "bf16"),
            "data": "synthetic token ids, random-init weights",
            "config": {
                "model": args.model + ("" if args.n_layer is None else f"-{args.n_layer}L(debug)"),
                "global_batch": args.mbs * (world if data_parallel else 1),
                "micro_batch": args.mbs,
                "seq_len": args.seq,
                "parallelism": f"{parallel}{world}" if world > 1 else "single",
                "mode": args.mode + (f"+lora-r{args.lora}" if args.lora else ""),
                "optimizer": "AdamW" + (" (fused, update issued inside the backward on a side stream)"
                                        if getattr(args, "overlap_used", False) else ""),
            },
            "tokens_per_sec_per_gpu": round(per_gpu, 2),
            "model_tflops_per_gpu": round(tflops, 1),
            "peak_mem_gb": round(mem, 2),
            "speedup_vs_eager": None if speedup is None else round(speedup, 3),
            "rccl": _rccl_record(world),
            "eager_ms_per_step": None if eager_ms is None else round(eager_ms, 3),
            "lr": args.lr,
            "lr_warmup_steps": args.lr_warmup,
            # per-step training loss (warmup steps first) from identical init and data
            "loss_curve_" + args.mode: curve,
            "loss_curve_eager": curve_eager if args.mode == "thunder" else curve,
        }
        print(json.dumps(out), flush=True)
    if torch.distributed.is_available() and torch.distributed.is_initialized():
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
