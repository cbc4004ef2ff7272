"""Bandwidth roofline of the hipfuse-generated kernels of a GPT-2-medium training step.

Runs one jitted NanoGPT gpt2-medium step (B=8, T=1024, bf16, dropout 0.1) with every hipFusion call
recorded, then re-launches each distinct generated kernel on copies of the inputs of its first call.
Timing: HIP events around a batch of back-to-back launches that rotate over k copies of every
input / output storage (k x bytes >= 1.5 GB, so no launch finds its operands in the 256 MB
Infinity Cache left by the previous one); per-launch time = batch / k, median of 7 batches.  (One
event pair per launch, the round-4 method, adds the event / launch gap to every kernel: ~6 us on a
15 us kernel.)  Bytes = the storage actually addressed by every input (broadcast operands counted
once) + every output; TB/s against the MI355X's ~8 TB/s HBM3E.

    python scripts/hipfuse_roofline.py [--json gpurun_out/hipfuse_roofline.json]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

import lightning_thunder_amd as thunder
from lightning_thunder_amd.executors import hipfuse
from lightning_thunder_amd.models.nanogpt import NanoGPT

HBM_TBS = 8.0


def _addressed_bytes(t: torch.Tensor) -> int:
    """Bytes spanned by the elements of ``t`` (a broadcast / expanded view counts its storage once)."""
    if t.numel() == 0:
        return 0
    n = 1 + sum((s - 1) * st for s, st in zip(t.shape, t.stride()) if st != 0)
    return min(n, t.numel()) * t.element_size()


def _copy(t: torch.Tensor) -> torch.Tensor:
    """A tensor with the same size / strides / offset over a copy of ``t``'s storage (broadcast and
    sliced views keep their layout, index operands their in-range values)."""
    st = t.untyped_storage().clone()
    return torch.empty(0, dtype=t.dtype, device=t.device).set_(st, t.storage_offset(), t.size(), t.stride())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--json", default="gpurun_out/hipfuse_roofline.json")
    ap.add_argument("--top", type=int, default=12)
    args = ap.parse_args()
    torch.manual_seed(0)
    B, T = 8, 1024
    m = NanoGPT.from_name("gpt2-medium", seq_len=T).to(device="cuda", dtype=torch.bfloat16)
    m.train()
    jm = thunder.jit(m)
    x = torch.randint(0, m.config.vocab_size, (B, T), device="cuda")
    y = torch.randint(0, m.config.vocab_size, (B, T), device="cuda")
    _, loss = jm(x, y)  # compile + first run
    loss.backward()
    torch.cuda.synchronize()

    seen: dict = {}
    orig = hipfuse.HipFusion._call

    def rec(self, a):
        outs = orig(self, a)
        tensors = [a[i] for i in self.tensor_pos]
        if tensors and tensors[0].is_cuda:
            fns, ks = self._variant(tensors)
            if ks.name not in seen:
                seen[ks.name] = dict(fusion=self, ks=ks, fns=fns, tensors=tensors, outs=outs,
                                     numbers=[a[i] for i in self.number_pos], calls=0,
                                     prims=[b.sym.name for b in self.nodes])
            seen[ks.name]["calls"] += 1
        return outs

    hipfuse.HipFusion._call = rec
    try:
        _, loss = jm(x, y)
        loss.backward()
    finally:
        hipfuse.HipFusion._call = orig
    torch.cuda.synchronize()

    rows = []
    for name, r in seen.items():
        ks = r["ks"]
        nbytes = sum(_addressed_bytes(t) for t in r["tensors"]) + sum(_addressed_bytes(o) for o in r["outs"])

        store = sum(t.untyped_storage().nbytes() for t in r["tensors"]) + \
            sum(o.untyped_storage().nbytes() for o in r["outs"])
        k = max(2, min(64, -(-int(1.5e9) // max(store, 1))))
        sets = [([_copy(t) for t in r["tensors"]], [_copy(o) for o in r["outs"]]) for _ in range(k)]

        def batch():
            for ins, outs in sets:
                hipfuse.launch(ks, r["fns"], ins, outs, r["numbers"])

        batch()
        ts = []
        for _ in range(7):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            batch()
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e3 / k)
        ts.sort()
        us = ts[len(ts) // 2]
        del sets
        tbs = nbytes / (us * 1e-6) / 1e12
        rows.append(dict(kernel=name, mode=ks.mode, calls_per_step=r["calls"], us=round(us, 2),
                         mbytes=round(nbytes / 1e6, 2), tb_s=round(tbs, 2), pct_hbm=round(100 * tbs / HBM_TBS, 1),
                         step_ms=round(us * r["calls"] / 1e3, 3), domain=list(r["fusion"].plan.domain or ()),
                         prims=len(r["prims"]), ops=sorted(set(r["prims"]))))
    rows.sort(key=lambda d: -d["step_ms"])
    total = sum(d["step_ms"] for d in rows)
    print(f"{len(rows)} distinct generated kernels, {sum(d['calls_per_step'] for d in rows)} launches per step, "
          f"{total:.2f} ms per step (isolated timings)")
    print(f"{'kernel':28s} {'mode':10s} {'calls':>5s} {'us':>8s} {'MB':>8s} {'TB/s':>6s} {'%HBM':>5s}  domain")
    for d in rows[:args.top]:
        print(f"{d['kernel']:28s} {d['mode']:10s} {d['calls_per_step']:5d} {d['us']:8.2f} {d['mbytes']:8.2f} "
              f"{d['tb_s']:6.2f} {d['pct_hbm']:5.1f}  {d['domain']}  {','.join(d['ops'])[:80]}")
    os.makedirs(os.path.dirname(args.json) or ".", exist_ok=True)
    with open(args.json, "w") as f:
        json.dump(dict(model="gpt2-medium", B=B, T=T, dtype="bf16", hbm_tb_s=HBM_TBS, kernels=rows), f, indent=1)


if __name__ == "__main__":
    main()
