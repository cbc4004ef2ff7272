"""Multi-process data/tensor-parallel tests on CPU with gloo (reference analogue: thunder/tests/distributed/).

Each test spawns ``world_size`` ranks (127.0.0.1 rendezvous), runs the compiled DDP/FSDP/TP
model and checks gradients against a single-process eager reference on the concatenated batch.
"""
import os
import socket
import tempfile

import pytest
import torch
import torch.multiprocessing as mp

WORLD = 2


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _model():
    torch.manual_seed(0)
    return torch.nn.Sequential(torch.nn.Linear(8, 16), torch.nn.GELU(), torch.nn.Linear(16, 5), torch.nn.Tanh(),
                               torch.nn.Linear(5, 3))


class _Blocks(torch.nn.Module):
    """Numbered blocks (``layers.<i>``): one FSDP block bucket each."""

    def __init__(self):
        super().__init__()
        torch.manual_seed(0)
        self.layers = torch.nn.ModuleList([torch.nn.Linear(8, 8) for _ in range(5)])

    def forward(self, x):
        for l in self.layers:
            x = torch.tanh(l(x))
        return x


def _data(rank):
    g = torch.Generator().manual_seed(100 + rank)
    return torch.randn(4, 8, generator=g, dtype=torch.float64)


def _reference_grads(make=None):
    m = (make or _model)().double()
    x = torch.cat([_data(r) for r in range(WORLD)])
    # each rank averages its local mean loss; the global objective is the mean over ranks
    loss = sum(m(_data(r)).pow(2).mean() for r in range(WORLD)) / WORLD
    loss.backward()
    return {n: p.grad.clone() for n, p in m.named_parameters()}, m


def _worker(rank, port, mode, out_dir):
    import lightning_thunder_amd as thunder
    from lightning_thunder_amd.distributed import ddp, fsdp
    from lightning_thunder_amd.distributed.transforms import FSDPType, FSDPBucketingStrategy

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    if mode.endswith("_coalesced"):
        # the grouped-collective bucket form RCCL runs by default: trace plumbing,
        # per-gradient futures / waits and shard shapes exercised on gloo
        os.environ["LTA_COALESCED_GRAD_SYNC"] = "1"
        mode = mode[: -len("_coalesced")]
    torch.distributed.init_process_group("gloo", rank=rank, world_size=WORLD)
    try:
        m = (_Blocks() if mode.startswith("blocks_") else _model()).double()
        jm = thunder.jit(m)
        if mode == "blocks_zero3":
            jm = fsdp(jm, sharding_strategy=FSDPType.ZERO3, bucketing_strategy=FSDPBucketingStrategy.BLOCK)
        elif mode == "blocks_zero2":
            # ~one block's gradients per bucket (8x8 weight + bias, fp64 = 576 B)
            jm = fsdp(jm, sharding_strategy=FSDPType.ZERO2, bucketing_strategy=FSDPBucketingStrategy.BLOCK,
                      bucket_size_in_mb=500 / 2 ** 20)
        elif mode == "ddp":
            jm = ddp(jm, bucket_size_in_mb=0.0005)
        elif mode == "ddp_nobucket":
            jm = ddp(jm, bucket_size_in_mb=0)
        elif mode == "fsdp":
            jm = fsdp(jm)
        elif mode == "fsdp_zero3":
            jm = fsdp(jm, sharding_strategy=FSDPType.ZERO3)
        elif mode == "fsdp_layer":
            jm = fsdp(jm, bucketing_strategy=FSDPBucketingStrategy.LAYER)
        elif mode == "fsdp_block_zero3":
            jm = fsdp(jm, sharding_strategy=FSDPType.ZERO3, bucketing_strategy=FSDPBucketingStrategy.BLOCK)
        elif mode == "fsdp_block":
            jm = fsdp(jm, bucketing_strategy=FSDPBucketingStrategy.BLOCK)
        out = jm(_data(rank))
        loss = out.pow(2).mean()
        loss.backward()
        grads = {n: p.grad.detach().clone() for n, p in m.named_parameters()}
        shapes = {n: tuple(p.shape) for n, p in m.named_parameters()}
        bw = str(thunder.last_backward_traces(jm)[-1])
        fw = str(thunder.last_traces(jm)[-1])
        torch.save({"grads": grads, "shapes": shapes, "bw": bw, "fw": fw, "out": out.detach()},
                   os.path.join(out_dir, f"rank{rank}.pt"))
    finally:
        torch.distributed.barrier()  # peers finish their collectives before gloo tears down
        torch.distributed.destroy_process_group()
    os._exit(0)  # skip interpreter teardown: gloo worker threads can abort it (rare SIGABRT)


def _run(mode):
    port = _free_port()
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_worker, args=(port, mode, d), nprocs=WORLD, join=True, start_method="spawn")
        return [torch.load(os.path.join(d, f"rank{r}.pt"), weights_only=False) for r in range(WORLD)]


@pytest.mark.parametrize("mode", ["ddp", "ddp_nobucket", "ddp_coalesced"])
def test_ddp_gloo(mode):
    ref, _ = _reference_grads()
    res = _run(mode)
    for r in res:
        for n, g in ref.items():
            torch.testing.assert_close(r["grads"][n], g)
    assert "all_reduce" in res[0]["bw"]
    if mode == "ddp":  # buckets: packed buffer (gloo) or one coalesced collective (RCCL)
        assert "pack" in res[0]["bw"] or "all_reduce_coalesced" in res[0]["bw"]
    if mode == "ddp_coalesced":
        assert "all_reduce_coalesced" in res[0]["bw"] and "pack(" not in res[0]["bw"]


@pytest.mark.parametrize("mode", ["fsdp", "fsdp_zero3", "fsdp_layer", "fsdp_block_zero3", "fsdp_block_coalesced",
                                  "fsdp_zero3_coalesced"])
def test_fsdp_gloo(mode):
    from lightning_thunder_amd.distributed.transforms import shard_tensor

    ref, _ = _reference_grads()
    res = _run(mode)
    for rank, r in enumerate(res):
        for n, g in ref.items():
            expected, _ = shard_tensor(g, rank, WORLD)
            assert r["shapes"][n] == tuple(expected.shape)
            torch.testing.assert_close(r["grads"][n], expected)
    assert "reduce_scatter" in res[0]["bw"]
    if mode.endswith("_coalesced"):
        assert "reduce_scatter_coalesced" in res[0]["bw"] and "pack_for_fsdp" not in res[0]["bw"]
    if mode == "fsdp_layer":
        # one coalesced gather per Linear (weight + bias), not one per parameter
        assert res[0]["fw"].count("all_gather_coalesced(") == 3, res[0]["fw"]
    if mode == "fsdp_block_zero3":
        # no numbered blocks in a Sequential: everything is one bucket, also for the backward's
        # re-gathers
        assert res[0]["fw"].count("all_gather_coalesced(") == 1
        assert res[0]["bw"].count("all_gather_coalesced(") == 1
    if "zero3" in mode:
        # ZeRO-3 saves shards and re-gathers (also when the padding trim follows the gather)
        assert "all_gather" in res[0]["bw"]


def test_fsdp_zero3_allgather_window():
    """ZeRO-3 with per-block buckets: the parameter all-gathers are issued in a 2-block sliding window
    (not all at the program start) in the forward and the backward re-gathers, and grads match."""
    from lightning_thunder_amd.distributed.transforms import shard_tensor

    ref, _ = _reference_grads(_Blocks)
    res = _run("blocks_zero3")
    for rank, r in enumerate(res):
        for n, g in ref.items():
            expected, _ = shard_tensor(g, rank, WORLD)
            torch.testing.assert_close(r["grads"][n], expected)
    for key in ("fw", "bw"):
        lines = [l.strip() for l in res[0][key].splitlines()]
        gathers = [i for i, l in enumerate(lines) if "all_gather_coalesced(" in l]
        waits = [i for i, l in enumerate(lines) if "wait(" in l]
        assert len(gathers) >= 4, res[0][key]
        # gather of block 2 comes after the first wait: at most two blocks in flight
        assert gathers[2] > waits[0], (key, gathers, waits)


def test_fsdp_zero2_reduce_scatter_overlaps_backward():
    """ZeRO-2 with one bucket per block: each block's gradient reduce-scatter is issued as soon as the
    block's gradients exist — before the next (earlier) block's backward matmuls — and every wait
    comes after all of them, so the collectives overlap the rest of the backward; grads match."""
    import re

    from lightning_thunder_amd.distributed.transforms import shard_tensor

    ref, _ = _reference_grads(_Blocks)
    res = _run("blocks_zero2_coalesced")
    for rank, r in enumerate(res):
        for n, g in ref.items():
            expected, _ = shard_tensor(g, rank, WORLD)
            torch.testing.assert_close(r["grads"][n], expected)
    lines = [l for l in res[0]["bw"].splitlines() if "=" in l and not l.strip().startswith("#")]
    mm = [i for i, l in enumerate(lines) if re.search(r"\bmatmul\(", l)]
    rs = [i for i, l in enumerate(lines) if "reduce_scatter" in l]
    waits = [i for i, l in enumerate(lines) if re.search(r"\bdist_wait\(|\bwait\(", l)]
    assert len(rs) == 5, res[0]["bw"]  # one coalesced reduce-scatter per block
    for k, i in enumerate(rs[:-1]):
        # compute of an earlier block runs between this block's issue and the next issue
        assert any(i < j < rs[k + 1] for j in mm), (k, res[0]["bw"])
    assert rs[0] < mm[-1] and min(waits) > mm[-1], res[0]["bw"]
