"""FSDP distributed checkpoint (DCP) and hybrid (ddp x fsdp) mesh tests on CPU/gloo."""
import os
import socket
import tempfile

import torch
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _model():
    torch.manual_seed(0)
    return torch.nn.Sequential(torch.nn.Linear(8, 15), torch.nn.GELU(), torch.nn.Linear(15, 3)).double()


def _tiny_rows_model():
    # dim 0 smaller than the world size (3 rows on 4 ranks) and padding spanning several ranks
    # (5 rows -> shards of 2, 2, 1, 0)
    torch.manual_seed(0)
    return torch.nn.Sequential(torch.nn.Linear(8, 3), torch.nn.Tanh(), torch.nn.Linear(3, 5)).double()


def _ckpt_worker(rank, world, port, d, make=None):
    make = make or _model
    import lightning_thunder_amd as thunder
    from lightning_thunder_amd.distributed import fsdp
    from lightning_thunder_amd.distributed import checkpoint as ck

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.distributed.init_process_group("gloo", rank=rank, world_size=world)
    try:
        jm = fsdp(thunder.jit(make()))
        with torch.no_grad():
            for p in jm.parameters():
                p.mul_(1.5)
        sd = ck.get_model_state_dict(jm, ck.StateDictOptions(full_state_dict=False))
        ck.save(sd, os.path.join(d, "ckpt"))
        full = ck.get_model_state_dict(jm, ck.StateDictOptions(full_state_dict=True, rank0_only=True))
        # a fresh sharded model, loaded from the sharded checkpoint
        jm2 = fsdp(thunder.jit(make()))
        sd2 = ck.get_model_state_dict(jm2, ck.StateDictOptions(full_state_dict=False))
        ck.load(sd2, os.path.join(d, "ckpt"))
        ck.load_model_state_dict(sd2, jm2, ck.StateDictOptions(full_state_dict=False))
        diff = max((a - b).abs().max().item() for a, b in zip(jm.parameters(), jm2.parameters()))
        # every sharded entry reassembles to the full (scaled) parameter
        ref = {k: v * 1.5 for k, v in make().state_dict().items()}
        full_err = max((sd[k].full_tensor() - ref[k]).abs().max().item() for k in ref)
        local_rows = {k: tuple(sd[k].to_local().shape) for k in ref}
        torch.save({"diff": diff, "full_err": full_err, "local_rows": local_rows, "full_keys": sorted(full), "full_shapes": {k: tuple(v.shape) for k, v in full.items()}},
                   os.path.join(d, f"r{rank}.pt"))
    finally:
        torch.distributed.barrier()  # peers finish their collectives before gloo tears down
        torch.distributed.destroy_process_group()
    os._exit(0)  # skip interpreter teardown: gloo worker threads can abort it (rare SIGABRT)


def test_fsdp_dcp_roundtrip():
    world = 2
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_ckpt_worker, args=(world, _free_port(), d), nprocs=world, join=True, start_method="spawn")
        r0 = torch.load(os.path.join(d, "r0.pt"), weights_only=False)
        r1 = torch.load(os.path.join(d, "r1.pt"), weights_only=False)
    assert r0["diff"] == 0.0 and r1["diff"] == 0.0
    assert r0["full_shapes"]["0.weight"] == (15, 8) and r1["full_keys"] == []
    assert r0["full_err"] == 0.0 and r1["full_err"] == 0.0


def test_fsdp_dcp_roundtrip_padding_spans_ranks():
    world = 4
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_ckpt_worker, args=(world, _free_port(), d, _tiny_rows_model), nprocs=world, join=True,
                           start_method="spawn")
        res = [torch.load(os.path.join(d, f"r{r}.pt"), weights_only=False) for r in range(world)]
    for r in res:
        assert r["diff"] == 0.0 and r["full_err"] == 0.0
    assert [r["local_rows"]["2.bias"] for r in res] == [(2,), (2,), (1,), (0,)]
    assert [r["local_rows"]["0.weight"] for r in res] == [(1, 8), (1, 8), (1, 8), (0, 8)]
    assert res[0]["full_shapes"]["2.weight"] == (5, 3)


def _hybrid_worker(rank, world, port, d, coalesced=False):
    if coalesced:
        os.environ["LTA_COALESCED_GRAD_SYNC"] = "1"
    import lightning_thunder_amd as thunder
    from lightning_thunder_amd.plugins import FSDP
    from torch.distributed.device_mesh import init_device_mesh

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.distributed.init_process_group("gloo", rank=rank, world_size=world)
    try:
        mesh = init_device_mesh("cpu", (2, 2), mesh_dim_names=("ddp", "fsdp"))
        m = _model()
        tm = thunder.compile(m, plugins=[FSDP(process_group=mesh)])
        g = torch.Generator().manual_seed(10 + rank)
        x = torch.randn(4, 8, generator=g, dtype=torch.float64)
        tm(x).pow(2).mean().backward()
        grads = {n: p.grad.clone() for n, p in m.named_parameters()}
        bw = str(thunder.last_backward_traces(tm)[-1])
        torch.save({"grads": grads, "bw": bw}, os.path.join(d, f"r{rank}.pt"))
    finally:
        torch.distributed.barrier()  # peers finish their collectives before gloo tears down
        torch.distributed.destroy_process_group()
    os._exit(0)  # skip interpreter teardown: gloo worker threads can abort it (rare SIGABRT)


import pytest


@pytest.mark.parametrize("coalesced", [False, True])
def test_hybrid_mesh_fsdp_plugin(coalesced):
    from lightning_thunder_amd.distributed.transforms import shard_tensor

    world = 4
    ref = _model()
    loss = 0
    for r in range(world):
        g = torch.Generator().manual_seed(10 + r)
        loss = loss + ref(torch.randn(4, 8, generator=g, dtype=torch.float64)).pow(2).mean() / world
    loss.backward()
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_hybrid_worker, args=(world, _free_port(), d, coalesced), nprocs=world, join=True,
                           start_method="spawn")
        res = [torch.load(os.path.join(d, f"r{r}.pt"), weights_only=False) for r in range(world)]
    for rank, r in enumerate(res):
        fsdp_rank = rank % 2
        for n, p in ref.named_parameters():
            expected, _ = shard_tensor(p.grad, fsdp_rank, 2)
            torch.testing.assert_close(r["grads"][n], expected)
        if coalesced:  # grouped reduce-scatter per bucket, then the replica-group all-reduce per gradient
            assert "reduce_scatter_coalesced" in r["bw"] and "all_reduce" in r["bw"], r["bw"]


def _sd_worker(rank, world, port, d):
    import lightning_thunder_amd as thunder
    from lightning_thunder_amd.distributed import fsdp

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.distributed.init_process_group("gloo", rank=rank, world_size=world)
    try:
        jm = fsdp(thunder.jit(_model()))
        x = torch.randn(4, 8, dtype=torch.float64, generator=torch.Generator().manual_seed(rank))
        y0 = jm(x).detach()
        sd = jm.state_dict()  # this rank's shards
        full = jm.original_state_dict()  # reverse hooks: full tensors
        ref = _model().state_dict()
        full_err = max((full[k] - ref[k]).abs().max().item() for k in ref)
        shapes_ok = all(tuple(full[k].shape) == tuple(ref[k].shape) for k in ref)
        # assign-load of the transformed state: new Parameter objects keep the sharding metadata
        jm.load_state_dict({k: v.clone() * 2 for k, v in sd.items()}, assign=True)
        y2 = jm(x).detach()
        # forward hooks: loading the full (original) dict re-shards it
        jm.load_original_state_dict(full)
        y3 = jm(x).detach()
        bad_shape = False
        try:
            jm.load_state_dict({k: v for k, v in full.items()})
        except RuntimeError:
            bad_shape = True
        torch.save({"full_err": full_err, "shapes_ok": shapes_ok, "changed": (y2 - y0).abs().max().item(),
                    "restored": (y3 - y0).abs().max().item(), "bad_shape": bad_shape}, os.path.join(d, f"r{rank}.pt"))
    finally:
        torch.distributed.barrier()  # peers finish their collectives before gloo tears down
        torch.distributed.destroy_process_group()
    os._exit(0)  # skip interpreter teardown: gloo worker threads can abort it (rare SIGABRT)


def test_thunder_module_state_dict_hooks_fsdp():
    """state_dict = transformed shards, original_state_dict = reverse hooks (full tensors),
    load_state_dict(assign=True) keeps the program working, load_original_state_dict re-shards."""
    world = 2
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_sd_worker, args=(world, _free_port(), d), nprocs=world, join=True, start_method="spawn")
        res = [torch.load(os.path.join(d, f"r{r}.pt"), weights_only=False) for r in range(world)]
    for r in res:
        assert r["full_err"] == 0.0 and r["shapes_ok"], r
        assert r["changed"] > 0 and r["restored"] < 1e-12 and r["bad_shape"], r


def _zero3_window_worker(rank, world, port, d):
    """ZeRO-3 + block bucketing with coalesced gathers and the prefetch window (the RCCL program's
    schedule, on gloo): the bucket of parameters outside the blocks is waited on at the start (the
    embedding) and at the end (the LM head), so the window must not place a block's gather after
    that bucket's last wait (it did: the forward read a future before its gather)."""
    import lightning_thunder_amd as thunder
    from lightning_thunder_amd.distributed import fsdp
    from lightning_thunder_amd.distributed.transforms import FSDPType
    from lightning_thunder_amd.models.litgpt import GPT

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), LTA_COALESCED_GRAD_SYNC="1")
    torch.distributed.init_process_group("gloo", rank=rank, world_size=world)
    try:
        res = {}
        for strategy in ("none", "block"):
            torch.manual_seed(0)
            m = GPT.from_name("llama2-like")
            m.set_rope_cache(64, device="cpu")
            jm = fsdp(thunder.jit(m), bucketing_strategy=strategy, sharding_strategy=FSDPType.ZERO3)
            x = torch.randint(0, m.config.vocab_size, (2, 64), generator=torch.Generator().manual_seed(1))
            out = jm(x)
            out.float().pow(2).mean().backward()
            res[strategy] = (out.detach().clone(), {n: p.grad.clone() for n, p in m.named_parameters()},
                             str(thunder.last_traces(jm)[-1]).count("all_gather_coalesced("))
        torch.save(res, os.path.join(d, f"r{rank}.pt"))
    finally:
        torch.distributed.barrier()
        torch.distributed.destroy_process_group()
    os._exit(0)  # skip interpreter teardown: gloo worker threads can abort it (rare SIGABRT)


def test_zero3_block_bucketing_window_order():
    import tempfile

    import torch.multiprocessing as mp

    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_zero3_window_worker, args=(1, _free_port(), d), nprocs=1, join=True, start_method="spawn")
        res = torch.load(os.path.join(d, "r0.pt"), weights_only=True)
    out0, g0, _ = res["none"]
    out1, g1, n_coalesced = res["block"]
    assert n_coalesced >= 3
    torch.testing.assert_close(out1, out0)
    for n in g0:
        torch.testing.assert_close(g1[n], g0[n])


def test_rccl_policy_defaults_and_presets():
    from lightning_thunder_amd.distributed import rccl_policy

    env = {}
    # the measured decision (profiles/cu_contention_r6.txt): finish collectives fast, every CU a channel
    # holds costs the one-tile-per-CU GEMMs a whole extra wave however many channels there are
    assert rccl_policy.apply(env) == {"TORCH_NCCL_AVOID_RECORD_STREAMS": "1", "NCCL_MIN_NCHANNELS": "32"}
    env = {"LTA_RCCL_POLICY": "narrow"}
    rccl_policy.apply(env)
    assert env["NCCL_MAX_NCHANNELS"] == "8" and "NCCL_MIN_NCHANNELS" not in env
    env = {"LTA_RCCL_POLICY": "rccl"}
    assert rccl_policy.apply(env) == {"TORCH_NCCL_AVOID_RECORD_STREAMS": "1"}
    env = {"LTA_RCCL_POLICY": "wide", "NCCL_MIN_NCHANNELS": "8"}
    rccl_policy.apply(env)
    assert env["NCCL_MIN_NCHANNELS"] == "8"  # an explicit setting wins
    env = {"LTA_RCCL_POLICY": "ring"}
    rccl_policy.apply(env)
    assert env["NCCL_ALGO"] == "Ring"
    assert rccl_policy.apply({"LTA_RCCL_POLICY": "off"}) == {}
    d = rccl_policy.describe({"LTA_RCCL_POLICY": "wide", "NCCL_MIN_NCHANNELS": "32"})
    assert d["LTA_RCCL_POLICY"] == "wide" and d["NCCL_MIN_NCHANNELS"] == "32"
    with pytest.raises(ValueError):
        rccl_policy.apply({"LTA_RCCL_POLICY": "bogus"})
