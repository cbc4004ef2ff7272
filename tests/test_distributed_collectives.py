"""User collectives and DDP ``no_sync`` inside compiled programs (gloo, 2 ranks, 127.0.0.1).

Reference analogues: ``thunder/tests/distributed/test_ops.py`` (all_reduce / all_gather /
reduce_scatter / broadcast inside ``thunder.jit``) and ``helper.py:329``
``run_test_no_sync_grad_accumulation`` (no collectives in the no-sync backward; accumulated
gradients equal the synchronized ones).
"""
import os
import socket
import tempfile

import torch
import torch.multiprocessing as mp

WORLD = 2


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _init(rank, port):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.distributed.init_process_group("gloo", rank=rank, world_size=WORLD)


def _collectives_worker(rank, port, out_dir):
    import lightning_thunder_amd as thunder
    from lightning_thunder_amd import torch as ltorch

    _init(rank, port)
    try:
        x = torch.full((4,), float(rank + 1))

        def f_allreduce(x):
            y = x * 2
            torch.distributed.all_reduce(y)
            return y + 1

        def f_gather(x):
            out = torch.empty(WORLD * 4)
            torch.distributed.all_gather_into_tensor(out, x)
            return out

        def f_scatter(x):
            out = torch.empty(2)
            torch.distributed.reduce_scatter_tensor(out, x)
            return out

        def f_broadcast(x):
            y = x.clone()
            torch.distributed.broadcast(y, 1)
            return y

        def f_functional(x):
            m = ltorch.all_reduce(x, "max")
            fut = ltorch.all_gather(x, async_op=True)
            return m, ltorch.wait(fut)

        jf = thunder.jit(f_allreduce)
        res = {
            "allreduce": jf(x),
            "gather": thunder.jit(f_gather)(x),
            "scatter": thunder.jit(f_scatter)(x),
            "broadcast": thunder.jit(f_broadcast)(x),
            "functional": thunder.jit(f_functional)(x),
            "trace": str(thunder.last_traces(jf)[-1]),
        }
        torch.save(res, os.path.join(out_dir, f"rank{rank}.pt"))
    finally:
        torch.distributed.barrier()  # peers finish their collectives before gloo tears down
        torch.distributed.destroy_process_group()
    os._exit(0)  # skip interpreter teardown: gloo worker threads can abort it (rare SIGABRT)


def _model():
    torch.manual_seed(0)
    return torch.nn.Sequential(torch.nn.Linear(8, 16), torch.nn.GELU(), torch.nn.Linear(16, 3)).double()


def _data(rank, mb):
    g = torch.Generator().manual_seed(1000 * mb + rank)
    return torch.randn(4, 8, generator=g, dtype=torch.float64)


def _nosync_worker(rank, port, out_dir):
    import lightning_thunder_amd as thunder
    from lightning_thunder_amd.distributed import ddp

    _init(rank, port)
    try:
        m = _model()
        jm = ddp(thunder.jit(m))
        with jm.no_sync():
            jm(_data(rank, 0)).pow(2).mean().backward()
        bw_nosync = str(thunder.last_backward_traces(jm)[-1])
        jm(_data(rank, 1)).pow(2).mean().backward()
        bw_sync = str(thunder.last_backward_traces(jm)[-1])
        grads = {n: p.grad.detach().clone() for n, p in m.named_parameters()}
        torch.save({"grads": grads, "bw_nosync": bw_nosync, "bw_sync": bw_sync},
                   os.path.join(out_dir, f"rank{rank}.pt"))
    finally:
        torch.distributed.barrier()  # peers finish their collectives before gloo tears down
        torch.distributed.destroy_process_group()
    os._exit(0)  # skip interpreter teardown: gloo worker threads can abort it (rare SIGABRT)


def _fsdp_nosync_worker(rank, port, out_dir):
    import lightning_thunder_amd as thunder
    from lightning_thunder_amd.distributed import fsdp

    _init(rank, port)
    try:
        m = _model()
        jm = fsdp(thunder.jit(m))
        with jm.no_sync():
            for mb in range(2):
                jm(_data(rank, mb)).pow(2).mean().backward()
            stashed = sorted(n for n, p in m.named_parameters() if getattr(p, "_lc_unsharded_grad", None) is not None)
        bw_nosync = str(thunder.last_backward_traces(jm)[-1])
        jm(_data(rank, 2)).pow(2).mean().backward()
        bw_sync = str(thunder.last_backward_traces(jm)[-1])
        grads = {n: p.grad.detach().clone() for n, p in m.named_parameters()}
        left = [n for n, p in m.named_parameters() if getattr(p, "_lc_unsharded_grad", None) is not None]
        torch.save({"grads": grads, "bw_nosync": bw_nosync, "bw_sync": bw_sync, "stashed": stashed, "left": left},
                   os.path.join(out_dir, f"rank{rank}.pt"))
    finally:
        torch.distributed.barrier()  # peers finish their collectives before gloo tears down
        torch.distributed.destroy_process_group()
    os._exit(0)  # skip interpreter teardown: gloo worker threads can abort it (rare SIGABRT)


def _run(worker):
    port = _free_port()
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(worker, args=(port, d), nprocs=WORLD, join=True, start_method="spawn")
        return [torch.load(os.path.join(d, f"rank{r}.pt"), weights_only=False) for r in range(WORLD)]


def test_user_collectives_in_jit():
    res = _run(_collectives_worker)
    total = sum(range(1, WORLD + 1))
    gathered = torch.cat([torch.full((4,), float(r + 1)) for r in range(WORLD)])
    for rank, r in enumerate(res):
        torch.testing.assert_close(r["allreduce"], torch.full((4,), 2.0 * total + 1))
        torch.testing.assert_close(r["gather"], gathered)
        torch.testing.assert_close(r["scatter"], torch.full((2,), float(total)))
        torch.testing.assert_close(r["broadcast"], torch.full((4,), 2.0))
        m, g = r["functional"]
        torch.testing.assert_close(m, torch.full((4,), float(WORLD)))
        torch.testing.assert_close(g, gathered)
    assert "all_reduce" in res[0]["trace"]


def test_ddp_no_sync_grad_accumulation():
    res = _run(_nosync_worker)
    m = _model()
    loss = sum(m(_data(r, mb)).pow(2).mean() for r in range(WORLD) for mb in range(2)) / WORLD
    loss.backward()
    for r in res:
        for n, p in m.named_parameters():
            torch.testing.assert_close(r["grads"][n], p.grad)
        assert "all_reduce" not in r["bw_nosync"]
        assert "all_reduce" in r["bw_sync"]


def test_fsdp_no_sync_grad_accumulation():
    """FSDP under no_sync: the backward stashes unsharded gradients (no reduce-scatter); leaving the
    context reduce-scatters them once; a later synced step accumulates on top (reference
    test_fsdp.py no_sync tests)."""
    from lightning_thunder_amd.distributed.transforms import shard_tensor

    res = _run(_fsdp_nosync_worker)
    m = _model()
    loss = sum(m(_data(r, mb)).pow(2).mean() for r in range(WORLD) for mb in range(3)) / WORLD
    loss.backward()
    for rank, r in enumerate(res):
        assert r["stashed"] == sorted(n for n, _ in m.named_parameters()) and r["left"] == []
        for n, p in m.named_parameters():
            expected, _ = shard_tensor(p.grad, rank, WORLD)
            torch.testing.assert_close(r["grads"][n], expected)
        assert "reduce_scatter" not in r["bw_nosync"] and "stash_grad_for_fsdp" in r["bw_nosync"]
        assert "reduce_scatter" in r["bw_sync"]
