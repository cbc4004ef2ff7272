"""DTensor inputs and DTensor tensor parallelism under jit (parity: reference
``thunder/tests/distributed/test_dtensor.py`` — basic ops fwd+bwd, unsupported mixed input,
column/row-wise ``parallelize_module``).  CPU, gloo, world size 2."""
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


_FNS = {
    "mul": lambda x, w: torch.mul(x, w),
    "add": lambda x, w: x + w,
    "matmul": lambda x, w: x @ w,
    "exp_neg": lambda x, w: torch.exp(-x) * w,
    "linear": lambda x, w: torch.nn.functional.linear(x, w),
    "reshape": lambda x, w: (x * w).reshape(-1, 8),
    "silu": lambda x, w: torch.nn.functional.silu(x) + w,
}


def _worker(rank, world, port, d):
    import lightning_thunder_amd as thunder
    from torch.distributed.tensor import Shard, distribute_tensor
    from torch.distributed.device_mesh import DeviceMesh
    from torch.distributed.tensor.parallel import parallelize_module, ColwiseParallel, RowwiseParallel

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.distributed.init_process_group("gloo", rank=rank, world_size=world)
    res = {}
    try:
        mesh = DeviceMesh("cpu", list(range(world)))
        torch.manual_seed(0)
        for k, fn in _FNS.items():
            w = distribute_tensor(torch.randn(16, 16, requires_grad=True), mesh, [Shard(0)])
            x = distribute_tensor(torch.randn(16, 16, requires_grad=True), mesh, [Shard(0)])
            e = fn(x, w)
            a = thunder.jit(fn)(x, w)
            g = distribute_tensor(torch.ones(e.shape), mesh, e.placements)
            eg = torch.autograd.grad(e, (x, w), g)
            ag = torch.autograd.grad(a, (x, w), g)
            res[k] = (torch.allclose(a.full_tensor(), e.full_tensor(), atol=1e-5)
                      and all(torch.allclose(p.full_tensor(), q.full_tensor(), atol=1e-5) for p, q in zip(eg, ag)))
        try:
            thunder.jit(lambda x, w: x * w)(x, torch.randn(16, 16))
            res["mixed_raises"] = False
        except Exception:  # noqa: BLE001
            res["mixed_raises"] = True

        m = torch.nn.Sequential(torch.nn.Linear(16, 32), torch.nn.ReLU(), torch.nn.Linear(32, 16))
        ref = torch.nn.Sequential(torch.nn.Linear(16, 32), torch.nn.ReLU(), torch.nn.Linear(32, 16))
        ref.load_state_dict(m.state_dict())
        pm = parallelize_module(m, mesh, {"0": ColwiseParallel(), "2": RowwiseParallel()})
        xin = torch.randn(4, 16)
        out_ref = ref(xin)
        out = thunder.jit(pm)(xin)
        out.sum().backward()
        out_ref.sum().backward()
        res["tp_fwd"] = torch.allclose(out, out_ref, atol=1e-5)
        res["tp_bwd"] = all(
            torch.allclose(pm[i].weight.grad.full_tensor(), ref[i].weight.grad, atol=1e-5) for i in (0, 2))
        torch.save(res, os.path.join(d, f"r{rank}.pt"))
    finally:
        torch.distributed.barrier()  # peers finish their collectives before gloo tears down
        torch.distributed.destroy_process_group()
    os._exit(0)  # skip interpreter teardown: gloo worker threads can abort it (rare SIGABRT)


def test_dtensor_ops_and_tensor_parallel():
    world = 2
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_worker, args=(world, _free_port(), d), nprocs=world, join=True, start_method="spawn")
        for r in range(world):
            res = torch.load(os.path.join(d, f"r{r}.pt"), weights_only=True)
            bad = {k: v for k, v in res.items() if v is not True}
            assert not bad, bad
