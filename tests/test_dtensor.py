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


import pytest  # noqa: E402


@pytest.mark.gpu
def test_dtensor_column_parallel_products_on_hand_kernels_gpu():
    """Column-parallel DTensor products (replicated input, weight sharded on the output features)
    need no communication: their forward runs the hand-written GEMMs on the local shards
    (distributed/dtensor.py ``_local_product``) and the result keeps DTensor's placement."""
    import torch.nn.functional as F
    from torch.distributed.device_mesh import DeviceMesh
    from torch.distributed.tensor import DTensor, Replicate, Shard

    import lightning_thunder_amd as thunder
    from lightning_thunder_amd.ops.gemm import last_gemm_backend_counts

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    torch.distributed.init_process_group("gloo", rank=0, world_size=1)
    try:
        mesh = DeviceMesh("cuda", [0])
        torch.manual_seed(0)
        W = torch.randn(512, 256, device="cuda", dtype=torch.bfloat16) / 16
        X = torch.randn(128, 256, device="cuda", dtype=torch.bfloat16)
        w = DTensor.from_local(W, mesh, [Shard(0)], run_check=False)
        x = DTensor.from_local(X, mesh, [Replicate()], run_check=False)
        last_gemm_backend_counts(reset=True)
        y = thunder.jit(lambda x, w: F.linear(x, w))(x, w)
        assert last_gemm_backend_counts(reset=True).get("gemm4", 0) >= 1
        assert isinstance(y, DTensor) and tuple(y.placements) == (Shard(1),)
        ref = X.float() @ W.float().t()
        assert (y.to_local().float() - ref).abs().max().item() < 2e-2 * ref.abs().max().item()

        G, K, N = 4, 256, 384
        offs = torch.tensor([100, 160, 300, 512], device="cuda", dtype=torch.int32)
        WG = torch.randn(G, K, N, device="cuda", dtype=torch.bfloat16) / 16
        XG = torch.randn(512, K, device="cuda", dtype=torch.bfloat16)
        wg = DTensor.from_local(WG, mesh, [Shard(2)], run_check=False)
        xg = DTensor.from_local(XG, mesh, [Replicate()], run_check=False)
        og = DTensor.from_local(offs, mesh, [Replicate()], run_check=False)
        last_gemm_backend_counts(reset=True)
        yg = thunder.jit(lambda x, w, o: torch._grouped_mm(x, w, o))(xg, wg, og)
        assert last_gemm_backend_counts(reset=True).get("gemm4", 0) >= 1
        assert tuple(yg.placements) == (Shard(1),)
        refg = torch._grouped_mm(XG, WG, offs).float()
        assert (yg.to_local().float() - refg).abs().max().item() < 2e-2 * refg.abs().max().item()
    finally:
        torch.distributed.destroy_process_group()
