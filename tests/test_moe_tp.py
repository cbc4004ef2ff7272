"""MoE expert tensor parallelism with DTensor (parity: reference
``thunder/tests/distributed/test_moe.py:29-195``): routed-expert ``GroupedLinear`` weights
``[E, out, in]`` sharded column-wise on dim 1 (gate/up) and row-wise on dim -1 (down) by custom
``ParallelStyle``s built on ``distribute_module``, run through ``jit`` and ``thunderfx``;
outputs and full weight gradients match the unsharded module.  CPU, gloo, world size 2, bf16
(``_grouped_mm`` requires it).  Also: forward (pre-)hooks are interpreted, so hook code sees
traced tensors as ``torch.Tensor``."""
import math
import os
import socket
import tempfile

import pytest
import torch
import torch.multiprocessing as mp
import torch.nn as nn
import torch.nn.functional as F

import lightning_thunder_amd as thunder


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class GroupedLinear(nn.Module):
    def __init__(self, groups, in_features, out_features):
        super().__init__()
        self.weight = nn.Parameter(torch.empty(groups, out_features, in_features))
        nn.init.kaiming_uniform_(self.weight, a=math.sqrt(5))

    def forward(self, x, offsets):
        return torch._grouped_mm(x, self.weight.transpose(-1, -2), offsets)


class GroupedSwiGLU(nn.Module):
    def __init__(self, groups, hidden, inter):
        super().__init__()
        self.gate_proj = GroupedLinear(groups, hidden, inter)
        self.up_proj = GroupedLinear(groups, hidden, inter)
        self.down_proj = GroupedLinear(groups, inter, hidden)

    def forward(self, x, offsets):
        return self.down_proj(F.silu(self.gate_proj(x, offsets)) * self.up_proj(x, offsets), offsets)


def _styles():
    from torch.distributed.tensor import DTensor, Replicate, Shard, distribute_module, distribute_tensor
    from torch.distributed.tensor.parallel import ParallelStyle

    def replicate_inputs(mod, inputs, mesh):
        return tuple(DTensor.from_local(i, mesh, (Replicate(),), run_check=False)
                     if isinstance(i, torch.Tensor) and not isinstance(i, DTensor) else i for i in inputs)

    class GroupedColwise(ParallelStyle):
        def _apply(self, module, mesh):
            def part(name, m, mesh):
                m.register_parameter("weight", nn.Parameter(distribute_tensor(m.weight, mesh, [Shard(1)])))

            return distribute_module(module, mesh, part, replicate_inputs, None)

    class GroupedRowwise(ParallelStyle):
        def _apply(self, module, mesh):
            def part(name, m, mesh):
                m.register_parameter("weight", nn.Parameter(distribute_tensor(m.weight, mesh, [Shard(-1)])))

            def out(mod, o, mesh):
                return o.redistribute(placements=(Replicate(),)).to_local()

            return distribute_module(module, mesh, part, replicate_inputs, out)

    return GroupedColwise, GroupedRowwise


def _worker(rank, world, port, d):
    from torch.distributed.device_mesh import init_device_mesh
    from torch.distributed.tensor.parallel import parallelize_module
    from lightning_thunder_amd.dynamo import thunderfx

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.distributed.init_process_group("gloo", rank=rank, world_size=world)
    res = {}
    try:
        mesh = init_device_mesh("cpu", (world,))
        Col, Row = _styles()
        for mode in ("jit", "thunderfx"):
            torch.manual_seed(0)
            m = GroupedSwiGLU(4, 16, 32).bfloat16()
            ref = GroupedSwiGLU(4, 16, 32).bfloat16()
            ref.load_state_dict(m.state_dict())
            pm = parallelize_module(m, mesh, {"gate_proj": Col(), "up_proj": Col(), "down_proj": Row()})
            x = torch.randn(24, 16, dtype=torch.bfloat16)
            offs = torch.tensor([5, 12, 20, 24], dtype=torch.int32)
            f = thunder.jit(pm) if mode == "jit" else thunderfx(pm)
            out, want = f(x, offs), ref(x, offs)
            res[f"{mode}_fwd"] = torch.allclose(out, want, atol=3e-2, rtol=3e-2)
            out.float().pow(2).sum().backward()
            want.float().pow(2).sum().backward()
            res[f"{mode}_bwd"] = all(
                torch.allclose(getattr(pm, n).weight.grad.full_tensor().float(), getattr(ref, n).weight.grad.float(),
                               atol=5e-2, rtol=5e-2) for n in ("gate_proj", "up_proj", "down_proj"))
        # the full Llama-4 MoE block with the reference's plan (test_moe.py:parallelize_moe_model)
        from torch.distributed.tensor import Shard
        from torch.distributed.tensor.parallel import ColwiseParallel, RowwiseParallel
        from lightning_thunder_amd.models.llama4_moe import Llama4MoE, MoEConfig

        torch.manual_seed(0)
        cfg = MoEConfig(hidden_size=32, intermediate_size=64, num_routed_experts=4)
        m = Llama4MoE(cfg).bfloat16()
        ref = Llama4MoE(cfg).bfloat16()
        ref.load_state_dict(m.state_dict())
        plan = {
            "shared_experts.gate_proj": ColwiseParallel(use_local_output=False, output_layouts=Shard(2)),
            "shared_experts.up_proj": ColwiseParallel(use_local_output=False, output_layouts=Shard(2)),
            "shared_experts.down_proj": RowwiseParallel(),
            "routed_experts.gate_proj": Col(),
            "routed_experts.up_proj": Col(),
            "routed_experts.down_proj": Row(),
        }
        pm = parallelize_module(m, mesh, plan)
        x = torch.randn(1, 16, 32, dtype=torch.bfloat16)
        out, want = thunder.jit(pm)(x), ref(x)
        res["llama4_fwd"] = torch.allclose(out.float(), want.float(), atol=5e-2, rtol=5e-2)
        out.float().pow(2).sum().backward()
        want.float().pow(2).sum().backward()
        names = ["routed_experts.gate_proj", "routed_experts.down_proj", "shared_experts.up_proj", "shared_experts.down_proj"]
        gp, gr = dict(pm.named_parameters()), dict(ref.named_parameters())
        res["llama4_bwd"] = all(
            torch.allclose(gp[n + ".weight"].grad.full_tensor().float(), gr[n + ".weight"].grad.float(), atol=8e-2, rtol=8e-2)
            for n in names)
        torch.save(res, os.path.join(d, f"r{rank}.pt"))
    finally:
        torch.distributed.barrier()  # peers finish their collectives before gloo tears down
        torch.distributed.destroy_process_group()
    os._exit(0)  # skip interpreter teardown: gloo worker threads can abort it (rare SIGABRT)


def test_moe_grouped_expert_tensor_parallel():
    world = 2
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_worker, args=(world, _free_port(), d), nprocs=world, join=True, start_method="spawn")
        for r in range(world):
            res = torch.load(os.path.join(d, f"r{r}.pt"), weights_only=True)
            assert set(res) == {"jit_fwd", "jit_bwd", "thunderfx_fwd", "thunderfx_bwd", "llama4_fwd", "llama4_bwd"}, res
            bad = {k: v for k, v in res.items() if v is not True}
            assert not bad, bad


def test_forward_hooks_are_interpreted():
    seen = []

    class M(nn.Module):
        def __init__(self):
            super().__init__()
            self.lin = nn.Linear(8, 8)

        def forward(self, x):
            return self.lin(x)

    m = M()

    def pre(mod, inputs):
        seen.append(isinstance(inputs[0], torch.Tensor))
        return (inputs[0] * 2,)

    def post(mod, inputs, out):
        return out + 1

    def pre_kw(mod, args, kwargs):
        return args, kwargs

    m.lin.register_forward_pre_hook(pre)
    m.lin.register_forward_hook(post)
    m.register_forward_pre_hook(pre_kw, with_kwargs=True)
    x = torch.randn(3, 8)
    jm = thunder.jit(m)
    torch.testing.assert_close(jm(x), m(x))
    assert seen and all(seen), seen
    names = {b.sym.name for b in thunder.last_traces(jm)[0].bound_symbols}
    assert any("mul" in n for n in names), names  # the hook's scaling is part of the program
