"""RCCL paths of the distributed transforms on one MI355X (world size 1, backend "nccl" = RCCL):
the coalesced FSDP all-gather (grouped RCCL launch), bucketed reduce-scatter and the LitGPT
block bucket names, checked against the unbucketed program."""
import os
import socket

import pytest
import torch


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.fixture
def nccl_world1():
    import torch.distributed as tdist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(_free_port())
    torch.cuda.set_device(0)
    tdist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        yield
    finally:
        tdist.destroy_process_group()


def _step(strategy, zero3=False):
    import lightning_thunder_amd as thunder
    from lightning_thunder_amd.distributed import fsdp
    from lightning_thunder_amd.distributed.transforms import FSDPType
    from lightning_thunder_amd.models.litgpt import GPT

    torch.manual_seed(0)
    m = GPT.from_name("llama2-like").to(device="cuda", dtype=torch.bfloat16)
    m.set_rope_cache(64, device="cuda")
    jm = fsdp(thunder.jit(m), bucketing_strategy=strategy,
              sharding_strategy=FSDPType.ZERO3 if zero3 else FSDPType.ZERO2)
    x = torch.randint(0, m.config.vocab_size, (2, 64), device="cuda", generator=torch.Generator("cuda").manual_seed(1))
    out = jm(x)
    out.float().pow(2).mean().backward()
    grads = {n: p.grad.float().clone() for n, p in m.named_parameters()}
    return out.float(), grads, str(thunder.last_traces(jm)[-1]), str(thunder.last_backward_traces(jm)[-1])


@pytest.mark.gpu
@pytest.mark.parametrize("zero3", [False, True])
def test_fsdp_block_bucketing_rccl(nccl_world1, zero3):
    ref_out, ref_grads, fw0, _ = _step("none", zero3)
    out, grads, fw, bw = _step("block", zero3)
    assert "all_gather_coalesced(" not in fw0
    n_blocks = fw.count("all_gather_coalesced(")
    assert n_blocks >= 2, fw  # every transformer block + the parameters outside blocks
    torch.testing.assert_close(out, ref_out)
    for n, g in ref_grads.items():
        torch.testing.assert_close(grads[n], g)
    if zero3:
        assert "all_gather_coalesced(" in bw
