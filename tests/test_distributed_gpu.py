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


@pytest.mark.gpu
@pytest.mark.parametrize("vocab_start", [0, 96])
def test_vocab_parallel_cross_entropy_hand_kernels(nccl_world1, vocab_start):
    """The vocab-parallel CE's per-rank passes on the hand CE kernels (distributed/prims.py): at world 1
    this rank's slice [vocab_start, vocab_start + V) is the whole reduction, so rows / lse / dlogits must
    equal fp32 torch over that slice, with targets outside the slice contributing no one-hot term (their
    owner is another rank) and ignore_index rows a zero gradient."""
    import torch.distributed as tdist
    from lightning_thunder_amd.distributed.prims import _vp_ce_fwd_impl, _vp_ce_bwd_impl, _vp_ce_hand_kernels

    torch.manual_seed(0)
    rows, V = 300, 1000
    logits = (torch.randn(rows, V, device="cuda") * 3).to(torch.bfloat16)
    target = torch.randint(vocab_start, vocab_start + V + 200, (rows,), device="cuda")
    target[:7] = -100
    assert _vp_ce_hand_kernels(logits)
    g = tdist.distributed_c10d._get_default_group()
    out_rows, lse = _vp_ce_fwd_impl(logits, target, g, vocab_start)
    x = logits.float()
    ref_lse = torch.logsumexp(x, -1)
    t = target - vocab_start
    local = (t >= 0) & (t < V) & (target != -100)
    xt = torch.where(local, x.gather(1, t.clamp(0, V - 1)[:, None]).squeeze(1), torch.zeros((), device="cuda"))
    ref_rows = torch.where(target != -100, ref_lse - xt, torch.zeros((), device="cuda"))
    torch.testing.assert_close(lse, ref_lse, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(out_rows, ref_rows, rtol=1e-5, atol=1e-5)
    gr = torch.randn(rows, device="cuda")
    dl = _vp_ce_bwd_impl(gr, logits, target, lse, vocab_start)
    p = (x - ref_lse[:, None]).exp()
    p[local.nonzero().squeeze(1), t[local]] -= 1.0
    ref_dl = p * torch.where(target != -100, gr, torch.zeros((), device="cuda"))[:, None]
    assert dl.dtype == logits.dtype
    torch.testing.assert_close(dl.float(), ref_dl, rtol=2e-2, atol=2e-3)
