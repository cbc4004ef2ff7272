"""Host-side dispatch rules of the attention wrappers (ops/attention.py), no GPU needed."""
import pytest

from lightning_thunder_amd.ops import attention as A


def test_dq_from_ds_auto_caps_the_workspace(monkeypatch):
    monkeypatch.delenv("LTA_ATTN_DQ_FROM_DS", raising=False)
    monkeypatch.delenv("LTA_ATTN_DS_MAX_GB", raising=False)
    # Llama-2-7B layer at T = 4096: 32 heads x 4096^2 bf16 = 1 GiB -> on
    assert A._dq_from_ds(32 * 4096 * 4096 * 2)
    # 4 GiB (T = 8192, 32 heads) is the default cap, inclusive
    assert A._dq_from_ds(4 * 2 ** 30)
    assert not A._dq_from_ds(4 * 2 ** 30 + 1)
    monkeypatch.setenv("LTA_ATTN_DS_MAX_GB", "0.5")
    assert not A._dq_from_ds(2 ** 30)


@pytest.mark.parametrize("mode,expect", [("0", False), ("1", True)])
def test_dq_from_ds_forced(monkeypatch, mode, expect):
    monkeypatch.setenv("LTA_ATTN_DQ_FROM_DS", mode)
    assert A._dq_from_ds(1 << 40) is expect
    assert A._dq_from_ds(0) is expect


@pytest.mark.parametrize("D,Dp", [(64, 64), (128, 128), (256, 256), (80, 96), (192, 256), (8, 64), (264, None), (100, None)])
def test_padded_head_dim(D, Dp):
    assert A.padded_head_dim(D) == Dp


def test_gqa_head_split_rule(monkeypatch):
    """dK/dV head split: only GQA, only while the (batch, kv head, 256-key block) grid is under two
    waves of 256 CUs, by a divisor of the group size, capped by LTA_ATTN_GQA_SPLIT."""
    from lightning_thunder_amd.ops import attention as A

    assert A.gqa_split(1, 32, 32, 4096) == 1            # MHA: no split
    assert A.gqa_split(1, 32, 8, 4096) == 4             # Mistral / Llama-3-8B: 128 workgroups -> 512
    assert A.gqa_split(4, 32, 8, 4096) == 1             # 512 workgroups already
    assert A.gqa_split(1, 64, 8, 4096) == 4             # Llama-2-70B: group 8, 128 -> 512
    assert A.gqa_split(1, 8, 1, 320) == 8               # MQA, one key block: the largest divisor
    monkeypatch.setenv("LTA_ATTN_GQA_SPLIT", "2")
    assert A.gqa_split(1, 32, 8, 4096) == 2
    monkeypatch.setenv("LTA_ATTN_GQA_SPLIT", "1")
    assert A.gqa_split(1, 32, 8, 4096) == 1
