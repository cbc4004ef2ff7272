"""Static GEMM dispatch rules (ops/gemm.py): the K-split choice for under-filled tile grids."""
import pytest

from lightning_thunder_amd.ops.gemm import splitk_factor


@pytest.mark.parametrize("M,N,K", [(4096, 4096, 4096), (8192, 4096, 1024), (4096, 12288, 4096)])
def test_splitk_off_for_full_waves(M, N, K):
    assert splitk_factor(M, N, K, 256) == 0


def test_splitk_off_for_short_k():
    # 128 tiles x K=1024: the partial traffic costs more than the idle half of the chip
    assert splitk_factor(8192, 1024, 1024, 256) == 0
    assert splitk_factor(8192, 1024, 1000, 256) == 0  # K % 128: not a gemm4 shape


@pytest.mark.parametrize("M,N,K", [(1024, 1024, 8192), (3072, 1024, 8192), (4096, 1024, 8192), (8192, 1024, 4096),
                                   (8192, 1024, 50304), (1000, 1000, 4096)])
def test_splitk_fills_at_most_one_wave(M, N, K):
    nwg = -(-M // 256) * -(-N // 256)
    s = splitk_factor(M, N, K, 256)
    assert s >= 2
    assert nwg * s <= 256
    assert K // 128 >= s  # every slice gets at least one 128-deep K pair
    # fewer CUs: fewer slices
    assert splitk_factor(M, N, K, 128) <= s
