"""Greedy-sampling kernel (``csrc/sampling.hip``): row-wise argmax of decode logits."""
from __future__ import annotations

import torch

from ._lib import require, dcode, stream_ptr, check, register_signature, c_int, c_int64, c_void_p

register_signature("lta_argmax_rows", [c_int, c_void_p, c_void_p, c_int, c_int64, c_int64, c_void_p])


def argmax_last(x: torch.Tensor, keepdim: bool = False) -> torch.Tensor:
    """``x.argmax(-1)`` for [..., V] logits; the HIP kernel on MI355X, torch elsewhere."""
    V = x.shape[-1]
    x2 = x.reshape(-1, V) if x.dim() != 2 else x
    ok = (x.is_cuda and x.dtype in (torch.bfloat16, torch.float16, torch.float32)
          and x2.stride(-1) == 1 and x2.stride(0) % 8 == 0 and x2.data_ptr() % 16 == 0 and x2.shape[0] > 0)
    if not ok:
        return x.argmax(-1, keepdim=keepdim)
    out = torch.empty(x2.shape[0], dtype=torch.int64, device=x.device)
    check(require().lta_argmax_rows(dcode(x2), x2.data_ptr(), out.data_ptr(), x2.shape[0], V, x2.stride(0),
                                    stream_ptr(x.device)), "lta_argmax_rows")
    out = out.reshape(x.shape[:-1])
    return out.unsqueeze(-1) if keepdim else out
