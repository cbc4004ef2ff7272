"""Devices in the IR (parity: reference ``thunder/core/devices.py:13,85,170,188``).

The IR stores ``torch.device`` objects.  On PyTorch-ROCm the ``"cuda"`` device
type *is* the HIP device (MI355X), so ``cuda:N`` in a trace means HIP device N.
"""
from __future__ import annotations

from enum import Enum

import torch


class DeviceType(Enum):
    CPU = "cpu"
    CUDA = "cuda"  # HIP on PyTorch-ROCm
    META = "meta"


Device = torch.device

cpu = torch.device("cpu")


def to_device(x) -> torch.device | None:
    if x is None:
        return None
    if isinstance(x, torch.device):
        if x.type == "cuda" and x.index is None:
            return torch.device("cuda", torch.cuda.current_device() if torch.cuda.is_available() else 0)
        return x
    if isinstance(x, str):
        return to_device(torch.device(x))
    if isinstance(x, int):
        return torch.device("cuda", x)
    d = getattr(x, "device", None)
    if d is not None:
        return to_device(d)
    raise ValueError(f"Cannot convert {x} to a device")


def device_str(d: torch.device) -> str:
    if d.index is None:
        return d.type
    return f"{d.type}:{d.index}"


def is_gpu(d) -> bool:
    return d is not None and to_device(d).type == "cuda"
