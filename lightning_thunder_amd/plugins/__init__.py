"""Plugin registry for ``lightning_thunder_amd.compile(model, plugins=[...])`` (reference ``thunder/plugins``)."""
from __future__ import annotations

from .distributed import DDP, FSDP
from .fp8 import FP8
from .quantization import QuantizeInt4
from .reduce_overhead import ReduceOverhead
from .profile import Profile

_names: dict[str, type] = {
    "ddp": DDP,
    "fsdp": FSDP,
    "fp8": FP8,
    "quantize-int4": QuantizeInt4,
    "reduce-overhead": ReduceOverhead,
    "profile": Profile,
}


def get_plugin(name: str):
    if name not in _names:
        raise ValueError(f"unknown plugin {name!r}; known: {sorted(_names)}")
    return _names[name]


def get_plugin_names() -> list[str]:
    return list(_names)


def register_plugin(name: str, cls) -> None:
    _names[name] = cls


__all__ = ["DDP", "FSDP", "FP8", "QuantizeInt4", "ReduceOverhead", "Profile", "get_plugin", "get_plugin_names",
           "register_plugin"]
