"""Trace transforms (parity: reference ``thunder/transforms/``)."""
from __future__ import annotations

from .autocast import autocast  # noqa: F401


def __getattr__(name):
    # Lazily resolve heavier transforms so importing the package stays cheap.
    if name in ("HipGraphTransform", "CUDAGraphTransform"):
        from .hipgraph import HipGraphTransform

        return HipGraphTransform
    if name == "MaterializationTransform":
        from .materialization import MaterializationTransform

        return MaterializationTransform
    if name == "ConstantFolding":
        from .constant_folding import ConstantFolding

        return ConstantFolding
    if name == "PrunePrologueChecks":
        from .prune_prologue_checks import PrunePrologueChecks

        return PrunePrologueChecks
    if name in ("LORATransform",):
        from .qlora import LORATransform

        return LORATransform
    raise AttributeError(name)
