"""FP8 training plugin (reference ``thunder/plugins/fp8.py`` -> TransformerEngine): every eligible
``linear`` runs as an OCP-fp8 (e4m3 activations/weights, e5m2 gradients) GEMM on CDNA4."""
from __future__ import annotations

from ..core.recipe import Plugin


class FP8(Plugin):
    def __init__(self, recipe: str = "delayed", amax_history_len: int = 16):
        self.recipe = recipe
        self.amax_history_len = amax_history_len

    def setup_transforms(self):
        from ..transforms.fp8 import FP8LinearTransform

        return [FP8LinearTransform(recipe=self.recipe, amax_history_len=self.amax_history_len)]
