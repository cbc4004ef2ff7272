"""4-bit weight quantization plugin (reference ``thunder/plugins/quantization.py`` -> bitsandbytes NF4)."""
from __future__ import annotations

from ..core.recipe import Plugin


class QuantizeInt4(Plugin):
    def __init__(self, blocksize: int = 64):
        self.blocksize = blocksize

    def setup_transforms(self):
        from ..transforms.quantization import NF4LinearQuant4bit

        return [NF4LinearQuant4bit(blocksize=self.blocksize)]
