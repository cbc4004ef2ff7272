"""``reduce-overhead``: capture execution traces in hipGraphs (reference: CUDAGraphTransform plugin)."""
from __future__ import annotations

from ..core.recipe import Plugin, PluginPolicy


class ReduceOverhead(Plugin):
    policy = PluginPolicy.POST

    def __init__(self, **kwargs):
        self.kwargs = kwargs

    def setup_transforms(self):
        from ..transforms.hipgraph import HipGraphTransform

        return [HipGraphTransform(**self.kwargs)]
