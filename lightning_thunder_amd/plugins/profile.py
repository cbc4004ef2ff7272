"""Profiling plugin: roctx ranges around a matched region of the execution trace
(reference ``thunder/plugins/profile.py`` -> ``ProfileTransform``)."""
from __future__ import annotations

from ..core.recipe import Plugin, PluginPolicy


class Profile(Plugin):
    policy = PluginPolicy.POST

    def __init__(self, input_match=None, from_match_idx: int = 0, to_match_idx: int = 1):
        from ..dev_utils.profile_transform import ProfileTransform

        self.profile_transform = ProfileTransform(input_match=input_match, start_idx=from_match_idx,
                                                  end_idx=to_match_idx)

    def setup_transforms(self):
        return [self.profile_transform]
