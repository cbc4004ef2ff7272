"""Profiling-range transform under the reference's module path
(``thunder/dev_utils/nvtx_profile_transform.py:41-76``).  On MI355X the ranges are roctx ranges
(``torch.cuda.nvtx`` is backed by roctx on ROCm); the implementation is
:class:`lightning_thunder_amd.dev_utils.profile_transform.RoctxProfileTransform`."""
from .profile_transform import RoctxProfileTransform

NvtxProfileTransform = RoctxProfileTransform

__all__ = ["NvtxProfileTransform", "RoctxProfileTransform"]
