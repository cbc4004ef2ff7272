"""einops backend for traced tensors (parity: the reference runs einops inside ``jit`` —
``thunder/tests/test_einops.py``).

einops picks a backend by the tensor's type; while tracing, tensors are :class:`TensorProxy`.
This backend reuses einops' torch backend (every operation is a torch call or tensor method,
which the acquisition routes to ``ltorch``) and only claims proxies.  einops discovers it through
``AbstractBackend.__subclasses__()`` because its ``framework_name`` module is imported.
"""
from __future__ import annotations

try:
    from einops._backends import TorchBackend
except Exception:  # einops not installed
    TorchBackend = None

if TorchBackend is not None:

    class ThunderProxyBackend(TorchBackend):
        framework_name = "lightning_thunder_amd"

        def is_appropriate_type(self, tensor):
            from ..core.proxies import TensorProxy

            return isinstance(tensor, TensorProxy)
