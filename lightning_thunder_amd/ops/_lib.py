"""ctypes binding of ``_lta_kernels.so`` (the in-tree native library).

On a machine with a HIP device the library MUST load: ``require()`` raises instead
of silently falling back, so a GPU run can never pass on an eager fallback.
"""
from __future__ import annotations

import ctypes
import os
import threading

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
# LTA_KERNELS_SO: load another build of the library (e.g. the diagnostic build of
# ``python -m lightning_thunder_amd.ops.build --diag``: phase-stamp / ablation kernels)
LIB_PATH = os.environ.get("LTA_KERNELS_SO") or os.path.join(HERE, "_lta_kernels.so")

_lib = None
_lock = threading.Lock()
_load_error: Exception | None = None

c_void_p = ctypes.c_void_p
c_int = ctypes.c_int
c_int64 = ctypes.c_int64
c_float = ctypes.c_float

# name -> argtypes (restype is always int: a hipError_t code)
_SIGNATURES: dict[str, list] = {
    "lta_rmsnorm_fwd": [c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_int64, c_float, c_void_p],
    "lta_rmsnorm_bwd": [c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_int64, c_int, c_void_p],
}


def register_signature(name: str, argtypes: list) -> None:
    _SIGNATURES[name] = argtypes
    if _lib is not None and hasattr(_lib, name):
        f = getattr(_lib, name)
        f.argtypes = argtypes
        f.restype = c_int


def _load():
    global _lib, _load_error
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            _load_error = FileNotFoundError(
                f"{LIB_PATH} not built; run `python -m lightning_thunder_amd.ops.build` (or __graft_entry__.build())"
            )
            raise _load_error
        lib = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
        for name, argtypes in _SIGNATURES.items():
            if hasattr(lib, name):
                f = getattr(lib, name)
                f.argtypes = argtypes
                f.restype = c_int
        _lib = lib
        return lib


def available() -> bool:
    """True if the library is loadable and a HIP device is present."""
    if not torch.cuda.is_available():
        return False
    try:
        _load()
        return True
    except Exception:
        return False


def require():
    """The loaded library; raises loudly when it is missing on a GPU box."""
    return _load()


DTYPE_CODE = {torch.float32: 0, torch.float16: 1, torch.bfloat16: 2, torch.float64: 3}


def dcode(t: torch.Tensor) -> int:
    return DTYPE_CODE[t.dtype]


def ptr(t: torch.Tensor | None):
    return None if t is None else t.data_ptr()


_raw_stream = getattr(torch._C, "_cuda_getCurrentRawStream", None)


def stream_ptr(device=None) -> int:
    """The current HIP stream of ``device`` as an integer handle.  Every kernel launch asks for it, so
    it takes the raw-stream accessor (one C call) instead of building a torch.cuda.Stream object."""
    if _raw_stream is not None:
        if device is None:
            idx = torch.cuda.current_device()
        elif isinstance(device, int):
            idx = device
        else:
            if isinstance(device, str):
                device = torch.device(device)
            idx = device.index if device.index is not None else torch.cuda.current_device()
        return _raw_stream(idx)
    return torch.cuda.current_stream(device).cuda_stream


def check(rc: int, what: str) -> None:
    if rc != 0:
        raise RuntimeError(f"{what} failed with HIP error code {rc}")
