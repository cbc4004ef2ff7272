"""User HIP kernels as compiler operators: runtime-compiled with hiprtc, launched on the current stream.

Reference parity: ``notebooks/extend_thunder_with_cuda_python.ipynb`` (a CUDA kernel compiled at
run time with NVRTC and registered as a Thunder operator of a new executor, optionally replacing a
torch function and given a gradient).  MI355X design: the source is compiled for gfx950 by the
same native hiprtc runtime the fusion executor uses (``ops/csrc/runtime/rtc.cpp``: compile without
a GPU, disk-cached code objects, ``hipModuleLaunchKernel`` with the packed argument buffer).

    src = r'''
    extern "C" __global__ void scale_add(const float* x, const float* y, float* out, float a, long n) {
      long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
      if (i < n) out[i] = a * x[i] + y[i];
    }'''
    k = HipKernel(src, "scale_add", ("ptr", "ptr", "ptr", "f32", "i64"))

    def impl(x, y, a):
        out = torch.empty_like(x)
        k(((x.numel() + 255) // 256,), (256,), x, y, out, a, x.numel())
        return out

    ex = OperatorExecutor("my_kernels")
    scale_add = register_hip_kernel(ex, "scale_add", impl, meta=lambda x, y, a: TensorProxy(like=x))
    jm = thunder.jit(fn, executors=[ex, *thunder.get_default_executors()])

Argument kinds: ``ptr`` (a tensor's device pointer, or None), ``i32``, ``i64``, ``u32``, ``u64``,
``f32``, ``f64``; packed with the C ABI's natural alignment, as the kernel's parameter list is.
"""
from __future__ import annotations

import ctypes
import hashlib
import struct
from typing import Callable, Sequence

import torch

_KINDS = {"ptr": ("Q", 8), "i32": ("i", 4), "u32": ("I", 4), "i64": ("q", 8), "u64": ("Q", 8), "f32": ("f", 4),
          "f64": ("d", 8)}


class HipKernel:
    """A ``extern "C" __global__`` kernel in HIP source, compiled once per (source, defines) for
    gfx950 and callable as ``kernel(grid, block, *args, shared_mem=0, stream=None)``.  ``defines``
    become ``#define`` lines ahead of the source (tile sizes, unroll factors)."""

    def __init__(self, source: str, name: str, signature: Sequence[str], defines: dict | None = None):
        for kind in signature:
            if kind not in _KINDS:
                raise ValueError(f"unknown argument kind {kind!r}; known: {sorted(_KINDS)}")
        self.source = source
        self.name = name
        self.signature = tuple(signature)
        self.defines = dict(defines or {})
        self._fn = None

    # -- compilation (no GPU needed) ----------------------------------------------------------
    def compile(self) -> bytes:
        """The gfx950 code object (hiprtc; cached on disk next to the fusion executor's)."""
        from ..executors import hipfuse
        from ..executors.hipfuse_codegen import KernelSource

        ks = KernelSource(self.name, self._full_source(), None, None, None, None)
        return hipfuse.compile_source(ks)

    def _full_source(self) -> str:
        head = "#include <hip/hip_runtime.h>\n#include <hip/hip_bf16.h>\n#include <hip/hip_fp16.h>\n"
        defs = "".join(f"#define {k} {v}\n" for k, v in sorted(self.defines.items()))
        return head + defs + self.source

    def _function(self):
        if self._fn is None:
            from ..executors import hipfuse
            from ..executors.hipfuse_codegen import KernelSource

            self._fn = hipfuse.load_kernel(KernelSource(self.name, self._full_source(), None, None, None, None))
        return self._fn

    # -- launch ---------------------------------------------------------------------------------
    def pack(self, *args) -> bytes:
        """The kernel's argument struct: each argument at its natural alignment."""
        if len(args) != len(self.signature):
            raise TypeError(f"{self.name} takes {len(self.signature)} arguments, got {len(args)}")
        buf = bytearray()
        for kind, a in zip(self.signature, args):
            fmt, size = _KINDS[kind]
            buf.extend(b"\0" * ((-len(buf)) % size))
            if kind == "ptr":
                a = 0 if a is None else (a.data_ptr() if isinstance(a, torch.Tensor) else int(a))
            elif isinstance(a, torch.Tensor):
                raise TypeError(f"{self.name}: argument of kind {kind} got a tensor")
            buf.extend(struct.pack("<" + fmt, a))
        buf.extend(b"\0" * ((-len(buf)) % 8))
        return bytes(buf)

    def __call__(self, grid, block, *args, shared_mem: int = 0, stream=None) -> None:
        from ..executors import hipfuse

        grid = tuple(grid) + (1,) * (3 - len(grid))
        block = tuple(block) + (1,) * (3 - len(block))
        if stream is None:
            dev = next((a.device for a in args if isinstance(a, torch.Tensor) and a.is_cuda), None)
            stream = torch.cuda.current_stream(dev)
        packed = self.pack(*args)
        buf = ctypes.create_string_buffer(packed, len(packed))
        rc = hipfuse._lib().lta_rtc_launch(self._function(), *[int(g) for g in grid], *[int(b) for b in block],
                                           int(shared_mem), ctypes.c_void_p(stream.cuda_stream),
                                           ctypes.cast(buf, ctypes.c_void_p), len(packed))
        if rc != 0:
            raise RuntimeError(f"launching {self.name} failed with HIP error {rc}")

    def __repr__(self):
        h = hashlib.sha1(self.source.encode()).hexdigest()[:8]
        return f"HipKernel({self.name!r}, {self.signature}, src={h})"


def register_hip_kernel(executor, name: str, fn: Callable, *, meta: Callable, replaces: Callable | None = None,
                        checker: Callable | None = None, vjp: Callable | None = None):
    """Registers ``fn`` (a Python function launching :class:`HipKernel` s on torch tensors) as operator
    ``name`` of ``executor``.  ``meta`` gives the outputs' proxies; ``replaces`` makes traced calls of
    that torch function run this operator (e.g. ``torch.nn.functional.gelu``); ``vjp(*args) ->
    (outputs, backward)`` gives it a gradient (the backward may call other operators).  Returns the
    operator symbol, callable inside jitted functions."""
    op = executor.register_operator(name, meta=meta, fn=fn, replaces=replaces)
    executor.register_implementation(op, op, checker=checker)
    if vjp is not None:
        from ..core.transforms import register_vjp

        register_vjp(op)(vjp)
    return op
