"""In-tree build of the native library ``_lta_kernels.so`` (HIP kernels for gfx950 + C++ runtime).

``python -m lightning_thunder_amd.ops.build`` compiles every ``csrc/*.hip`` kernel
translation unit and every ``csrc/runtime/*.cpp`` host unit with ``hipcc
--offload-arch=gfx950`` and links them (plus hiprtc for the fusion JIT) into
``ops/_lta_kernels.so``.  Incremental: objects are rebuilt only when a source or
header is newer.
"""
from __future__ import annotations

import concurrent.futures as cf
import glob
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
BUILD = os.path.join(HERE, "_build")
LIB = os.path.join(HERE, "_lta_kernels.so")
ARCH = os.environ.get("LTA_OFFLOAD_ARCH", "gfx950")


def _hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found (ROCm required to build lightning_thunder_amd kernels)")


def _headers_mtime() -> float:
    hs = glob.glob(os.path.join(CSRC, "**", "*.h"), recursive=True)
    return max((os.path.getmtime(h) for h in hs), default=0.0)


def _sources():
    hip = sorted(glob.glob(os.path.join(CSRC, "*.hip")))
    cpp = sorted(glob.glob(os.path.join(CSRC, "runtime", "*.cpp")))
    return hip, cpp


# Per-file device flags.  attention_fwd4: no SLP vectorisation (it packs the softmax row-sum chain
# into v_pk_add_f32, an anti-lever beside MFMAs: MI355X_MICROARCH.md constants table).  attention_bwd: MFMAs written as intrinsics take VGPR destinations, so the
# S / dP tiles stay where their softmax reads them while the dK / dV accumulators (inline-asm MFMAs)
# own the AGPR file (without it hipcc swaps them through AGPRs every tile).
FILE_FLAGS = {"attention_bwd.hip": ["-mllvm", "-amdgpu-mfma-vgpr-form=1"],
              "attention_fwd4.hip": ["-mllvm", "-amdgpu-mfma-vgpr-form=1", "-fno-slp-vectorize"],
              "attention_fwd_d256.hip": ["-mllvm", "-amdgpu-mfma-vgpr-form=1"]}


def _compile(src: str, obj: str, is_device: bool, verbose: bool, defines=()) -> str:
    cmd = [_hipcc(), "-c", src, "-o", obj, "-fPIC", "-O3", "-std=c++17", f"-I{CSRC}", "-Wno-unused-result",
           *[f"-D{d}" for d in defines]]
    if is_device:
        cmd += [f"--offload-arch={ARCH}", "-munsafe-fp-atomics"] + FILE_FLAGS.get(os.path.basename(src), [])
    else:
        cmd += ["-D__HIP_PLATFORM_AMD__"]
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"compilation failed for {src}:\n{r.stderr[-8000:]}")
    return obj


def build(force: bool = False, verbose: bool = False, jobs: int | None = None, defines=(), build_dir: str | None = None,
          lib_path: str | None = None) -> str:
    """Incremental hipcc build of every csrc source for gfx950 into one shared library.  ``defines``
    / ``build_dir`` / ``lib_path`` make a separate variant (the diagnostic build: ``--diag OUT``
    compiles the measurement-only kernels behind -DLTA_ATTN_DIAG into OUT, loaded with
    LTA_KERNELS_SO=OUT; the production library is untouched)."""
    BUILD = build_dir or globals()["BUILD"]
    LIB = lib_path or globals()["LIB"]
    os.makedirs(BUILD, exist_ok=True)
    hip, cpp = _sources()
    hdr = _headers_mtime()
    todo = []
    objs = []
    for src in hip + cpp:
        obj = os.path.join(BUILD, os.path.basename(src) + ".o")
        objs.append(obj)
        if force or not os.path.exists(obj) or os.path.getmtime(obj) < max(os.path.getmtime(src), hdr):
            todo.append((src, obj, src.endswith(".hip")))
    jobs = jobs or min(8, max(1, (os.cpu_count() or 4) // 2))
    if todo:
        with cf.ThreadPoolExecutor(jobs) as pool:
            futs = [pool.submit(_compile, s, o, d, verbose, defines) for s, o, d in todo]
            for f in futs:
                f.result()
    newest = max((os.path.getmtime(o) for o in objs), default=0.0)
    if force or todo or not os.path.exists(LIB) or os.path.getmtime(LIB) < newest:
        cmd = [_hipcc(), "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", LIB + ".tmp", *objs, "-lhiprtc"]
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stderr[-8000:]}")
        os.replace(LIB + ".tmp", LIB)
    return LIB


if __name__ == "__main__":
    if "--diag" in sys.argv:
        out = os.path.abspath(sys.argv[sys.argv.index("--diag") + 1])
        path = build(force="--force" in sys.argv, verbose="-v" in sys.argv, defines=("LTA_ATTN_DIAG",),
                     build_dir=os.path.join(os.path.dirname(out), "_build_diag"), lib_path=out)
    else:
        path = build(force="--force" in sys.argv, verbose="-v" in sys.argv)
    print(path)
