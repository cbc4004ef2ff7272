"""Native CDNA4 kernels (``_lta_kernels.so``) and their torch-tensor wrappers.

Kernel inventory: K4 RMSNorm, K6 RoPE/qkv-split, K7 softmax
cross-entropy, K3 flash attention, K1 fusion JIT (hiprtc), SwiGLU, fused AdamW,
K8 FP8 GEMM/quantize.  Each wrapper allocates outputs with the torch caching
allocator and launches on the current HIP stream (graph-capture safe).
"""
from ._lib import available, require  # noqa: F401
