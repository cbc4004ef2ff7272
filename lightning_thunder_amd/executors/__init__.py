"""Executors: hipex (hand-written CDNA4 kernels), hipfuse (HIP fusion codegen), torch (ATen), python."""
