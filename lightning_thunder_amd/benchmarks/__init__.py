"""Benchmarks (parity: reference ``thunder/benchmarks/`` — ``benchmark_litgpt.py``, ``targets.py``,
the HF ``generate`` quickstart ``examples/quickstart/hf_llm.py``).

* ``python bench.py`` (repo root): the headline LitGPT pretraining step (tokens/s).
* ``python -m lightning_thunder_amd.benchmarks.generate``: greedy generation latency with the static KV
  cache (eager vs compiled vs compiled + hipGraph), the reference README's Llama-3.2-1B / 100-token number.
* ``python -m lightning_thunder_amd.benchmarks.targets``: per-component micro-benchmarks (NanoGPT GPT-2
  block, LitGPT QKV-split+RoPE, RMSNorm, SDPA, cross-entropy) fwd/bwd, eager vs compiled.
"""
