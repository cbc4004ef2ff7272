"""RCCL policy for the data-parallel collectives over xGMI.

What the framework's collectives look like on one 8 x MI355X node:
* FSDP (ZeRO-2, ``bucketing_strategy="block"``): one coalesced all-gather of a transformer block's
  parameters (~405 MB gathered, ~50 MB per rank) per block in the forward, one coalesced
  reduce-scatter of the same size per block in the backward;
* DDP: 256 MB gradient buckets as coalesced all-reduces;
* TP: 32-64 MB activation all-reduces.
All are large messages.  The fabric is fully connected: every GPU has 7 xGMI links (~153 GB/s each)
to its 7 peers.  One ring uses one outgoing link per GPU, so its bandwidth is bounded by a single
link; RCCL reaches the aggregate by running many channels whose rings are laid over different link
permutations of the fully connected topology.

What decides the default (measured, ``profiles/cu_contention_r6.txt``, ``scripts/cu_contention.py``):
* an RCCL channel is one workgroup of ``ncclDevKernel_Generic`` resident on a CU for the whole
  collective; on gfx950 that kernel takes 37,664 B of LDS and 248-256 VGPRs (librccl 7.2 code-object
  metadata, read with ``llvm-readelf --notes``).  The hand GEMM's workgroup takes 128 KiB of LDS
  (two 64 KiB stages), so the two cannot share a CU (37 + 128 > 160 KiB): every CU a channel holds
  is a CU the GEMM loses;
* one-GPU emulation (workgroups of that shape held resident on a high-priority stream while the
  compute stream runs): the one-wave GEMMs (256 tiles, the o-projection and MLP down-projection)
  run 1.50-1.65x slower as soon as 8 CUs are taken, and no slower with 64 taken — any loss turns
  one wave into two; the three-wave qkv GEMM +13 %;
* so what costs compute is how LONG a collective overlaps the GEMMs, not how many channels it
  uses: the default finishes each collective as fast as the links allow, i.e. enough channels to
  stripe every shard over all seven xGMI links (``NCCL_MIN_NCHANNELS=32``).  ``narrow``
  (``NCCL_MAX_NCHANNELS=8``) is the opposite trade-off, kept as an A/B preset.

Policy (``apply``; environment defaults only, an explicit user setting always wins):
* ``LTA_RCCL_POLICY=default``: ``NCCL_MIN_NCHANNELS=32``, ``TORCH_NCCL_AVOID_RECORD_STREAMS=1``, and
  the high-priority communicator stream
  (:func:`~lightning_thunder_amd.distributed.high_priority_pg_options`) so collectives get a
  hardware queue of their own and overlap compute; RCCL's own tuning picks algorithm / protocol;
* ``LTA_RCCL_POLICY=narrow``: ``NCCL_MAX_NCHANNELS=8`` instead (fewer CUs held, longer overlap);
* ``LTA_RCCL_POLICY=ring``: additionally ``NCCL_ALGO=Ring`` (A/B hook);
* ``LTA_RCCL_POLICY=rccl``: RCCL's own channel count (round-5 behaviour);
* ``LTA_RCCL_POLICY=off``: the environment is left untouched.

The policy is set before ``init_process_group`` (RCCL reads it when the communicator is created)
and recorded: :func:`describe` returns the effective values, which ``bench.py`` prints on rank 0 and
puts into its JSON line (``rccl``), so every multi-GPU run states the policy it ran with.  No
8-GPU node is available to this build: the CU-contention curve is measured on one GPU; the
link-side gain of more channels is RCCL's, not measured here.
"""
from __future__ import annotations

import os

POLICY_ENV = "LTA_RCCL_POLICY"
_KEYS = ("NCCL_MIN_NCHANNELS", "NCCL_MAX_NCHANNELS", "NCCL_ALGO", "NCCL_PROTO", "TORCH_NCCL_AVOID_RECORD_STREAMS",
         "TORCH_NCCL_ASYNC_ERROR_HANDLING", "LTA_NCCL_HIGH_PRIORITY", "RCCL_MSCCL_ENABLE")

DEFAULTS = {"TORCH_NCCL_AVOID_RECORD_STREAMS": "1"}
PRESETS = {"default": {"NCCL_MIN_NCHANNELS": "32"}, "wide": {"NCCL_MIN_NCHANNELS": "32"},
           "narrow": {"NCCL_MAX_NCHANNELS": "8"}, "ring": {"NCCL_MIN_NCHANNELS": "32", "NCCL_ALGO": "Ring"},
           "rccl": {}}


def apply(env=None) -> dict:
    """Set the policy's defaults in ``env`` (``os.environ``) unless disabled; returns what it set."""
    env = os.environ if env is None else env
    mode = env.get(POLICY_ENV, "default").lower()
    if mode == "off":
        return {}
    if mode not in PRESETS:
        raise ValueError(f"{POLICY_ENV}={mode!r}: expected one of {sorted(PRESETS) + ['off']}")
    set_now = {}
    for k, v in {**DEFAULTS, **PRESETS[mode]}.items():
        if k not in env:
            env[k] = v
            set_now[k] = v
    return set_now


def describe(env=None) -> dict:
    """The RCCL-related settings in effect (None = RCCL's own default)."""
    env = os.environ if env is None else env
    out = {k: env.get(k) for k in _KEYS}
    out[POLICY_ENV] = env.get(POLICY_ENV, "default")
    return out
