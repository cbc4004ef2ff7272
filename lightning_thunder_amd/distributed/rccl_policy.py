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

Trade-off that decides the default: every RCCL channel is a workgroup resident on a CU for the
collective's duration.  The collectives here run CONCURRENTLY with the backward's GEMMs (waits
sorted late, high-priority stream), and those GEMMs are sized one 256x256 tile per CU: a
256-tile wave that loses 32 CUs to RCCL channels becomes two waves.  More channels buy link
parallelism but cost compute throughput while overlapped, so the channel count is not forced up.

Policy (``apply``; environment defaults only, an explicit user setting always wins):
* ``LTA_RCCL_POLICY=default``: RCCL's own topology tuning (it detects the fully connected xGMI
  graph and sizes channels / algorithm / protocol per message), ``TORCH_NCCL_AVOID_RECORD_STREAMS=1``,
  and the high-priority communicator stream
  (:func:`~lightning_thunder_amd.distributed.high_priority_pg_options`) so collectives get a
  hardware queue of their own and overlap compute;
* ``LTA_RCCL_POLICY=wide``: additionally ``NCCL_MIN_NCHANNELS=32`` (stripe every per-rank shard
  over all links from the first collective on; for communication-bound configurations);
* ``LTA_RCCL_POLICY=ring``: additionally ``NCCL_ALGO=Ring`` (A/B hook);
* ``LTA_RCCL_POLICY=off``: the environment is left untouched.

The policy is set before ``init_process_group`` (RCCL reads it when the communicator is created)
and recorded: :func:`describe` returns the effective values, which ``bench.py`` prints on rank 0 and
puts into its JSON line (``rccl``), so every multi-GPU run states the policy it ran with.  No
8-GPU node is available to this build: the default is RCCL's tuning, not a sweep measured here.
"""
from __future__ import annotations

import os

POLICY_ENV = "LTA_RCCL_POLICY"
_KEYS = ("NCCL_MIN_NCHANNELS", "NCCL_MAX_NCHANNELS", "NCCL_ALGO", "NCCL_PROTO", "TORCH_NCCL_AVOID_RECORD_STREAMS",
         "TORCH_NCCL_ASYNC_ERROR_HANDLING", "LTA_NCCL_HIGH_PRIORITY", "RCCL_MSCCL_ENABLE")

DEFAULTS = {"TORCH_NCCL_AVOID_RECORD_STREAMS": "1"}
PRESETS = {"default": {}, "wide": {"NCCL_MIN_NCHANNELS": "32"}, "ring": {"NCCL_ALGO": "Ring"}}


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
