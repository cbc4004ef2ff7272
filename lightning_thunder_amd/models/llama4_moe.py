"""Llama-4-style mixture-of-experts block (model family of the reference's MoE tests,
``thunder/tests/llama4_moe.py`` and ``thunder/tests/distributed/test_moe.py:158-195``).

    out = shared_experts(x) + unsort(routed_experts(sort_by_expert(x * sigmoid(top1 router logit))))

* the router picks one expert per token (top-1 of ``gate(x)``), scales the token by the sigmoid
  of its logit, and tokens are sorted by expert id so each expert owns a contiguous row range;
* the routed experts are a :class:`GroupedSwiGLU`: three ``[E, out, in]`` weights applied with
  ``torch._grouped_mm`` over int32 cumulative offsets (one grouped GEMM per projection — on
  MI355X the grouped MFMA kernel K10, ``ops/csrc/gemm.hip``), no per-expert Python loop and
  no host synchronisation (the offsets stay on the device);
* the shared expert is a dense SwiGLU MLP of width ``intermediate_size * num_shared_experts``.

Expert weights ``[E, out, in]`` shard naturally for expert tensor parallelism on dim 1
(gate/up, column-wise) and dim -1 (down, row-wise); see ``tests/test_moe_tp.py``.
``torch._grouped_mm`` requires bf16 operands and 16-byte-aligned strides (hidden and
intermediate sizes multiples of 8).
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import torch
import torch.nn as nn
import torch.nn.functional as F


@dataclass(frozen=True)
class MoEConfig:
    name: str = "small"
    hidden_size: int = 256
    intermediate_size: int = 512
    num_routed_experts: int = 8
    num_shared_experts: int = 1


class SwiGLU(nn.Module):
    def __init__(self, hidden: int, inter: int):
        super().__init__()
        self.gate_proj = nn.Linear(hidden, inter, bias=False)
        self.up_proj = nn.Linear(hidden, inter, bias=False)
        self.down_proj = nn.Linear(inter, hidden, bias=False)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return self.down_proj(F.silu(self.gate_proj(x)) * self.up_proj(x))


class GroupedLinear(nn.Module):
    """``y[rows of expert e] = x[rows of expert e] @ weight[e].T`` for all experts in one grouped GEMM."""

    def __init__(self, groups: int, in_features: int, out_features: int):
        super().__init__()
        self.weight = nn.Parameter(torch.empty(groups, out_features, in_features))
        for w in self.weight.data:  # each expert initialised like an nn.Linear
            nn.init.kaiming_uniform_(w, a=math.sqrt(5))

    def forward(self, x: torch.Tensor, offsets: torch.Tensor) -> torch.Tensor:
        return torch._grouped_mm(x, self.weight.transpose(-1, -2), offsets)


class GroupedSwiGLU(nn.Module):
    def __init__(self, groups: int, hidden: int, inter: int):
        super().__init__()
        self.gate_proj = GroupedLinear(groups, hidden, inter)
        self.up_proj = GroupedLinear(groups, hidden, inter)
        self.down_proj = GroupedLinear(groups, inter, hidden)

    def forward(self, x: torch.Tensor, offsets: torch.Tensor) -> torch.Tensor:
        return self.down_proj(F.silu(self.gate_proj(x, offsets)) * self.up_proj(x, offsets), offsets)


class Llama4MoE(nn.Module):
    def __init__(self, config: MoEConfig):
        super().__init__()
        self.config = config
        self.gate = nn.Linear(config.hidden_size, config.num_routed_experts, bias=False)
        self.shared_experts = SwiGLU(config.hidden_size, config.intermediate_size * config.num_shared_experts)
        self.routed_experts = GroupedSwiGLU(config.num_routed_experts, config.hidden_size, config.intermediate_size)

    def route(self, x2: torch.Tensor):
        """(tokens sorted by expert and scaled by their router score, int32 expert end offsets,
        the sorting permutation)."""
        logits = self.gate(x2)  # [S, E]
        top_logit, top_id = logits.topk(1)  # [S, 1]
        scaled = x2 * top_logit.sigmoid()
        counts = torch.zeros(top_id.shape[0], self.config.num_routed_experts, device=x2.device, dtype=torch.int32)
        counts = counts.scatter(1, top_id, 1)
        offsets = torch.cumsum(counts.sum(0), 0, dtype=torch.int32)  # [E]
        order = top_id.view(-1).argsort()  # token ids grouped by expert
        return scaled[order], offsets, order

    def run_routed_experts(self, x: torch.Tensor) -> torch.Tensor:
        x2 = x.reshape(-1, x.shape[-1])
        tokens, offsets, order = self.route(x2)
        out_sorted = self.routed_experts(tokens, offsets)
        return out_sorted[order.argsort()].reshape(x.shape)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return self.shared_experts(x) + self.run_routed_experts(x)
