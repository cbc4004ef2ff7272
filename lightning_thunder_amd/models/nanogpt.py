"""NanoGPT (GPT-2 architecture) in plain PyTorch (parity: the reference's test/benchmark model
``thunder/tests/nanogpt_model.py`` and ``thunder/benchmarks/__init__.py`` ``NanoGPTConfig`` :1139-1165).

Pre-LayerNorm GPT-2 blocks: fused ``c_attn`` (3*C), causal SDPA with attention dropout, tanh-GELU
MLP (4*C), learned position embeddings, weight tying between ``wte`` and ``lm_head``.  ``forward``
returns ``(logits, loss)`` (loss is ``None`` without targets), like nanoGPT.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, replace

import torch
import torch.nn as nn
import torch.nn.functional as F


@dataclass
class NanoGPTConfig:
    block_size: int = 1024
    seq_len: int = 128
    vocab_size: int = 50304  # GPT-2's 50257 padded to a multiple of 64
    n_layer: int = 12
    n_head: int = 12
    n_embd: int = 768
    dropout: float = 0.1
    bias: bool = True

    @classmethod
    def from_name(cls, name: str, **kwargs) -> "NanoGPTConfig":
        return replace(cls(**nanogpt_configs[name]), **kwargs)


nanogpt_configs = {
    "test": dict(n_layer=1, n_head=1, n_embd=64, seq_len=2, dropout=0.0, block_size=6, vocab_size=1024),
    "gpt2": dict(n_layer=12, n_head=12, n_embd=768),  # 124M
    "gpt2-medium": dict(n_layer=24, n_head=16, n_embd=1024),  # 350M
    "gpt2-large": dict(n_layer=36, n_head=20, n_embd=1280),  # 774M
    "gpt2-xl": dict(n_layer=48, n_head=25, n_embd=1600),  # 1558M
}


class CausalSelfAttention(nn.Module):
    def __init__(self, config: NanoGPTConfig):
        super().__init__()
        assert config.n_embd % config.n_head == 0
        self.c_attn = nn.Linear(config.n_embd, 3 * config.n_embd, bias=config.bias)
        self.c_proj = nn.Linear(config.n_embd, config.n_embd, bias=config.bias)
        self.resid_dropout = nn.Dropout(config.dropout)
        self.n_head = config.n_head
        self.dropout = config.dropout

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        B, T, C = x.shape
        hs = C // self.n_head
        q, k, v = self.c_attn(x).split(C, dim=2)
        q = q.view(B, T, self.n_head, hs).transpose(1, 2)
        k = k.view(B, T, self.n_head, hs).transpose(1, 2)
        v = v.view(B, T, self.n_head, hs).transpose(1, 2)
        y = F.scaled_dot_product_attention(q, k, v, dropout_p=self.dropout if self.training else 0.0, is_causal=True)
        y = y.transpose(1, 2).reshape(B, T, C)
        return self.resid_dropout(self.c_proj(y))


class MLP(nn.Module):
    def __init__(self, config: NanoGPTConfig):
        super().__init__()
        self.c_fc = nn.Linear(config.n_embd, 4 * config.n_embd, bias=config.bias)
        self.c_proj = nn.Linear(4 * config.n_embd, config.n_embd, bias=config.bias)
        self.dropout = nn.Dropout(config.dropout)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return self.dropout(self.c_proj(F.gelu(self.c_fc(x), approximate="tanh")))


class Block(nn.Module):
    def __init__(self, config: NanoGPTConfig):
        super().__init__()
        self.ln_1 = nn.LayerNorm(config.n_embd, bias=config.bias)
        self.attn = CausalSelfAttention(config)
        self.ln_2 = nn.LayerNorm(config.n_embd, bias=config.bias)
        self.mlp = MLP(config)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        x = x + self.attn(self.ln_1(x))
        return x + self.mlp(self.ln_2(x))


class NanoGPT(nn.Module):
    def __init__(self, config: NanoGPTConfig):
        super().__init__()
        self.config = config
        self.transformer = nn.ModuleDict(dict(
            wte=nn.Embedding(config.vocab_size, config.n_embd),
            wpe=nn.Embedding(config.block_size, config.n_embd),
            drop=nn.Dropout(config.dropout),
            h=nn.ModuleList(Block(config) for _ in range(config.n_layer)),
            ln_f=nn.LayerNorm(config.n_embd, bias=config.bias),
        ))
        self.lm_head = nn.Linear(config.n_embd, config.vocab_size, bias=False)
        self.transformer.wte.weight = self.lm_head.weight  # weight tying
        self.apply(self._init)
        for name, p in self.named_parameters():
            if name.endswith("c_proj.weight"):  # GPT-2 scaled residual init
                nn.init.normal_(p, mean=0.0, std=0.02 / math.sqrt(2 * config.n_layer))

    @staticmethod
    def _init(m):
        if isinstance(m, nn.Linear):
            nn.init.normal_(m.weight, mean=0.0, std=0.02)
            if m.bias is not None:
                nn.init.zeros_(m.bias)
        elif isinstance(m, nn.Embedding):
            nn.init.normal_(m.weight, mean=0.0, std=0.02)

    def forward(self, idx: torch.Tensor, targets: torch.Tensor | None = None):
        B, T = idx.shape
        pos = torch.arange(0, T, dtype=torch.long, device=idx.device)
        x = self.transformer.drop(self.transformer.wte(idx) + self.transformer.wpe(pos))
        for block in self.transformer.h:
            x = block(x)
        logits = self.lm_head(self.transformer.ln_f(x))
        loss = None
        if targets is not None:
            loss = F.cross_entropy(logits.view(-1, logits.size(-1)), targets.view(-1), ignore_index=-1)
        return logits, loss

    @classmethod
    def from_name(cls, name: str, **kwargs) -> "NanoGPT":
        return cls(NanoGPTConfig.from_name(name, **kwargs))
