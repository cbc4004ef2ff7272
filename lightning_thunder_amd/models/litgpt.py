"""LitGPT-architecture decoder models in plain PyTorch (parity: the LitGPT configs/model used by the
reference's ``thunder/benchmarks/benchmark_litgpt.py:295,335`` and ``thunder/tests/litgpt_model.py:1-131``).

LitGPT itself is not installed in this image, so the architecture is defined
here with LitGPT's module names (``transformer.wte``, ``transformer.h[i].attn.attn``,
``mlp.fc_1/fc_2/proj``, ``lm_head`` …) so checkpoints and traces line up.

Hot spots live in small module-level helpers (``apply_rope``, ``qkv_split_rope``)
written in plain torch; the HIP executor registers lookasides for them so a
compiled model runs the fused CDNA4 kernels while eager PyTorch runs the same
math unfused (that is the "speedup vs eager" baseline).
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field, replace
from typing import Optional

import torch
import torch.nn as nn
import torch.utils.checkpoint
import torch.nn.functional as F


@dataclass
class Config:
    name: str = ""
    block_size: int = 4096
    vocab_size: int = 32000
    padded_vocab_size: Optional[int] = None
    padding_multiple: int = 512
    n_layer: int = 32
    n_head: int = 32
    n_embd: int = 4096
    head_size: Optional[int] = None
    n_query_groups: Optional[int] = None
    rotary_percentage: float = 1.0
    parallel_residual: bool = False
    bias: bool = False
    norm_class_name: str = "RMSNorm"
    norm_eps: float = 1e-5
    mlp_class_name: str = "LLaMAMLP"
    intermediate_size: Optional[int] = None
    rope_base: int = 10000
    rope_condense_ratio: int = 1
    shared_attention_norm: bool = False
    gelu_approximate: str = "none"
    tie_embeddings: bool = False
    n_expert: int = 0
    n_expert_per_token: int = 0
    # Gemma: token embeddings scaled by sqrt(n_embd), RMSNorm scale (1 + weight)
    scale_embeddings: bool = False
    norm_unit_offset: bool = False

    def __post_init__(self):
        if self.head_size is None:
            self.head_size = self.n_embd // self.n_head
        if self.padded_vocab_size is None:
            self.padded_vocab_size = ((self.vocab_size + self.padding_multiple - 1) // self.padding_multiple) * self.padding_multiple
        if self.n_query_groups is None:
            self.n_query_groups = self.n_head
        if self.intermediate_size is None:
            self.intermediate_size = 4 * self.n_embd
        self.rope_n_elem = int(self.rotary_percentage * self.head_size)

    @classmethod
    def from_name(cls, name: str, **kwargs) -> "Config":
        base = name_to_config[name]
        return replace(base, **kwargs)

    @property
    def qkv_size(self) -> int:
        return (self.n_head + 2 * self.n_query_groups) * self.head_size


configs = [
    # Meta Llama 2
    Config(name="Llama-2-7b-hf", vocab_size=32000, padding_multiple=64, n_layer=32, n_head=32, n_embd=4096,
           intermediate_size=11008, norm_eps=1e-5),
    Config(name="Llama-2-13b-hf", vocab_size=32000, padding_multiple=64, n_layer=40, n_head=40, n_embd=5120,
           intermediate_size=13824, norm_eps=1e-5),
    Config(name="Llama-2-70b-hf", vocab_size=32000, padding_multiple=64, n_layer=80, n_head=64, n_embd=8192,
           n_query_groups=8, intermediate_size=28672, norm_eps=1e-5),
    # Meta Llama 3
    Config(name="Llama-3-8B", block_size=8192, vocab_size=128000, padded_vocab_size=128256, n_layer=32, n_head=32,
           n_embd=4096, n_query_groups=8, intermediate_size=14336, rope_base=500000),
    Config(name="Llama-3-70B", block_size=8192, vocab_size=128000, padded_vocab_size=128256, n_layer=80, n_head=64,
           n_embd=8192, n_query_groups=8, intermediate_size=28672, rope_base=500000),
    Config(name="Llama-3.2-1B", block_size=8192, vocab_size=128000, padded_vocab_size=128256, n_layer=16, n_head=32,
           n_embd=2048, n_query_groups=8, intermediate_size=8192, rope_base=500000, tie_embeddings=True),
    # Mistral
    Config(name="Mistral-7B-v0.1", block_size=4096, vocab_size=32000, padded_vocab_size=32000, n_layer=32, n_head=32,
           n_embd=4096, n_query_groups=8, intermediate_size=14336),
    Config(name="Mistral-7B-v0.2", block_size=32768, vocab_size=32000, padded_vocab_size=32000, n_layer=32, n_head=32,
           n_embd=4096, n_query_groups=8, intermediate_size=14336, rope_base=1000000),
    # Google Gemma (the reference's multi-model chart and GemmaMLP target, BASELINE.md:26):
    # head_size 256 (n_head * head_size != n_embd), GeGLU (tanh) MLP, scaled embeddings, (1 + w) RMSNorm
    Config(name="Gemma-2b", block_size=8192, vocab_size=256000, padding_multiple=64, n_layer=18, n_head=8,
           n_query_groups=1, n_embd=2048, head_size=256, intermediate_size=16384, mlp_class_name="GemmaMLP",
           gelu_approximate="tanh", scale_embeddings=True, norm_unit_offset=True, norm_eps=1e-6, tie_embeddings=True),
    Config(name="Gemma-7b", block_size=8192, vocab_size=256000, padding_multiple=64, n_layer=28, n_head=16,
           n_query_groups=16, n_embd=3072, head_size=256, intermediate_size=24576, mlp_class_name="GemmaMLP",
           gelu_approximate="tanh", scale_embeddings=True, norm_unit_offset=True, norm_eps=1e-6, tie_embeddings=True),
    # Microsoft Phi-3
    Config(name="Phi-3-mini-4k-instruct", block_size=4096, vocab_size=32064, padded_vocab_size=32064, n_layer=32,
           n_head=32, n_embd=3072, intermediate_size=8192, norm_eps=1e-5),
    # Llama-1-architecture fine-tunes of the chart
    Config(name="Nous-Hermes-13b", block_size=2048, vocab_size=32000, padded_vocab_size=32001, n_layer=40, n_head=40,
           n_embd=5120, intermediate_size=13824, norm_eps=1e-6),
    Config(name="Platypus-30B", block_size=2048, vocab_size=32000, padded_vocab_size=32000, n_layer=60, n_head=52,
           n_embd=6656, intermediate_size=17920, norm_eps=1e-6),
    # CodeLlama
    Config(name="CodeLlama-34b-hf", block_size=16384, vocab_size=32000, padded_vocab_size=32000, n_layer=48, n_head=64,
           n_embd=8192, n_query_groups=8, intermediate_size=22016, rope_base=1000000),
    # Small test configs (reference thunder/tests/litgpt_model.py)
    Config(name="llama2-like", vocab_size=320, padding_multiple=64, n_layer=2, n_head=4, n_embd=64, intermediate_size=86,
           block_size=128),
    Config(name="llama3-like", vocab_size=320, padded_vocab_size=320, n_layer=2, n_head=4, n_embd=64, n_query_groups=2,
           intermediate_size=96, block_size=128, rope_base=500000),
    Config(name="gpt-neox-like", vocab_size=320, padding_multiple=64, n_layer=2, n_head=4, n_embd=64, block_size=128,
           norm_class_name="LayerNorm", mlp_class_name="GptNeoxMLP", bias=True, parallel_residual=True,
           rotary_percentage=0.25),
    # Mixtral-style sparse MoE (litgpt "LLaMAMoE"): 8 experts, top-2 routing
    Config(name="Mixtral-8x7B-v0.1", vocab_size=32000, padding_multiple=512, n_layer=32, n_head=32, n_embd=4096,
           n_query_groups=8, intermediate_size=14336, mlp_class_name="LLaMAMoE", n_expert=8, n_expert_per_token=2,
           rope_base=1000000, norm_eps=1e-5),
    Config(name="mixtral-like", vocab_size=320, padding_multiple=64, n_layer=2, n_head=4, n_embd=256, n_query_groups=2,
           intermediate_size=512, mlp_class_name="LLaMAMoE", n_expert=4, n_expert_per_token=2),
    Config(name="llama2-7b-shape-2l", vocab_size=32000, padding_multiple=64, n_layer=2, n_head=32, n_embd=4096,
           intermediate_size=11008),
    Config(name="gemma-like", vocab_size=320, padding_multiple=64, n_layer=2, n_head=2, n_query_groups=1, n_embd=64,
           head_size=256, intermediate_size=128, block_size=128, mlp_class_name="GemmaMLP", gelu_approximate="tanh",
           scale_embeddings=True, norm_unit_offset=True, norm_eps=1e-6, tie_embeddings=True),
]
name_to_config = {c.name: c for c in configs}


def build_rope_cache(seq_len: int, n_elem: int, device=None, base: int = 10000, condense_ratio: int = 1):
    theta = 1.0 / (base ** (torch.arange(0, n_elem, 2, device=device).float() / n_elem))
    seq_idx = torch.arange(seq_len, device=device) / condense_ratio
    idx_theta = torch.outer(seq_idx, theta).repeat(1, 2)
    return torch.cos(idx_theta), torch.sin(idx_theta)


def apply_rope(x: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor) -> torch.Tensor:
    """x: [B, H, T, hs]; cos/sin: [T, hs]  (LitGPT's rotate-half formulation)."""
    head_size = x.size(-1)
    x1 = x[..., : head_size // 2]
    x2 = x[..., head_size // 2:]
    rotated = torch.cat((-x2, x1), dim=-1)
    roped = (x * cos) + (rotated * sin)
    return roped.to(dtype=x.dtype)


def qkv_split_rope(qkv: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor, n_head: int, n_query_groups: int,
                   head_size: int, rope_n_elem: int):
    """Splits fused qkv [B, T, (nh+2*ng)*hs] into q [B, nh, T, hs], k/v [B, ng, T, hs] and applies RoPE to q, k."""
    B, T, _ = qkv.shape
    q_size = n_head * head_size
    kv_size = n_query_groups * head_size
    q, k, v = qkv.split((q_size, kv_size, kv_size), dim=-1)
    q = q.view(B, T, n_head, head_size).transpose(1, 2)
    k = k.view(B, T, n_query_groups, head_size).transpose(1, 2)
    v = v.view(B, T, n_query_groups, head_size).transpose(1, 2)
    if rope_n_elem == head_size:
        q = apply_rope(q, cos, sin)
        k = apply_rope(k, cos, sin)
    else:
        q = torch.cat((apply_rope(q[..., :rope_n_elem], cos, sin), q[..., rope_n_elem:]), dim=-1)
        k = torch.cat((apply_rope(k[..., :rope_n_elem], cos, sin), k[..., rope_n_elem:]), dim=-1)
    return q, k, v


def swiglu(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """LLaMA MLP gate: silu(a) * b."""
    return F.silu(a) * b


class RMSNorm(nn.Module):
    """RMSNorm; ``add_unit_offset`` (Gemma) scales by ``1 + weight`` with the weight initialised to
    zero, so the stored parameter is the deviation from identity."""

    def __init__(self, size: int, dim: int = -1, eps: float = 1e-6, add_unit_offset: bool = False):
        super().__init__()
        self.add_unit_offset = add_unit_offset
        self.weight = nn.Parameter(torch.zeros(size) if add_unit_offset else torch.ones(size))
        self.eps = eps
        self.dim = dim

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        w = self.weight + 1.0 if self.add_unit_offset else self.weight
        return F.rms_norm(x, (x.shape[-1],), w, self.eps)

    def reset_parameters(self) -> None:
        (nn.init.zeros_ if self.add_unit_offset else nn.init.ones_)(self.weight)


def _norm(config: Config, size: int) -> nn.Module:
    if config.norm_class_name == "RMSNorm":
        return RMSNorm(size, eps=config.norm_eps, add_unit_offset=config.norm_unit_offset)
    return nn.LayerNorm(size, eps=config.norm_eps)


class KVCache(nn.Module):
    """Static key/value cache (LitGPT ``KVCache``): [B, n_query_groups, max_seq, head_size] buffers
    updated in place at ``input_pos``.  Static storage keeps the decode step's addresses fixed, so
    a compiled decode step is a cache hit every token and can be replayed as one hipGraph."""

    def __init__(self, k_shape, v_shape, device=None, dtype=None):
        super().__init__()
        self.register_buffer("k", torch.zeros(k_shape, device=device, dtype=dtype), persistent=False)
        self.register_buffer("v", torch.zeros(v_shape, device=device, dtype=dtype), persistent=False)

    def forward(self, input_pos: torch.Tensor, k: torch.Tensor, v: torch.Tensor):
        k_all = self.k.index_copy_(2, input_pos, k.to(self.k.dtype))
        v_all = self.v.index_copy_(2, input_pos, v.to(self.v.dtype))
        return k_all, v_all

    def reset_parameters(self) -> None:
        torch.nn.init.zeros_(self.k)
        torch.nn.init.zeros_(self.v)


class CausalSelfAttention(nn.Module):
    def __init__(self, config: Config):
        super().__init__()
        self.attn = nn.Linear(config.n_embd, config.qkv_size, bias=config.bias)
        self.proj = nn.Linear(config.n_head * config.head_size, config.n_embd, bias=config.bias)
        self.config = config
        self.kv_cache: Optional[KVCache] = None

    def forward(self, x: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor, mask: Optional[torch.Tensor] = None,
                input_pos: Optional[torch.Tensor] = None) -> torch.Tensor:
        B, T, C = x.shape
        c = self.config
        qkv = self.attn(x)
        q, k, v = qkv_split_rope(qkv, cos, sin, c.n_head, c.n_query_groups, c.head_size, c.rope_n_elem)
        if input_pos is not None:
            if self.kv_cache is None:
                raise TypeError("call model.set_kv_cache(...) before passing input_pos")
            k, v = self.kv_cache(input_pos, k, v)
            y = F.scaled_dot_product_attention(q, k, v, attn_mask=mask, enable_gqa=c.n_query_groups != c.n_head)
        else:
            y = F.scaled_dot_product_attention(q, k, v, is_causal=True, enable_gqa=c.n_query_groups != c.n_head)
        y = y.transpose(1, 2).reshape(B, T, c.n_head * c.head_size)
        return self.proj(y)


class LLaMAMLP(nn.Module):
    def __init__(self, config: Config):
        super().__init__()
        self.fc_1 = nn.Linear(config.n_embd, config.intermediate_size, bias=config.bias)
        self.fc_2 = nn.Linear(config.n_embd, config.intermediate_size, bias=config.bias)
        self.proj = nn.Linear(config.intermediate_size, config.n_embd, bias=config.bias)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        x_fc_1 = self.fc_1(x)
        x_fc_2 = self.fc_2(x)
        return self.proj(swiglu(x_fc_1, x_fc_2))


def geglu(a: torch.Tensor, b: torch.Tensor, approximate: str = "tanh") -> torch.Tensor:
    """Gemma MLP gate: gelu(a) * b."""
    return F.gelu(a, approximate=approximate) * b


class GemmaMLP(nn.Module):
    """LitGPT ``GemmaMLP`` (the reference benchmarks it, thunder/benchmarks/targets.py:578): the
    LLaMA MLP layout with a GeGLU gate."""

    def __init__(self, config: Config):
        super().__init__()
        self.fc_1 = nn.Linear(config.n_embd, config.intermediate_size, bias=config.bias)
        self.fc_2 = nn.Linear(config.n_embd, config.intermediate_size, bias=config.bias)
        self.proj = nn.Linear(config.intermediate_size, config.n_embd, bias=config.bias)
        self.config = config

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return self.proj(geglu(self.fc_1(x), self.fc_2(x), self.config.gelu_approximate))


class GptNeoxMLP(nn.Module):
    def __init__(self, config: Config):
        super().__init__()
        self.fc = nn.Linear(config.n_embd, config.intermediate_size, bias=config.bias)
        self.proj = nn.Linear(config.intermediate_size, config.n_embd, bias=config.bias)
        self.config = config

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        x = self.fc(x)
        x = F.gelu(x, approximate=self.config.gelu_approximate)
        return self.proj(x)


class LLaMAMoE(nn.Module):
    """Sparse MoE MLP (litgpt ``LLaMAMoE``): softmax top-k router, tokens sorted by expert and run
    through *grouped* GEMMs (``torch._grouped_mm`` -> the K10 HIP kernel on MI355X), combined with
    the routing weights.  Expert weights are stored [E, out, in] like ``nn.Linear``."""

    def __init__(self, config: Config):
        super().__init__()
        E, D, I = config.n_expert, config.n_embd, config.intermediate_size
        self.gate = nn.Linear(D, E, bias=False)
        self.fc_1 = nn.Parameter(torch.empty(E, I, D))
        self.fc_2 = nn.Parameter(torch.empty(E, I, D))
        self.proj = nn.Parameter(torch.empty(E, D, I))
        self.config = config
        self.reset_parameters()

    def reset_parameters(self, std: float = 0.02) -> None:
        for w in (self.fc_1, self.fc_2, self.proj):
            nn.init.normal_(w, std=std)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        B, T, D = x.shape
        E, k = self.config.n_expert, self.config.n_expert_per_token
        xf = x.reshape(-1, D)
        probs = torch.softmax(self.gate(xf).float(), dim=-1)
        weights, experts = torch.topk(probs, k, dim=-1)                       # [N, k]
        weights = (weights / weights.sum(-1, keepdim=True)).to(x.dtype)
        flat_e = experts.reshape(-1)                                          # [N*k]
        order = torch.argsort(flat_e, stable=True)
        token = torch.div(order, k, rounding_mode="floor")
        counts = torch.nn.functional.one_hot(flat_e, E).sum(0)
        offs = torch.cumsum(counts, 0).to(torch.int32)
        xs = xf[token]                                                        # [N*k, D] sorted by expert
        a = torch._grouped_mm(xs, self.fc_1.transpose(1, 2), offs)
        b = torch._grouped_mm(xs, self.fc_2.transpose(1, 2), offs)
        h = swiglu(a, b)
        ys = torch._grouped_mm(h, self.proj.transpose(1, 2), offs)            # [N*k, D]
        ys = ys * weights.reshape(-1)[order].unsqueeze(-1)
        out = torch.zeros_like(xf).index_add(0, token, ys)
        return out.reshape(B, T, D)


class Block(nn.Module):
    def __init__(self, config: Config):
        super().__init__()
        self.norm_1 = _norm(config, config.n_embd)
        self.attn = CausalSelfAttention(config)
        self.norm_2 = None if config.shared_attention_norm else _norm(config, config.n_embd)
        if config.mlp_class_name == "LLaMAMLP":
            self.mlp = LLaMAMLP(config)
        elif config.mlp_class_name == "LLaMAMoE":
            self.mlp = LLaMAMoE(config)
        elif config.mlp_class_name == "GemmaMLP":
            self.mlp = GemmaMLP(config)
        else:
            self.mlp = GptNeoxMLP(config)
        self.config = config

    def forward(self, x: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor, mask: Optional[torch.Tensor] = None,
                input_pos: Optional[torch.Tensor] = None) -> torch.Tensor:
        x_normed = self.norm_1(x)
        h = self.attn(x_normed, cos, sin, mask, input_pos)
        if self.config.parallel_residual:
            n2 = x_normed if self.norm_2 is None else self.norm_2(x)
            return self.mlp(n2) + h + x
        x = h + x
        return self.mlp(self.norm_2(x)) + x


class GPT(nn.Module):
    def __init__(self, config: Config):
        super().__init__()
        self.config = config
        self.activation_checkpointing = False  # per-Block torch.utils.checkpoint in training forwards
        self.lm_head = nn.Linear(config.n_embd, config.padded_vocab_size, bias=config.lm_head_bias if hasattr(config, "lm_head_bias") else False)
        self.transformer = nn.ModuleDict(
            dict(
                wte=nn.Embedding(config.padded_vocab_size, config.n_embd),
                h=nn.ModuleList(Block(config) for _ in range(config.n_layer)),
                ln_f=_norm(config, config.n_embd),
            )
        )
        if config.tie_embeddings:
            self.lm_head.weight = self.transformer.wte.weight
        self.max_seq_length = config.block_size
        self.register_buffer("cos", torch.empty(0), persistent=False)
        self.register_buffer("sin", torch.empty(0), persistent=False)
        self.mask_cache: Optional[torch.Tensor] = None
        self._rope_seq = 0

    def set_rope_cache(self, seq_len: int, device=None) -> None:
        cos, sin = build_rope_cache(seq_len, self.config.rope_n_elem, device=device, base=self.config.rope_base,
                                    condense_ratio=self.config.rope_condense_ratio)
        self.cos = cos
        self.sin = sin
        self._rope_seq = seq_len

    def set_kv_cache(self, batch_size: int, max_seq_length: Optional[int] = None, device=None,
                     dtype: Optional[torch.dtype] = None) -> None:
        """Allocates a static KV cache in every block and the causal mask for incremental decoding."""
        c = self.config
        max_seq_length = max_seq_length or c.block_size
        dtype = dtype or self.lm_head.weight.dtype
        device = device or self.lm_head.weight.device
        for block in self.transformer.h:
            # sized from the attention module's own config: under head-parallel TP it holds only
            # this rank's kv groups (distributed/tensor_parallel swaps in a localized config)
            ac = getattr(block.attn, "config", c)
            shape = (batch_size, ac.n_query_groups, max_seq_length, ac.head_size)
            block.attn.kv_cache = KVCache(shape, shape, device=device, dtype=dtype)
        if self.cos.numel() == 0 or self.cos.shape[0] < max_seq_length:
            self.set_rope_cache(max_seq_length, device=device)
        ones = torch.ones((max_seq_length, max_seq_length), device=device, dtype=torch.bool)
        self.mask_cache = torch.tril(ones).unsqueeze(0).unsqueeze(0)
        self.max_seq_length = max_seq_length

    def clear_kv_cache(self) -> None:
        for block in self.transformer.h:
            block.attn.kv_cache = None
        self.mask_cache = None

    def forward(self, idx: torch.Tensor, input_pos: Optional[torch.Tensor] = None) -> torch.Tensor:
        T = idx.size(1)
        if self.cos.numel() == 0 or self.cos.shape[0] < T:
            raise RuntimeError("call model.set_rope_cache(seq_len, device) before forward")
        if input_pos is not None:  # incremental decoding against the KV cache
            cos = self.cos.index_select(0, input_pos)
            sin = self.sin.index_select(0, input_pos)
            mask = self.mask_cache.index_select(2, input_pos)
        else:
            cos = self.cos[:T]
            sin = self.sin[:T]
            mask = None
        x = self.transformer.wte(idx)
        if self.config.scale_embeddings:
            x = x * math.sqrt(self.config.n_embd)
        for block in self.transformer.h:
            if self.activation_checkpointing and input_pos is None:
                # recompute the block's intermediates in the backward (LitGPT / benchmark_litgpt
                # ``--checkpoint_activations``); traced as ltorch.checkpoint
                x = torch.utils.checkpoint.checkpoint(block, x, cos, sin, mask, None, use_reentrant=False)
            else:
                x = block(x, cos, sin, mask, input_pos)
        x = self.transformer.ln_f(x)
        return self.lm_head(x)

    @classmethod
    def from_name(cls, name: str, **kwargs) -> "GPT":
        return cls(Config.from_name(name, **kwargs))


def init_weights(model: GPT, std: float = 0.02) -> None:
    """Random init (synthetic benchmark weights; no checkpoints are available offline).

    Every parameter and buffer is initialised — a model materialised with ``to_empty`` holds
    uninitialised memory otherwise: Linear/Embedding weights N(0, std), biases zero, and every other
    module with a ``reset_parameters`` (RMSNorm/LayerNorm weights to one, KV caches to zero, MoE
    routers) through it."""
    for m in model.modules():
        if isinstance(m, nn.Linear):
            nn.init.normal_(m.weight, mean=0.0, std=std)
            if m.bias is not None:
                nn.init.zeros_(m.bias)
        elif isinstance(m, nn.Embedding):
            nn.init.normal_(m.weight, mean=0.0, std=std)
        elif isinstance(m, nn.LayerNorm):
            if m.weight is not None:
                nn.init.ones_(m.weight)
            if m.bias is not None:
                nn.init.zeros_(m.bias)
        elif hasattr(m, "reset_parameters"):
            m.reset_parameters()


def flops_per_token(config: Config, seq_len: int, training: bool = True) -> float:
    """Model FLOPs per token (matmuls + attention), as used for MFU/TFLOP/s reporting."""
    c = config
    n_params_linear = c.n_layer * (c.n_embd * c.qkv_size + c.n_head * c.head_size * c.n_embd
                                   + 3 * c.n_embd * c.intermediate_size) + c.n_embd * c.padded_vocab_size
    attn = c.n_layer * 2 * 2 * seq_len * c.n_head * c.head_size / 2  # causal: half of QK^T and PV
    fwd = 2 * n_params_linear + attn
    return fwd * (3 if training else 1)


@torch.no_grad()
def generate(model, prompt: torch.Tensor, max_new_tokens: int, *, forward=None, temperature: float = 0.0,
             top_k: Optional[int] = None, eos_id: Optional[int] = None) -> torch.Tensor:
    """Autoregressive generation with the static KV cache (LitGPT ``generate``).

    ``forward`` is the callable used for every step (default: ``model``; pass ``thunder.jit(model)``).
    Prefill runs the prompt with ``input_pos = arange(T)``; every decode step feeds one token with
    the *same* ``input_pos`` tensor advanced in place, so a compiled decode step keeps its input
    addresses (hipGraph-replayable) and is a cache hit after the first token.
    Greedy when ``temperature == 0``.  Returns ``[B, T + max_new_tokens]`` token ids.
    """
    from ..ops.sampling import argmax_last

    forward = forward or model
    B, T = prompt.shape
    if model.transformer.h[0].attn.kv_cache is None:
        raise RuntimeError("call model.set_kv_cache(batch_size, max_seq_length) first")
    device = prompt.device
    input_pos = torch.arange(T, device=device)
    logits = forward(prompt, input_pos)
    out = [prompt]
    pos = torch.tensor([T], device=device, dtype=torch.int64)
    for i in range(max_new_tokens):
        last = logits[:, -1]
        if temperature > 0:
            last = last / temperature
            if top_k is not None:
                v, _ = torch.topk(last, min(top_k, last.size(-1)))
                last = torch.where(last < v[:, [-1]], torch.full_like(last, -float("inf")), last)
            nxt = torch.multinomial(torch.softmax(last.float(), -1), 1)
        else:
            nxt = argmax_last(last, keepdim=True)
        out.append(nxt)
        if eos_id is not None and bool((nxt == eos_id).all()):
            break
        if i + 1 < max_new_tokens:
            logits = forward(nxt, pos)
            pos.add_(1)
    return torch.cat(out, dim=1)
