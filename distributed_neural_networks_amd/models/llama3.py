"""Llama-3 golden model and stage modules (north-star config 4; not in the reference).

RMSNorm, RoPE (theta 500000, rotate-half convention as HF), grouped-query
attention (32 q / 8 kv heads of 128 for 8B), SwiGLU MLP, untied ``lm_head``.
State-dict keys follow the Hugging Face layout so safetensors shards load:

    model.embed_tokens.weight
    model.layers.{i}.input_layernorm.weight
    model.layers.{i}.self_attn.{q,k,v,o}_proj.weight
    model.layers.{i}.post_attention_layernorm.weight
    model.layers.{i}.mlp.{gate,up,down}_proj.weight
    model.norm.weight   lm_head.weight

Stage split mirrors the GPT stages (``partitions/gpt_model_parts.py``): the
first stage owns the embedding, the last owns ``norm`` + ``lm_head``.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, List, Optional, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F


@dataclass(frozen=True)
class LlamaConfig:
    vocab_size: int = 128256
    n_layer: int = 32
    n_head: int = 32
    n_kv_head: int = 8
    n_embd: int = 4096
    ffn_dim: int = 14336
    rope_theta: float = 500000.0
    norm_eps: float = 1e-5
    max_seq: int = 8192

    @property
    def head_dim(self) -> int:
        return self.n_embd // self.n_head


LLAMA_CONFIGS: Dict[str, LlamaConfig] = {
    "llama3-8b": LlamaConfig(),
    "llama3-tiny": LlamaConfig(vocab_size=512, n_layer=4, n_head=4, n_kv_head=2, n_embd=512,
                               ffn_dim=1024, max_seq=512),
}


class RMSNorm(nn.Module):
    def __init__(self, d: int, eps: float):
        super().__init__()
        self.eps = eps
        self.weight = nn.Parameter(torch.ones(d))

    def forward(self, x):
        xf = x.float()
        y = xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + self.eps)
        return (y * self.weight.float()).to(x.dtype)


def rope_tables(cfg: LlamaConfig, seq: int, device=None) -> Tuple[torch.Tensor, torch.Tensor]:
    hd = cfg.head_dim
    inv = 1.0 / (cfg.rope_theta ** (torch.arange(0, hd, 2, dtype=torch.float64) / hd))
    t = torch.arange(seq, dtype=torch.float64)
    f = torch.outer(t, inv)  # (seq, hd/2)
    return f.cos().float().to(device), f.sin().float().to(device)


def apply_rope(x: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor) -> torch.Tensor:
    """x: (B, H, T, hd); cos/sin: (T, hd/2). Rotate-half convention."""
    h = x.shape[-1] // 2
    x1, x2 = x[..., :h].float(), x[..., h:].float()
    c, s = cos[None, None], sin[None, None]
    return torch.cat([x1 * c - x2 * s, x2 * c + x1 * s], dim=-1).to(x.dtype)


class Attention(nn.Module):
    def __init__(self, cfg: LlamaConfig):
        super().__init__()
        self.cfg = cfg
        hd = cfg.head_dim
        self.q_proj = nn.Linear(cfg.n_embd, cfg.n_head * hd, bias=False)
        self.k_proj = nn.Linear(cfg.n_embd, cfg.n_kv_head * hd, bias=False)
        self.v_proj = nn.Linear(cfg.n_embd, cfg.n_kv_head * hd, bias=False)
        self.o_proj = nn.Linear(cfg.n_head * hd, cfg.n_embd, bias=False)

    def forward(self, x, cos, sin, kv=None, pos: int = 0):
        B, T, _ = x.shape
        c = self.cfg
        hd = c.head_dim
        q = self.q_proj(x).view(B, T, c.n_head, hd).transpose(1, 2)
        k = self.k_proj(x).view(B, T, c.n_kv_head, hd).transpose(1, 2)
        v = self.v_proj(x).view(B, T, c.n_kv_head, hd).transpose(1, 2)
        q = apply_rope(q, cos[pos:pos + T], sin[pos:pos + T])
        k = apply_rope(k, cos[pos:pos + T], sin[pos:pos + T])
        if kv is not None:
            kc, vc = kv
            kc[:, :, pos:pos + T] = k
            vc[:, :, pos:pos + T] = v
            k, v = kc[:, :, :pos + T], vc[:, :, :pos + T]
        rep = c.n_head // c.n_kv_head
        k = k.repeat_interleave(rep, dim=1)
        v = v.repeat_interleave(rep, dim=1)
        S = k.shape[2]
        mask = torch.ones(T, S, dtype=torch.bool, device=x.device).tril(diagonal=S - T)
        y = F.scaled_dot_product_attention(q, k, v, attn_mask=mask)
        return self.o_proj(y.transpose(1, 2).reshape(B, T, c.n_head * hd))


class FeedForward(nn.Module):
    def __init__(self, cfg: LlamaConfig):
        super().__init__()
        self.gate_proj = nn.Linear(cfg.n_embd, cfg.ffn_dim, bias=False)
        self.up_proj = nn.Linear(cfg.n_embd, cfg.ffn_dim, bias=False)
        self.down_proj = nn.Linear(cfg.ffn_dim, cfg.n_embd, bias=False)

    def forward(self, x):
        return self.down_proj(F.silu(self.gate_proj(x)) * self.up_proj(x))


class DecoderLayer(nn.Module):
    def __init__(self, cfg: LlamaConfig):
        super().__init__()
        self.input_layernorm = RMSNorm(cfg.n_embd, cfg.norm_eps)
        self.self_attn = Attention(cfg)
        self.post_attention_layernorm = RMSNorm(cfg.n_embd, cfg.norm_eps)
        self.mlp = FeedForward(cfg)

    def forward(self, x, cos, sin, kv=None, pos: int = 0):
        x = x + self.self_attn(self.input_layernorm(x), cos, sin, kv, pos)
        return x + self.mlp(self.post_attention_layernorm(x))


class LlamaStage(nn.Module):
    """Layers ``[start, end]`` inclusive; embedding on the first stage, norm+head on the last."""

    def __init__(self, cfg: LlamaConfig, start: int, end: int, first: bool, last: bool):
        super().__init__()
        self.config, self.start, self.end, self.first, self.last = cfg, start, end, first, last
        if first:
            self.embed_tokens = nn.Embedding(cfg.vocab_size, cfg.n_embd)
        self.layers = nn.ModuleList([DecoderLayer(cfg) for _ in range(start, end + 1)])
        if last:
            self.norm = RMSNorm(cfg.n_embd, cfg.norm_eps)
            self.lm_head = nn.Linear(cfg.n_embd, cfg.vocab_size, bias=False)
        self._rope = None

    def rope(self, seq: int, device):
        if self._rope is None or self._rope[0].shape[0] < seq or self._rope[0].device != torch.device(device):
            self._rope = rope_tables(self.config, max(seq, 16), device)
        return self._rope

    def forward(self, x, kv: Optional[List] = None, pos: int = 0, last_only: bool = False):
        if self.first:
            x = self.embed_tokens(x)
        cos, sin = self.rope(pos + x.shape[1], x.device)
        for j, layer in enumerate(self.layers):
            x = layer(x, cos, sin, None if kv is None else kv[j], pos)
        if self.last:
            if last_only:
                x = x[:, -1:, :]
            x = self.lm_head(self.norm(x))
        return x


def init_random_(stage: nn.Module, std: float = 0.02, seed: int = 0) -> None:
    g = torch.Generator().manual_seed(seed)
    for n, p in stage.named_parameters():
        with torch.no_grad():
            if n.endswith("layernorm.weight") or n.endswith("norm.weight"):
                p.fill_(1.0)
            else:
                p.copy_(torch.randn(p.shape, generator=g) * std)


def stage_key_map(cfg: LlamaConfig, start: int, end: int, first: bool, last: bool) -> Dict[str, str]:
    m: Dict[str, str] = {}
    if first:
        m["embed_tokens.weight"] = "model.embed_tokens.weight"
    sub = ["input_layernorm.weight", "self_attn.q_proj.weight", "self_attn.k_proj.weight",
           "self_attn.v_proj.weight", "self_attn.o_proj.weight", "post_attention_layernorm.weight",
           "mlp.gate_proj.weight", "mlp.up_proj.weight", "mlp.down_proj.weight"]
    for j, i in enumerate(range(start, end + 1)):
        for s in sub:
            m[f"layers.{j}.{s}"] = f"model.layers.{i}.{s}"
    if last:
        m["norm.weight"] = "model.norm.weight"
        m["lm_head.weight"] = "lm_head.weight"
    return m


def flops_per_token(cfg: LlamaConfig, n_layers: int, ctx: int, lm_head: bool = True) -> float:
    d, hd = cfg.n_embd, cfg.head_dim
    qkvo = 2 * d * (cfg.n_head * hd) + 2 * d * (cfg.n_kv_head * hd)
    mlp = 3 * d * cfg.ffn_dim
    attn = 2 * 2 * ctx * cfg.n_head * hd
    head = 2 * d * cfg.vocab_size if lm_head else 0
    return float(n_layers * (2 * (qkvo + mlp) + attn) + head)
