"""GPT-2 (nanoGPT-compatible) golden model and pipeline stage modules.

The reference's GPT path (``partitions/gpt_model_parts.py:6-50``) imports the
absent nanoGPT ``model.py`` and is never wired into ``node.py``; this module
provides the model itself with **nanoGPT state-dict keys** so nanoGPT ``.pth``
files load:

    transformer.wte.weight (V,d)     transformer.wpe.weight (block_size,d)
    transformer.h.{i}.ln_1.{weight,bias}
    transformer.h.{i}.attn.c_attn.{weight (3d,d), bias}
    transformer.h.{i}.attn.c_proj.{weight (d,d), bias}
    transformer.h.{i}.ln_2.{weight,bias}
    transformer.h.{i}.mlp.c_fc.{weight (4d,d), bias}
    transformer.h.{i}.mlp.c_proj.{weight (d,4d), bias}
    transformer.ln_f.{weight,bias}   lm_head.weight (tied to wte)

Stage semantics mirror the reference part classes:

* first stage (``ModelPart0``, ``gpt_model_parts.py:6-22``): ``wte(idx)+wpe(arange(T))``
  then blocks ``[start..end]`` inclusive, asserting ``T <= block_size``;
* middle stage (``ModelPartIntermediate``, ``:26-34``): blocks only;
* last stage (``ModelPartFinal_GPT``, ``:36-50``): blocks, ``ln_f``, ``lm_head``.
  ``last_only=True`` restricts the head to the final position (decode/serving);
  the default computes logits for all T like the reference.

This is the fp32/bf16 torch oracle; the MI355X path is ``runtime/transformer.py``.
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Dict, List, Optional, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F


@dataclass(frozen=True)
class GPTConfig:
    block_size: int = 1024
    vocab_size: int = 50257
    n_layer: int = 12
    n_head: int = 12
    n_embd: int = 768
    bias: bool = True

    @property
    def head_dim(self) -> int:
        return self.n_embd // self.n_head

    def params_per_block(self) -> int:
        d = self.n_embd
        return 12 * d * d + 13 * d


GPT_CONFIGS: Dict[str, GPTConfig] = {
    "gpt2": GPTConfig(n_layer=12, n_head=12, n_embd=768),
    "gpt2-medium": GPTConfig(n_layer=24, n_head=16, n_embd=1024),
    "gpt2-large": GPTConfig(n_layer=36, n_head=20, n_embd=1280),
    "gpt2-xl": GPTConfig(n_layer=48, n_head=25, n_embd=1600),
    # small config for CPU tests / smoke (same code paths, head_dim 64)
    "gpt2-tiny": GPTConfig(block_size=256, vocab_size=512, n_layer=4, n_head=4, n_embd=256),
}


class CausalSelfAttention(nn.Module):
    def __init__(self, cfg: GPTConfig):
        super().__init__()
        self.n_head = cfg.n_head
        self.c_attn = nn.Linear(cfg.n_embd, 3 * cfg.n_embd, bias=cfg.bias)
        self.c_proj = nn.Linear(cfg.n_embd, cfg.n_embd, bias=cfg.bias)

    def forward(self, x: torch.Tensor, kv: Optional[Tuple[torch.Tensor, torch.Tensor]] = None,
                pos: int = 0):
        B, T, C = x.shape
        q, k, v = self.c_attn(x).split(C, dim=2)
        hd = C // self.n_head
        q = q.view(B, T, self.n_head, hd).transpose(1, 2)
        k = k.view(B, T, self.n_head, hd).transpose(1, 2)
        v = v.view(B, T, self.n_head, hd).transpose(1, 2)
        if kv is not None:
            kc, vc = kv
            kc[:, :, pos:pos + T] = k
            vc[:, :, pos:pos + T] = v
            k, v = kc[:, :, :pos + T], vc[:, :, :pos + T]
        if kv is None or pos == 0:
            y = F.scaled_dot_product_attention(q, k, v, is_causal=True)
        else:
            # queries at absolute positions pos..pos+T-1 see keys 0..pos+t
            S = pos + T
            mask = torch.ones(T, S, dtype=torch.bool, device=x.device).tril(diagonal=pos)
            y = F.scaled_dot_product_attention(q, k, v, attn_mask=mask)
        y = y.transpose(1, 2).contiguous().view(B, T, C)
        return self.c_proj(y)


class MLP(nn.Module):
    def __init__(self, cfg: GPTConfig):
        super().__init__()
        self.c_fc = nn.Linear(cfg.n_embd, 4 * cfg.n_embd, bias=cfg.bias)
        self.c_proj = nn.Linear(4 * cfg.n_embd, cfg.n_embd, bias=cfg.bias)

    def forward(self, x):
        return self.c_proj(F.gelu(self.c_fc(x)))  # exact erf GELU, as nanoGPT


class Block(nn.Module):
    def __init__(self, cfg: GPTConfig):
        super().__init__()
        self.ln_1 = nn.LayerNorm(cfg.n_embd, bias=cfg.bias)
        self.attn = CausalSelfAttention(cfg)
        self.ln_2 = nn.LayerNorm(cfg.n_embd, bias=cfg.bias)
        self.mlp = MLP(cfg)

    def forward(self, x, kv=None, pos: int = 0):
        x = x + self.attn(self.ln_1(x), kv, pos)
        return x + self.mlp(self.ln_2(x))


class GPT(nn.Module):
    """Full model with nanoGPT key layout (``transformer.*`` + tied ``lm_head``)."""

    def __init__(self, cfg: GPTConfig):
        super().__init__()
        self.config = cfg
        self.transformer = nn.ModuleDict(dict(
            wte=nn.Embedding(cfg.vocab_size, cfg.n_embd),
            wpe=nn.Embedding(cfg.block_size, cfg.n_embd),
            h=nn.ModuleList([Block(cfg) for _ in range(cfg.n_layer)]),
            ln_f=nn.LayerNorm(cfg.n_embd, bias=cfg.bias),
        ))
        self.lm_head = nn.Linear(cfg.n_embd, cfg.vocab_size, bias=False)
        self.lm_head.weight = self.transformer.wte.weight
        self.apply(_init_weights)
        for n, p in self.named_parameters():
            if n.endswith("c_proj.weight"):
                nn.init.normal_(p, 0.0, 0.02 / math.sqrt(2 * cfg.n_layer))

    def forward(self, idx: torch.Tensor) -> torch.Tensor:
        B, T = idx.shape
        assert T <= self.config.block_size, "Cannot forward, model block size is exhausted."
        pos = torch.arange(T, device=idx.device)
        x = self.transformer.wte(idx) + self.transformer.wpe(pos)
        for blk in self.transformer.h:
            x = blk(x)
        return self.lm_head(self.transformer.ln_f(x))


def _init_weights(m):
    if isinstance(m, nn.Linear):
        nn.init.normal_(m.weight, 0.0, 0.02)
        if m.bias is not None:
            nn.init.zeros_(m.bias)
    elif isinstance(m, nn.Embedding):
        nn.init.normal_(m.weight, 0.0, 0.02)


class GPTStage(nn.Module):
    """Blocks ``[start, end]`` (inclusive) plus embeddings on the first stage and
    ``ln_f``/``lm_head`` on the last.  Stage-local parameter names:
    ``wte, wpe, h.{j}.*, ln_f, lm_head``; ``checkpoint.gpt_stage_state`` maps the
    nanoGPT keys onto them (``transformer.h.{start+j}.* -> h.{j}.*``)."""

    def __init__(self, cfg: GPTConfig, start: int, end: int, first: bool, last: bool):
        super().__init__()
        self.config, self.start, self.end, self.first, self.last = cfg, start, end, first, last
        if first:
            self.wte = nn.Embedding(cfg.vocab_size, cfg.n_embd)
            self.wpe = nn.Embedding(cfg.block_size, cfg.n_embd)
        self.h = nn.ModuleList([Block(cfg) for _ in range(start, end + 1)])
        if last:
            self.ln_f = nn.LayerNorm(cfg.n_embd, bias=cfg.bias)
            self.lm_head = nn.Linear(cfg.n_embd, cfg.vocab_size, bias=False)

    def forward(self, x: torch.Tensor, kv: Optional[List] = None, pos: int = 0,
                last_only: bool = False) -> torch.Tensor:
        if self.first:
            B, T = x.shape
            assert pos + T <= self.config.block_size, "Cannot forward, model block size is exhausted."
            p = torch.arange(pos, pos + T, device=x.device)
            x = self.wte(x) + self.wpe(p)
        for j, blk in enumerate(self.h):
            x = blk(x, None if kv is None else kv[j], pos)
        if self.last:
            if last_only:
                x = x[:, -1:, :]
            x = self.lm_head(self.ln_f(x))
        return x


def stage_key_map(cfg: GPTConfig, start: int, end: int, first: bool, last: bool) -> Dict[str, str]:
    """stage-local key -> nanoGPT full-model key."""
    m: Dict[str, str] = {}
    if first:
        m["wte.weight"] = "transformer.wte.weight"
        m["wpe.weight"] = "transformer.wpe.weight"
    sub = ["ln_1.weight", "ln_1.bias", "attn.c_attn.weight", "attn.c_attn.bias", "attn.c_proj.weight",
           "attn.c_proj.bias", "ln_2.weight", "ln_2.bias", "mlp.c_fc.weight", "mlp.c_fc.bias",
           "mlp.c_proj.weight", "mlp.c_proj.bias"]
    if not cfg.bias:
        sub = [s for s in sub if not s.endswith("bias")]
    for j, i in enumerate(range(start, end + 1)):
        for s in sub:
            m[f"h.{j}.{s}"] = f"transformer.h.{i}.{s}"
    if last:
        m["ln_f.weight"] = "transformer.ln_f.weight"
        if cfg.bias:
            m["ln_f.bias"] = "transformer.ln_f.bias"
        m["lm_head.weight"] = "lm_head.weight"
    return m


def flops_per_token(cfg: GPTConfig, n_layers: int, ctx: int, lm_head: bool = True) -> float:
    """Forward FLOPs per token: 2*params for the dense part + attention scores/values."""
    d = cfg.n_embd
    dense = 2 * n_layers * 12 * d * d
    attn = 2 * n_layers * 2 * ctx * d
    head = 2 * d * cfg.vocab_size if lm_head else 0
    return float(dense + attn + head)
