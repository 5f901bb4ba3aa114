"""Token sampling: greedy, or temperature + top-k by the Gumbel-max trick.

The device kernel is ``sample_topk`` (csrc/kernels/sampler.hip); this module is
its bit-compatible torch mirror for the CPU/gloo golden path and the tests:

    token = argmax_{i : key(x_i) >= key(k-th largest)} ( x_i / T + G_i ),
    G_i = -log(-log(U_i)),  U_i = hash(seed, row, step[row], i)

The counter-based hash needs no RNG state (one captured HIP graph serves every
decode step; runs are reproducible from ``seed``).  The reference has no
sampler at all: ``np.argmax`` on the host (``node.py:61,190``).
"""
from __future__ import annotations

from typing import Optional

import torch

_M32 = 0xFFFFFFFF


def _mix32(x: torch.Tensor) -> torch.Tensor:
    x = x & _M32
    x = x ^ (x >> 16)
    x = (x * 0x7feb352d) & _M32
    x = x ^ (x >> 15)
    x = (x * 0x846ca68b) & _M32
    return x ^ (x >> 16)


def _keys(x_bf16: torch.Tensor) -> torch.Tensor:
    u = x_bf16.contiguous().view(torch.int16).to(torch.int64) & 0xFFFF
    return torch.where((u & 0x8000) != 0, (~u) & 0xFFFF, u | 0x8000)


def sample_topk_ref(logits: torch.Tensor, temperature: float, top_k: int = 0, seed: int = 0,
                    step: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Torch mirror of the device sampler; ``logits`` (M, N) (rounded to bf16)."""
    x = logits.to(torch.bfloat16).cpu()
    M, N = x.shape
    keys = _keys(x)
    if 0 < top_k < N:
        thr = keys.sort(dim=1, descending=True).values[:, top_k - 1:top_k]
    else:
        thr = torch.zeros((M, 1), dtype=torch.int64)
    st = (step.cpu().to(torch.int64) if step is not None else torch.zeros(M, dtype=torch.int64)) & _M32
    rows = torch.arange(M, dtype=torch.int64)
    inner = _mix32(st + 0x632BE5AB)
    base = _mix32((seed & _M32) ^ _mix32(((rows * 0x9E3779B9) & _M32) ^ inner))
    idx = torch.arange(N, dtype=torch.int64)
    h = _mix32(base[:, None] ^ ((idx[None, :] * 0x85EBCA6B) & _M32))
    u = ((h >> 8).to(torch.float32) + 0.5) * (1.0 / 16777216.0)
    inv_t = torch.tensor(1.0, dtype=torch.float32) / torch.tensor(temperature, dtype=torch.float32)
    score = x.float() * inv_t - torch.log(-torch.log(u))
    score = torch.where(keys >= thr, score, torch.full_like(score, float("-inf")))
    return score.argmax(dim=1).to(torch.int32)


def pick(logits: torch.Tensor, temperature: float = 0.0, top_k: int = 0, seed: int = 0,
         step: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Greedy when temperature <= 0, else the Gumbel top-k sample (CPU path)."""
    if temperature <= 0:
        return logits.argmax(dim=-1).to(torch.int32)
    return sample_topk_ref(logits, temperature, top_k, seed, step)
