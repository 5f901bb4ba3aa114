"""Model registry: model name -> golden torch stage modules and layer counts."""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Tuple

from . import cifar, gpt2, llama3


@dataclass(frozen=True)
class ModelInfo:
    name: str
    family: str           # "cifar" | "gpt2" | "llama3"
    num_layers: int       # layer units that can be split across stages
    cfg: object = None


def model_info(name: str) -> ModelInfo:
    if name == "cifar10":
        return ModelInfo(name, "cifar", cifar.NUM_UNITS)
    if name in gpt2.GPT_CONFIGS:
        c = gpt2.GPT_CONFIGS[name]
        return ModelInfo(name, "gpt2", c.n_layer, c)
    if name in llama3.LLAMA_CONFIGS:
        c = llama3.LLAMA_CONFIGS[name]
        return ModelInfo(name, "llama3", c.n_layer, c)
    raise KeyError(f"unknown model {name!r}")


def default_ranges(name: str, num_stages: int) -> List[Tuple[int, int]]:
    from ..parallel.partition import balanced_ranges
    info = model_info(name)
    if info.family == "cifar":
        return cifar.stage_ranges(num_stages)
    if info.family == "gpt2":
        # lm_head on the last stage ~ 2*d*V FLOPs/token vs 24*d^2 per block
        c = info.cfg
        head = (2 * c.n_embd * c.vocab_size) / (24 * c.n_embd * c.n_embd)
        return balanced_ranges(info.num_layers, num_stages, 0.0, min(head, 2.0))
    c = info.cfg
    head = (2 * c.n_embd * c.vocab_size) / (2 * (2 * c.n_embd * c.n_embd * 2 + 3 * c.n_embd * c.ffn_dim))
    return balanced_ranges(info.num_layers, num_stages, 0.0, min(head, 2.0))


def build_golden_stage(name: str, start: int, end: int, first: bool, last: bool):
    info = model_info(name)
    if info.family == "cifar":
        return cifar.CifarStage(start, end)
    if info.family == "gpt2":
        return gpt2.GPTStage(info.cfg, start, end, first, last)
    return llama3.LlamaStage(info.cfg, start, end, first, last)
