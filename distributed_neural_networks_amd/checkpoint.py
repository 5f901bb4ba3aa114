"""Checkpoint loading: one full-model file, each stage takes its own slice.

Reference behaviour (``node.py:294-325``): every stage ``torch.load``s the full
state dict on CPU, wraps a throw-away full model in its part class and calls
``load_state_dict(full_sd, strict=False)``; missing/unexpected keys are only
printed.  That trick silently loads nothing for GPT stages (their attribute
names do not match ``transformer.h.{i}.*``).  Here:

* ``load_full_state_dict`` accepts a plain ``.pth`` state dict (reference), a
  nanoGPT ``ckpt.pt`` dict (``{"model": sd}``, ``_orig_mod.`` prefixes
  stripped), Hugging Face GPT-2 ``Conv1D`` layouts (transposed to
  ``nn.Linear``), and ``.safetensors`` files/directories (lazy: a stage reads
  only its own tensors).  Loading is always ``weights_only=True``.
* ``stage_state_dict`` remaps full-model keys to stage-local keys (explicit
  ``transformer.h.{start+j} -> h.{j}``), fills the tied ``lm_head`` from ``wte``
  and raises on missing keys instead of hiding them.
* ``"synthetic"`` / ``"random"`` / ``"random:<seed>"`` as ``model_weights``
  means random-init weights of the named architecture (no file), which is what
  the benchmarks use (no network, no real checkpoints).
"""
from __future__ import annotations

import glob
import os
from typing import Dict, Iterable, List, Optional, Tuple

import torch

from .models import cifar, gpt2, llama3, model_info


class CheckpointError(Exception):
    pass


def is_synthetic(path: Optional[str]) -> bool:
    return path is not None and (path in ("synthetic", "random") or path.startswith("random:")
                                 or path.startswith("synthetic:"))


def synthetic_seed(path: str) -> int:
    return int(path.split(":", 1)[1]) if ":" in path else 0


class LazyStateDict:
    """Read-on-demand view over safetensors shards (or an in-memory dict)."""

    def __init__(self, files: List[str]):
        from safetensors import safe_open
        self._index: Dict[str, str] = {}
        for f in files:
            with safe_open(f, framework="pt") as h:
                for k in h.keys():
                    self._index[k] = f
        self._files = files

    def keys(self) -> Iterable[str]:
        return self._index.keys()

    def __contains__(self, k) -> bool:
        return k in self._index

    def __getitem__(self, k: str) -> torch.Tensor:
        from safetensors import safe_open
        with safe_open(self._index[k], framework="pt") as h:
            return h.get_tensor(k)

    def get(self, k, default=None):
        return self[k] if k in self._index else default


def load_full_state_dict(path: str):
    """Full-model state dict from ``path`` (see module doc).  Raises FileNotFoundError."""
    if os.path.isdir(path):
        files = sorted(glob.glob(os.path.join(path, "*.safetensors")))
        if not files:
            raise FileNotFoundError(path)
        return LazyStateDict(files)
    if path.endswith(".safetensors"):
        if not os.path.exists(path):
            raise FileNotFoundError(path)
        return LazyStateDict([path])
    obj = torch.load(path, map_location=torch.device("cpu"), weights_only=True)
    if isinstance(obj, dict) and "model" in obj and isinstance(obj["model"], dict):
        obj = obj["model"]  # nanoGPT training checkpoint
    if not isinstance(obj, dict):
        raise CheckpointError(f"{path} does not contain a state dict (got {type(obj).__name__})")
    sd = {}
    for k, v in obj.items():
        if k.startswith("_orig_mod."):
            k = k[len("_orig_mod."):]
        sd[k] = v
    return sd


def _gpt2_normalise(sd) -> Dict[str, torch.Tensor]:
    """HF GPT2LMHeadModel / GPT2Model -> nanoGPT key + layout conventions."""
    if isinstance(sd, LazyStateDict):
        sd = {k: sd[k] for k in sd.keys()}
    out = {}
    for k, v in sd.items():
        if k.endswith(".attn.bias") or k.endswith(".attn.masked_bias"):
            continue  # causal-mask buffers
        if k.startswith("h.") or k in ("wte.weight", "wpe.weight", "ln_f.weight", "ln_f.bias"):
            k = "transformer." + k
        out[k] = v
    w = out.get("transformer.h.0.attn.c_attn.weight")
    if w is not None and w.shape[0] * 3 == w.shape[1]:  # Conv1D: (in, out)
        for k in list(out):
            if any(k.endswith(s) for s in ("attn.c_attn.weight", "attn.c_proj.weight",
                                           "mlp.c_fc.weight", "mlp.c_proj.weight")):
                out[k] = out[k].t().contiguous()
    if "lm_head.weight" not in out and "transformer.wte.weight" in out:
        out["lm_head.weight"] = out["transformer.wte.weight"]  # weight tying
    return out


def stage_state_dict(model: str, full_sd, start: int, end: int, first: bool,
                     last: bool) -> Dict[str, torch.Tensor]:
    """Stage-local state dict; raises CheckpointError listing any missing keys."""
    info = model_info(model)
    if info.family == "cifar":
        stage = cifar.CifarStage(start, end)
        want = {k: k for k in stage.state_dict().keys()}
    elif info.family == "gpt2":
        full_sd = _gpt2_normalise(full_sd)
        want = gpt2.stage_key_map(info.cfg, start, end, first, last)
    else:
        want = llama3.stage_key_map(info.cfg, start, end, first, last)
        if last and "lm_head.weight" not in full_sd and "model.embed_tokens.weight" in full_sd:
            want["lm_head.weight"] = "model.embed_tokens.weight"  # tied-embedding variants
    missing = [f for f in want.values() if f not in full_sd]
    if missing:
        raise CheckpointError(f"missing keys for stage layers [{start},{end}]: {missing[:8]}"
                              + (f" (+{len(missing) - 8} more)" if len(missing) > 8 else ""))
    return {local: full_sd[full] for local, full in want.items()}


def unexpected_keys(model: str, full_sd, start: int, end: int, first: bool, last: bool) -> List[str]:
    """Keys of the full checkpoint this stage does not use (the reference prints these)."""
    info = model_info(model)
    if info.family == "cifar":
        mine = set(cifar.CifarStage(start, end).state_dict().keys())
    elif info.family == "gpt2":
        full_sd = _gpt2_normalise(full_sd)
        mine = set(gpt2.stage_key_map(info.cfg, start, end, first, last).values())
    else:
        mine = set(llama3.stage_key_map(info.cfg, start, end, first, last).values())
    return [k for k in full_sd.keys() if k not in mine]


def random_stage_state_dict(model: str, start: int, end: int, first: bool, last: bool,
                            seed: int = 0, device=None, nontrivial: bool = False) -> Dict[str, torch.Tensor]:
    """Random-init weights for one stage, identical to slicing a random full model
    generated with the same seed (layer-indexed seeding).  ``device`` generates
    directly on that device (billion-parameter stages without a host copy);
    values then follow the device RNG, so compare only within one device.

    The default follows nanoGPT's init (zero biases, unit norm gains).
    ``nontrivial=True`` (tests) draws biases ~ N(0, 0.02^2) and norm gains
    ~ 1 + N(0, 0.1^2) so folded-norm / bias epilogues are actually exercised."""
    info = model_info(model)
    if info.family == "cifar":
        return {k: v for k, v in cifar.random_state_dict(seed).items()
                if k.split(".")[0] in {n for u in range(start, end + 1) for n in cifar.UNIT_KEYS[u]}}
    dev = torch.device(device) if device is not None else torch.device("cpu")
    shapes = _stage_shapes(model, start, end, first, last)
    sd = {}
    for local, shape in shapes.items():
        g = torch.Generator(device=dev).manual_seed(_key_seed(seed, _global_key(model, local, start)))
        if local.endswith("bias"):
            sd[local] = (torch.randn(shape, generator=g, device=dev) * 0.02 if nontrivial
                         else torch.zeros(shape, device=dev))
        elif "ln" in local.split(".")[-2] or local.endswith("norm.weight") or "layernorm" in local:
            sd[local] = (1.0 + 0.1 * torch.randn(shape, generator=g, device=dev) if nontrivial
                         else torch.ones(shape, device=dev))
        else:
            sd[local] = torch.randn(shape, generator=g, device=dev) * 0.02
    if info.family == "gpt2" and last and first:
        sd["lm_head.weight"] = sd["wte.weight"]
    elif info.family == "gpt2" and last:
        g = torch.Generator(device=dev).manual_seed(_key_seed(seed, "transformer.wte.weight"))
        sd["lm_head.weight"] = torch.randn(sd["lm_head.weight"].shape, generator=g, device=dev) * 0.02
    return sd


def _stage_shapes(model: str, start: int, end: int, first: bool, last: bool) -> Dict[str, Tuple[int, ...]]:
    """Parameter shapes of a stage without materialising it (meta device)."""
    from .models import build_golden_stage
    with torch.device("meta"):
        stage = build_golden_stage(model, start, end, first, last)
    return {k: tuple(v.shape) for k, v in stage.state_dict().items()}


def _global_key(model: str, local: str, start: int) -> str:
    parts = local.split(".")
    if parts[0] in ("h", "layers") and len(parts) > 1 and parts[1].isdigit():
        parts[1] = str(start + int(parts[1]))
    key = ".".join(parts)
    if model_info(model).family == "gpt2" and key == "lm_head.weight":
        return "transformer.wte.weight"
    if model_info(model).family == "gpt2" and key == "wte.weight":
        return "transformer.wte.weight"
    return key


def _key_seed(seed: int, key: str) -> int:
    h = 1469598103934665603
    for ch in key.encode():
        h = ((h ^ ch) * 1099511628211) & 0xFFFFFFFFFFFF
    return (h + seed * 7919) & 0x7FFFFFFF


def make_full_checkpoint(model: str, path: str, seed: int = 0) -> None:
    """Write a random-init full-model ``.pth`` with the reference/nanoGPT key layout."""
    info = model_info(model)
    if info.family == "cifar":
        sd = cifar.random_state_dict(seed)
    else:
        n = info.num_layers
        st = random_stage_state_dict(model, 0, n - 1, True, True, seed)
        if info.family == "gpt2":
            km = gpt2.stage_key_map(info.cfg, 0, n - 1, True, True)
        else:
            km = llama3.stage_key_map(info.cfg, 0, n - 1, True, True)
        sd = {km[k]: v for k, v in st.items()}
    torch.save(sd, path)
