"""What fp8 weights cost at the model level.

The fp8 kernel tests pin the GPT-2 XL fp8 stage against an fp32 golden on its
own *dequantised* e4m3 weights: kernel fidelity.  This harness instead runs
the device stage against the fp32 torch golden (``models/gpt2.py`` nanoGPT
``Block``, the reference's ``partitions/gpt_model_parts.py:17-21,44-50``) on
the *original, unquantised* weights, so the numbers include the e4m3 weight
rounding itself:

* logits relative error (Frobenius) of the prefill and of every decode step;
* greedy-token agreement: per step, the fraction of rows whose device argmax
  equals the golden's argmax on the same prefix.  The device's own tokens are
  fed to both sides (teacher forcing), so one early disagreement does not
  cascade into every later step.

Variants share one golden (built once): fp8 weights with the ``split``
prefill (e4m3 hi + residual activations) or the ``e4m3`` prefill (one byte
per activation), and bf16 weights as the comparator.

    python -m distributed_neural_networks_amd.tools.fp8_fidelity --layers 48 --batch 64 --prompt 512
"""
from __future__ import annotations

import argparse
import json
from typing import Dict, Sequence

import torch


def _rel(a: torch.Tensor, b: torch.Tensor) -> float:
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


@torch.no_grad()
def measure(model: str = "gpt2-xl", layers: int = 2, B: int = 64, T: int = 512, steps: int = 8,
            variants: Sequence[str] = ("fp8-split", "fp8-e4m3", "bf16"), device=None, seed: int = 17,
            nontrivial: bool = True) -> Dict[str, dict]:
    """One device stage of ``layers`` blocks + embeddings + ln_f + head per
    variant, against the fp32 golden on the same unquantised weights.
    Returns {variant: {prefill_logits_rel, decode_logits_rel_max,
    decode_logits_rel_mean, prefill_greedy_agreement, decode_greedy_agreement}}."""
    from .. import checkpoint as ckpt
    from ..models import build_golden_stage, model_info
    from ..runtime.transformer import TransformerStage
    dev = torch.device(device or "cuda")
    cfg = model_info(model).cfg
    S = T + steps + 1
    sd = ckpt.random_stage_state_dict(model, 0, layers - 1, True, True, seed, device=dev, nontrivial=nontrivial)
    with torch.device(dev):  # parameter init on the device (1.5 B of them for the whole XL)
        gold = build_golden_stage(model, 0, layers - 1, True, True)
    gold.load_state_dict({k: v.float() for k, v in sd.items()})
    gold = gold.float().eval()
    H = cfg.n_head
    hd = cfg.n_embd // H
    kv = [(torch.zeros(B, H, S, hd, device=dev), torch.zeros(B, H, S, hd, device=dev)) for _ in range(layers)]
    ids = torch.randint(0, cfg.vocab_size, (B, T), generator=torch.Generator().manual_seed(seed + 1)).to(dev)
    tf32 = torch.backends.cuda.matmul.allow_tf32
    torch.backends.cuda.matmul.allow_tf32 = False
    out: Dict[str, dict] = {}
    try:
        for var in variants:
            fp8 = var.startswith("fp8")
            st = TransformerStage(model, sd, 0, layers - 1, True, True, dev, max_batch=B, max_seq=S, fp8=fp8,
                                  fp8_prefill=var.split("-", 1)[1] if fp8 else "split")
            pos = torch.zeros(B, dtype=torch.int32, device=dev)
            x, Tn, p = ids, T, 0
            rels, agree = [], []
            for _ in range(steps + 1):
                o = st.step(x.to(torch.int32).contiguous(), pos, B, Tn)
                pos.add_(Tn)
                ref = gold(x.long(), kv, p, last_only=True)[:, -1]
                rels.append(_rel(o.probs, ref))
                agree.append(float((o.pred.long().view(B) == ref.argmax(-1)).float().mean().item()))
                x = o.pred.long().view(B, 1)
                p += Tn
                Tn = 1
            out[var] = {"prefill_logits_rel": round(rels[0], 5),
                        "decode_logits_rel_max": round(max(rels[1:]), 5) if steps else None,
                        "decode_logits_rel_mean": round(sum(rels[1:]) / steps, 5) if steps else None,
                        "prefill_greedy_agreement": round(agree[0], 4),
                        "decode_greedy_agreement": round(sum(agree[1:]) / steps, 4) if steps else None}
            del st
            torch.cuda.empty_cache()
    finally:
        torch.backends.cuda.matmul.allow_tf32 = tf32
    return out


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="gpt2-xl")
    ap.add_argument("--layers", type=int, default=2)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--prompt", type=int, default=512)
    ap.add_argument("--steps", type=int, default=8)
    ap.add_argument("--variants", default="fp8-split,fp8-e4m3,bf16")
    ap.add_argument("--default_init", action="store_true", help="nanoGPT init (zero biases, unit gains)")
    a = ap.parse_args()
    r = measure(a.model, a.layers, a.batch, a.prompt, a.steps, a.variants.split(","),
                nontrivial=not a.default_init)
    print(json.dumps({"model": a.model, "layers": a.layers, "batch": a.batch, "prompt": a.prompt,
                      "decode_steps": a.steps, "weights_vs": "fp32 golden on the unquantised weights", **r}))
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
