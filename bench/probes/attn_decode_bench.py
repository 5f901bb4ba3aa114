#!/usr/bin/env python3
"""Fused decode-attention microbenchmark (``attn_decode_qkv``: RoPE + KV write
+ split-K attention from the QKV projection rows): device time per launch as
HIP-graph replays, per shape and split count, plus the bytes-per-second of the
K/V stream, for both score paths (suffix ``m``: MFMA key tiles,
the GQA default; none: DPP row reductions).  Shapes are the decode benches' (Llama-3 8B B=1 / B=32, GPT-2
B=64 / B=256).

    python bench/probes/attn_decode_bench.py [--iters 50] [--splits 1,2,4,8,16]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

SHAPES = {  # name: (B, H, Hkv, hd, S capacity, pos, rope)
    "llama_b1": (1, 32, 8, 128, 151, 140, True),
    "llama_b1_4k": (1, 32, 8, 128, 4096, 4000, True),
    "llama_b32": (32, 32, 8, 128, 161, 150, True),
    "gpt2_b64": (64, 12, 12, 64, 567, 540, False),
    "gpt2_b256": (256, 12, 12, 64, 567, 540, False),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--splits", default="1,2,4,8,16")
    ap.add_argument("--shapes", default=",".join(SHAPES))
    args = ap.parse_args()
    from distributed_neural_networks_amd.ops.transformer_ops import attn_decode_qkv, decode_splits
    dev = torch.device("cuda", 0)
    for name in args.shapes.split(","):
        B, H, Hkv, hd, S, pos, rope = SHAPES[name]
        G = H // Hkv
        g = torch.Generator(device=dev).manual_seed(0)
        kc = torch.randn(B, Hkv, S, hd, device=dev, generator=g).bfloat16()
        vc = torch.randn(B, Hkv, S, hd, device=dev, generator=g).bfloat16()
        qkv = torch.randn(B, (H + 2 * Hkv) * hd, device=dev, generator=g).bfloat16()
        out = torch.empty(B, H * hd, device=dev, dtype=torch.bfloat16)
        p = torch.full((B,), pos, device=dev, dtype=torch.int32)
        cos = sin = None
        if rope:
            t = torch.arange(S, device=dev, dtype=torch.float32)[:, None] * torch.rand(hd // 2, device=dev)[None]
            cos, sin = torch.cos(t), torch.sin(t)
        res = {"shape": name, "B": B, "H": H, "Hkv": Hkv, "hd": hd, "S": S, "pos": pos,
               "auto_splits": decode_splits(S, B, Hkv, G)}
        kv_bytes = 2 * B * Hkv * (pos + 1) * hd * 2
        ref = None
        modes = {"": "0", "m": "1"}
        for sp, mode in [(int(v), m) for v in args.splits.split(",") for m in modes]:
            sp = sp or res["auto_splits"]
            if sp < decode_splits(S, B, Hkv, G) and sp < res["auto_splits"]:
                continue
            os.environ["DNN_DECODE_MFMA"] = modes[mode]
            ws = torch.empty(B * Hkv * sp * G * (hd + 2), device=dev, dtype=torch.float32)

            def run():
                attn_decode_qkv(qkv, kc, vc, out, B, H, Hkv, hd, p, ws, sp, cos, sin)

            run()
            torch.cuda.synchronize()
            if ref is None:
                ref = out.float().clone()
            err = (out.float() - ref).abs().max().item()
            gr = torch.cuda.CUDAGraph()
            with torch.cuda.graph(gr):
                for _ in range(args.iters):
                    run()
            gr.replay()
            torch.cuda.synchronize()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(5):
                gr.replay()
            b.record()
            torch.cuda.synchronize()
            us = a.elapsed_time(b) / (5 * args.iters) * 1e3
            key = f"s{sp}{mode}"
            res[f"{key}_us"] = round(us, 2)
            res[f"{key}_GBs"] = round(kv_bytes / us / 1e3, 1)
            res[f"{key}_maxdiff"] = round(err, 4)
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
