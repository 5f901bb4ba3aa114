#!/usr/bin/env python3
"""Decode attention at the decode benches' shapes, batched kernel vs the
one-pass kernel and its switches (attention.hip attn_decode_1p_kernel).

The K/V caches rotate over enough copies (> 640 MB) that every launch streams
from HBM as in a real decode step (one layer's cache is evicted from the
256 MB MALL by the other layers' before it is read again); a single-copy
microbenchmark would time MALL hits.  Device time per launch from HIP-graph
replays; GB/s counts the K/V rows attended.

    python bench/probes/attn_1p_probe.py [--iters 24] [--shapes gpt2_b64,...]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

SHAPES = {  # name: (B, H, Hkv, hd, S capacity, pos, rope)
    "gpt2_b64": (64, 12, 12, 64, 567, 540, False),
    "gpt2xl_b64": (64, 25, 25, 64, 567, 540, False),
    "llama_b32": (32, 32, 8, 128, 567, 540, True),
    "llama_b32_p270": (32, 32, 8, 128, 567, 270, True),   # fixed vs per-byte cost
    "llama_b48": (48, 32, 8, 128, 567, 540, True),
    "llama_b64": (64, 32, 8, 128, 567, 540, True),        # two workgroups per CU
}
VARIANTS = {  # name: env
    "batched": {"DNN_DECODE_1P": "0"},
    "1p": {"DNN_DECODE_1P": "1"},
    "1p_force": {"DNN_DECODE_1P": "2"},
    "1p_kf0": {"DNN_DECODE_1P": "1", "DNN_DECODE_1P_KF": "0"},
    "1p_kf1": {"DNN_DECODE_1P": "1", "DNN_DECODE_1P_KF": "1"},
    "1p_knt0": {"DNN_DECODE_1P": "1", "DNN_DECODE_1P_KNT": "0"},
    "1p_knt1": {"DNN_DECODE_1P": "1", "DNN_DECODE_1P_KNT": "1"},
    "1p_rs0": {"DNN_DECODE_1P": "1", "DNN_DECODE_1P_RS": "0"},
}
KEYS = ("DNN_DECODE_1P", "DNN_DECODE_1P_KNT", "DNN_DECODE_1P_RS", "DNN_DECODE_1P_KF")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=24)
    ap.add_argument("--shapes", default=",".join(SHAPES))
    ap.add_argument("--variants", default=",".join(VARIANTS))
    ap.add_argument("--rounds", type=int, default=2)
    args = ap.parse_args()
    from distributed_neural_networks_amd.ops.transformer_ops import attn_decode_qkv, decode_splits
    dev = torch.device("cuda", 0)
    for name in args.shapes.split(","):
        B, H, Hkv, hd, S, pos, rope = SHAPES[name]
        G = H // Hkv
        one = 2 * B * Hkv * S * hd * 2
        nc = max(2, -(-640 * 2 ** 20 // one))
        g = torch.Generator(device=dev).manual_seed(0)
        caches = [(torch.randn(B, Hkv, S, hd, device=dev, generator=g).bfloat16(),
                   torch.randn(B, Hkv, S, hd, device=dev, generator=g).bfloat16()) for _ in range(nc)]
        qkv = torch.randn(B, (H + 2 * Hkv) * hd, device=dev, generator=g).bfloat16()
        out = torch.empty(B, H * hd, device=dev, dtype=torch.bfloat16)
        p = torch.full((B,), pos, device=dev, dtype=torch.int32)
        cos = sin = None
        if rope:
            t = torch.arange(S, device=dev, dtype=torch.float32)[:, None] * torch.rand(hd // 2, device=dev)[None]
            cos, sin = torch.cos(t), torch.sin(t)
        splits = decode_splits(S, B, Hkv, G)
        ws = torch.empty(B * Hkv * max(splits, 2) * G * (hd + 2), device=dev, dtype=torch.float32)
        kv_bytes = 2 * B * Hkv * (pos + 1) * hd * 2
        res = {"shape": name, "B": B, "H": H, "Hkv": Hkv, "hd": hd, "S": S, "pos": pos, "splits": splits,
               "copies": nc}
        ref = None
        times = {v: [] for v in args.variants.split(",")}
        graphs = {}
        for v in times:
            for k in KEYS:
                os.environ.pop(k, None)
            os.environ.update(VARIANTS[v])
            kc, vc = caches[0]
            attn_decode_qkv(qkv, kc, vc, out, B, H, Hkv, hd, p, ws, splits, cos, sin)
            torch.cuda.synchronize()
            if ref is None:
                ref = out.float().clone()
            res[f"{v}_maxdiff"] = round((out.float() - ref).abs().max().item(), 4)
            gr = torch.cuda.CUDAGraph()
            with torch.cuda.graph(gr):
                for i in range(args.iters):
                    kc, vc = caches[i % nc]
                    attn_decode_qkv(qkv, kc, vc, out, B, H, Hkv, hd, p, ws, splits, cos, sin)
            graphs[v] = gr
        for _ in range(args.rounds):
            for v, gr in graphs.items():
                gr.replay()
                torch.cuda.synchronize()
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                for _ in range(4):
                    gr.replay()
                b.record()
                torch.cuda.synchronize()
                times[v].append(a.elapsed_time(b) / (4 * args.iters) * 1e3)
        for v, ts in times.items():
            us = min(ts)
            res[f"{v}_us"] = round(us, 2)
            res[f"{v}_GBs"] = round(kv_bytes / us / 1e3, 1)
        for k in KEYS:
            os.environ.pop(k, None)
        print(json.dumps(res), flush=True)
        del caches, graphs
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
