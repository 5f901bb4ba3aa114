#!/usr/bin/env python3
"""A/B of the decode stream GEMM (csrc/kernels/gemm_stream.h) against the
skinny kernel it replaces (the production plan: shapes the plan rejects
fall back to the skinny kernel in both arms), on the decode projection shapes (Llama-3 8B at
M = 32, GPT-2 XL W8 at M = 64, ...): device time per launch from HIP-graph
replays of rotating weight copies (>= 1 GiB between reuses, so no MALL
hits), the two kernels interleaved in one process.

    python bench/stream_gemm_ab.py [--m 32] [--shapes llama] [--w8 0] [--rounds 3]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SHAPES = {
    "llama": [("qkv", 6144, 4096, 1), ("o", 4096, 4096, 0), ("gate_up", 28672, 4096, 1), ("down", 4096, 14336, 0),
              ("head", 128256, 4096, 1)],
    "gpt2xl": [("qkv", 4800, 1600, 2), ("o", 1600, 1600, 0), ("fc", 6400, 1600, 2), ("proj", 1600, 6400, 0),
               ("head", 50304, 1600, 2)],
    "gpt2": [("qkv", 2304, 768, 2), ("o", 768, 768, 0), ("fc", 3072, 768, 2), ("proj", 768, 3072, 0),
             ("head", 50304, 768, 2)],
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", default="32")
    ap.add_argument("--shapes", default="llama")
    ap.add_argument("--w8", type=int, default=0)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--arms", default="stream,skinny", help="stream (plan), skinny, forced (every shape streamed)")
    args = ap.parse_args()
    from distributed_neural_networks_amd.ops.fp8 import linear_w8, quantize_weight
    from distributed_neural_networks_amd.ops.gemm import (attach_shuffled, decode_workspace, fold_norm, linear,
                                                          linear_norm, set_stream_gemm)
    dev = torch.device("cuda", 0)
    ws = decode_workspace(dev, 0)
    for M in [int(v) for v in args.m.split(",")]:
        for name, N, K, norm in [s for k in args.shapes.split(",") for s in SHAPES[k]]:
            wbytes = N * K * (1 if args.w8 else 2)
            copies = max(2, min(48, (1 << 30) // wbytes + 1))
            x = torch.randn(M, K, device=dev).bfloat16()
            out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            gamma = torch.rand(K, device=dev) + 0.5
            mats = []
            for _ in range(copies):
                W = torch.randn(N, K, device=dev) / K ** 0.5
                if norm:
                    mats.append(attach_shuffled(fold_norm(W, gamma, None, None, norm == 1, 1e-5, dev, bool(args.w8))))
                elif args.w8:
                    mats.append(attach_shuffled(quantize_weight(W, dev)))
                else:
                    Wb = W.bfloat16()
                    mats.append((Wb, attach_shuffled(Wb)))
                del W

            def call(w):
                if norm:
                    return linear_norm(x, w, out=out, ws=ws)
                if args.w8:
                    return linear_w8(x, w, out=out, ws=ws)
                return linear(x, w[0], out=out, w_shuf=w[1], ws=ws)

            def timed():
                for i in range(3):
                    call(mats[i % copies])
                torch.cuda.synchronize()
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g):
                    for i in range(args.iters):
                        call(mats[i % copies])
                g.replay()
                torch.cuda.synchronize()
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                for _ in range(3):
                    g.replay()
                b.record()
                torch.cuda.synchronize()
                return a.elapsed_time(b) / (3 * args.iters) * 1e3

            res = {"shape": name, "M": M, "N": N, "K": K, "w8": args.w8, "norm": norm, "MB": round(wbytes / 1e6, 1)}
            arms = {"stream": 1, "skinny": 0, "forced": 2, "f2": 2, "f3": 2, "f4": 2, "f6": 2}
            ts = {k: [] for k in args.arms.split(",")}
            for _ in range(args.rounds):
                for k in ts:
                    set_stream_gemm(arms[k], 8 << 20)
                    if k[0] == "f" and k[1:].isdigit():  # forced with a pinned split count
                        os.environ["DNN_STREAM_SPLITK"] = k[1:]
                    ts[k].append(timed())
                    os.environ.pop("DNN_STREAM_SPLITK", None)
            set_stream_gemm(1, 8 << 20)
            for k in ts:
                us = min(ts[k])
                res[k + "_us"] = round(us, 2)
                res[k + "_TBs"] = round(wbytes / us / 1e6, 2)
            print(json.dumps(res), flush=True)
            del mats
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
