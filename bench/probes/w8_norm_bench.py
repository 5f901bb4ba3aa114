#!/usr/bin/env python3
"""Decode W8A16 projections at batch 1 as the Llama-3 8B layer issues them:
plain, with the fused RMSNorm statistics (norm=1), and the SwiGLU gate|up
(act=3), each with and without the fragment-order weight copy.  Device time
per launch as HIP-graph replays, weight copies rotated past the 256 MB MALL.

    python bench/probes/w8_norm_bench.py [--iters 20] [--m 1]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

CASES = [  # name, N, K, act, norm
    ("qkv", 6144, 4096, 0, 1), ("qkv_nonorm", 6144, 4096, 0, 0), ("o", 4096, 4096, 0, 0),
    ("gate_up", 28672, 4096, 3, 1), ("down", 4096, 14336, 0, 0),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--m", type=int, default=1)
    ap.add_argument("--cases", default=",".join(c[0] for c in CASES))
    ap.add_argument("--env", default="", help="NAME=v1,v2,...: repeat each case per value of an A/B env var")
    args = ap.parse_args()
    from distributed_neural_networks_amd.ops.fp8 import linear_w8, quantize_weight
    from distributed_neural_networks_amd.ops.gemm import attach_shuffled
    dev = torch.device("cuda", 0)
    M = args.m
    want = set(args.cases.split(","))
    for name, N, K, act, norm in CASES:
        if name not in want:
            continue
        copies = max(2, min(48, (1 << 30) // (N * K) + 1))
        ws = [quantize_weight(torch.randn(N, K, device=dev) / K ** 0.5, dev) for _ in range(copies)]
        x = torch.randn(M, K, device=dev).bfloat16()
        out = torch.empty(M, N // 2 if act == 3 else N, device=dev, dtype=torch.bfloat16)
        res = {"case": name, "M": M, "N": N, "K": K, "MB": round(N * K / 1e6, 1)}
        envs = [None]
        if args.env:
            ename, vals = args.env.split("=")
            envs = [(ename, v) for v in vals.split(",")]
        for shuf, ev in [(s_, e_) for s_ in (False, True) for e_ in envs]:
            if ev is not None:
                if not shuf:
                    continue
                os.environ[ev[0]] = ev[1]
            if shuf and ws[0].shuf is None:
                for w in ws:
                    attach_shuffled(w)

            def run(w):
                linear_w8(x, w, act=act, out=out, norm=norm, eps=1e-5)

            for i in range(3):
                run(ws[i % copies])
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                for i in range(args.iters):
                    run(ws[i % copies])
            g.replay()
            torch.cuda.synchronize()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(3):
                g.replay()
            b.record()
            torch.cuda.synchronize()
            us = a.elapsed_time(b) / (3 * args.iters) * 1e3
            key = ("shuf" if shuf else "rowmajor") + (f"_{ev[0]}{ev[1]}" if ev else "")
            res[f"{key}_us"] = round(us, 2)
            res[f"{key}_TBs"] = round(N * K / us / 1e6, 2)
        print(json.dumps(res), flush=True)
        del ws


if __name__ == "__main__":
    main()
