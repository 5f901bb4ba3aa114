#!/usr/bin/env python3
"""Decode vocabulary head, fused (csrc/kernels/gemm_head.h: logits + argmax
partials, then the merge launch) vs unfused (linear_norm + the row-split
argmax_rows), at the bench batch of the GPT-2 (bf16) and GPT-2 XL (fp8 W8A16)
heads.  Each arm is a HIP-graph replay of ``--iters`` head+argmax calls over
weight copies rotated past the 256 MB MALL (as in a decode step, where the
head's weights are not cache-resident).  One JSON line per shape.

    python bench/head_probe.py [--shapes gpt2,gpt2xl] [--iters 10]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SHAPES = {"gpt2": (64, 768, 50257, False), "gpt2xl": (64, 1600, 50257, True)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="gpt2,gpt2xl")
    ap.add_argument("--iters", type=int, default=10)
    args = ap.parse_args()
    from distributed_neural_networks_amd.ops import transformer_ops as T_
    from distributed_neural_networks_amd.ops.gemm import (HEAD_PART_PER_ROW, attach_shuffled, fold_norm, head_argmax,
                                                          linear_norm)
    dev = torch.device("cuda", 0)
    for name in args.shapes.split(","):
        M, K, N, w8 = SHAPES[name]
        g = torch.Generator(device=dev).manual_seed(0)
        gamma = 1 + 0.1 * torch.randn(K, device=dev, generator=g)
        beta = 0.1 * torch.randn(K, device=dev, generator=g)
        wbytes = N * K * (1 if w8 else 2)
        copies = max(2, min(32, (1 << 30) // wbytes + 1))
        fs = [attach_shuffled(fold_norm(torch.randn(N, K, device=dev, generator=g) / K ** 0.5, gamma, beta, None,
                                        False, 1e-5, dev, fp8=w8)) for _ in range(copies)]
        x = (torch.randn(M, K, device=dev, generator=g)).bfloat16()
        logits = torch.empty((M, (N + 7) // 8 * 8), device=dev, dtype=torch.bfloat16)
        part = torch.empty(2 * HEAD_PART_PER_ROW * M, dtype=torch.int32, device=dev)
        apart = torch.empty(2 * T_.ARGMAX_PART_PER_ROW * M, dtype=torch.int32, device=dev)
        out = torch.empty(M, dtype=torch.int32, device=dev)
        std = torch.empty((M, K), device=dev, dtype=torch.bfloat16)
        ones = torch.ones(K, device=dev)

        def fused(i):
            assert head_argmax(x, fs[i % copies], logits[:, :N], part, out)

        def unfused(i):
            linear_norm(x, fs[i % copies], out=logits[:, :N], std_buf=std, ones=ones)
            T_.argmax_rows(logits[:, :N], out, n=N, part=apart)

        def timed(fn):
            for i in range(3):
                fn(i)
            torch.cuda.synchronize()
            gr = torch.cuda.CUDAGraph()
            with torch.cuda.graph(gr):
                for i in range(args.iters):
                    fn(i)
            gr.replay()
            torch.cuda.synchronize()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(3):
                gr.replay()
            b.record()
            torch.cuda.synchronize()
            return round(a.elapsed_time(b) / (3 * args.iters) * 1e3, 2)

        res = {"shape": name, "M": M, "N": N, "K": K, "w8": w8, "weight_MB": round(wbytes / 1e6, 1)}
        for arm, fn in (("fused", fused), ("unfused", unfused), ("fused2", fused), ("unfused2", unfused)):
            res[arm + "_us"] = timed(fn)
        fused(0)
        torch.cuda.synchronize()
        o1 = out.clone()
        unfused(0)
        torch.cuda.synchronize()
        res["same_ids"] = bool(torch.equal(o1, out))
        best = min(res["fused_us"], res["fused2_us"])
        res["fused_TBs"] = round(wbytes / best / 1e6, 2)
        print(json.dumps(res), flush=True)
        del fs


if __name__ == "__main__":
    main()
