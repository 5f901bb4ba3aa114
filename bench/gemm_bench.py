#!/usr/bin/env python3
"""bf16 GEMM throughput: our 128^2 and 256^2 kernels vs torch.matmul (hipBLASLt).

Random operands (uniform-ish normal, never zero-filled: guide §5.4 rule 25).
Prints one JSON line per shape with TFLOP/s of every arm.

    python bench/gemm_bench.py [--shapes 65536x512x4096,32768x2304x768,...] [--iters 50]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

DEFAULT = ("65536x512x4096,16384x512x4096,32768x2304x768,32768x768x768,32768x3072x768,32768x768x3072,"
           "4096x4096x4096,8192x8192x8192,32768x1024x4096")


def timeit(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a = torch.cuda.Event(enable_timing=True)
    b = torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default=DEFAULT)
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--act", default="none")
    ap.add_argument("--residual", action="store_true", help="residual epilogue (R = a separate (M,N) bf16 tensor)")
    ap.add_argument("--inplace", action="store_true", help="residual epilogue in place (R = C, the decoder's h += ...)")
    ap.add_argument("--torch", action="store_true", help="also time torch.nn.functional.linear (hipBLASLt)")
    ap.add_argument("--tiles", default="128,256", help="tile arms: 128, 256, 255 (= 256x128), 0 (auto)")
    ap.add_argument("--rounds", type=int, default=1, help="interleaved repetitions of the arms")
    args = ap.parse_args()
    from distributed_neural_networks_amd.ops.gemm import linear, set_gemm_tile
    dev = torch.device("cuda", 0)
    for s in args.shapes.split(","):
        M, N, K = (int(v) for v in s.split("x"))
        x = torch.randn(M, K, device=dev).bfloat16()
        w = (torch.randn(N, K, device=dev) * 0.05).bfloat16()
        bias = torch.randn(N, device=dev)
        out = torch.randn(M, N, device=dev).bfloat16()
        res = out if args.inplace else (torch.randn(M, N, device=dev).bfloat16() if args.residual else None)
        flop = 2.0 * M * N * K
        row = {"M": M, "N": N, "K": K}
        ref = None
        for tile in [int(t) for t in args.tiles.split(",")] * args.rounds:
            set_gemm_tile(tile)
            ms = timeit(lambda: linear(x, w, bias, act=args.act, residual=res, out=out), args.iters)
            row[f"tile{tile}_tflops"] = max(row.get(f"tile{tile}_tflops", 0.0), round(flop / ms / 1e9, 1))
            if not args.inplace:
                if ref is None:
                    ref = out.clone()
                else:
                    row[f"tile{tile}_maxdiff"] = (out.float() - ref.float()).abs().max().item()
        set_gemm_tile(0)
        if args.torch:
            ms = timeit(lambda: torch.nn.functional.linear(x, w, bias.bfloat16()), args.iters)
            row["torch_tflops"] = round(flop / ms / 1e9, 1)
        row["epilogue"] = args.act + ("+residual_inplace" if args.inplace else "+residual" if args.residual else "")
        print(json.dumps(row), flush=True)
        del x, w, out


if __name__ == "__main__":
    main()
