#!/usr/bin/env python3
"""fp8 (e4m3, per-token x per-channel scales) GEMM throughput: the 128^2 and the
256^2 4-phase kernels, GEMM only (operands pre-quantised), vs torch bf16
matmul on the same shape for scale.  One JSON line per shape.

    python bench/probes/gemm_fp8_bench.py [--shapes 32768x4800x1600,...] [--iters 30]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

DEFAULT = "32768x4800x1600,32768x1600x1600,32768x6400x1600,32768x1600x6400,16384x6144x4096,16384x28672x4096,16384x4096x14336,8192x8192x8192"


def timeit(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
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
    args = ap.parse_args()
    from distributed_neural_networks_amd.ops._lib import lib, ptr, stream_ptr
    from distributed_neural_networks_amd.ops.fp8 import kpad_of, quant_rows, quantize_weight, set_fp8_tile
    dev = torch.device("cuda", 0)
    L = lib()
    for s in args.shapes.split(","):
        M, N, K = (int(v) for v in s.split("x"))
        x = torch.randn(M, K, device=dev).bfloat16()
        wq = quantize_weight(torch.randn(N, K, device=dev) * 0.05, dev)
        kp = kpad_of(K)
        qb = torch.empty(M, kp, dtype=torch.uint8, device=dev)
        sb = torch.empty(M, device=dev)
        quant_rows(x, qb, sb)
        out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        flop = 2.0 * M * N * K
        row = {"M": M, "N": N, "K": K}
        ref = None
        for tile in (128, 256):
            set_fp8_tile(tile)
            ms = timeit(lambda: L.gemm_fp8(ptr(qb), ptr(sb), ptr(wq.q), ptr(wq.scale), ptr(out), N, 0, 0, 0, M, N, kp,
                                           0, stream_ptr()), args.iters)
            row[f"fp8_tile{tile}_tflops"] = round(flop / ms / 1e9, 1)
            if ref is None:
                ref = out.clone()
            else:
                row[f"tile{tile}_rel"] = ((out.float() - ref.float()).norm() / ref.float().norm()).item()
        set_fp8_tile(0)
        wb = torch.randn(N, K, device=dev).bfloat16()
        ms = timeit(lambda: torch.nn.functional.linear(x, wb), args.iters)
        row["torch_bf16_tflops"] = round(flop / ms / 1e9, 1)
        print(json.dumps(row), flush=True)
        del x, wq, qb, out, wb


if __name__ == "__main__":
    main()
