#!/usr/bin/env python3
"""Anatomy of a 256^2 prefill GEMM tile: the same
launch with the epilogue's stores skipped (probe bit 1), with the main loop
skipped (bit 2: prologue DMAs, their wait and the epilogue), and both (3),
against the product launch (0), interleaved ``--rounds`` times.  Per shape:
microseconds per launch and per round of 256 tiles, so a tile's fixed cost
(prologue + epilogue + hand-over to the next workgroup) separates from its
per-K-tile cost.  bf16 (``linear``) and fp8 (per-token scales, ``gemm_fp8``)
arms; one JSON line per (dtype, shape).

    python bench/probes/gemm_anatomy.py [--shapes MxNxK,...] [--dtypes bf16,fp8,fp8mx] [--act none|gelu]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

DEFAULT = "32768x6400x1600,32768x6400x6400,32768x3072x768,32768x768x3072"


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
    return a.elapsed_time(b) * 1e3 / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default=DEFAULT)
    ap.add_argument("--dtypes", default="bf16,fp8")
    ap.add_argument("--act", default="none")
    ap.add_argument("--residual", action="store_true", help="bf16 / fp8mx: residual epilogue")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--arms", default="0,1,2,3",
                    help="anatomy bits per arm: 0 product, 1 no epilogue (no stores), 2 no main loop, "
                         "4 the residual by per-lane gathers (no LDS-DMA tile), "
                         "8 the epilogue with its plain-path stores predicated off")
    a = ap.parse_args()
    from distributed_neural_networks_amd.ops._lib import lib, ptr, stream_ptr
    from distributed_neural_networks_amd.ops.fp8 import (kpad_of, mx_scale_bytes, quant_rows, quant_rows_mx,
                                                         quantize_weight, set_fp8_tile)
    from distributed_neural_networks_amd.ops.gemm import linear, set_gemm_tile
    L = lib()
    dev = torch.device("cuda", 0)
    act_code = {"none": 0, "gelu": 2}[a.act]
    try:
        for s in a.shapes.split(","):
            M, N, K = (int(v) for v in s.split("x"))
            x = torch.randn(M, K, device=dev).bfloat16()
            out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            tiles = ((M + 255) // 256) * ((N + 255) // 256)
            for dt in a.dtypes.split(","):
                if dt == "bf16":
                    set_gemm_tile(256)
                    w = (torch.randn(N, K, device=dev) * 0.05).bfloat16()
                    rb = torch.randn(M, N, device=dev).bfloat16() if a.residual else None
                    fn = lambda: linear(x, w, None, act=a.act, residual=rb, out=out)  # noqa: E731
                elif dt == "fp8mx":  # the MX W8A8 product path (GPT-2 XL prefill); GELU: quantised output (QOUT)
                    wq = quantize_weight(torch.randn(N, K, device=dev) * 0.05, dev)
                    kp = kpad_of(K)
                    qb = torch.empty(M, kp, dtype=torch.uint8, device=dev)
                    sx = torch.empty(mx_scale_bytes(M, kp), dtype=torch.uint8, device=dev)
                    quant_rows_mx(x, qb, sx)
                    bias = torch.randn(N, device=dev)
                    kpo = kpad_of(N)
                    qo = torch.empty(M, kpo, dtype=torch.uint8, device=dev) if a.act == "gelu" else None
                    sxo = torch.empty(mx_scale_bytes(M, kpo), dtype=torch.uint8, device=dev) if qo is not None else None
                    res_t = torch.randn(M, N, device=dev).bfloat16() if a.residual else None
                    fn = lambda: L.gemm_fp8_mx(ptr(qb), ptr(sx), ptr(wq.q), ptr(wq.scale),  # noqa: E731
                                               0 if qo is not None else ptr(out), N, ptr(bias),
                                               ptr(res_t) if res_t is not None else 0, N, M, N, kp, act_code,
                                               ptr(qo) if qo is not None else 0, kpo if qo is not None else 0,
                                               ptr(sxo) if sxo is not None else 0, kpo if qo is not None else 0,
                                               stream_ptr())
                else:
                    set_fp8_tile(256)
                    wq = quantize_weight(torch.randn(N, K, device=dev) * 0.05, dev)
                    kp = kpad_of(K)
                    qb = torch.empty(M, kp, dtype=torch.uint8, device=dev)
                    sb = torch.empty(M, device=dev)
                    quant_rows(x, qb, sb)
                    fn = lambda: L.gemm_fp8(ptr(qb), ptr(sb), ptr(wq.q), ptr(wq.scale), ptr(out), N, 0, 0, 0,  # noqa: E731
                                            M, N, kp, act_code, stream_ptr())
                res = {}
                arms = [int(v) for v in a.arms.split(",")]
                for _ in range(a.rounds):
                    for bits in arms:
                        assert L.gemm_set_anatomy(bits) == 0
                        us = timeit(fn, a.iters)
                        res[bits] = min(res.get(bits, 1e30), us)
                L.gemm_set_anatomy(0)
                rounds = -(-tiles // 256)
                names = {0: "product", 1: "no_stores", 2: "no_main_loop", 3: "neither", 4: "residual_gathers",
                         8: "epilogue_no_store_instr"}
                row = {"dtype": dt, "M": M, "N": N, "K": K, "act": a.act, "tiles": tiles, "tile_rounds": rounds,
                       "us": {names.get(b, str(b)): round(v, 2) for b, v in res.items()},
                       "us_per_round": {names.get(b, str(b)): round(v / rounds, 2) for b, v in res.items()},
                       "tflops": round(2.0 * M * N * K / res[0] / 1e6, 1) if 0 in res else None}
                print(json.dumps(row), flush=True)
    finally:
        L.gemm_set_anatomy(0)
        set_gemm_tile(0)
        set_fp8_tile(0)


if __name__ == "__main__":
    main()
