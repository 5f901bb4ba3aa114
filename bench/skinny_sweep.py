#!/usr/bin/env python3
"""Decode-GEMM (M <= 64) configuration sweep: achieved weight-stream GB/s per
(column tiles NT, chunks in flight U, waves/WG KS, software pipeline) on the
Llama-3 8B / GPT-2 shapes.  Weight copies are rotated so >= 1 GiB is streamed
between reuses (the 256 MB MALL would otherwise serve repeats).

    python bench/skinny_sweep.py [--m 1,32] [--iters 20]
"""
from __future__ import annotations

import argparse
import itertools
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SHAPES = [(6144, 4096), (4096, 4096), (28672, 4096), (4096, 14336), (128256, 4096), (4800, 1600), (6400, 1600),
          (1600, 6400), (50304, 1600)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", default="1,32")
    ap.add_argument("--iters", type=int, default=20)
    args = ap.parse_args()
    from distributed_neural_networks_amd.ops._lib import lib, ptr, stream_ptr
    from distributed_neural_networks_amd.ops.gemm import linear
    dev = torch.device("cuda", 0)
    L = lib()
    for (N, K), M in itertools.product(SHAPES, [int(v) for v in args.m.split(",")]):
        wbytes = N * K * 2
        copies = max(2, min(64, (1 << 30) // wbytes + 1))
        ws = [torch.randn(N, K, device=dev).bfloat16() for _ in range(copies)]
        x = torch.randn(M, K, device=dev).bfloat16()
        out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        ref = (x.float() @ ws[0].float().t())
        res = {"M": M, "N": N, "K": K}

        def timed(fn):
            for i in range(3):
                fn(ws[i % copies])
            torch.cuda.synchronize()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for i in range(args.iters):
                fn(ws[i % copies])
            b.record()
            torch.cuda.synchronize()
            return a.elapsed_time(b) / args.iters * 1e3  # us

        us = timed(lambda w: linear(x, w, out=out))
        res["auto_us"] = round(us, 2)
        res["auto_GBs"] = round(wbytes / us / 1e3, 1)
        best = None
        for nt, u, ks, pipe in itertools.product((1, 2, 4), (2, 4, 8), (2, 4, 8), (0, 1)):
            if nt == 4 and u == 8:
                continue
            rc = L.gemm_skinny_sweep(ptr(x), K, ptr(ws[0]), K, ptr(out), N, M, N, K, nt, u, ks, pipe, stream_ptr())
            if rc != 0:
                continue
            torch.cuda.synchronize()
            err = ((out.float() - ref).norm() / ref.norm()).item()
            if err > 2e-2:
                res[f"bad_{nt}_{u}_{ks}_{pipe}"] = err
                continue
            us = timed(lambda w: L.gemm_skinny_sweep(ptr(x), K, ptr(w), K, ptr(out), N, M, N, K, nt, u, ks, pipe,
                                                     stream_ptr()))
            res.setdefault("all", {})[f"{nt}/{u}/{ks}/{pipe}"] = round(us, 2)
            if best is None or us < best[0]:
                best = (us, nt, u, ks, pipe)
        res["best_us"] = round(best[0], 2)
        res["best_GBs"] = round(wbytes / best[0] / 1e3, 1)
        res["best_cfg"] = {"nt": best[1], "u": best[2], "ks": best[3], "pipe": best[4]}
        print(json.dumps(res), flush=True)
        del ws


if __name__ == "__main__":
    main()
