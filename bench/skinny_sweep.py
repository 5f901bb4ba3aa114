#!/usr/bin/env python3
"""Decode-GEMM (M <= 64) configuration sweep: achieved weight-stream GB/s per
(column tiles NT, chunks in flight U, waves/WG KS, software pipeline) on the
Llama-3 8B / GPT-2 / GPT-2 XL projection shapes, for bf16 weights and for
weight-only fp8 (``--w8``: e4m3 weights, bf16 activations).  Weight copies are
rotated so >= 1 GiB is streamed between reuses (the 256 MB MALL would
otherwise serve repeats, which a decode step never does).

    python bench/skinny_sweep.py [--m 1,32] [--w8 0,1] [--shapes llama,gpt2,gpt2xl] [--iters 20]

Configs: pipe bit 0 = software pipeline, bit 1 = M split (one 16-row tile per
workgroup).  Kernels are timed as HIP-graph replays (device time per launch).
One JSON line per (shape, M, w8): the auto-dispatch time and the best config;
``csrc/kernels/gemm_skinny.hip`` launch_skinny's table is fitted to these.
"""
from __future__ import annotations

import argparse
import itertools
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SHAPES = {
    "llama": [(6144, 4096), (4096, 4096), (28672, 4096), (4096, 14336), (128256, 4096)],
    "gpt2": [(2304, 768), (768, 768), (3072, 768), (768, 3072)],
    "gpt2head": [(50304, 768)],
    "gpt2xl": [(4800, 1600), (1600, 1600), (6400, 1600), (1600, 6400), (50304, 1600)],
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", default="1,32")
    ap.add_argument("--w8", default="0")
    ap.add_argument("--shapes", default="llama,gpt2xl")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--pipes", default="0,1,2,3", help="pipe codes: bit0 pipeline, bit1 M split, bit2 shuffled W")
    ap.add_argument("--shuf", action="store_true", help="also build pre-shuffled weight copies (pipe bit 2)")
    args = ap.parse_args()
    from distributed_neural_networks_amd.ops._lib import lib, ptr, stream_ptr
    from distributed_neural_networks_amd.ops.fp8 import linear_w8, quantize_weight
    from distributed_neural_networks_amd.ops.gemm import linear
    dev = torch.device("cuda", 0)
    L = lib()
    shapes = [s for k in args.shapes.split(",") for s in SHAPES[k]]
    for (N, K), M, w8 in itertools.product(shapes, [int(v) for v in args.m.split(",")],
                                           [int(v) for v in args.w8.split(",")]):
        wbytes = N * K * (1 if w8 else 2)
        copies = max(2, min(64, (1 << 30) // wbytes + 1))
        if w8:
            ws = [quantize_weight(torch.randn(N, K, device=dev), dev) for _ in range(copies)]
            sw = ws[0].scale
            ldw = ws[0].q.shape[1]
            wref = ws[0].q[:, :K].float() * ws[0].scale[:, None]
        else:
            ws = [torch.randn(N, K, device=dev).bfloat16() for _ in range(copies)]
            sw, ldw = None, K
            wref = ws[0].float()
        x = torch.randn(M, K, device=dev).bfloat16()
        out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        ref = x.float() @ wref.t()
        res = {"M": M, "N": N, "K": K, "w8": w8}

        def wptr(w):
            return ptr(w.q) if w8 else ptr(w)

        def timed(fn):
            # One HIP graph of `iters` launches (rotating weight copies), replayed:
            # the device time per kernel, as in the decode graphs, without the
            # ~7 us per-call Python/launch floor of an eager loop.
            for i in range(3):
                fn(ws[i % copies])
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                for i in range(args.iters):
                    fn(ws[i % copies])
            g.replay()
            torch.cuda.synchronize()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(3):
                g.replay()
            b.record()
            torch.cuda.synchronize()
            return a.elapsed_time(b) / (3 * args.iters) * 1e3  # us

        if w8:
            us = timed(lambda w: linear_w8(x, w, out=out))
        else:
            us = timed(lambda w: linear(x, w, out=out))
        res["auto_us"] = round(us, 2)
        res["auto_GBs"] = round(wbytes / us / 1e3, 1)
        best = None
        shuf = {}
        if args.shuf:
            from distributed_neural_networks_amd.ops.gemm import shuffle_weight
            shuf = {id(w): shuffle_weight(w.q[:, :K] if w8 else w) for w in ws}
        pipes = [int(p) for p in args.pipes.split(",")]
        for nt, u, ks, pipe in itertools.product((1, 2, 4), (2, 4, 8), (2, 4, 8), pipes):
            if nt == 4 and u == 8:
                continue
            if pipe & 2 and M <= 16:
                continue  # M split (pipe bit 1) only splits M > 16
            if pipe & 4 and not args.shuf:
                continue

            def run(w, pipe=pipe, nt=nt, u=u, ks=ks):
                wp = ptr(shuf[id(w)]) if pipe & 4 else wptr(w)
                return L.gemm_skinny_sweep(ptr(x), K, wp, ldw, ptr(sw if not w8 else w.scale), ptr(out), N, M,
                                           N, K, nt, u, ks, pipe, w8, stream_ptr())

            if run(ws[0]) != 0:
                continue
            torch.cuda.synchronize()
            err = ((out.float() - ref).norm() / ref.norm()).item()
            if err > 2e-2:
                res[f"bad_{nt}_{u}_{ks}_{pipe}"] = err
                continue
            us = timed(run)
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
