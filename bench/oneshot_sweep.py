#!/usr/bin/env python3
"""One-shot decode GEMM (csrc/kernels/gemm_oneshot.h) configuration sweep
against the current decode dispatch (gemm_skinny / gemm_stream), on the
decode projection shapes of BASELINE configs 3-5 at their bench batch:
GPT-2 small (bf16, M = 64), GPT-2 XL (fp8 e4m3 weights, W8A16, M = 64) and
Llama-3 8B (bf16, M = 32).  Every kernel is timed as a HIP-graph replay of
``--iters`` launches over rotating weight copies (>= 1 GiB between reuses, so
the 256 MB MALL never serves a repeat, as in a decode step), and checked
against an fp32 product first.

    python bench/oneshot_sweep.py [--shapes gpt2,gpt2xl,llama] [--iters 20]
    python bench/oneshot_sweep.py --epi ln,ln_gelu [--shapes gpt2xl]

``--epi``: instead of the config sweep, time the folded-LayerNorm decode path
(``linear_norm``: row statistics accumulated inside the GEMM, optional GELU)
with the one-shot kernel off / planned, next to the plain product, to price the
in-kernel statistics.

One JSON line per shape: the dispatch's time, every config's time
(``mt/ntw/steps/splitk``), the best, and GB/s of weight bytes.
"""
from __future__ import annotations

import argparse
import itertools
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SHAPES = {  # (N, K, M, w8)
    "gpt2": [(2304, 768, 64, 0), (768, 768, 64, 0), (3072, 768, 64, 0), (768, 3072, 64, 0)],
    "gpt2xl": [(4800, 1600, 64, 1), (1600, 1600, 64, 1), (6400, 1600, 64, 1), (1600, 6400, 64, 1)],
    "llama": [(6144, 4096, 32, 0), (4096, 4096, 32, 0), (28672, 4096, 32, 0), (4096, 14336, 32, 0)],
    "heads": [(50304, 768, 64, 0), (50304, 1600, 64, 1)],  # the tied GPT-2 / GPT-2 XL heads at B = 64
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="gpt2,gpt2xl,llama")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--mts", default="1,2,4")
    ap.add_argument("--ntws", default="1,2,4")
    ap.add_argument("--splits", default="1,2,3,4,6,8")
    ap.add_argument("--epi", default="", help="comma list of ln | ln_gelu: folded-norm path A/B instead")
    args = ap.parse_args()
    if args.epi:
        return epi_ab(args)
    from distributed_neural_networks_amd.ops._lib import lib, ptr, stream_ptr
    from distributed_neural_networks_amd.ops.fp8 import linear_w8, quantize_weight
    from distributed_neural_networks_amd.ops.gemm import decode_workspace, linear, shuffle_weight
    dev = torch.device("cuda", 0)
    L = lib()
    ws_buf = decode_workspace(dev)
    wsb = ws_buf.numel()
    shapes = [s for k in args.shapes.split(",") for s in SHAPES[k]]
    for N, K, M, w8 in shapes:
        wbytes = N * K * (1 if w8 else 2)
        copies = max(2, min(64, (1 << 30) // wbytes + 1))
        if w8:
            ws = [quantize_weight(torch.randn(N, K, device=dev), dev) for _ in range(copies)]
            for w in ws:
                w.shuf = shuffle_weight(w.q[:, :K])
            wref = ws[0].q[:, :K].float() * ws[0].scale[:, None]
        else:
            ws = [torch.randn(N, K, device=dev).bfloat16() for _ in range(copies)]
            shuf = {id(w): shuffle_weight(w) for w in ws}
            wref = ws[0].float()
        x = torch.randn(M, K, device=dev).bfloat16()
        out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        ref = x.float() @ wref.t()
        res = {"M": M, "N": N, "K": K, "w8": w8}

        def timed(fn):
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

        def err():
            torch.cuda.synchronize()
            return ((out.float() - ref).norm() / ref.norm()).item()

        L.gemm_set_oneshot(0, 0, 0, 0, 0)  # the current dispatch (skinny / stream)
        if w8:
            def auto(w):
                linear_w8(x, w, out=out, ws=ws_buf)
        else:
            def auto(w):
                linear(x, w, out=out, w_shuf=shuf[id(w)], ws=ws_buf)
        auto(ws[0])
        res["dispatch_err"] = round(err(), 5)
        us = timed(auto)
        res["dispatch_us"] = round(us, 2)
        res["dispatch_GBs"] = round(wbytes / us / 1e3, 1)
        best = None
        for mt, ntw, steps, sk in itertools.product([int(v) for v in args.mts.split(",")],
                                                    [int(v) for v in args.ntws.split(",")], (1, 2),
                                                    [int(v) for v in args.splits.split(",")]):
            def run(w, mt=mt, ntw=ntw, steps=steps, sk=sk):
                wp = ptr(w.shuf) if w8 else ptr(shuf[id(w)])
                return L.gemm_oneshot_sweep(ptr(x), K, wp, ptr(w.scale) if w8 else 0, ptr(out), N, M, N, K, mt, ntw,
                                            steps, sk, w8, ptr(ws_buf), wsb, stream_ptr())

            out.zero_()
            if run(ws[0]) != 0:
                continue
            e = err()
            key = f"{mt}/{ntw}/{steps}/{sk}"
            if e > 2e-2:
                res[f"bad_{key}"] = round(e, 4)
                continue
            us = timed(run)
            res.setdefault("all", {})[key] = round(us, 2)
            if best is None or us < best[0]:
                best = (us, key)
        if best is not None:
            res["best_us"] = round(best[0], 2)
            res["best_GBs"] = round(wbytes / best[0] / 1e3, 1)
            res["best_cfg"] = best[1]
        print(json.dumps(res), flush=True)
        del ws


def epi_ab(args):
    """one-shot off / planned on the folded-LayerNorm decode path (linear_norm)."""
    from distributed_neural_networks_amd.ops.gemm import (attach_shuffled, decode_workspace, fold_norm, linear,
                                                          linear_norm, set_oneshot_gemm, shuffle_weight)
    from distributed_neural_networks_amd.ops.fp8 import linear_w8, quantize_weight
    dev = torch.device("cuda", 0)
    ws_buf = decode_workspace(dev)
    shapes = [s for k in args.shapes.split(",") for s in SHAPES[k]]
    for N, K, M, w8 in shapes:
        wbytes = N * K * (1 if w8 else 2)
        copies = max(2, min(64, (1 << 30) // wbytes + 1))
        g = torch.Generator(device=dev).manual_seed(0)
        gamma = 1 + 0.1 * torch.randn(K, device=dev, generator=g)
        beta = 0.1 * torch.randn(K, device=dev, generator=g)
        bias = 0.1 * torch.randn(N, device=dev, generator=g)
        w32 = [torch.randn(N, K, device=dev, generator=g) / K ** 0.5 for _ in range(2)]
        fs = [attach_shuffled(fold_norm(w32[i % 2], gamma, beta, bias, False, 1e-5, dev, fp8=bool(w8)))
              for i in range(copies)]
        plain = [quantize_weight(w32[i % 2], dev) if w8 else w32[i % 2].bfloat16() for i in range(copies)]
        pshuf = [attach_shuffled(p) if w8 else shuffle_weight(p) for p in plain]
        x = (3 + torch.randn(M, K, device=dev, generator=g)).bfloat16()
        out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        xn = torch.nn.functional.layer_norm(x.float(), (K,), gamma, beta, 1e-5)
        res = {"M": M, "N": N, "K": K, "w8": w8}

        def timed(fn):
            for i in range(3):
                fn(i % copies)
            torch.cuda.synchronize()
            gr = torch.cuda.CUDAGraph()
            with torch.cuda.graph(gr):
                for i in range(args.iters):
                    fn(i % copies)
            gr.replay()
            torch.cuda.synchronize()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(3):
                gr.replay()
            b.record()
            torch.cuda.synchronize()
            return round(a.elapsed_time(b) / (3 * args.iters) * 1e3, 2)

        for on in (0, 1):
            set_oneshot_gemm(on)
            if w8:
                res[f"plain_os{on}_us"] = timed(lambda i: linear_w8(x, pshuf[i], out=out, ws=ws_buf))
            else:
                res[f"plain_os{on}_us"] = timed(lambda i: linear(x, plain[i], out=out, w_shuf=pshuf[i], ws=ws_buf))
            for epi in args.epi.split(","):
                act = "gelu" if epi == "ln_gelu" else None
                linear_norm(x, fs[0], act, out=out, ws=ws_buf)
                torch.cuda.synchronize()
                ref = xn @ w32[0].t() + bias
                if act:
                    ref = torch.nn.functional.gelu(ref)
                res[f"{epi}_os{on}_err"] = round(((out.float() - ref).norm() / ref.norm()).item(), 5)
                res[f"{epi}_os{on}_us"] = timed(lambda i: linear_norm(x, fs[i], act, out=out, ws=ws_buf))
        set_oneshot_gemm(1)
        print(json.dumps(res), flush=True)
        del fs, plain, pshuf


if __name__ == "__main__":
    main()
