#!/usr/bin/env python3
"""Where a one-shot decode GEMM launch spends its time (csrc/kernels/gemm_oneshot.h,
template parameter ABL): the planned configuration of each GPT-2 / GPT-2 XL
decode projection at B = 64, timed whole and with parts removed —

    full      the product launch (ABL 0)
    no_w      no weight loads (registers filled with constants)
    no_a      no activation image (LDS-DMA skipped)
    no_ld     neither (launch + MFMAs + reduction + epilogue only)
    no_mfma   loads, no MFMAs
    no_store  everything but the epilogue stores
    empty     the launch alone (every wave returns at once)
    no_red    no cross-wave reduction through LDS (each wave's partial stored)
    no_ld_no_red  neither loads nor the reduction
    counted_wait  the round-4/5 image wait (vmcnt(weights after the image)
                  instead of vmcnt(0)): with two steps, step 0 computes while
                  step 1's weights land — racy (gemm_oneshot.h "Retiring the
                  image"), measured here only for what the fix costs

Each arm is a HIP-graph replay of ``--iters`` launches over weight copies
rotated past the 256 MB MALL (as bench/oneshot_sweep.py), interleaved over
``--rounds``; the minimum per arm is reported.

    python bench/probes/oneshot_anatomy.py [--iters 20 --rounds 3]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

SHAPES = [  # name, N, K, cfg (gemm_skinny.hip dnn_gemm_oneshot_ablate), w8
    ("xl_c_attn", 4800, 1600, 0, True), ("xl_c_fc", 6400, 1600, 0, True), ("xl_o", 1600, 1600, 1, True),
    ("gpt2_c_attn", 2304, 768, 2, False), ("gpt2_c_fc", 3072, 768, 2, False),
]
ARMS = {"full": 0, "no_w": 1, "no_a": 2, "no_ld": 3, "no_mfma": 4, "no_store": 8, "empty": 32, "no_red": 64,
        "no_ld_no_red": 67, "counted_wait": 128}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--M", type=int, default=64)
    args = ap.parse_args()
    from distributed_neural_networks_amd.ops._lib import lib, ptr, stream_ptr
    from distributed_neural_networks_amd.ops.fp8 import quantize_weight
    from distributed_neural_networks_amd.ops.gemm import shuffle_weight
    dev = torch.device("cuda", 0)
    L = lib()
    M = args.M
    for name, N, K, cfg, w8 in SHAPES:
        wbytes = N * K * (1 if w8 else 2)
        copies = max(2, min(64, (1 << 30) // wbytes + 1))
        if w8:
            qs = [quantize_weight(torch.randn(N, K, device=dev), dev) for _ in range(copies)]
            ws = [(shuffle_weight(q.q[:, :K]), q.scale) for q in qs]
            wref = qs[0].q[:, :K].float() * qs[0].scale[:, None]
            del qs
        else:
            wb = [torch.randn(N, K, device=dev).bfloat16() for _ in range(copies)]
            ws = [(shuffle_weight(w), None) for w in wb]
            wref = wb[0].float()
            del wb
        x = torch.randn(M, K, device=dev).bfloat16()
        out = torch.zeros(M, N, device=dev, dtype=torch.bfloat16)

        def launch(w, abl):
            return L.gemm_oneshot_ablate(ptr(x), K, ptr(w[0]), ptr(w[1]) if w[1] is not None else 0, ptr(out), N, M, N,
                                         K, cfg, abl, stream_ptr())

        rc = launch(ws[0], 0)
        torch.cuda.synchronize()
        res = {"shape": name, "M": M, "N": N, "K": K, "w8": w8, "weight_MB": round(wbytes / 1e6, 2)}
        if rc != 0:
            res["error"] = rc
            print(json.dumps(res), flush=True)
            continue
        ref = x.float() @ wref.t()
        res["full_err"] = round(((out.float() - ref).norm() / ref.norm()).item(), 5)
        graphs = {}
        for arm, abl in ARMS.items():
            for i in range(3):
                launch(ws[i % copies], abl)
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                for i in range(args.iters):
                    launch(ws[i % copies], abl)
            graphs[arm] = g
        best = {}
        for _ in range(args.rounds):
            for arm, g in graphs.items():
                g.replay()
                torch.cuda.synchronize()
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                for _ in range(3):
                    g.replay()
                b.record()
                torch.cuda.synchronize()
                us = a.elapsed_time(b) / (3 * args.iters) * 1e3
                best[arm] = min(best.get(arm, 1e9), us)
        res.update({f"{k}_us": round(v, 2) for k, v in best.items()})
        print(json.dumps(res), flush=True)
        del ws, graphs
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
