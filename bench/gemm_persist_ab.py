"""Interleaved in-process A/B of the persistent 256^2 GEMM grid
(``gemm_set_persist(2)``: one workgroup per CU walking the tiles, the next
tile's prologue DMA under this tile's epilogue) against one workgroup per
tile, on the prefill projection shapes (GPT-2, GPT-2 XL, Llama-3 8B) with their
epilogues, plus the GPT-2 4-stage and Llama-3 8B prefill tokens/s either way.
Outputs must match bit for bit (same tiles, same math).  One JSON line per
shape, then one for the pipelines."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "bench"))

# (M, N, K, epilogue)
SHAPES = [(32768, 2304, 768, "none"), (32768, 768, 768, "res"), (32768, 3072, 768, "gelu"),
          (32768, 768, 3072, "res"), (32768, 4800, 1600, "none"), (32768, 6400, 1600, "gelu"),
          (16384, 6144, 4096, "none"), (16384, 4096, 14336, "res"), (8192, 8192, 8192, "none"),
          (65536, 512, 4096, "relu")]


def timeit(fn, iters=20):
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
    from distributed_neural_networks_amd.ops._lib import lib
    from distributed_neural_networks_amd.ops.gemm import linear
    dev = torch.device("cuda", 0)
    only_gemm = "--gemm_only" in sys.argv
    for (M, N, K, epi) in SHAPES:
        x = torch.randn(M, K, device=dev).bfloat16()
        w = (torch.randn(N, K, device=dev) * 0.05).bfloat16()
        bias = torch.randn(N, device=dev)
        r = torch.randn(M, N, device=dev).bfloat16() if epi == "res" else None
        act = epi if epi in ("gelu", "relu") else None
        outs = {f: torch.empty(M, N, device=dev, dtype=torch.bfloat16) for f in (0, 1)}
        t = {0: [], 1: []}
        for _ in range(3):
            for flag in (1, 0):
                lib().gemm_set_persist(2 * flag)
                t[flag].append(timeit(lambda: linear(x, w, bias, act=act, residual=r, out=outs[flag])))
        same = bool(torch.equal(outs[0], outs[1]))
        res = {"M": M, "N": N, "K": K, "epilogue": epi, "bit_identical": same}
        for flag in (0, 1):
            ms = sorted(t[flag])[len(t[flag]) // 2]
            res[f"persist{flag}_ms"] = round(ms, 4)
            res[f"persist{flag}_tflops"] = round(2.0 * M * N * K / ms / 1e9, 1)
        print(json.dumps(res), flush=True)
        del x, w, r, outs
        torch.cuda.empty_cache()
    lib().gemm_set_persist(1)
    if only_gemm:
        return
    import gpt_bench
    res = {}
    for name, argv in (("gpt2_4stage", ["--steps", "4", "--warmup", "1", "--prefill_iters", "3"]),
                       ("llama3_8b_b32", ["--model", "llama3-8b", "--stages", "8", "--batch", "32", "--steps", "2",
                                          "--warmup", "1", "--prefill_iters", "2"])):
        pf = {0: [], 1: []}
        for flag in (1, 0, 1, 0):
            lib().gemm_set_persist(2 * flag)
            g = gpt_bench.run(gpt_bench.parse(argv))
            pf[flag].append(g["prefill_tokens_per_s"])
            torch.cuda.empty_cache()
        res[f"{name}_prefill_tok_s_persist1"] = max(pf[1])
        res[f"{name}_prefill_tok_s_persist0"] = max(pf[0])
    lib().gemm_set_persist(1)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
