"""Interleaved in-process A/B of the 256^2 GEMM's residual-prefetch epilogue
(``gemm_set_res_prefetch``): the 768-wide GPT-2 prefill projections with the
residual in place (R = C, the decoder's h += ...) and separate, then the
GPT-2 4-stage prefill tokens/s with the switch on and off.  One JSON line."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "bench"))


def timeit(fn, iters=30):
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
    res = {}
    for (M, N, K) in ((32768, 768, 768), (32768, 768, 3072)):
        x = torch.randn(M, K, device=dev).bfloat16()
        w = (torch.randn(N, K, device=dev) * 0.05).bfloat16()
        bias = torch.randn(N, device=dev)
        out = torch.randn(M, N, device=dev).bfloat16()
        r = torch.randn(M, N, device=dev).bfloat16()
        for mode in ("inplace", "separate"):
            R = out if mode == "inplace" else r
            t = {0: [], 1: []}
            for _ in range(4):
                for flag in (1, 0):
                    lib().gemm_set_res_prefetch(flag)
                    t[flag].append(timeit(lambda: linear(x, w, bias, residual=R, out=out)))
            for flag in (0, 1):
                ms = sorted(t[flag])[len(t[flag]) // 2]
                res[f"{N}x{K}_{mode}_pre{flag}_tflops"] = round(2.0 * M * N * K / ms / 1e9, 1)
    import gpt_bench
    pf = {0: [], 1: []}
    for flag in (1, 0, 1, 0):
        lib().gemm_set_res_prefetch(flag)
        g = gpt_bench.run(gpt_bench.parse(["--steps", "4", "--warmup", "1", "--prefill_iters", "3"]))
        pf[flag].append(g["prefill_tokens_per_s"])
        torch.cuda.empty_cache()
    res["gpt2_prefill_tok_s_pre1"] = max(pf[1])
    res["gpt2_prefill_tok_s_pre0"] = max(pf[0])
    lib().gemm_set_res_prefetch(1)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
