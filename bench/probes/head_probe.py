"""LM-head shapes at decode batch: the fused-norm skinny GEMM (weight
streaming, default for M <= 64) vs LayerNorm + the 128^2 / 256^2 MFMA tile
GEMMs (``set_skinny_max_m``).  Graph-replayed, one JSON line per shape."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def timed(fn, reps=50):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            for _ in range(10):
                fn()
    torch.cuda.synchronize()
    g.replay()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        g.replay()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps / 10 * 1e6


def main():
    from distributed_neural_networks_amd.ops.gemm import attach_shuffled, fold_norm, linear_norm, set_gemm_tile, \
        set_skinny_max_m
    dev = torch.device("cuda", 0)
    for M, N, K, rms in ((64, 50304, 768, False), (16, 50304, 768, False), (64, 50304, 1600, False),
                         (32, 128256, 4096, True), (64, 4096 * 7, 4096, True)):
        torch.manual_seed(0)
        w = torch.randn(N, K, device=dev) * 0.02
        f = attach_shuffled(fold_norm(w, torch.rand(K, device=dev) + 0.5, None if rms else torch.randn(K, device=dev),
                                      None, rms, 1e-5, dev))
        x = torch.randn(M, K, device=dev).bfloat16()
        out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        std = torch.empty(M, K, device=dev, dtype=torch.bfloat16)
        ones = torch.ones(K, device=dev)
        fn = lambda: linear_norm(x, f, out=out, std_buf=std, ones=ones)  # noqa: E731
        r = {"M": M, "N": N, "K": K, "MB": round(N * K * 2 / 2**20, 1)}
        set_skinny_max_m(64)  # force the skinny kernels at every M <= 64
        r["skinny_us"] = round(timed(fn), 2)
        ref = out.clone()
        set_skinny_max_m(0)
        for tile in (128, 256):
            set_gemm_tile(tile)
            r[f"ln_tile{tile}_us"] = round(timed(fn), 2)
            r[f"tile{tile}_maxdiff"] = (out.float() - ref.float()).abs().max().item()
        set_gemm_tile(0)
        set_skinny_max_m()
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
