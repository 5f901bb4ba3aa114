"""Row pass costs of the fp8 prefill at the GPT-2 XL bench shape (64 x 512 rows
x 1600): LayerNorm + MX e4m3 quantisation (norm_q8, R rows per wave),
plain MX quantisation, bf16 LayerNorm and row statistics, each timed alone
(events over repeated launches) with its effective HBM TB/s.

    python bench/probes/norm_q8_probe.py [--M 32768 --N 1600]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


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
    return a.elapsed_time(b) / iters * 1e3  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, default=32768)
    ap.add_argument("--N", type=int, default=1600)
    a = ap.parse_args()
    from distributed_neural_networks_amd.ops import fp8
    from distributed_neural_networks_amd.ops import transformer_ops as T
    dev = torch.device("cuda", 0)
    M, N = a.M, a.N
    kp = fp8.kpad_of(N)
    x = (torch.randn(M, N, device=dev) * 3 + 1).bfloat16()
    w = torch.rand(N, device=dev) + 0.5
    bvec = torch.randn(N, device=dev) * 0.1
    q = torch.empty(M, kp, device=dev, dtype=torch.uint8)
    sx = torch.empty(fp8.mx_scale_bytes(M, kp), device=dev, dtype=torch.uint8)
    y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    st = torch.empty(M, 2, device=dev, dtype=torch.float32)
    rd, wq, wy = M * N * 2, M * kp + sx.numel(), M * N * 2
    res = {"M": M, "N": N, "kpad": kp}
    for r in ("1", "2", "4"):
        os.environ["DNN_NORMQ8_R"] = r
        t = timeit(lambda: T.layernorm_q8_mx(x, w, bvec, q, sx, kp))
        res[f"norm_q8_mx_R{r}_us"] = round(t, 2)
        res[f"norm_q8_mx_R{r}_TBs"] = round((rd + wq) / t / 1e6, 2)
    os.environ.pop("DNN_NORMQ8_R", None)
    t = timeit(lambda: fp8.quant_rows_mx(x, q, sx))
    res["quant_mx_us"], res["quant_mx_TBs"] = round(t, 2), round((rd + wq) / t / 1e6, 2)
    t = timeit(lambda: T.layernorm(x, w, bvec, y))
    res["layernorm_bf16_us"], res["layernorm_bf16_TBs"] = round(t, 2), round((rd + wy) / t / 1e6, 2)
    t = timeit(lambda: T.row_stats(x, st))
    res["row_stats_us"], res["row_stats_TBs"] = round(t, 2), round(rd / t / 1e6, 2)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
