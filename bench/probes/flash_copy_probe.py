"""Probe: GPT-2 prefill attention straight from the c_attn output (QKV mode:
reads K/V rows from qkv and copies them into the cache) vs the head-major
kernel on an already-filled cache (no copy, contiguous K/V): the cost of the
in-kernel cache write + strided K/V reads.  One JSON line per shape."""
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
    return a.elapsed_time(b) / iters


def main():
    from distributed_neural_networks_amd.ops import transformer_ops as T_
    dev = torch.device("cuda", 0)
    for (B, T, H, hd) in [(64, 512, 12, 64), (64, 512, 25, 64)]:
        qkv = torch.randn(B * T, 3 * H * hd, device=dev).bfloat16()
        kc = torch.zeros(B, H, T, hd, device=dev, dtype=torch.bfloat16)
        vc = torch.zeros_like(kc)
        out = torch.empty(B * T, H * hd, device=dev, dtype=torch.bfloat16)
        pos = torch.zeros(B, dtype=torch.int32, device=dev)
        q = torch.empty(B * H * T * hd, device=dev, dtype=torch.bfloat16)
        T_.qkv_split(qkv, q, kc, vc, B, T, H, H, hd, pos)
        t_qkv = timeit(lambda: T_.flash_attn_qkv(qkv, kc, vc, out, B, T, H, H, hd, pos))
        t_hm = timeit(lambda: T_.flash_attn(q, kc, vc, out, B, T, H, H, hd, pos))
        t_split = timeit(lambda: T_.qkv_split(qkv, q, kc, vc, B, T, H, H, hd, pos))
        print(json.dumps({"B": B, "T": T, "H": H, "hd": hd, "qkv_mode_ms": round(t_qkv, 4),
                          "head_major_no_copy_ms": round(t_hm, 4), "qkv_split_ms": round(t_split, 4)}), flush=True)


if __name__ == "__main__":
    main()
