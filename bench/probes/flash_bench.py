"""Prefill attention: our flash_attn (QKV mode, GPT-2 shapes; Llama GQA) vs
torch scaled_dot_product_attention (the ROCm library kernel), causal, bf16.
One JSON line per shape: ms and effective TFLOP/s (causal half counted)."""
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


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
    from distributed_neural_networks_amd.ops import transformer_ops as T_
    dev = torch.device("cuda", 0)
    shapes = [(64, 512, 12, 12, 64), (8, 2048, 12, 12, 64), (32, 512, 32, 8, 128), (4, 4096, 32, 8, 128)]
    pick = os.environ.get("FLASH_SHAPES")  # e.g. "0" (GPT-2 B=64 T=512 only, for PMC passes)
    if pick:
        shapes = [shapes[int(i)] for i in pick.split(",")]
    for (B, T, H, Hkv, hd) in shapes:
        qkv = torch.randn(B * T, (H + 2 * Hkv) * hd, device=dev).bfloat16()
        kc = torch.zeros(B, Hkv, T, hd, device=dev, dtype=torch.bfloat16)
        vc = torch.zeros_like(kc)
        out = torch.empty(B * T, H * hd, device=dev, dtype=torch.bfloat16)
        pos = torch.zeros(B, dtype=torch.int32, device=dev)
        qh = torch.empty(B * H * T * hd, device=dev, dtype=torch.bfloat16)
        if Hkv == H:
            ours = lambda: T_.flash_attn_qkv(qkv, kc, vc, out, B, T, H, Hkv, hd, pos)  # noqa: E731
        else:
            def ours():
                T_.qkv_split(qkv, qh, kc, vc, B, T, H, Hkv, hd, pos)
                T_.flash_attn(qh, kc, vc, out, B, T, H, Hkv, hd, pos)
        q = torch.randn(B, H, T, hd, device=dev).bfloat16()
        k = torch.randn(B, H, T, hd, device=dev).bfloat16()
        v = torch.randn(B, H, T, hd, device=dev).bfloat16()
        ref = lambda: torch.nn.functional.scaled_dot_product_attention(q, k, v, is_causal=True)  # noqa: E731
        flop = 4.0 * B * H * T * T * hd / 2
        t_o, t_r = timeit(ours), timeit(ref)
        dbs = {}
        # A/B in one process (attention.hip): DNN_FLASH_DB single vs double
        # K/V buffer, DNN_FLASH_PIPE the hd-64 three-buffer software pipeline
        for _ in range(3):
            for db, pipe in ((0, 0), (1, 0), (1, 1)):
                os.environ["DNN_FLASH_DB"], os.environ["DNN_FLASH_PIPE"] = str(db), str(pipe)
                t = timeit(ours)
                k = f"db{db}_pipe{pipe}_ms"
                dbs[k] = round(min(t, dbs.get(k, 1e9)), 4)
        os.environ.pop("DNN_FLASH_DB", None)
        os.environ.pop("DNN_FLASH_PIPE", None)
        print(json.dumps({"B": B, "T": T, "H": H, "Hkv": Hkv, "hd": hd, "ours_ms": round(t_o, 4),
                          "ours_tflops": round(flop / t_o / 1e9, 1), "torch_sdpa_ms": round(t_r, 4),
                          "torch_tflops": round(flop / t_r / 1e9, 1), **dbs}), flush=True)


if __name__ == "__main__":
    main()
