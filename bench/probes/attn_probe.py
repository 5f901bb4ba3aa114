#!/usr/bin/env python3
"""Phase timing of one decode-attention workgroup (block (0,0)): builds
``csrc/kernels/attention.hip`` with ``-DDNN_DEC_PROBE`` into
``bench/_attn_probe.so`` (``--build``, on the CPU host) and prints, per shape,
the s_memrealtime (100 MHz) deltas between the kernel's phase marks:

    0 entry  1 lens read  2 q (+RoPE) packed  3 scores in LDS  4 softmax
    5 P.V done  6 reduction scratch written  7 output written

    python bench/probes/attn_probe.py --build        # CPU host
    python bench/probes/attn_probe.py                # GPU box
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
SO = os.path.join(ROOT, "bench", "_attn_probe.so")
sys.path.insert(0, ROOT)

SHAPES = {  # name: (B, H, Hkv, hd, S, pos, rope, splits)
    "llama_b1": (1, 32, 8, 128, 151, 140, True, 1),
    "llama_b32_s16": (32, 32, 8, 128, 161, 150, True, 16),
    "gpt2_b64": (64, 12, 12, 64, 567, 540, False, 1),
}


def build():
    src = os.path.join(ROOT, "csrc", "kernels", "attention.hip")
    cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "-shared", "--offload-arch=gfx950",
           "-DDNN_DEC_PROBE", "-I" + os.path.join(ROOT, "csrc", "kernels"), src, "-o", SO]
    subprocess.run(cmd, check=True)
    print("built", SO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", action="store_true")
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    if args.build:
        return build()
    import torch
    lib = ctypes.CDLL(SO)
    lib.dnn_attn_decode_qkv.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                        ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                        ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                        ctypes.c_float, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
    ts = (ctypes.c_ulonglong * 32)()
    dev = torch.device("cuda", 0)
    modes = {"dpp": "0", "mfma": "1"}
    for (name, (B, H, Hkv, hd, S, pos, rope, sp)), mode in [(x, m) for x in SHAPES.items() for m in modes]:
        os.environ["DNN_DECODE_MFMA"] = modes[mode]
        G = H // Hkv
        kc = torch.randn(B, Hkv, S, hd, device=dev).bfloat16()
        vc = torch.randn(B, Hkv, S, hd, device=dev).bfloat16()
        qkv = torch.randn(B, (H + 2 * Hkv) * hd, device=dev).bfloat16()
        out = torch.empty(B, H * hd, device=dev, dtype=torch.bfloat16)
        p = torch.full((B,), pos, device=dev, dtype=torch.int32)
        cos = torch.rand(S, hd // 2, device=dev) if rope else None
        sin = torch.rand(S, hd // 2, device=dev) if rope else None
        ws = torch.empty(B * Hkv * sp * G * (hd + 2), device=dev)
        rows = []
        for _ in range(args.reps):
            rc = lib.dnn_attn_decode_qkv(qkv.data_ptr(), qkv.stride(0), kc.data_ptr(), vc.data_ptr(), out.data_ptr(),
                                         B, H, Hkv, hd, S, p.data_ptr(), cos.data_ptr() if rope else None,
                                         sin.data_ptr() if rope else None, 1.0 / hd ** 0.5, sp, ws.data_ptr(),
                                         torch.cuda.current_stream().cuda_stream)
            assert rc == 0, rc
            torch.cuda.synchronize()
            assert lib.dnn_dec_probe_read(ts) == 0
            t = list(ts)[:8]
            clk = list(ts)[16:32]
            sub = [(ts[i] - ts[2]) * 10 for i in (8, 9, 10)] if mode == "mfma" else []
            ghz = (clk[7] - clk[0]) / max(1, (t[7] - t[0]) * 10)
            rows.append([(t[i + 1] - t[i]) * 10 for i in (0, 1, 2, 3)] + [(t[7] - t[0]) * 10, round(ghz, 2)] + sub)
        print(json.dumps({"shape": name, "mode": mode, "ns: lens,q,scores,softmax,total,GHz[,mfma: K landed,mfma done,LDS written (from q)]": rows}), flush=True)


if __name__ == "__main__":
    main()
