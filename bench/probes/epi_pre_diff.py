"""Run-to-run and prefetch on/off differences of the forced one-shot decode
GEMM with the folded LayerNorm + GELU epilogue (test_epilogue_prefetch_bit_identical
diagnostics): prints max |diff| and count for (off, off), (on, on), (off, on)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def bias_res_w8(N, K):
    """linear_w8 with bias + residual (GPT-2 XL O / c_proj) under the same arms."""
    from distributed_neural_networks_amd.ops._lib import lib
    from distributed_neural_networks_amd.ops.fp8 import linear_w8, quantize_weight
    from distributed_neural_networks_amd.ops.gemm import decode_workspace, set_oneshot_gemm, shuffle_weight
    dev = torch.device("cuda", 0)
    M = 64
    g = torch.Generator(device=dev).manual_seed(N + K)
    x = (torch.randn(M, K, device=dev, generator=g) * 2 + 0.5).bfloat16()
    w = torch.randn(N, K, device=dev, generator=g) / K ** 0.5
    bias = torch.randn(N, device=dev, generator=g)
    res = torch.randn(M, N, device=dev, generator=g).bfloat16()
    ws = decode_workspace(dev)
    q = quantize_weight(w, dev)
    q.shuf = shuffle_weight(q.q[:, :K])
    res_ = {"N": N, "K": K, "epi": "bias_res_w8"}
    for mode in (2, 0):
        outs = {}
        set_oneshot_gemm(mode)
        for tag, on in (("off1", 0), ("off2", 0), ("on1", 1), ("on2", 1)):
            lib().gemm_set_epi_prefetch(on)
            outs[tag] = linear_w8(x, q, bias, 0, res, ws=ws).float().clone()
        torch.cuda.synchronize()
        for a, b in (("off1", "off2"), ("on1", "on2"), ("off1", "on1")):
            d = (outs[a] - outs[b]).abs()
            res_[f"mode{mode}_{a}_{b}"] = {"max": d.max().item(), "n": int((d > 0).sum())}
    lib().gemm_set_epi_prefetch(1)
    set_oneshot_gemm(1)
    print(json.dumps(res_), flush=True)


def main():
    bias_res_w8(1600, 6400)
    bias_res_w8(1600, 1600)
    from distributed_neural_networks_amd.ops._lib import lib
    from distributed_neural_networks_amd.ops.gemm import (attach_shuffled, decode_workspace, fold_norm, linear_norm,
                                                          set_oneshot_gemm)
    dev = torch.device("cuda", 0)
    for (N, K), test_data in (((2304, 768), True), ((2304, 768), False), ((3072, 768), True), ((4800, 1600), False)):
        M = 64
        g = torch.Generator(device=dev).manual_seed(N + K)
        x = (torch.randn(M, K, device=dev, generator=g) * 2 + 0.5).bfloat16()
        w = torch.randn(N, K, device=dev, generator=g) / K ** 0.5
        bias = torch.randn(N, device=dev, generator=g)
        if test_data:  # the draw order of test_epilogue_prefetch_bit_identical (a residual before gamma / beta)
            torch.randn(M, N, device=dev, generator=g)
        ws = decode_workspace(dev)
        gam = torch.rand(K, device=dev, generator=g) + 0.5
        bet = torch.randn(K, device=dev, generator=g) * 0.1
        f = fold_norm(w, gam, bet, bias, False, 1e-5, dev, False)
        attach_shuffled(f)
        xf = x.float()
        xn = (xf - xf.mean(1, keepdim=True)) / torch.sqrt(xf.var(1, unbiased=False, keepdim=True) + 1e-5)
        ref = torch.nn.functional.gelu((xn * gam + bet) @ w.t() + bias, approximate="tanh")
        outs = {}
        set_oneshot_gemm(2)
        for tag, on in (("off1", 0), ("off2", 0), ("on1", 1), ("on2", 1)):
            lib().gemm_set_epi_prefetch(on)
            outs[tag] = linear_norm(x, f, act="gelu", ws=ws).float().clone()
        torch.cuda.synchronize()
        lib().gemm_set_epi_prefetch(1)
        set_oneshot_gemm(1)
        res = {"N": N, "K": K}
        res["test_data"] = test_data
        for a in ("off1", "on1"):
            d = (outs[a] - ref).abs()
            i = int(d.argmax())
            res[f"{a}_vs_fp32"] = {"max": d.max().item(), "at": [i // N, i % N], "ref": ref.view(-1)[i].item()}
        for a, b in (("off1", "off2"), ("on1", "on2"), ("off1", "on1")):
            d = (outs[a] - outs[b]).abs()
            i = int(d.argmax())
            res[f"{a}_{b}"] = {"max": d.max().item(), "n": int((d > 0).sum()), "at": [i // N, i % N],
                               "vals": [outs[a].view(-1)[i].item(), outs[b].view(-1)[i].item()],
                                "ref": ref.view(-1)[i].item(), "n_gt_step": int((d > outs[a].abs().maximum(
                                    outs[b].abs()) * 2.0 ** -7).sum())}
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
