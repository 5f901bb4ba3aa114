"""A/B of the fp32 fc1 paths at large batch: split3 + K-concat bf16 GEMM vs the
fused cifar_fc1_x3 kernel (same math, same weights).  Prints one JSON line."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    from distributed_neural_networks_amd.ops import cifar as cops
    from distributed_neural_networks_amd.ops.gemm import ACT_RELU, linear
    from distributed_neural_networks_amd.ops._lib import check, lib, ptr, stream_ptr
    from distributed_neural_networks_amd import checkpoint as ckpt
    dev = torch.device("cuda", 0)
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    sd = ckpt.random_stage_state_dict("cifar10", 2, 3, False, True, 0)
    w = cops.pack_head(sd, dev)
    h = torch.randn(B, 4096, device=dev).relu_()
    out_a = torch.empty(B, 512, device=dev)
    out_b = torch.empty(B, 512, device=dev)
    scratch = torch.empty(B, 3 * 4096, dtype=torch.bfloat16, device=dev)

    def a():
        check(lib().cifar_split3(ptr(h), 4096, ptr(scratch), 3 * 4096, B, 4096, stream_ptr()), "split3")
        linear(scratch, w.w_fc1, w.b_fc1, act=ACT_RELU, out=out_a)

    def b():
        check(lib().cifar_fc1_x3(ptr(h), 4096, ptr(w.w_fc1h), ptr(w.w_fc1l), 4096, ptr(w.b_fc1), ptr(out_b), 512,
                                 B, 512, 4096, stream_ptr()), "fc1_x3")

    res = {"B": B}
    outs = {}
    for name, fn in (("split3_concat_gemm", a), ("fused_fc1_x3", b)):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 20
        res[name + "_ms"] = round(ms, 4)
        res[name + "_pflops"] = round(3 * 2 * B * 512 * 4096 / ms / 1e12, 3)
        outs[name] = (out_a if fn is a else out_b).clone()
    res["max_abs_diff"] = (outs["split3_concat_gemm"] - outs["fused_fc1_x3"]).abs().max().item()
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
