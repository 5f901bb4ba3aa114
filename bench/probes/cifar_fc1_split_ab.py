"""A/B of the fused fp32 fc1 (cifar_fc1_x3) on its two A encodings, interleaved
in one process: fp32 boundary rows split in registers (current) vs the blocked
hi/lo boundary encoding staged by DMA (SPLIT_IN).  Same operands, so the
outputs must be bit-identical.  Also times the fp32 -> blocked conversion and
its inverse.  Prints one JSON line."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    from distributed_neural_networks_amd.ops import cifar as cops
    from distributed_neural_networks_amd.ops._lib import check, lib, ptr, stream_ptr
    from distributed_neural_networks_amd import checkpoint as ckpt
    dev = torch.device("cuda", 0)
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    sd = ckpt.random_stage_state_dict("cifar10", 2, 3, False, True, 0)
    w = cops.pack_head(sd, dev)
    h = torch.randn(B, 4096, device=dev).relu_()
    hb = torch.empty_like(h)
    back = torch.empty_like(h)
    check(lib().cifar_split_blocked(ptr(h), ptr(hb), B, 4096, 0, stream_ptr()), "split_blocked")
    outs = {k: torch.empty(B, 512, device=dev) for k in ("fp32_in", "split_in")}

    def run(name, a, split):
        def f():
            check(lib().cifar_fc1_x3(ptr(a), 4096, ptr(w.w_fc1h), ptr(w.w_fc1l), 4096, ptr(w.b_fc1), ptr(outs[name]),
                                     512, B, 512, 4096, stream_ptr(), split), name)
        return f

    fns = {"fp32_in": run("fp32_in", h, 0), "split_in": run("split_in", hb, 1),
           "to_blocked": lambda: check(lib().cifar_split_blocked(ptr(h), ptr(hb), B, 4096, 0, stream_ptr()), "sb"),
           "from_blocked": lambda: check(lib().cifar_split_blocked(ptr(hb), ptr(back), B, 4096, 1, stream_ptr()), "fb")}
    res = {"B": B}
    times = {k: [] for k in fns}
    for _ in range(3):
        for name, fn in fns.items():
            for _ in range(2):
                fn()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                fn()
            e1.record()
            torch.cuda.synchronize()
            times[name].append(e0.elapsed_time(e1) / 20)
    for k, v in times.items():
        res[k + "_ms"] = round(min(v), 4)
    res["split_in_pflops"] = round(3 * 2 * B * 512 * 4096 / min(times["split_in"]) / 1e12, 3)
    res["max_abs_diff"] = (outs["fp32_in"] - outs["split_in"]).abs().max().item()
    ref = torch.relu(h @ sd["fc1.weight"].float().to(dev).T + sd["fc1.bias"].float().to(dev))
    res["split_in_max_rel_vs_fp32"] = ((outs["split_in"] - ref).abs().max() / ref.abs().max()).item()
    res["roundtrip_max_rel"] = ((back - h).abs() / h.abs().clamp_min(1e-30)).max().item()
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
