#!/usr/bin/env python3
"""Would concurrent prefill microbatches fill the GEMM tile tails?  GPT-2
4-stage prefill of 64 x 512 tokens as one microbatch on one stream, against
two 32 x 512 microbatches on two HIP streams (two stage copies, so no buffer
is shared).  The 768-wide projections run 384 256^2 tiles on 256 CUs (a
half-empty second round); a second stream's kernels can fill it.

    python bench/probes/prefill_lanes_probe.py [--model gpt2] [--reps 5]
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "bench"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="gpt2")
    ap.add_argument("--stages", type=int, default=4)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--prompt", type=int, default=512)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    from gpt_bench import _build_group
    from distributed_neural_networks_amd.models import default_ranges, model_info
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    ranges = default_ranges(a.model, a.stages)
    ids = list(range(a.stages))
    B, T = a.batch, a.prompt
    full = _build_group(a.model, ranges, ids, dev, B, T + 8, False)
    halves = [_build_group(a.model, ranges, ids, dev, B // 2, T + 8, False) for _ in range(2)]
    V = model_info(a.model).cfg.vocab_size
    x = torch.randint(0, V, (B, T), device=dev, dtype=torch.int32)
    xs = [x[:B // 2].contiguous(), x[B // 2:].contiguous()]
    pos = torch.zeros((B,), dtype=torch.int32, device=dev)
    posh = [torch.zeros((B // 2,), dtype=torch.int32, device=dev) for _ in range(2)]
    streams = [torch.cuda.Stream(dev) for _ in range(2)]

    def run(stages, inp, p, b):
        h = inp
        for s in stages:
            h = s.step(h, p, b, T)
        return h

    def one():
        run(full, x, pos, B)

    def two_seq():
        for i in range(2):
            run(halves[i], xs[i], posh[i], B // 2)

    def two_lanes():
        cur = torch.cuda.current_stream(dev)
        for s in streams:
            s.wait_stream(cur)
        for i in range(2):
            with torch.cuda.stream(streams[i]):
                run(halves[i], xs[i], posh[i], B // 2)
        for s in streams:
            cur.wait_stream(s)

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        best = 1e9
        for _ in range(a.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fn()
            e1.record()
            torch.cuda.synchronize()
            best = min(best, e0.elapsed_time(e1))
        return best

    res = {"model": a.model, "stages": a.stages, "batch": B, "prompt": T}
    for name, fn in (("one_mb", one), ("two_mb_one_stream", two_seq), ("two_mb_two_streams", two_lanes)):
        ms = timed(fn)
        res[name + "_ms"] = round(ms, 3)
        res[name + "_tok_s"] = round(B * T / ms * 1e3, 1)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
