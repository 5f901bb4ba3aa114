#!/usr/bin/env python3
"""A/B: the colocated CIFAR 2-stage step serial (one stream, one graph: the
bench headline) vs stage 1 (fc1 + fc2/softmax/argmax) of microbatch m running
on a second stream under stage 0 of microbatch m+1, with the persistent
stage-0 grid leaving ``spare`` CUs free for fc1.  Both
arms are single HIP graphs (the overlapped one forks/joins streams inside the
capture), fp32 (bf16x3) precision, B = 65536 images per step, interleaved
rounds in one process.  Outputs must be identical to the serial arm.

    python bench/probes/cifar_overlap_ab.py [--batch 65536] [--rounds 3] [--steps 20]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=65536)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--arms", default="1x0,2x0,2x16,2x32,4x16,4x32,4x64", help="MxSPARE overlapped arms")
    args = ap.parse_args()
    from distributed_neural_networks_amd import checkpoint as ckpt
    from distributed_neural_networks_amd.ops import cifar as cops
    from distributed_neural_networks_amd.runtime.stages import CifarHipStage
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    sd0 = ckpt.random_stage_state_dict("cifar10", 0, 1, True, False, 0)
    sd1 = ckpt.random_stage_state_dict("cifar10", 2, 3, False, True, 0)
    s0, s1 = CifarHipStage(sd0, 0, 1, dev), CifarHipStage(sd1, 2, 3, dev)
    B = args.batch
    x = torch.randn((B, 3, 32, 32), device=dev, generator=torch.Generator(device=dev).manual_seed(0))
    n_cu = torch.cuda.get_device_properties(dev).multi_processor_count
    side = torch.cuda.Stream(dev)

    def build(M, spare):
        mb = B // M
        hs = [torch.empty((mb, 4096), dtype=torch.float32, device=dev) for _ in range(M)]
        ps = [torch.empty((mb, 10), dtype=torch.float32, device=dev) for _ in range(M)]

        def step():
            cops.set_stage0_grid(n_cu - spare if spare else 0)
            main = torch.cuda.current_stream(dev)
            if M == 1:
                s1.forward(s0.forward(x, hs[0]), ps[0])
                return
            side.wait_stream(main)
            for m in range(M):
                s0.forward(x[m * mb:(m + 1) * mb], hs[m])      # stage 0 chain on the main stream
                ev = torch.cuda.Event()
                ev.record(main)
                side.wait_event(ev)
                with torch.cuda.stream(side):                  # stage 1 of m under stage 0 of m+1
                    s1.forward(hs[m], ps[m])
            main.wait_stream(side)
        for _ in range(2):
            step()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            step()
        cops.set_stage0_grid(0)
        return g, ps

    def timed(g):
        g.replay()
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(args.steps):
            g.replay()
        b.record()
        torch.cuda.synchronize()
        return a.elapsed_time(b) / args.steps

    from distributed_neural_networks_amd.runtime.pipeline import ColocatedPipeline
    ref = ColocatedPipeline([s0, s1], B)(x).probs.clone()  # eager, serial: what every arm must reproduce
    torch.cuda.synchronize()
    arms = {}
    for a in args.arms.split(","):
        M, spare = (int(v) for v in a.split("x"))
        arms[a] = build(M, spare)
    res = {a: [] for a in arms}
    for _ in range(args.rounds):
        for a, (g, ps) in arms.items():
            res[a].append(round(timed(g), 4))
            p = torch.cat(ps)
            d = float((p - ref).abs().max())
            res[a + "_maxdiff_vs_eager"] = max(res.get(a + "_maxdiff_vs_eager", 0.0), d)
    out = {"batch": B, "ms_per_step": res,
           "img_per_s": {a: round(B / (min(v) / 1e3), 1) for a, v in res.items() if isinstance(v, list)}}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
