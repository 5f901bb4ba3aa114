"""Quick single-GPU CIFAR-10 2-stage (colocated) throughput probe: per-kernel timing
and HIP-graph replay of one step, across batch sizes."""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from distributed_neural_networks_amd.models.cifar import NeuralNetwork
from distributed_neural_networks_amd.ops import cifar as cops


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", default="1,256,4096,65536")
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--precision", default="fp32", choices=["fp32", "bf16"])
    a = ap.parse_args()
    torch.manual_seed(0)
    sd = NeuralNetwork().state_dict()
    w0, wh = cops.pack_stage0(sd, "cuda", a.precision), cops.pack_head(sd, "cuda", precision=a.precision)
    adt = cops.act_dtype(a.precision)
    res = []
    for B in [int(b) for b in a.batches.split(",")]:
        x = torch.randn(B, 3, 32, 32, device="cuda")
        mid = torch.empty(B, 4096, dtype=adt, device="cuda")
        hid = torch.empty(B, 512, dtype=adt, device="cuda")
        spl = (torch.empty(B, 3 * 4096, dtype=torch.bfloat16, device="cuda")
               if a.precision == "fp32" and B < cops.FC1_X3_MIN_ROWS else None)
        probs = torch.empty(B, 10, device="cuda")
        pred = torch.empty(B, dtype=torch.int32, device="cuda")

        def step():
            cops.stage0_forward(x, w0, mid)
            cops.fc1_forward(mid, wh, hid, scratch=spl)
            cops.head_tail(hid, wh, probs, pred)

        for _ in range(3):
            step()
        torch.cuda.synchronize()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        g = torch.cuda.CUDAGraph()
        with torch.cuda.stream(s):
            step()
            torch.cuda.synchronize()
            with torch.cuda.graph(g, stream=s):
                step()
        torch.cuda.synchronize()
        for _ in range(5):
            g.replay()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.iters):
            g.replay()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / a.iters
        # per-stage timing with events
        e = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
        e[0].record()
        for _ in range(a.iters):
            cops.stage0_forward(x, w0, mid)
        e[1].record()
        for _ in range(a.iters):
            cops.fc1_forward(mid, wh, hid, scratch=spl)
        e[2].record()
        for _ in range(a.iters):
            cops.head_tail(hid, wh, probs, pred)
        e[3].record()
        torch.cuda.synchronize()
        r = {"precision": a.precision, "B": B, "ms_per_step": dt * 1e3, "img_per_s": B / dt,
             "stage0_ms": e[0].elapsed_time(e[1]) / a.iters, "fc1_ms": e[1].elapsed_time(e[2]) / a.iters,
             "tail_ms": e[2].elapsed_time(e[3]) / a.iters}
        print(json.dumps(r), flush=True)
        res.append(r)


if __name__ == "__main__":
    main()
