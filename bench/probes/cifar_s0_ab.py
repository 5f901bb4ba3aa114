"""Interleaved in-process A/B of a stage-0 kernel switch (box-to-box clock
differences cancel): stage-0 time at B=65536 for each setting, plus the
max |difference| of the two outputs (must be 0).  One JSON line.

    python bench/probes/cifar_s0_ab.py [--switch wide_store] [--batch 65536]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from distributed_neural_networks_amd.models.cifar import NeuralNetwork  # noqa: E402
from distributed_neural_networks_amd.ops import _lib, cifar as cops  # noqa: E402

SWITCHES = {"wide_store": lambda v: _lib.lib().cifar_s0_set_wide_store(v)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--switch", default="wide_store")
    ap.add_argument("--batch", type=int, default=65536)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    torch.manual_seed(0)
    sd = NeuralNetwork().state_dict()
    w0 = cops.pack_stage0(sd, "cuda")
    x = torch.randn(a.batch, 3, 32, 32, device="cuda")
    outs = {v: torch.empty(a.batch, 4096, device="cuda") for v in (0, 1)}
    times = {0: [], 1: []}
    for _ in range(a.rounds):
        for v in (0, 1):
            assert SWITCHES[a.switch](v) == 0
            cops.stage0_forward(x, w0, outs[v])
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                cops.stage0_forward(x, w0, outs[v])
            e1.record()
            torch.cuda.synchronize()
            times[v].append(e0.elapsed_time(e1) / a.iters)
    SWITCHES[a.switch](1)
    print(json.dumps({"switch": a.switch, "B": a.batch,
                      **{f"{a.switch}{v}_ms": round(sorted(t)[len(t) // 2], 4) for v, t in times.items()},
                      "max_abs_diff": (outs[0] - outs[1]).abs().max().item()}), flush=True)


if __name__ == "__main__":
    main()
