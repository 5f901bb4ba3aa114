#!/usr/bin/env python3
"""Replay determinism of the colocated CIFAR pipeline graph (the headline's
timed region): the probabilities after 1, 2 and 50 graph replays, after other
graphs of the same stages ran in between, and the eager result, all against
the fp32 torch model.  One JSON line.

    python bench/probes/cifar_replay_check.py [--batch 65536]
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
    args = ap.parse_args()
    from distributed_neural_networks_amd import checkpoint as ckpt
    from distributed_neural_networks_amd.models.cifar import NeuralNetwork
    from distributed_neural_networks_amd.runtime.pipeline import ColocatedPipeline
    from distributed_neural_networks_amd.runtime.stages import CifarHipStage
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    sd0 = ckpt.random_stage_state_dict("cifar10", 0, 1, True, False, 0)
    sd1 = ckpt.random_stage_state_dict("cifar10", 2, 3, False, True, 0)
    s0, s1 = CifarHipStage(sd0, 0, 1, dev), CifarHipStage(sd1, 2, 3, dev)
    B = args.batch
    x = torch.randn((B, 3, 32, 32), device=dev, generator=torch.Generator(device=dev).manual_seed(0))
    ref_m = NeuralNetwork().to(dev).eval()
    ref_m.load_state_dict(ckpt.random_stage_state_dict("cifar10", 0, 3, True, True, 0))
    torch.backends.cudnn.allow_tf32 = torch.backends.cuda.matmul.allow_tf32 = False
    with torch.no_grad():
        ref = ref_m(x)
    out = {}
    eager = ColocatedPipeline([s0, s1], B)(x)
    torch.cuda.synchronize()
    out["eager"] = float((eager.probs - ref).abs().max())
    pipe = ColocatedPipeline([s0, s1], B)
    pipe.x.copy_(x)
    pipe.capture()
    for n in (1, 2, 50):
        for _ in range(n if n == 1 else n - (1 if n == 2 else 2)):
            r = pipe()
        torch.cuda.synchronize()
        out[f"replay_{n}"] = float((r.probs - ref).abs().max())
    other = ColocatedPipeline([s0, s1], B // 2)
    other.x.copy_(x[: B // 2])
    other.capture()
    for _ in range(3):
        o = other()
    torch.cuda.synchronize()
    out["other_graph_half_batch"] = float((o.probs - ref[: B // 2]).abs().max())
    r = pipe()
    torch.cuda.synchronize()
    out["replay_after_other"] = float((r.probs - ref).abs().max())
    out["argmax_agreement_after_other"] = float((r.pred.long() == ref.argmax(1)).float().mean())
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
