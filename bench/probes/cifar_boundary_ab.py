"""In-process A/B of the fp32 CIFAR 2-stage pipeline (bench.py's colocated
headline step, B=65536, HIP graph) with the plain fp32 boundary vs the blocked
hi/lo boundary encoding.  Prints one JSON line: ms/step and img/s per variant
(min over interleaved rounds) and whether the probabilities match bitwise."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    from distributed_neural_networks_amd import checkpoint as ckpt
    from distributed_neural_networks_amd.runtime.pipeline import ColocatedPipeline
    from distributed_neural_networks_amd.runtime.stages import CifarHipStage
    dev = torch.device("cuda", 0)
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    sd0 = ckpt.random_stage_state_dict("cifar10", 0, 1, True, False, 0)
    sd1 = ckpt.random_stage_state_dict("cifar10", 2, 3, False, True, 0)
    x = torch.randn(B, 3, 32, 32, device=dev)
    pipes = {}
    for bd in ("fp32", "split"):
        p = ColocatedPipeline([CifarHipStage(sd0, 0, 1, dev, boundary=bd), CifarHipStage(sd1, 2, 3, dev, boundary=bd)], B)
        p.x.copy_(x)
        p.capture()
        pipes[bd] = p
    times = {k: [] for k in pipes}
    for _ in range(4):
        for k, p in pipes.items():
            for _ in range(3):
                p()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                p()
            e1.record()
            torch.cuda.synchronize()
            times[k].append(e0.elapsed_time(e1) / 20)
    res = {"B": B}
    for k, v in times.items():
        res[f"{k}_ms"] = round(min(v), 4)
        res[f"{k}_img_s"] = round(B / min(v) * 1e3, 1)
    outs = {k: p() for k, p in pipes.items()}
    torch.cuda.synchronize()
    res["probs_bitwise_equal"] = bool(torch.equal(outs["fp32"].probs, outs["split"].probs))
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
