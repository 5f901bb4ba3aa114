"""Interleaved A/B of CIFAR stage-0 kernel variants in one process (guide §5.4 rule 24)."""
import json
import statistics
import sys

import torch

from distributed_neural_networks_amd.models.cifar import NeuralNetwork, CifarStage
from distributed_neural_networks_amd.ops import cifar as cops


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    # a variant is "V" or "V@PT" (v3/v4: conv1 tiles run by the producer waves)
    variants = (sys.argv[2] if len(sys.argv) > 2 else "3,4").split(",")
    torch.manual_seed(0)
    model = NeuralNetwork().eval()
    sd = model.state_dict()
    w0 = cops.pack_stage0(sd, "cuda")
    x = torch.randn(B, 3, 32, 32, device="cuda")
    outs = {v: torch.empty(B, 4096, dtype=torch.bfloat16, device="cuda") for v in variants}
    ref_mod = CifarStage(0, 1).eval()
    ref_mod.load_state_dict(sd, strict=False)
    with torch.no_grad():
        ref = ref_mod(x[:256].cpu())
    from distributed_neural_networks_amd.ops._lib import lib

    def run(v):
        var, _, pt = v.partition("@")
        if pt:
            assert getattr(lib(), f"cifar_set_v{var}_pt")(int(pt)) == 0
        cops.stage0_forward(x, w0, outs[v], variant=int(var))

    for v in variants:
        run(v)
    torch.cuda.synchronize()
    for v in variants:
        err = ((outs[v][:256].float().cpu() - ref).norm() / ref.norm()).item()
        print(json.dumps({"variant": v, "rel_err_vs_fp32": err}))
    times = {v: [] for v in variants}
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    for rnd in range(12):
        for v in variants:
            ev[0].record()
            for _ in range(5):
                run(v)
            ev[1].record()
            torch.cuda.synchronize()
            times[v].append(ev[0].elapsed_time(ev[1]) / 5)
    for v in variants:
        med = statistics.median(times[v][2:])
        print(json.dumps({"variant": v, "B": B, "ms_median": med, "ms_min": min(times[v]), "img_per_s": B / med * 1e3}))


if __name__ == "__main__":
    main()
