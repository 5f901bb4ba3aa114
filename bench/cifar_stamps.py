"""Diagnostic: per-phase cycle split of stage-0 v3 (s_memtime stamps build).
Prints mean cycles per image for producer (wave 0) and consumer (wave 4):
[phase A, barrier 1 wait, phase B, barrier 2 wait], and the plain kernel's
time, for each producer conv1 tile count ``--pt`` (comma list)."""
import json
import sys

import torch

from distributed_neural_networks_amd.models.cifar import NeuralNetwork
from distributed_neural_networks_amd.ops import cifar as cops
from distributed_neural_networks_amd.ops._lib import lib, ptr, stream_ptr

B = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
PTS = [int(v) for v in (sys.argv[2] if len(sys.argv) > 2 else "24").split(",")]
torch.manual_seed(0)
w = cops.pack_stage0(NeuralNetwork().state_dict(), "cuda")
x = torch.randn(B, 3, 32, 32, device="cuda")
out = torch.empty(B, 4096, dtype=torch.bfloat16, device="cuda")
grid = min(256, B)
for pt in PTS:
    assert lib().cifar_set_v3_pt(pt) == 0
    st = torch.zeros(grid * 2 * 4, dtype=torch.int64, device="cuda")
    for _ in range(3):
        st.zero_()
        lib().cifar_stage0_v3_stamps(ptr(x), ptr(out), ptr(w.w1p2), ptr(w.b1), ptr(w.w2p), ptr(w.b2), B, grid,
                                     ptr(st), stream_ptr())
    torch.cuda.synchronize()
    s = st.view(grid, 2, 4).double().cpu()
    imgs = B / grid
    res = {}
    for role, name in ((0, "producer"), (1, "consumer")):
        m = s[:, role, :].mean(0) / (imgs + 1)
        res[name] = {"phaseA": round(m[0].item()), "barrier1": round(m[1].item()), "phaseB": round(m[2].item()),
                     "barrier2": round(m[3].item())}
    ts = []
    for _ in range(3):
        lib().cifar_stage0_v3(ptr(x), ptr(out), ptr(w.w1p2), ptr(w.b1), ptr(w.w2p), ptr(w.b2), B, grid, stream_ptr())
    for _ in range(10):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        lib().cifar_stage0_v3(ptr(x), ptr(out), ptr(w.w1p2), ptr(w.b1), ptr(w.w2p), ptr(w.b2), B, grid, stream_ptr())
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    ts.sort()
    print(json.dumps({"B": B, "pt": pt, "kernel_ms_median": round(ts[len(ts) // 2], 4),
                      "img_per_s": round(B / ts[len(ts) // 2] * 1e3), "cycles_per_image_per_wave": res}), flush=True)
assert lib().cifar_set_v3_pt(24) == 0
