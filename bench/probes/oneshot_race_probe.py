"""Root-cause probe of the one-shot decode GEMM race (VERDICT r5 item 2;
csrc/kernels/gemm_oneshot.h "Retiring the image").

Symptom (profiles/r5_oneshot_race_screen_*.jsonl): in ~2 % of forced
LN + GELU calls at 2/1/1 (288 or 384 workgroups, two per CU) one workgroup's
second 16-row tile (rows 16-31 of its m-group) comes out a few bf16 ulp off,
in one 16-column tile.  Cause (found with the 32768 dump, see
profiles/r6_oneshot_race_root_cause.md): one element of that tile's row
statistics summed without its shift in lanes 48-63 of one wave -- the SLP
vectoriser's cross-half packed subtract, not the LDS image; the library builds
the kernel with -fno-slp-vectorize (ops/build.py).  Run with
``DNN_HIP_LIB=<an SLP build>`` to see the failure again.

Each experiment compares ``--iters`` calls bit for bit with a settled
reference of the same launch; every call follows a call on other activations
(the LDS holds someone else's bytes).  Probe bits (gemm_oneshot.h) select
instrumented or alternative image syncs; profiles/r6_oneshot_race_root_cause.md
tells the story of the round-6 runs (LDS floors 0 / 72 / 82 KB, an entry
barrier, a detector, CK's split waits, ck_tile's vmcnt-only wait, a short
s_sleep, a second barrier, register-staged images, the dump, the SLP A/B).
One JSON line per experiment."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

WORDS = 1024  # OS_PROBE_WORDS
SAVE_DIR = os.environ.get("RACE_SAVE_DIR", "")


def cu_key(rec):
    hw, xcc = int(rec[0]), int(rec[1])
    return (xcc & 0xF, (hw >> 13) & 0x7, (hw >> 12) & 1, (hw >> 8) & 0xF)


def stamp(rec, i):
    return (int(rec[i]) & 0xFFFFFFFF) | ((int(rec[i + 1]) & 0xFFFFFFFF) << 32)


def setup(N, K, dev):
    from distributed_neural_networks_amd.ops.gemm import attach_shuffled, decode_workspace, fold_norm, linear_norm
    M = 64
    g = torch.Generator(device=dev).manual_seed(N + K)
    x = (torch.randn(M, K, device=dev, generator=g) * 2 + 0.5).bfloat16()
    w = torch.randn(N, K, device=dev, generator=g) / K ** 0.5
    bias = torch.randn(N, device=dev, generator=g)
    x2 = (torch.randn(M, K, device=dev, generator=g) * 3 - 1.0).bfloat16()
    ws = decode_workspace(dev)
    f = fold_norm(w, torch.rand(K, device=dev, generator=g) + 0.5, torch.randn(K, device=dev, generator=g) * 0.1,
                  bias, False, 1e-5, dev, False)
    attach_shuffled(f)
    out = torch.empty((M, N), dtype=torch.bfloat16, device=dev)
    return (lambda a: linear_norm(a, f, act="gelu", ws=ws, out=out)), x, x2


def experiment(name, N, K, pin, floor, abl, iters, dev):
    from distributed_neural_networks_amd.ops._lib import lib
    from distributed_neural_networks_amd.ops.gemm import set_oneshot_gemm
    set_oneshot_gemm(2, *pin)
    lib().gemm_set_oneshot_lds_floor(floor)
    run, x, x2 = setup(N, K, dev)
    det = bool(abl & 256)
    dump = bool(abl & 32768)
    rec = torch.zeros((4096, WORDS if not dump else 2 * 64 * 24), dtype=torch.int32, device=dev)
    check(lib().gemm_set_oneshot_probe(rec.data_ptr() if abl else 0, abl))
    try:
        run(x)
        ref = run(x).clone()
        torch.cuda.synchronize()
        ref_dump = rec.clone() if dump else None
        nwg = int((rec[:, 15] != 0).sum().item()) + 1 if det else None  # blockIdx 0 writes 0
        bad_calls, det_calls, both, worst, fails = 0, 0, 0, 0.0, []
        for i in range(iters):
            run(x2)
            if det:
                rec[:, 16:16 + 256].zero_()
            o = run(x)
            d = (o.float() - ref.float()).abs()
            mism = bool((d > 0).any())
            ev = 0
            if det:
                ev = int((rec[:nwg, 16:16 + 256] != 0).sum().item())
                det_calls += ev > 0
                both += ev > 0 and mism
            if mism:
                bad_calls += 1
                worst = max(worst, d.max().item())
            if (mism or ev) and len(fails) < 8:
                nz = (d > 0).nonzero()
                f = {"call": i, "out_mismatch": mism, "n": int(nz.shape[0]),
                     "rows": sorted(set(nz[:, 0].tolist()))[:32], "col16_tiles": sorted(set((nz[:, 1] // 16).tolist())),
                     "max": d.max().item()}
                if det:
                    f.update(analyse(rec[:nwg].cpu(), pin[1], f["col16_tiles"]))
                if dump and mism:
                    f.update(analyse_dump(rec, ref_dump))
                    if SAVE_DIR:  # the raw records and the activations, for offline forensics
                        import numpy as np
                        tag = f"{SAVE_DIR}/{name}_call{i}"
                        wgs = (rec.view(rec.shape[0], 2, 64, 24)[..., :15] !=
                               ref_dump.view(rec.shape[0], 2, 64, 24)[..., :15]).flatten(1).any(1).nonzero().flatten()
                        np.save(tag + "_wgs.npy", wgs.cpu().numpy())
                        np.save(tag + "_got.npy", rec[wgs].cpu().numpy())
                        np.save(tag + "_ref.npy", ref_dump[wgs].cpu().numpy())
                        np.save(f"{SAVE_DIR}/{name}_x.npy", x.float().cpu().numpy())
                fails.append(f)
        return {"exp": name, "N": N, "K": K, "pin": list(pin), "lds_floor": floor, "abl": abl, "iters": iters,
                "workgroups": nwg, "mismatched_calls": bad_calls, "max": worst, "detector_calls": det_calls,
                "detector_and_output_calls": both, "fails": fails}
    finally:
        lib().gemm_set_oneshot_probe(0, 0)


def check(rc):
    if rc != 0:
        raise RuntimeError(f"probe call failed: {rc}")


FIELDS = ["v0", "v1", "v2", "v3", "a_w0", "a_w1", "a_w2", "a_w3", "q_w0", "q_w1", "q_w2", "q_w3", "shift", "mean",
          "rstd"]


def analyse_dump(rec, ref):
    """Probe bit 32768: which epilogue inputs of which workgroup / lane differ
    from the reference call's (v = the cross-wave GEMM sum, a_w / q_w = the row
    statistics partial of wave w, shift, mean, rstd), with the hardware ids of
    the workgroup and of the wave that wrote the record."""
    a = rec.view(-1, 2, 64, 24).cpu()
    b = ref.view(-1, 2, 64, 24).cpu()
    af, bf = a[..., :15].view(torch.float32), b[..., :15].view(torch.float32)
    diff = (af != bf)
    wgs = diff.any(-1).any(-1).any(-1).nonzero().flatten().tolist()
    out = []
    for lg in wgs[:3]:
        for k in range(2):
            d = diff[lg, k]
            if not bool(d.any()):
                continue
            lanes = d.any(-1).nonzero().flatten().tolist()
            fields = sorted({FIELDS[i] for i in d.any(0).nonzero().flatten().tolist()})
            l0 = lanes[0]
            rel = {FIELDS[i]: (float(af[lg, k, l0, i]), float(bf[lg, k, l0, i])) for i in range(15) if d[l0, i]}
            hw, xcc = int(a[lg, k, l0, 16]), int(a[lg, k, l0, 17])
            wv = int(a[lg, k, l0, 18:19].view(torch.float32))
            out.append({"lg": lg, "slot": k, "q": float(a[lg, k, l0, 15:16].view(torch.float32)), "wave": wv, "lanes": lanes[:16],
                        "n_lanes": len(lanes), "fields": fields, "first_lane_got_vs_ref": rel,
                        "cu": [xcc & 0xF, (hw >> 13) & 7, (hw >> 12) & 1, (hw >> 8) & 0xF, (hw >> 4) & 3]})
    return {"dump_diff_wgs": len(wgs), "dump": out}


def analyse(r, ntw, tiles):
    """Per workgroup whose detector fired: which statistics-pass reads changed
    after they were made, decoded into (row of the m-group, 16-B K slot, the
    LDS slot it sits in, and the DMA instruction / lane that wrote it); plus
    the output tiles of the same call and who shared the CU."""
    out = []
    keys = [cu_key(r[i]) for i in range(r.shape[0])]
    for lg in range(r.shape[0]):
        m = r[lg, 16:16 + 256]
        if not bool((m != 0).any()):
            continue
        reads = []
        for w in range(4):
            for lane in range(64):
                mask = int(m[w * 64 + lane]) & 0xFFFFFFFF
                for bit in range(32):
                    if mask >> bit & 1:
                        c, t = bit // 2, bit % 2
                        fr, fg = lane & 15, lane >> 4
                        row = 16 * t + fr
                        slot = c * 4 + fg                      # 16-B K slot within the wave's 512-B step row
                        phys = slot ^ (row & 15)               # LDS slot it sits in
                        reads.append({"wave": w, "row": row, "k_slot": slot, "lds_slot": phys,
                                      "dma_instr": row // 2, "dma_lane": (row & 1) * 32 + phys})
        mg, rest = lg % 2, lg // 2
        out.append({"lg": lg, "mgroup": mg, "col_tile": rest, "cu": list(keys[lg]),
                    "same_cu_lg": [j for j in range(r.shape[0]) if j != lg and keys[j] == keys[lg]][:8],
                    "n_reads": len(reads), "reads": reads[:12]})
    return {"detector_wgs": out[:4], "n_detector_wgs": len(out)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=2000)
    ap.add_argument("--exps", default="")
    ap.add_argument("--control_iters", type=int, default=3000)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    from distributed_neural_networks_amd.ops._lib import lib
    from distributed_neural_networks_amd.ops.gemm import set_oneshot_gemm
    KB = 1024
    exps = [
        # the product launch (ABL 0), two WG/CU (floors 0 and 72 KB) and one (82 KB)
        ("p0_3072_floor0", 3072, 768, (2, 1, 1, 1), 0, 0),
        ("p0_2304_floor0", 2304, 768, (2, 1, 1, 1), 0, 0),
        ("p0_3072_floor72", 3072, 768, (2, 1, 1, 1), 72 * KB, 0),
        ("p0_2304_floor82", 2304, 768, (2, 1, 1, 1), 82 * KB, 0),
        # epilogue-input dump (32768): the forensics of profiles/r6_oneshot_race_root_cause.md
        ("d32768_3072_floor0", 3072, 768, (2, 1, 1, 1), 0, 32768),
        ("d32768_2304_floor0", 2304, 768, (2, 1, 1, 1), 0, 32768),
        # image-sync variants: the wait and two barriers (16384), CK's split waits (2048)
        ("c16384_3072_floor0", 3072, 768, (2, 1, 1, 1), 0, 16384),
        ("c2048_3072_floor0", 3072, 768, (2, 1, 1, 1), 0, 2048),
    ]
    try:
        for name, N, K, pin, floor, abl in exps:
            if a.exps and name not in a.exps.replace("+", ",").split(","):
                continue
            it = a.control_iters if name.startswith(("c", "d")) else a.iters
            print(json.dumps(experiment(name, N, K, pin, floor, abl, it, dev)), flush=True)
    finally:
        set_oneshot_gemm(1)
        lib().gemm_set_oneshot_lds_floor(0)  # the library default


if __name__ == "__main__":
    main()
