"""Root-cause probe of the one-shot decode GEMM race (VERDICT r5 item 2;
csrc/kernels/gemm_oneshot.h "Retiring the image").

Symptom (profiles/r5_oneshot_race_screen_*.jsonl): in ~1 of 150 forced
LN + GELU calls at 2/1/1 (288 or 384 workgroups, two per CU) one workgroup's
second 16-row tile (rows 16-31 of its m-group) comes out a few bf16 ulp off,
in one 16-column tile; an 82 KB LDS floor (one workgroup per CU) hides it.

Experiments, each a bit-for-bit comparison with a settled reference of the
same launch over ``--iters`` calls, every call preceded by a call on other
activations (the LDS holds someone else's data):

  (a) floors: 0 (the kernel's own 66.5 KB: two workgroups per CU), 72 KB (two
      per CU with an unused tail: an out-of-range LDS write would land in the
      workgroup's own padding) and 82 KB (one per CU);
  (b) the instrumented kernel (ABL 256): the LDS past the kernel's own size is
      filled with a canary at entry and checked at exit (an out-of-range write
      by the workgroup itself), and the row statistics are taken twice from
      the image, right after the image sync (as the product does) and again
      after the MFMAs: early != late means the image changed after it was
      read; per-workgroup records also carry the hardware ids and
      s_memrealtime stamps, so a failing workgroup's co-residents are named;
  (c) the failing records' early / late statistics against the reference
      call's: which of the two is the correct one.
One JSON line per experiment."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

WORDS = 1024  # OS_PROBE_WORDS


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


def experiment(name, N, K, pin, floor, probe, iters, dev):
    from distributed_neural_networks_amd.ops._lib import lib
    from distributed_neural_networks_amd.ops.gemm import set_oneshot_gemm
    set_oneshot_gemm(2, *pin)
    lib().gemm_set_oneshot_lds_floor(floor)
    run, x, x2 = setup(N, K, dev)
    rec = torch.zeros((4096, WORDS), dtype=torch.int32, device=dev) if probe else None
    lib().gemm_set_oneshot_probe(rec.data_ptr() if probe else 0)
    try:
        run(x)
        ref = run(x).clone()
        ref_rec = rec.clone() if probe else None
        nwg = int((ref_rec[:, 15] != 0).sum().item()) + 1 if probe else None  # blockIdx 0 writes 0
        bad_calls, early_late_calls, canary_calls, worst, fails = 0, 0, 0, 0.0, []
        for i in range(iters):
            run(x2)
            o = run(x)
            d = (o.float() - ref.float()).abs()
            mism = bool((d > 0).any())
            el = can = 0
            if probe:
                r = rec[:nwg]
                el = int(r[:, 10:14].sum().item())
                can = int(r[:, 6:10].sum().item())
                early_late_calls += el > 0
                canary_calls += can > 0
            if mism:
                bad_calls += 1
                worst = max(worst, d.max().item())
            if (mism or el or can) and len(fails) < 8:
                nz = (d > 0).nonzero()
                f = {"call": i, "out_mismatch": mism, "n": int(nz.shape[0]),
                     "rows": sorted(set(nz[:, 0].tolist()))[:32], "col16_tiles": sorted(set((nz[:, 1] // 16).tolist())),
                     "max": d.max().item()}
                if probe:
                    f.update(analyse(rec[:nwg].cpu(), ref_rec[:nwg].cpu()))
                fails.append(f)
        return {"exp": name, "N": N, "K": K, "pin": list(pin), "lds_floor": floor, "probe": probe, "iters": iters,
                "workgroups": nwg, "mismatched_calls": bad_calls, "max": worst,
                "early_late_calls": early_late_calls, "canary_calls": canary_calls, "fails": fails}
    finally:
        lib().gemm_set_oneshot_probe(0)


def analyse(r, ref):
    """Which workgroups / waves / tiles saw early != late, how each compares
    with the reference call's statistics, and who shared their CU."""
    out = {"wg_early_late": [], "wg_canary": []}
    keys = [cu_key(r[i]) for i in range(r.shape[0])]
    span = [(stamp(r[i], 2), stamp(r[i], 4)) for i in range(r.shape[0])]
    for lg in range(r.shape[0]):
        el = r[lg, 10:14].tolist()
        if any(el):
            f = r[lg, 16:16 + 4 * 2 * 16 * 4].view(torch.float32).view(4, 2, 16, 4)
            fr = ref[lg, 16:16 + 4 * 2 * 16 * 4].view(torch.float32).view(4, 2, 16, 4)
            waves = []
            for w in range(4):
                for t in range(2):
                    e, late, refv = f[w, t, :, :2], f[w, t, :, 2:], fr[w, t, :, :2]
                    de = (e - refv).abs().max().item()
                    dl = (late - refv).abs().max().item()
                    if de > 0 or dl > 0:
                        rows = ((e - refv).abs().sum(1) > 0).nonzero().flatten().tolist()
                        waves.append({"wave": w, "t": t, "early_vs_ref": de, "late_vs_ref": dl,
                                      "rows_early_off": rows, "ref_s1_mean_abs": refv[:, 0].abs().mean().item()})
            co = [j for j in range(r.shape[0]) if j != lg and keys[j] == keys[lg]
                  and span[j][0] < span[lg][1] and span[lg][0] < span[j][1]]
            out["wg_early_late"].append({"lg": lg, "lanes_per_wave": el, "cu": list(keys[lg]),
                                         "co_resident_lg": co, "waves": waves[:8]})
        if any(r[lg, 6:10].tolist()):
            out["wg_canary"].append({"lg": lg, "bad_words_per_wave": r[lg, 6:10].tolist()})
    out["wg_early_late"] = out["wg_early_late"][:6]
    out["wg_canary"] = out["wg_canary"][:6]
    # co-residency census of the whole call
    from collections import Counter
    c = Counter(keys)
    out["cus_used"] = len(c)
    out["max_wg_per_cu"] = max(c.values())
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=2000)
    ap.add_argument("--exps", default="")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    from distributed_neural_networks_amd.ops._lib import lib
    from distributed_neural_networks_amd.ops.gemm import set_oneshot_gemm
    KB = 1024
    exps = [
        # (a) plain product kernel, three floors, two grids
        ("a_2304_floor0", 2304, 768, (2, 1, 1, 1), 0, False),
        ("a_2304_floor72", 2304, 768, (2, 1, 1, 1), 72 * KB, False),
        ("a_2304_floor82", 2304, 768, (2, 1, 1, 1), 82 * KB, False),
        ("a_3072_floor0", 3072, 768, (2, 1, 1, 1), 0, False),
        ("a_3072_floor72", 3072, 768, (2, 1, 1, 1), 72 * KB, False),
        ("a_3072_ntw2_floor0", 3072, 768, (2, 2, 1, 1), 0, False),
        # (b)/(c) instrumented kernel
        ("b_2304_floor72", 2304, 768, (2, 1, 1, 1), 72 * KB, True),
        ("b_3072_floor72", 3072, 768, (2, 1, 1, 1), 72 * KB, True),
        ("b_3072_floor0", 3072, 768, (2, 1, 1, 1), 0, True),
        ("b_3072_ntw2_floor72", 3072, 768, (2, 2, 1, 1), 72 * KB, True),
    ]
    try:
        for name, N, K, pin, floor, probe in exps:
            if a.exps and name not in a.exps.split(","):
                continue
            print(json.dumps(experiment(name, N, K, pin, floor, probe, a.iters, dev)), flush=True)
    finally:
        set_oneshot_gemm(1)
        lib().gemm_set_oneshot_lds_floor(82 * KB)


if __name__ == "__main__":
    main()
