"""Offline forensics of the one-shot GEMM "race" dumps (CPU; no GPU).

Input: the records bench/probes/oneshot_race_probe.py saves with
``RACE_SAVE_DIR`` for probe bit 32768 (per differing workgroup: the epilogue's
inputs of both 16-row tiles for every lane -- the cross-wave GEMM sum, the four
waves' row-statistics partials a_w = sum(x - shift), q_w = sum((x - shift)^2),
the shift, mean, rstd -- of the failing call and of the settled reference
call) plus the activations x.

For every (call, workgroup, wave, row) whose partial differs the script tests
one hypothesis: ONE element x_k of the wave's own K range was summed as x_k
instead of x_k - shift.  Then delta a == shift exactly and
delta q == x_k^2 - (x_k - shift)^2, so x_k = (delta q + shift^2) / (2 shift)
must be an element of that row inside the wave's range -- and, if the
mechanism is one instruction, the SAME position k for all 16 rows of the
wave.  Prints one line per failing wave: k, its 16-B slot (k // 8 -> c = slot
// 4 the LDS step chunk, fg = slot % 4 the lane group, lanes 16 fg .. 16 fg + 15),
the element within the slot, and how many of the 16 rows agree.

    python bench/probes/oneshot_race_forensics.py [DIR]   (default profiles/r6_race_dump)
"""
import glob
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(d):
    out = []
    for xf in sorted(glob.glob(os.path.join(d, "*_x.npy"))):
        exp = os.path.basename(xf)[:-len("_x.npy")]
        x = np.load(xf).astype(np.float64)
        M, K = x.shape
        kw = K // 4  # each wave's K range
        for f in sorted(glob.glob(os.path.join(d, f"{exp}_call*_wgs.npy"))):
            call = int(f.split("_call")[1].split("_")[0])
            wgs = np.load(f)
            got = np.load(f.replace("_wgs", "_got")).view(np.float32).reshape(-1, 2, 64, 24)
            ref = np.load(f.replace("_wgs", "_ref")).view(np.float32).reshape(-1, 2, 64, 24)
            for n, lg in enumerate(wgs):
                mg = int(lg) % 2
                for slot in range(2):
                    g, r = got[n, slot], ref[n, slot]
                    if not (g[:, :15] != r[:, :15]).any():
                        continue
                    t = int(round(float(r[0, 15]))) % 2
                    for w in range(4):
                        ks, exact, rows = [], 0, 0
                        for lane in range(16):
                            row = mg * 32 + 16 * t + lane
                            s = x[row, 0]
                            da = float(g[lane, 4 + w]) - float(r[lane, 4 + w])
                            dq = float(g[lane, 8 + w]) - float(r[lane, 8 + w])
                            if da == 0 and dq == 0:
                                continue
                            rows += 1
                            exact += da == s
                            xk = (dq + s * s) / (2 * s)
                            rng = x[row, w * kw:(w + 1) * kw]
                            ks.append(set(np.nonzero(np.abs(rng - xk) < 1e-2 * max(1.0, abs(xk)))[0].tolist()))
                        if not rows:
                            continue
                        common = set.intersection(*ks) if ks else set()
                        k = min(common) if common else None
                        line = {"exp": exp, "call": call, "wg": int(lg), "tile_t": t, "wave": w, "rows": rows,
                                "delta_a_equals_shift": f"{exact}/{rows}", "k_common_to_all_rows": sorted(common)}
                        if k is not None:
                            line.update({"slot16": k // 8, "chunk_c": (k // 8) // 4, "lane_group": (k // 8) % 4,
                                         "element_in_slot": k % 8, "low_half_of_dword": k % 2 == 0})
                        out.append(line)
    import json
    for l in out:
        print(json.dumps(l))
    n = len(out)
    pinned = [l for l in out if l["k_common_to_all_rows"]]
    print(json.dumps({"failing_waves": n, "one_unshifted_element_all_rows": len(pinned),
                      "delta_a_exact_all_rows": sum(l["delta_a_equals_shift"].split("/")[0] ==
                                                    l["delta_a_equals_shift"].split("/")[1] for l in out),
                      "lane_groups": sorted({l.get("lane_group") for l in pinned}),
                      "tiles_t": sorted({l["tile_t"] for l in out}),
                      "elements_in_slot": sorted({l.get("element_in_slot") for l in pinned})}))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "profiles", "r6_race_dump"))
