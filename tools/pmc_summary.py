#!/usr/bin/env python3
"""Summarise rocprofv3 PMC passes (``-i tools/pmc_*.txt --output-format csv``)
into one markdown table per kernel: counter sums over the large dispatches plus
derived ratios.

    python tools/pmc_summary.py gpurun_out/pmc16 [--min_grid 65536] [--top 4]

Derived (per kernel, summed over its dispatches):
* ``MFMA busy / SIMD-cycle`` = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs * 1024 SIMDs):
  the fraction of every SIMD's cycles the matrix core was busy while the kernel ran;
* ``VALU : MFMA`` instruction ratio; ``LDS conflict %`` = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE;
* ``effective clock`` = GRBM_GUI_ACTIVE / 8 / wall time (MI355X_MICROARCH.md DVFS note).
"""
from __future__ import annotations

import argparse
import collections
import csv
import glob
import os


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--min_grid", type=int, default=65536, help="only dispatches with at least this many threads")
    ap.add_argument("--top", type=int, default=4)
    a = ap.parse_args()
    # per pass: a counter collected in several passes (GRBM_GUI_ACTIVE usually rides along in
    # each) is averaged over them, not summed
    per = collections.defaultdict(lambda: collections.defaultdict(lambda: collections.defaultdict(float)))
    wall = collections.defaultdict(dict)
    for f in sorted(glob.glob(os.path.join(a.dir, "**", "*counter_collection.csv"), recursive=True)):
        for r in csv.DictReader(open(f)):
            if int(r["Grid_Size"]) < a.min_grid:
                continue
            k = r["Kernel_Name"].split("(")[0].replace("void ", "")
            per[k][r["Counter_Name"]][f] += float(r["Counter_Value"])
            wall[k][(f, r["Dispatch_Id"])] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    sums = {k: {c: sum(v.values()) / len(v) for c, v in cs.items()} for k, cs in per.items()}
    kern = sorted(sums, key=lambda k: -sum(wall[k].values()))[: a.top]
    counters = sorted({c for k in kern for c in sums[k]})
    print("| counter | " + " | ".join(f"`{k}`" for k in kern) + " |")
    print("|---|" + "---|" * len(kern))
    for c in counters:
        print(f"| {c} | " + " | ".join(f"{sums[k].get(c, 0):.3g}" for k in kern) + " |")

    def ratio(k, num, den, scale=1.0):
        d = sums[k].get(den, 0)
        return f"{scale * sums[k].get(num, 0) / d:.3g}" if d else "-"

    rows = []
    for k in kern:
        s = sums[k]
        # dispatches of one pass (wall time is duplicated across passes)
        per_pass = collections.defaultdict(float)
        for (f, _), t in wall[k].items():
            per_pass[f] += t
        t = min(per_pass.values()) if per_pass else 0
        ga = s.get("GRBM_GUI_ACTIVE", 0)
        mfma = f"{s['SQ_VALU_MFMA_BUSY_CYCLES'] / (ga / 8 * 1024):.2f}" if ga and "SQ_VALU_MFMA_BUSY_CYCLES" in s else "-"
        clk = f"{ga / 8 / t / 1e9:.2f} GHz" if ga and t else "-"
        # FETCH_SIZE is in KiB; its own pass's wall time (the pass holding FETCH_SIZE)
        fetch = "-"
        if "FETCH_SIZE" in s:
            tf = [per_pass[f] for f in per_pass if any(r_ for r_ in [f] if "p2" in f)] or [t]
            if tf and tf[0] > 0:
                fetch = f"{s['FETCH_SIZE'] * 1024 / tf[0] / 1e12:.2f}"
        rows.append((k, mfma, ratio(k, "SQ_INSTS_VALU", "SQ_INSTS_MFMA"),
                     ratio(k, "SQ_LDS_BANK_CONFLICT", "SQ_LDS_IDX_ACTIVE", 100), clk, fetch))
    print()
    print("| kernel | MFMA busy / SIMD-cycle | VALU : MFMA | LDS conflict % | effective clock | HBM fetch TB/s (profiled) |")
    print("|---|---|---|---|---|---|")
    for r in rows:
        print("| `" + r[0] + "` | " + " | ".join(r[1:]) + " |")


if __name__ == "__main__":
    main()
