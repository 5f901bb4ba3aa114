#!/usr/bin/env python3
"""Per-call kernel sequence from a rocprofv3 ``--kernel-trace`` database: the
calls of one window (the N-th occurrence of a marker kernel onward), with
duration, grid and the gap before each, so the kernels of one layer can be
told apart when they share a template instance.

    python tools/rocprof_seq.py gpurun_out/prof_dir --marker flash_attn --occurrence 3 --count 12
"""
import argparse
import glob
import os
import re
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--marker", default="flash_attn")
    ap.add_argument("--occurrence", type=int, default=3)
    ap.add_argument("--before", type=int, default=2, help="calls listed before the marker")
    ap.add_argument("--count", type=int, default=12)
    args = ap.parse_args()
    db = glob.glob(os.path.join(args.dir, "**", "*results.db"), recursive=True)[0]
    con = sqlite3.connect(db)
    cols = [r[1] for r in con.execute("pragma table_info(kernels)")]
    cs = next(c for c in cols if c.lower() in ("start", "start_ns", "begin", "begin_ns"))
    ce = next(c for c in cols if c.lower() in ("end", "end_ns"))
    gx = next((c for c in cols if c.lower() in ("grid_size_x", "grid_x", "grid_size")), None)
    sel = f"select name, {cs}, {ce}" + (f", {gx}" if gx else "") + f" from kernels order by {cs}"
    rows = con.execute(sel).fetchall()
    hits = [i for i, r in enumerate(rows) if args.marker in r[0]]
    if len(hits) < args.occurrence:
        raise SystemExit(f"marker {args.marker!r} occurs {len(hits)} times")
    i0 = max(0, hits[args.occurrence - 1] - args.before)
    print("| # | kernel | us | grid | gap before us |")
    print("|---|---|---|---|---|")
    for k in range(i0, min(len(rows), i0 + args.count)):
        r = rows[k]
        gap = (r[1] - rows[k - 1][2]) / 1e3 if k > 0 else 0.0
        name = re.sub(r"\(.*", "", r[0]).replace("void ", "")[:70]
        print(f"| {k - i0} | `{name}` | {(r[2] - r[1]) / 1e3:.2f} | {r[3] if gx else ''} | {gap:.2f} |")


if __name__ == "__main__":
    main()
