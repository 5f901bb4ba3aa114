#!/usr/bin/env python3
"""Kernel-boundary cost of a decode run from a rocprofv3 ``--kernel-trace``
database or csv: over the kernels after the last prefill attention launch (the decode
graphs), the span, the summed kernel time, the idle gaps between consecutive
kernels (the per-launch boundary the HIP graph does not hide), and the mean
duration and gap per kernel name.

    python tools/rocprof_gaps.py gpurun_out/prof_dir [--after flash_attn] > profiles/xxx.md
"""
import argparse
import collections
import glob
import os
import re
import sqlite3


def short(name: str) -> str:
    return re.sub(r"\(.*", "", name).replace("void ", "")[:80]


def load(d):
    """(name, start_ns, end_ns) sorted by start, from the sqlite database or
    the csv kernel trace (``--output-format csv``) under ``d``."""
    dbs = glob.glob(os.path.join(d, "**", "*results.db"), recursive=True)
    if dbs:
        con = sqlite3.connect(dbs[0])
        cols = [r[1] for r in con.execute("pragma table_info(kernels)")]
        cs = next(c for c in cols if c.lower() in ("start", "start_ns", "begin", "begin_ns"))
        ce = next(c for c in cols if c.lower() in ("end", "end_ns"))
        return con.execute(f"select name, {cs}, {ce} from kernels order by {cs}").fetchall()
    import csv
    f = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
    with open(f, newline="") as fh:
        rows = [(r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in csv.DictReader(fh)]
    return sorted(rows, key=lambda r: r[1])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--after", default="flash_attn", help="decode region starts after the last kernel matching this")
    ap.add_argument("--detail", default="argmax_final",
                    help="also list every gap after the kernels matching this (sorted, us)")
    args = ap.parse_args()
    rows = load(args.dir)
    last = max((i for i, r in enumerate(rows) if args.after in r[0]), default=-1)
    dec = rows[last + 1:]
    if len(dec) < 2:
        raise SystemExit("no decode region")
    span = dec[-1][2] - dec[0][1]
    busy = sum(e - s for _, s, e in dec)
    gaps = [max(0, dec[i + 1][1] - dec[i][2]) for i in range(len(dec) - 1)]
    print(f"decode region: {len(dec)} kernels, span {span / 1e3:.1f} us, kernel time {busy / 1e3:.1f} us, "
          f"idle between kernels {sum(gaps) / 1e3:.1f} us ({100 * sum(gaps) / span:.1f} %), "
          f"mean gap {sum(gaps) / len(gaps) / 1e3:.2f} us")
    print()
    # the median gap is the steady-state boundary; the mean also carries the
    # few host-side pauses of the timing loop (synchronise, timers)
    srt = sorted(gaps)
    print(f"median gap {srt[len(srt) // 2] / 1e3:.2f} us, gaps under 20 us: "
          f"{sum(g for g in gaps if g < 20e3) / 1e3:.1f} us "
          f"({100 * sum(g for g in gaps if g < 20e3) / span:.1f} % of the span)")
    print()
    per = collections.defaultdict(lambda: [0, 0, []])
    for i, (n, s, e) in enumerate(dec[:-1]):
        p = per[short(n)]
        p[0] += 1
        p[1] += e - s
        p[2].append(gaps[i])
    if args.detail:
        det = sorted(round(gaps[i] / 1e3, 2) for i, (n, _, _) in enumerate(dec[:-1]) if args.detail in n)
        print(f"gaps after `{args.detail}` (sorted, us): {det}")
        print()
    print("| kernel | calls | mean us | mean gap after us | median gap after us |")
    print("|---|---|---|---|---|")
    for n, (c, d, g) in sorted(per.items(), key=lambda kv: -kv[1][1]):
        med = sorted(g)[len(g) // 2]
        print(f"| `{n}` | {c} | {d / c / 1e3:.2f} | {sum(g) / c / 1e3:.2f} | {med / 1e3:.2f} |")


if __name__ == "__main__":
    main()
