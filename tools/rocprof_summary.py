#!/usr/bin/env python3
"""Summarise a rocprofv3 run (``--kernel-trace --stats``) into a markdown table.

Reads the ``*_results.db`` (rocpd SQLite, ROCm 7.2 default output) or a
``kernel_stats.csv`` and prints per-kernel calls / total / mean / share, plus
registers and LDS from the dispatch records.

    python tools/rocprof_summary.py gpurun_out/prof1 > profiles/xxx.md
"""
import csv
import glob
import os
import re
import sqlite3
import sys


def short(name: str) -> str:
    name = re.sub(r"\(.*", "", name)
    return name.replace("void ", "")[:90]


def from_db(path):
    con = sqlite3.connect(path)
    rows = con.execute("select name, count(*), sum(duration), avg(duration), max(vgpr_count), max(accum_vgpr_count),"
                       " max(lds_size), max(grid_x), max(workgroup_x) from kernels group by name"
                       " order by sum(duration) desc").fetchall()
    tot = sum(r[2] for r in rows) or 1
    out = ["| kernel | calls | total us | mean us | share | VGPR | AGPR | LDS B | max grid_x | wg |",
           "|---|---|---|---|---|---|---|---|---|---|"]
    for n, c, s, a, v, ag, lds, gx, wg in rows:
        out.append(f"| `{short(n)}` | {c} | {s / 1e3:.1f} | {a / 1e3:.2f} | {100 * s / tot:.1f}% | {v} | {ag} | {lds} | {gx} | {wg} |")
    return "\n".join(out)


def from_csv(path):
    rows = list(csv.DictReader(open(path)))
    out = ["| kernel | calls | total us | mean us | share |", "|---|---|---|---|---|"]
    for r in rows:
        out.append(f"| `{short(r['Name'])}` | {r['Calls']} | {float(r['TotalDurationNs']) / 1e3:.1f} | "
                   f"{float(r['AverageNs']) / 1e3:.2f} | {float(r['Percentage']):.1f}% |")
    return "\n".join(out)


def main(d):
    dbs = glob.glob(os.path.join(d, "**", "*results.db"), recursive=True)
    if dbs:
        print(from_db(dbs[0]))
        return
    csvs = glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True)
    if csvs:
        print(from_csv(csvs[0]))
        return
    raise SystemExit(f"no rocprofv3 output under {d}")


if __name__ == "__main__":
    main(sys.argv[1])
