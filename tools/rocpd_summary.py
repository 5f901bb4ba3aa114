#!/usr/bin/env python3
"""Per-kernel table from a rocprofv3 kernel trace in its SQLite (rocpd)
output (``rocprofv3 --kernel-trace -d DIR -o run -- ...`` writes
``DIR/run_results.db`` on ROCm 7.2).

    python tools/rocpd_summary.py DIR/run_results.db [--match REGEX] [--last-ms 50] [--grid]

``--match`` keeps kernels whose name matches; ``--last-ms`` keeps dispatches
that start in the last N ms of the trace (e.g. a decode loop that follows the
setup); ``--grid`` splits rows by grid size (the same kernel at different
shapes).  Prints a markdown table: calls, mean / total us, share.
"""
from __future__ import annotations

import argparse
import re
import sqlite3
from collections import defaultdict


def load(db: str):
    c = sqlite3.connect(db)
    names = {r[0]: r[1] for r in c.execute("select id, kernel_name from rocpd_info_kernel_symbol")}
    rows = c.execute("select kernel_id, start, end, grid_size_x, grid_size_y, workgroup_size_x "
                     "from rocpd_kernel_dispatch order by start").fetchall()
    return [(names.get(k, str(k)), s, e, gx, gy, wx) for k, s, e, gx, gy, wx in rows]


def short(name: str, n: int = 90) -> str:
    name = re.sub(r"\(.*$", "", name)
    return name if len(name) <= n else name[:n]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--match", default=None)
    ap.add_argument("--last-ms", type=float, default=0.0)
    ap.add_argument("--grid", action="store_true")
    a = ap.parse_args()
    rows = load(a.db)
    if not rows:
        raise SystemExit("no kernel dispatches")
    if a.last_ms > 0:
        t_end = max(r[2] for r in rows)
        rows = [r for r in rows if r[1] >= t_end - a.last_ms * 1e6]
    if a.match:
        rx = re.compile(a.match)
        rows = [r for r in rows if rx.search(r[0])]
    agg = defaultdict(list)
    for name, s, e, gx, gy, wx in rows:
        key = (short(name), (gx // max(wx, 1), gy) if a.grid else None)
        agg[key].append((e - s) / 1e3)
    span = (max(r[2] for r in rows) - min(r[1] for r in rows)) / 1e3
    busy = sum(sum(v) for v in agg.values())
    print(f"{len(rows)} dispatches, span {span:.1f} us, kernel time {busy:.1f} us ({100 * busy / span:.1f} % busy)\n")
    print("| kernel | grid | calls | mean us | total us | share |")
    print("|---|---|---|---|---|---|")
    for (name, grid), v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
        print(f"| `{name}` | {grid if grid else ''} | {len(v)} | {sum(v) / len(v):.2f} | {sum(v):.1f} | "
              f"{100 * sum(v) / busy:.1f}% |")


if __name__ == "__main__":
    main()
