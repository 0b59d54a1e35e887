"""Kernel-time totals from a rocprofv3 trace database: per (kernel, grid) calls and time, divided by --div (e.g.
the number of prefills in the traced run).  Markdown table, heaviest first.

    python tools/prof_sum.py gpurun_out/x/run_results.db --div 3 [--min-us 1]
"""
from __future__ import annotations

import argparse
import collections
import re
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--div", type=float, default=1.0)
    ap.add_argument("--top", type=int, default=30)
    args = ap.parse_args()
    con = sqlite3.connect(args.db)
    per = collections.defaultdict(lambda: [0, 0.0])
    total = 0.0
    for s, e, n, gx, gy, wx in con.execute("select start, end, name, grid_x, grid_y, workgroup_x from kernels"):
        name = re.sub(r"\(.*", "", n).replace("void ", "").replace("dsse::", "")[:60]
        key = f"{name} grid={gx // max(1, wx)}x{gy}"
        per[key][0] += 1
        per[key][1] += (e - s) / 1e3
        total += (e - s) / 1e3
    d = args.div
    print(f"total kernel time {total / d:.1f} us per unit ({d:g} units)\n")
    print("| kernel | calls | us | % |")
    print("|---|---|---|---|")
    for k, (c, t) in sorted(per.items(), key=lambda kv: -kv[1][1])[:args.top]:
        print(f"| `{k}` | {c / d:.1f} | {t / d:.1f} | {100 * t / total:.1f} |")


if __name__ == "__main__":
    main()
