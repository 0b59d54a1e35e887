"""Per-decode-step kernel breakdown from a rocprofv3 kernel trace.

Usage: python tools/prof_step.py gpurun_out/prof/run_kernel_trace.csv (or rocprofv3's run_results.db) [--marker sample_pick] [--last 6]

A decode step ends with the sampler's pick kernel; the last `--last` steady-state steps (no admission,
prefill or slot-metadata uploads) are averaged: per kernel name, calls and GPU time per step, plus the step's wall time (end of one pick to
the end of the next) and the idle share (wall - busy).  Prints a markdown table.
"""
from __future__ import annotations

import argparse
import collections
import csv
import re


def short(name: str) -> str:
    grid = re.search(r" grid=\S+$", name)
    name = re.sub(r"\(.*", "", name) + (grid.group(0) if grid and "(" in name else "")
    name = name.replace("void ", "").replace("dsse::", "")
    return name[:70]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--marker", default="sample_pick")
    ap.add_argument("--last", type=int, default=6)
    ap.add_argument("--by-grid", action="store_true", help="one row per (kernel, grid): separates the projections")
    args = ap.parse_args()
    rows = []
    if args.trace.endswith(".db"):  # rocprofv3's default SQLite output (ROCm 7)
        import sqlite3

        con = sqlite3.connect(args.trace)
        q = "select start, end, name, grid_x, grid_y, workgroup_x from kernels"
        rows = [(int(s), int(e), f"{n} grid={gx // max(1, wx)}x{gy}" if args.by_grid else n)
                for s, e, n, gx, gy, wx in con.execute(q)]
    else:
        with open(args.trace) as f:
            for r in csv.DictReader(f):
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    ends = [i for i, (_, _, n) in enumerate(rows) if args.marker in n]
    # steady-state steps only: no slot-metadata uploads (at most the one token-ring drain copy) and the
    # most common kernel count (admission / finishing steps carry prefill or upload work)
    spans = [(a, b) for a, b in zip(ends[:-1], ends[1:])]
    ncopy = [sum(1 for _, _, n in rows[a + 1:b + 1] if "copyBuffer" in n) for a, b in spans]
    nk = [b - a for a, b in spans]
    mode = collections.Counter(k for k, c in zip(nk, ncopy) if c <= 1).most_common(1)
    steady = [sp for sp, k, c in zip(spans, nk, ncopy) if c <= 1 and mode and k == mode[0][0]]
    if len(steady) < args.last:
        raise SystemExit(f"only {len(steady)} steady-state steps found")
    per = collections.defaultdict(lambda: [0, 0.0])
    wall = busy = 0.0
    for a, b in steady[-args.last:]:
        wall += (rows[b][1] - rows[a][1]) / 1e3
        for s, e, n in rows[a + 1:b + 1]:
            per[short(n)][0] += 1
            per[short(n)][1] += (e - s) / 1e3
            busy += (e - s) / 1e3
    k = args.last
    print(f"decode step: wall {wall / k:.1f} us, kernel busy {busy / k:.1f} us, idle {(wall - busy) / k:.1f} us\n")
    print("| kernel | calls/step | us/step | % of busy |")
    print("|---|---|---|---|")
    for n, (c, t) in sorted(per.items(), key=lambda kv: -kv[1][1]):
        print(f"| `{n}` | {c / k:.0f} | {t / k:.1f} | {100 * t / busy:.1f} |")


if __name__ == "__main__":
    main()
