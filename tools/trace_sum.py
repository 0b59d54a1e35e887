"""Per-kernel totals from a rocprofv3 `--kernel-trace --output-format csv` run (run_kernel_trace.csv).

    python tools/trace_sum.py gpurun_out/x/prof/run_kernel_trace.csv --div 3 [--after-kernel flash_prefill]
        [--skip 'normal_|uniform_|fill_'] [--top 30] [--unit-kernel decode_prep --last 6 [--skip-last 20]]

Groups dispatches by (kernel, grid), divides by --div (e.g. the number of timed prefills) and prints a markdown
table, heaviest first.  --skip drops kernels by regex (the random weight initialisation of a benchmark's setup, torch
fills); --after-kernel drops every dispatch before the first one whose name matches (the setup and warm-up), so the
table is the steady-state work only; --unit-kernel R --last N keeps the last N units (each starting at a dispatch
matching R, e.g. the last 6 decode steps) and divides by N.
"""
from __future__ import annotations

import argparse
import collections
import csv
import re


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--div", type=float, default=1.0)
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("--skip", default=r"normal_kernel|uniform_kernel|random_|FillFunctor|distribution_")
    ap.add_argument("--after-kernel", default="")
    ap.add_argument("--title", default="")
    ap.add_argument("--unit-kernel", default="",
                    help="with --last: a unit starts at each dispatch matching this regex (e.g. decode_prep)")
    ap.add_argument("--last", type=int, default=0, help="keep only the last N complete units (sets --div to N)")
    ap.add_argument("--skip-last", type=int, default=0, help="with --last: ... that end this many units before the end")
    args = ap.parse_args()
    rows = sorted(csv.DictReader(open(args.csv, newline="")), key=lambda r: int(r["Start_Timestamp"]))
    if args.after_kernel:
        pat = re.compile(args.after_kernel)
        first = next((i for i, r in enumerate(rows) if pat.search(r["Kernel_Name"])), 0)
        rows = rows[first:]
    if args.unit_kernel and args.last:
        pat = re.compile(args.unit_kernel)
        starts = [i for i, r in enumerate(rows) if pat.search(r["Kernel_Name"])]
        k = args.skip_last
        if len(starts) > args.last + k:
            rows = rows[starts[-args.last - 1 - k]:starts[-1 - k]]
            args.div = float(args.last)
    skip = re.compile(args.skip) if args.skip else None
    per = collections.defaultdict(lambda: [0, 0.0])
    total = 0.0
    span0, span1 = None, None
    for r in rows:
        name = r["Kernel_Name"]
        if skip and skip.search(name):
            continue
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        span0 = s if span0 is None else min(span0, s)
        span1 = e if span1 is None else max(span1, e)
        short = re.sub(r"\(.*", "", name).replace("void ", "").replace("dsse::", "")[:70]
        gx, wx = int(r.get("Grid_Size_X") or 0), max(1, int(r.get("Workgroup_Size_X") or 1))
        key = f"{short} grid={gx // wx}x{r.get('Grid_Size_Y', '1')}"
        per[key][0] += 1
        per[key][1] += (e - s) / 1e3
        total += (e - s) / 1e3
    d = args.div
    if args.title:
        print(f"# {args.title}\n")
    print(f"kernel time {total / d:.1f} us per unit ({d:g} units); first-to-last dispatch span "
          f"{(span1 - span0) / 1e3 / d if span0 is not None else 0:.1f} us per unit\n")
    print("| kernel | calls / unit | us / unit | % |")
    print("|---|---|---|---|")
    for k, (c, t) in sorted(per.items(), key=lambda kv: -kv[1][1])[:args.top]:
        print(f"| `{k}` | {c / d:.1f} | {t / d:.1f} | {100 * t / max(total, 1e-9):.1f} |")


if __name__ == "__main__":
    main()
