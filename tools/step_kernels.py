"""Per-kernel breakdown of steady decode steps from a rocprofv3 kernel trace, one row per (kernel, grid).

    python tools/step_kernels.py gpurun_out/prof/run_kernel_trace.csv [LAST] [tail | has=SUBSTRING]

A step ends with the sampler's pick kernel.  The steps with the most common kernel count are steady (admission and
finishing steps carry prefill or upload work); the last LAST (default 6) of them are averaged: calls, us per step and
us per call per kernel, plus the steps' wall (pick to pick) and busy time.  Prints a markdown table.
"""
import collections
import csv
import re
import sys


def main():
    path = sys.argv[1]
    last = int(sys.argv[2]) if len(sys.argv) > 2 else 6
    tail = len(sys.argv) > 3 and sys.argv[3] == "tail"
    has = sys.argv[3][4:] if len(sys.argv) > 3 and sys.argv[3].startswith("has=") else None
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            wg = max(1, int(r.get("Workgroup_Size_X") or 1))
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"],
                         int(r.get("Grid_Size_X") or 0) // wg, int(r.get("Grid_Size_Y") or 0)))
    rows.sort()
    ends = [i for i, r in enumerate(rows) if "sample_pick" in r[2]]
    spans = list(zip(ends[:-1], ends[1:]))
    if not spans:
        raise SystemExit("no decode steps (sample_pick) in the trace")
    if has is not None:
        def label(k):
            return re.sub(r"\(.*", "", k[2]).replace("void ", "").replace("dsse::", "")[:55] + f" grid={k[3]}x{k[4]}"
        spans = [(a, b) for a, b in spans if any(has in label(k) for k in rows[a + 1:b + 1])]
        if not spans:
            raise SystemExit(f"no step has a kernel matching {has!r}")
    mode = collections.Counter(b - a for a, b in spans).most_common(1)[0][0]
    if tail:
        steady = spans[-last:]
        mode = collections.Counter(b - a for a, b in steady).most_common(1)[0][0]
        steady = [s for s in steady if s[1] - s[0] == mode]
    else:
        steady = [s for s in spans if s[1] - s[0] == mode][-last:]
    per = collections.defaultdict(lambda: [0, 0.0])
    wall = 0.0
    for a, b in steady:
        wall += (rows[b][1] - rows[a][1]) / 1e3
        for k in rows[a + 1:b + 1]:
            name = re.sub(r"\(.*", "", k[2]).replace("void ", "").replace("dsse::", "")[:55]
            key = f"{name} grid={k[3]}x{k[4]}"
            per[key][0] += 1
            per[key][1] += (k[1] - k[0]) / 1e3
    n = len(steady)
    busy = sum(v[1] for v in per.values()) / n
    print(f"{n} steps of {mode} kernels: wall {wall / n:.1f} us, busy {busy:.1f} us")
    print("| kernel | calls/step | us/step | us/call |\n|---|---|---|---|")
    for k, v in sorted(per.items(), key=lambda kv: -kv[1][1]):
        print(f"| `{k}` | {v[0] / n:.1f} | {v[1] / n:.1f} | {v[1] / v[0]:.2f} |")


if __name__ == "__main__":
    main()
