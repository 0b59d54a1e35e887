"""Per-kernel PMC averages from rocprofv3 `--pmc ... --output-format csv` runs (one or more passes).

    python tools/pmc_sum.py gpurun_out/x/pmc_a gpurun_out/x/pmc_b [--kernel flash_prefill] [--title ...]

Every `*counter_collection.csv` under the given directories is read; rows are grouped by (kernel, grid) and each
counter is averaged per dispatch.  Prints a markdown table (kernel, grid, VGPRs, dispatches, counter, value) and
the derived ratios the GEMM / attention tuning reads: MFMA busy share of the SIMD cycles, wait share of the wave
cycles, LDS bank-conflict share of the LDS cycles.  Kernels whose names do not match --kernel (regex) are
dropped, so the weight-init and random-fill kernels of a benchmark's setup never enter the table.
"""
from __future__ import annotations

import argparse
import collections
import csv
import glob
import os
import re


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--kernel", default=".")
    ap.add_argument("--title", default="PMC counters")
    ap.add_argument("--cus", type=int, default=256)
    ap.add_argument("--ghz", type=float, default=2.4, help="shader clock for the MFMA-busy share")
    args = ap.parse_args()
    pat = re.compile(args.kernel)
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    meta = {}
    dur = collections.defaultdict(list)
    for d in args.dirs:
        for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(path, newline="") as f:
                for row in csv.DictReader(f):
                    name = row.get("Kernel_Name", "")
                    if not pat.search(name):
                        continue
                    short = re.sub(r"\(.*", "", name).replace("void ", "").replace("dsse::", "")[:70]
                    key = (short, row.get("Grid_Size", "?"))
                    meta[key] = (row.get("VGPR_Count", "?"), row.get("Accum_VGPR_Count", "?"),
                                 row.get("LDS_Block_Size", "?"))
                    vals[key][row["Counter_Name"]].append(float(row["Counter_Value"]))
                    if row.get("Start_Timestamp") and row.get("End_Timestamp"):
                        dur[key].append((float(row["End_Timestamp"]) - float(row["Start_Timestamp"])) / 1e3)
    print(f"# {args.title}\n")
    print("| kernel | grid | VGPR/AGPR | LDS | counter | dispatches | per dispatch |")
    print("|---|---|---|---|---|---|---|")
    for key, counters in vals.items():
        v, a, lds = meta[key]
        for c in sorted(counters):
            xs = counters[c]
            print(f"| `{key[0]}` | {key[1]} | {v}/{a} | {lds} | {c} | {len(xs)} | {sum(xs) / len(xs):,.0f} |")
    print()
    for key, counters in vals.items():
        avg = {c: sum(xs) / len(xs) for c, xs in counters.items()}
        notes = []
        if dur[key]:
            us = sorted(dur[key])[len(dur[key]) // 2]
            notes.append(f"median dispatch {us:,.1f} us (profiled clock)")
            if "SQ_VALU_MFMA_BUSY_CYCLES" in avg:
                # summed over the SIMDs: share of 4 x CUs SIMDs x the dispatch's cycles at --ghz
                share = avg["SQ_VALU_MFMA_BUSY_CYCLES"] / (4 * args.cus * us * 1e3 * args.ghz)
                notes.append(f"MFMA busy share of SIMD cycles ~ {share:.2f} (at {args.ghz} GHz)")
        if "SQ_WAIT_INST_ANY" in avg and "SQ_WAVE_CYCLES" in avg and avg["SQ_WAVE_CYCLES"] > 0:
            notes.append(f"wait-on-dependency share of wave time = {avg['SQ_WAIT_INST_ANY'] / avg['SQ_WAVE_CYCLES']:.2f}")
        if "SQ_ACTIVE_INST_ANY" in avg and "SQ_WAVE_CYCLES" in avg and avg["SQ_WAVE_CYCLES"] > 0:
            notes.append(f"issuing share of wave time = {avg['SQ_ACTIVE_INST_ANY'] / avg['SQ_WAVE_CYCLES']:.2f}")
        if "SQ_LDS_BANK_CONFLICT" in avg and "SQ_LDS_IDX_ACTIVE" in avg and avg["SQ_LDS_IDX_ACTIVE"] > 0:
            notes.append(f"LDS bank-conflict share of LDS cycles = "
                         f"{avg['SQ_LDS_BANK_CONFLICT'] / avg['SQ_LDS_IDX_ACTIVE']:.2f}")
        if "SQ_INSTS_MFMA" in avg and "SQ_WAVES" in avg and avg["SQ_WAVES"] > 0:
            notes.append(f"MFMAs per wave = {avg['SQ_INSTS_MFMA'] / avg['SQ_WAVES']:,.0f}")
        if notes:
            print(f"- `{key[0]}` grid {key[1]}: " + "; ".join(notes))


if __name__ == "__main__":
    main()
