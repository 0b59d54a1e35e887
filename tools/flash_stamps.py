"""Phase anatomy of the flash prefill kernel from its diagnostic stamps (DSSE_FLASH_STAMPS, attention_prefill.hip).

    DSSE_FLASH_STAMPS=/tmp/fs.bin python tools/bench_prefill_attn.py --T 8192 && python tools/flash_stamps.py /tmp/fs.bin

The file holds [32 workgroups][8 waves][128 blocks][6] u32 shader-clock values per key block: a = before the barrier
in front of QKᵀ, b = after it, c = after QKᵀ, d = after the barrier in front of softmax + PV, e = after the DMA issue
of block j + 3, f = after the softmax (the next block's a closes PV).  Prints, per query half (leading waves 0-3, lagging waves 4-7), the median cycles per block of
each segment over the steady blocks (the first 4 and the last 2 of each wave are skipped).
"""
import argparse

import numpy as np


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--wgs", type=int, default=32)
    args = ap.parse_args()
    raw = np.fromfile(args.path, dtype=np.uint32).reshape(args.wgs, 8, 128, 6).astype(np.int64)
    rows = {"leading (w 0-3)": [], "lagging (w 4-7)": []}
    for g in range(args.wgs):
        for w in range(8):
            st = raw[g, w]
            n = int((st[:, 0] != 0).sum())
            if n < 8:
                continue
            a, b, c, d, e, f = (st[:n, i] for i in range(6))
            a_next = np.append(a[1:], np.nan)
            seg = np.stack([b - a, c - b, d - c, e - d, f - e, a_next - f, a_next - a], axis=1)[4:n - 2]
            seg = seg % (1 << 32)  # 32-bit clock wrap
            rows["leading (w 0-3)" if w < 4 else "lagging (w 4-7)"].append(seg)
    print("| half | barrier before QK | QK | barrier before SM+PV | DMA issue | softmax | PV | block |")
    print("|---|---|---|---|---|---|---|---|")
    for k, v in rows.items():
        if not v:
            continue
        m = np.median(np.concatenate(v), axis=0)
        print(f"| {k} | " + " | ".join(f"{x:.0f}" for x in m) + " |")


if __name__ == "__main__":
    main()
