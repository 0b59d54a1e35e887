"""Library-GEMM shapes of the engine (prefill and the >64-sequence decode path) under hipBLASLt defaults vs
PyTorch TunableOp (which times every hipBLASLt / rocBLAS solution per shape and keeps the fastest).

    python tools/tune_blas.py [--M 256,8192] [--tunableop-file profiles/tunableop_gfx950.csv]

Without the TunableOp environment it reports the default-heuristic times; with
``PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_FILENAME=<file>`` it tunes and
writes the results file that the serving process later loads (tuning off, results on).
"""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", default="256,8192")
    ap.add_argument("--iters", type=int, default=20)
    args = ap.parse_args()
    import torch

    dev = torch.device("cuda", 0)
    H, F, V = 4096, 14336, 32768
    shapes = {"qkv": (6144, H), "o": (H, H), "gate_up": (2 * F, H), "down": (H, F)}
    out = {}
    for M in [int(m) for m in args.M.split(",")]:
        for name, (N, K) in shapes.items():
            x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
            ws = [torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02 for _ in range(max(2, (600 << 20) // (N * K * 2) + 1))]
            for i in range(3):
                torch.matmul(x, ws[i % len(ws)].t())
            torch.cuda.synchronize()
            st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            st.record()
            for i in range(args.iters):
                torch.matmul(x, ws[i % len(ws)].t())
            en.record()
            torch.cuda.synchronize()
            us = st.elapsed_time(en) * 1000 / args.iters
            tf = 2 * M * N * K / us / 1e6
            out[f"{name}_M{M}"] = {"us": round(us, 2), "tflops": round(tf, 1), "weight_TBps": round(N * K * 2 / us / 1e6, 3)}
            print(f"{name:8s} M={M:5d} N={N:6d} K={K:6d} {us:9.2f} us {tf:7.1f} TFLOP/s", flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
