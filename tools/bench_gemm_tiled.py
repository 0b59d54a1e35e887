"""Tiled LDS-DMA GEMM (gemm_tiled.hip) vs the library GEMM (torch.matmul -> hipBLASLt) at the Mistral-7B
prefill and wide-decode shapes, on the same random bf16 operands, interleaved rounds in one process.

    python tools/bench_gemm_tiled.py [--M 8192,2048,256] [--cfg auto,0,1,2] [--iters 20] [--rounds 3]

Prints one line per (shape, M, kernel) with the median time and TFLOP/s, then a JSON summary.
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from distributed_sse_for_llm_response_amd import ops  # noqa: E402
from distributed_sse_for_llm_response_amd.ops import reference as R  # noqa: E402

SHAPES = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336)}


def timeit(fn, iters):
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    st.record()
    for _ in range(iters):
        fn()
    en.record()
    torch.cuda.synchronize()
    return st.elapsed_time(en) * 1000.0 / iters  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", default="8192,2048,256")
    ap.add_argument("--cfg", default="0")
    ap.add_argument("--shapes", default="qkv,o,gate_up,down")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--no-library", action="store_true")
    args = ap.parse_args()
    ops.load_library(required=True)
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(0)
    res = {}
    for name in args.shapes.split(","):
        N, K = SHAPES[name]
        w = (torch.rand(N, K, generator=g) * 2 - 1).bfloat16().to(dev) / 64
        wt = R.tile_weight(w)
        for M in [int(m) for m in args.M.split(",")]:
            x = (torch.rand(M, K, generator=g) * 2 - 1).bfloat16().to(dev)
            out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            flop = 2.0 * M * N * K
            arms = {}
            if not args.no_library:
                arms["library"] = lambda: torch.matmul(x, w.t(), out=out)
            for cfg in args.cfg.split(","):
                # "auto": the engine's default dispatch for this shape (any kernel family); else a gemm_tiled cfg
                arms["auto" if cfg == "auto" else f"tiled{cfg}"] = lambda: ops.gemm_out(x, wt, out)
            times = {k: [] for k in arms}
            for _ in range(args.rounds):
                for k, fn in arms.items():
                    os.environ.pop("DSSE_KERNEL_CFG", None)
                    if k.startswith("tiled"):
                        os.environ["DSSE_KERNEL_CFG"] = f"gemm_impl=4,t_cfg={k[5:]}"
                    ops.refresh_env()
                    times[k].append(timeit(fn, args.iters))
            for k, ts in times.items():
                us = sorted(ts)[len(ts) // 2]
                tf = flop / us / 1e6
                res[f"{name}_M{M}_{k}"] = {"us": round(us, 2), "tflops": round(tf, 1),
                                           "weight_TBps": round(N * K * 2 / us / 1e6, 3)}
                print(f"{name:8s} M={M:5d} N={N:6d} K={K:6d} {k:10s} {us:10.2f} us {tf:8.1f} TFLOP/s", flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
