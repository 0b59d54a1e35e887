"""hipBLASLt default heuristic vs PyTorch TunableOp (each GEMM shape benchmarked over the library's candidate
solutions once, the fastest kept) for the engine's library projections, same operands, one process.

    python tools/bench_tunable.py [--M 8192,1024,512] [--out tunableop_results.csv]

Prints one line per (shape, M) with both times, then writes the tuned solutions to --out (a TunableOp results file
the engine can load: DSSE_TUNABLEOP_FILE).
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

SHAPES = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336)}


def timeit(fn, iters=20):
    fn()
    torch.cuda.synchronize()
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    st.record()
    for _ in range(iters):
        fn()
    en.record()
    torch.cuda.synchronize()
    return st.elapsed_time(en) * 1000.0 / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", default="8192,4096,2048,1024,512,256")
    ap.add_argument("--out", default="tunableop_results.csv")
    ap.add_argument("--max-tuning-ms", type=int, default=300)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    tun = torch.cuda.tunable
    tun.set_filename(a.out, insert_device_ordinal=False)
    tun.set_max_tuning_duration(a.max_tuning_ms)
    g = torch.Generator().manual_seed(0)
    for name, (N, K) in SHAPES.items():
        w = ((torch.rand(N, K, generator=g) * 2 - 1) / 64).bfloat16().to(dev)
        for M in [int(m) for m in a.M.split(",")]:
            x = (torch.rand(M, K, generator=g) * 2 - 1).bfloat16().to(dev)
            out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            fn = lambda: torch.matmul(x, w.t(), out=out)  # noqa: E731
            tun.enable(False)
            base = [timeit(fn) for _ in range(3)]
            tun.enable(True)
            tun.tuning_enable(True)
            fn()  # tunes this shape
            torch.cuda.synchronize()
            tuned = [timeit(fn) for _ in range(3)]
            tun.enable(False)
            b, t = sorted(base)[1], sorted(tuned)[1]
            print(f"{name:8s} M={M:5d} default {b:9.2f} us  tuned {t:9.2f} us  ({100 * (b - t) / b:+.1f} %)", flush=True)
    print(f"results are written to {a.out} at exit (torch.cuda.tunable)", flush=True)


if __name__ == "__main__":
    main()
