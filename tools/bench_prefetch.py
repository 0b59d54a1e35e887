#!/usr/bin/env python3
"""Does a weight matrix read from the Infinity Cache (MALL) make a decode GEMM faster, and can the prefetch run
beside another kernel?  (Round-3 experiment for cross-kernel weight prefetch.)

    python tools/bench_prefetch.py [--rows 64] [--reps 20]

Per projection shape (o: 4096x4096, down: 4096x14336, half of gate_up: 14336x4096), 8 weight copies (cold: a 1 GiB
buffer is read between reps to evict the MALL):
  cold      flush, GEMM(W_i)                       -- GEMM time (events around the GEMM only)
  warm      flush, prefetch(W_i), GEMM(W_i)        -- GEMM time after a prefetch
  pf        the prefetch kernel alone (GB/s)
  overlap   flush, [GEMM(W_a) || prefetch(W_b) on a second stream], GEMM(W_b): total vs GEMM(W_a) + GEMM(W_b) cold
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from distributed_sse_for_llm_response_amd import ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=64)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--wgs", default="256,512")
    args = ap.parse_args()
    ops.load_library(required=True)
    dev = torch.device("cuda", 0)
    sink = ops.prefetch_sink(dev)
    flush = torch.empty(1 << 30, dtype=torch.uint8, device=dev)
    M = args.rows
    side = torch.cuda.Stream(dev)
    for name, N, K in (("o", 4096, 4096), ("down", 4096, 14336), ("gate_up/2", 14336, 4096)):
        ws = [torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.01 for _ in range(8)]
        x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
        out = torch.zeros(M, N, device=dev, dtype=torch.bfloat16)
        wbytes = N * K * 2

        def gemm(i):
            ops.gemm_out(x, ws[i % 8], out)

        def timed(body, reps):
            evs = []
            for i in range(reps):
                ops.prefetch(flush, sink, -1, 1024)
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                body(i, a, b)
                evs.append((a, b))
            torch.cuda.synchronize()
            t = sorted(a.elapsed_time(b) * 1e3 for a, b in evs)
            return t[len(t) // 2]

        for i in range(3):
            gemm(i)

        def cold(i, a, b):
            a.record(); gemm(i); b.record()

        t_cold = timed(cold, args.reps)
        print(f"{name:10s} M={M} {wbytes / 1e6:7.1f} MB  cold GEMM {t_cold:7.2f} us ({wbytes / t_cold / 1e6:5.2f} TB/s)",
              flush=True)
        for wgs in [int(v) for v in args.wgs.split(",")]:
            def warm(i, a, b):
                ops.prefetch(ws[i % 8], sink, -1, wgs)
                a.record(); gemm(i); b.record()

            def pf(i, a, b):
                a.record(); ops.prefetch(ws[i % 8], sink, -1, wgs); b.record()

            def overlap(i, a, b):
                a.record()
                side.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(side):
                    ops.prefetch(ws[(i + 1) % 8], sink, -1, wgs)
                gemm(i)
                torch.cuda.current_stream().wait_stream(side)
                ops.gemm_out(x, ws[(i + 1) % 8], out)
                b.record()

            def serial(i, a, b):
                a.record(); gemm(i); ops.gemm_out(x, ws[(i + 1) % 8], out); b.record()

            t_warm, t_pf = timed(warm, args.reps), timed(pf, args.reps)
            t_ov, t_se = timed(overlap, args.reps), timed(serial, args.reps)
            print(f"{'':10s} wgs={wgs:4d}  warm GEMM {t_warm:7.2f} us ({wbytes / t_warm / 1e6:5.2f} TB/s)  "
                  f"prefetch {t_pf:7.2f} us ({wbytes / t_pf / 1e6:5.2f} TB/s)  "
                  f"pair: overlapped {t_ov:7.2f} vs serial {t_se:7.2f} us", flush=True)
        del ws
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
