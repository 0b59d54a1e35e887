#!/usr/bin/env python3
"""Sweep the decode GEMM kernels over Mistral-7B shapes and tile configs; prints achieved HBM TB/s.

Usage (GPU box): python tools/tune_gemm.py [--M 1,16,32,64] [--tp 1] [--iters 50]
Weights are 2x the L3 (Infinity Cache, 256 MiB) per shape class by rotating over several copies,
so every timed call streams its weights from HBM as in a real decode step.
"""
import argparse
import itertools
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from distributed_sse_for_llm_response_amd import ops  # noqa: E402


def shapes(tp):
    H, F, V = 4096, 14336, 32768
    nh, nkv = 32 // tp, 8 // tp
    return {
        "qkv": ((nh + 2 * nkv) * 128, H),
        "o": (H, nh * 128),
        "gate_up": (2 * F // tp, H),
        "down": (H, F // tp),
        "lm_head": (V // tp, H),
    }


def time_op(fn, iters, graph=False):
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(3):
        fn(0)
    torch.cuda.synchronize()
    if graph:  # the decode step replays its kernels from a hipGraph: time them the same way
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for i in range(iters):
                fn(i)
        g.replay()
        torch.cuda.synchronize()
        st.record()
        g.replay()
        en.record()
        torch.cuda.synchronize()
        return st.elapsed_time(en) / iters * 1e3
    st.record()
    for i in range(iters):
        fn(i)
    en.record()
    torch.cuda.synchronize()
    return st.elapsed_time(en) / iters * 1e3  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", default="1,16,32,64")
    ap.add_argument("--ops", default="", help="comma-separated subset of qkv,o,gate_up,down,lm_head")
    ap.add_argument("--tp", type=int, default=1)
    ap.add_argument("--graph", action="store_true", help="time hipGraph replays of the calls")
    ap.add_argument("--iters", type=int, default=40)
    ap.add_argument("--configs", default="skinny;s;s:s_nw=8;w;t",
                    help="';'-separated; 'skinny', 's' (X-streaming), 'w' (wide, 32x32 MFMA) or 't' (tiled), "
                         "optionally ':key=V,key=V' DSSE_KERNEL_CFG overrides")
    ap.add_argument("--hot", action="store_true", help="one weight copy (Infinity-Cache resident when it fits)")
    ap.add_argument("--out", default="")
    ap.add_argument("--grid", action="store_true", help="sweep the X-streaming parameter grid")
    args = ap.parse_args()
    ops.load_library(required=True)
    dev = torch.device("cuda", 0)
    results = []
    if args.grid:
        cfgs = ["skinny"]
        for nw in (4, 8):
            for split in (1, 2, 4):
                for rd in (1, 2):
                    cfgs.append(f"s:s_nw={nw},s_split={split},s_rd={rd}")
        args.configs = ";".join(cfgs)
    for name, (N, K) in shapes(args.tp).items():
        if args.ops and name not in args.ops.split(","):
            continue
        nbytes = N * K * 2
        copies = 1 if args.hot else max(2, (600 << 20) // nbytes + 1)
        ws = [torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02 for _ in range(copies)]
        for M in [int(m) for m in args.M.split(",")]:
            x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
            for cfg in args.configs.split(";"):
                impl, _, kv = cfg.partition(":")
                gi = {"skinny": "0", "s": "2", "w": "3", "t": "4"}[impl]
                os.environ["DSSE_KERNEL_CFG"] = f"gemm_impl={gi}" + (f",{kv}" if kv else "")
                ops.refresh_env()
                if name == "gate_up":
                    out = torch.empty(M, N // 2, device=dev, dtype=torch.bfloat16)
                    fn = (lambda i, out=out, x=x: ops.gemm_silu(x, ws[i % copies], out))
                elif name == "lm_head":
                    out = torch.empty(M, N, device=dev, dtype=torch.float32)
                    fn = (lambda i, out=out, x=x: ops.gemm_out(x, ws[i % copies], out))
                else:
                    out = torch.zeros(M, N, device=dev, dtype=torch.float32)
                    fn = (lambda i, out=out, x=x: ops.gemm_resid(x, ws[i % copies], out))
                try:
                    us = time_op(fn, args.iters, args.graph)
                except RuntimeError as e:
                    print(f"{name} M={M} cfg={cfg}: {e}", flush=True)
                    continue
                tbs = nbytes / us / 1e6
                results.append({"op": name, "N": N, "K": K, "M": M, "cfg": cfg, "us": round(us, 2),
                                "TBps": round(tbs, 3)})
                print(f"{name:8s} N={N:6d} K={K:6d} M={M:3d} cfg={cfg:28s} {us:9.2f} us  {tbs:6.3f} TB/s",
                      flush=True)
        del ws
        torch.cuda.empty_cache()
    best = {}
    for r in results:
        k = (r["op"], r["M"])
        if k not in best or r["us"] < best[k]["us"]:
            best[k] = r
    print("\nbest per (op, M):")
    for k, r in sorted(best.items()):
        print(f"  {k[0]:8s} M={k[1]:3d} {r['us']:8.2f} us {r['TBps']:6.3f} TB/s  {r['cfg']}")
    if args.out:
        with open(args.out, "w") as f:
            json.dump(results, f, indent=1)


if __name__ == "__main__":
    main()
