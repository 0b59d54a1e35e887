#!/usr/bin/env python3
"""Decode paged-attention microbenchmark: B sequences x ctx tokens, Mistral-7B heads (32 q / 8 kv, d 128).

Usage (GPU box): python tools/bench_attn.py [--B 64] [--ctx 560] [--configs "KWV=4;KWV=1;KWV=1,PD=2"]
(KWV / PD = the attn_kwv / attn_pd keys of DSSE_KERNEL_CFG.)
Pages are randomly permuted over the cache and several layer caches are rotated (> 256 MiB Infinity
Cache), so every call streams its K/V from HBM as in a decode step.  Times hipGraph replays; prints us and
the achieved K/V bandwidth.
"""
import argparse
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from distributed_sse_for_llm_response_amd import ops  # noqa: E402
from distributed_sse_for_llm_response_amd.engine.model_runner import decode_partitioning  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", default="64")
    ap.add_argument("--ctx", default="560")
    ap.add_argument("--hq", type=int, default=32)
    ap.add_argument("--hkv", type=int, default=8)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--configs", default="KWV=4;KWV=1")
    ap.add_argument("--target-wgs", default="512", help="flash-decoding partition targets to sweep")
    ap.add_argument("--seq-pages", action="store_true", help="pages in cache order instead of a random permutation")
    args = ap.parse_args()
    ops.load_library(required=True)
    base_cfg = os.environ.get("DSSE_KERNEL_CFG", "")
    dev = torch.device("cuda", 0)
    for B in [int(b) for b in args.B.split(",")]:
        for ctx in [int(c) for c in args.ctx.split(",")]:
            npg = math.ceil(ctx / 32)
            total = B * npg
            kv_bytes = B * ctx * args.hkv * 128 * 2 * 2
            copies = max(2, (600 << 20) // max(1, kv_bytes) + 1)
            ks = [torch.randn(total, args.hkv, 32, 128, device=dev, dtype=torch.bfloat16) for _ in range(copies)]
            vs = [torch.randn(total, args.hkv, 128, 32, device=dev, dtype=torch.bfloat16) for _ in range(copies)]
            order = torch.arange(total, device=dev) if args.seq_pages else torch.randperm(total, device=dev)
            bt = order.to(torch.int32).view(B, npg)
            bt = torch.cat([bt, torch.zeros(B, 1, device=dev, dtype=torch.int32)], 1).contiguous()
            q = torch.randn(B, args.hq, 128, device=dev, dtype=torch.bfloat16)
            out = torch.empty_like(q)
            i32 = dict(device=dev, dtype=torch.int32)
            q_start, q_len = torch.arange(B, **i32), torch.ones(B, **i32)
            ctx_len = torch.full((B,), ctx, **i32)
            work_seq, work_tile = torch.arange(B, **i32), torch.zeros(B, **i32)
            for tw, cfg in [(int(t), c) for t in args.target_wgs.split(",") for c in args.configs.split(";")]:
                part, nparts = decode_partitioning(B, args.hkv, ctx + 64, target_wgs=tw)
                part_o = torch.empty(B * nparts * args.hkv * 16 * 128, device=dev)
                part_ml = torch.empty(B * nparts * args.hkv * 16 * 2, device=dev)
                keys = {"KWV": "attn_kwv", "PD": "attn_pd"}  # DSSE_KERNEL_CFG keys (csrc/kernels/bindings.cpp)
                os.environ["DSSE_KERNEL_CFG"] = base_cfg  # each config starts from the caller's environment
                os.environ["DSSE_KERNEL_CFG"] = ops.kernel_cfg_env(
                    **{keys[k]: v for k, v in (item.split("=") for item in filter(None, cfg.split(",")))})
                ops.refresh_env()

                def run(i):
                    ops.paged_attention(0, q, ks[i % copies], vs[i % copies], bt, q_start, q_len, ctx_len, work_seq,
                                        work_tile, out, part_o, part_ml, part, nparts)

                for i in range(3):
                    run(i)
                torch.cuda.synchronize()
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g):
                    for i in range(args.iters):
                        run(i)
                g.replay()
                torch.cuda.synchronize()
                st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                st.record()
                g.replay()
                en.record()
                torch.cuda.synchronize()
                us = st.elapsed_time(en) / args.iters * 1e3
                print(f"B={B:4d} ctx={ctx:5d} nparts={nparts:2d} cfg={cfg:16s} {us:8.2f} us  "
                      f"{kv_bytes / us / 1e6:6.3f} TB/s", flush=True)
            del ks, vs
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
