#!/usr/bin/env python3
"""Flash prefill attention microbenchmark (attention_prefill.hip, paged_attention mode 2): one causal prompt of
--T tokens, Mistral-7B heads (32 q / 8 kv, d 128), pages in random cache order, random bf16 operands.

    python tools/bench_prefill_attn.py [--T 8192,512] [--iters 10] [--rounds 3] [--sdpa]

Timed as a captured graph of --iters calls (the engine's form; --eager: back-to-back eager calls).  Prints us per call and TFLOP/s (causal FLOPs = 2 * 2 * Hq * d * T (T + 1) / 2), then a JSON summary.  --sdpa adds
torch's scaled_dot_product_attention on the same (contiguous) data as a library arm, interleaved in one process.
Under rocprofv3 --pmc use --rounds 1 --iters 3: the kernel trace then holds only this kernel (plus torch's
random fills, which run before the first timed call and have different names).
"""
import argparse
import json
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from distributed_sse_for_llm_response_amd import ops  # noqa: E402

PAGE = 32


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--T", default="8192,512")
    ap.add_argument("--hq", type=int, default=32)
    ap.add_argument("--hkv", type=int, default=8)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--sdpa", action="store_true")
    ap.add_argument("--mode1", default="", help="comma list of key partition counts for mode-1 arms")
    ap.add_argument("--eager", action="store_true", help="time eager back-to-back calls instead of a graph")
    args = ap.parse_args()
    ops.load_library(required=True)
    dev = torch.device("cuda", 0)
    i32 = dict(device=dev, dtype=torch.int32)
    res = {}
    for T in [int(t) for t in args.T.split(",")]:
        npg = math.ceil(T / PAGE)
        k_cache = torch.randn(npg, args.hkv, PAGE, 128, device=dev, dtype=torch.bfloat16)
        v_cache = torch.randn(npg, args.hkv, 128, PAGE, device=dev, dtype=torch.bfloat16)
        bt = torch.randperm(npg, device=dev).to(torch.int32).view(1, npg)
        q = torch.randn(T, args.hq, 128, device=dev, dtype=torch.bfloat16)
        out = torch.empty_like(q)
        q_start, q_len, ctx_len = torch.zeros(1, **i32), torch.full((1,), T, **i32), torch.full((1,), T, **i32)
        ntile = math.ceil(T / 64)
        work_tile = torch.arange(ntile - 1, -1, -1, **i32)  # heaviest first, as the engine orders them
        work_seq = torch.zeros(ntile, **i32)
        dummy = torch.empty(1, device=dev)
        flop = 2.0 * 2.0 * args.hq * 128 * T * (T + 1) / 2

        def flash():
            ops.paged_attention(2, q, k_cache, v_cache, bt, q_start, q_len, ctx_len, work_seq, work_tile, out,
                                dummy, dummy, 32 * math.ceil((T + 31) / 32), 1)

        arms = {"flash": flash}
        # --mode1 N,...: the decode-style kernel on 64-query work items (4 tiles of 16) with the keys in N partitions
        # merged by the combine kernel (paged_attention mode 1): more workgroups for short prompts
        # (a mode-1 work item is 4 tiles of 16 / G queries: 16 queries of all G heads at G = 4)
        n1 = math.ceil(T / 16)
        wt1, ws1 = torch.arange(n1 - 1, -1, -1, **i32), torch.zeros(n1, **i32)
        for npart in [int(v) for v in args.mode1.split(",") if v]:
            part = 32 * math.ceil(T / npart / 32)
            po = torch.empty(n1 * args.hkv * npart * 64 * 128, device=dev)
            pml = torch.empty(n1 * args.hkv * npart * 64 * 2, device=dev)
            arms[f"m1p{npart}"] = (lambda po=po, pml=pml, part=part, npart=npart: ops.paged_attention(
                1, q, k_cache, v_cache, bt, q_start, q_len, ctx_len, ws1, wt1, out, po, pml, part, npart))
        if args.sdpa:
            # contiguous [1, H, T, d] copies of the same K/V (GQA expanded), causal
            kk = k_cache[bt[0].long()].permute(1, 0, 2, 3).reshape(args.hkv, T, 128)
            # the V cache holds each page transposed with token t at column vperm(t) (gemm_epilogue.h vperm_tok)
            vperm = [((t & 15) >> 2) * 8 + ((t >> 4) & 1) * 4 + (t & 3) for t in range(PAGE)]
            vv = v_cache[bt[0].long()][..., vperm].permute(1, 0, 3, 2).reshape(args.hkv, T, 128)
            rep = args.hq // args.hkv
            kk = kk.repeat_interleave(rep, 0)[None].contiguous()
            vv = vv.repeat_interleave(rep, 0)[None].contiguous()
            qq = q.permute(1, 0, 2)[None].contiguous()
            arms["sdpa"] = lambda: torch.nn.functional.scaled_dot_product_attention(qq, kk, vv, is_causal=True)
        flash()
        torch.cuda.synchronize()
        first = out.clone()
        times = {k: [] for k in arms}
        # timed as a captured graph of `iters` calls (as the engine runs prefill): a short prompt's kernel is shorter
        # than the host's per-call dispatch, so eager back-to-back calls would time the host
        graphs = {}
        if not args.eager:
            for k, fn in arms.items():
                if k == "sdpa":
                    continue
                fn()
                torch.cuda.synchronize()
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g):
                    for _ in range(args.iters):
                        fn()
                graphs[k] = g
        for _ in range(args.rounds):
            for k, fn in arms.items():
                fn()
                torch.cuda.synchronize()
                st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                st.record()
                if k in graphs:
                    graphs[k].replay()
                else:
                    for _ in range(args.iters):
                        fn()
                en.record()
                torch.cuda.synchronize()
                times[k].append(st.elapsed_time(en) * 1e3 / args.iters)
        # race screen: the kernel is deterministic, so every call must reproduce the first output bit for bit
        flash()
        torch.cuda.synchronize()
        same = bool(torch.equal(first, out))
        for k in arms:
            if k.startswith("m1p"):
                out.zero_()
                arms[k]()
                torch.cuda.synchronize()
                err = (out.float() - first.float()).abs().max().item()
                res[f"T{T}_{k}_max_abs_vs_flash"] = round(err, 5)
                print(f"T={T:6d} {k} max |out - flash| = {err:.5f}", flush=True)
        flash()
        torch.cuda.synchronize()
        res[f"T{T}_repeat_identical"] = same
        print(f"T={T:6d} repeated calls bit-identical: {same}", flush=True)
        if args.sdpa:
            ref = arms["sdpa"]()[0].permute(1, 0, 2).float()
            err = (out.float() - ref).abs().max().item()
            res[f"T{T}_max_abs_err_vs_sdpa"] = round(err, 5)
            print(f"T={T:6d} max |flash - sdpa| = {err:.5f}", flush=True)
        for k, ts in times.items():
            us = sorted(ts)[len(ts) // 2]
            res[f"T{T}_{k}"] = {"us": round(us, 1), "tflops": round(flop / us / 1e6, 1), "min_us": round(min(ts), 1)}
            print(f"T={T:6d} {k:6s} {us:10.1f} us {flop / us / 1e6:8.1f} TFLOP/s", flush=True)
        del k_cache, v_cache, q, out
        torch.cuda.empty_cache()
    print(json.dumps(res))


if __name__ == "__main__":
    main()
