#!/usr/bin/env python3
"""Headline benchmark: concurrent SSE token streams + p50 inter-token latency, Mistral-7B on MI355X.

Contract (driver): ``python bench.py --gpus N --steps K --warmup W``; for N > 1 the driver launches one
rank per GPU with torchrun.  Each rank is a Mistral-7B engine replica (DP, one engine per GPU,
BASELINE config 2/3) serving ``--streams`` concurrent conversations (64 per GPU = config 2), so per-GPU
work is fixed as N grows (weak scaling).  With ``--delivery sse`` (default) one client process opens
all N x streams POST /chat SSE connections to rank 0's server, whose C++ data-parallel router spreads
them over the replicas through shared-memory rings (the ``serve --dp N`` path).  One timed step = one engine iteration for all
live streams on every rank: the hipGraph-captured decode step (all 32 layers, LM head, sampler,
token-ring append), the device->host token drain on a side stream, and host-side delivery of every
token as an SSE ``event: token`` frame carrying the reference's TokenMessage JSON
(``--delivery sse``: through the C++ bus + epoll SSE server to real socket clients; ``--delivery
frame``: frame formatting only).

Timing: W untimed warmup steps, then exactly K steps bracketed by a barrier + device synchronize on
both sides; the MAX elapsed time over ranks is used.  Rank 0 prints ONE JSON line.

value = total streamed tokens per second over all N GPUs (= streams / ITL); p50 ITL is reported
in ``p50_itl_ms``.  Weights are random-init bf16 of the exact Mistral-7B-v0.3 architecture and
prompts are synthetic (no network): ``data = "synthetic"``.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "concurrent SSE streams + p50 inter-token latency, Mistral-7B at 1/2/4/8 MI355X"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=64)
    ap.add_argument("--warmup", type=int, default=8)
    ap.add_argument("--streams", type=int, default=64, help="concurrent streams per GPU")
    ap.add_argument("--prompt-len", type=int, default=512)
    ap.add_argument("--model", default="mistral-7b-v0.3")
    ap.add_argument("--tp", type=int, default=1)
    ap.add_argument("--delivery", default="sse", choices=["sse", "frame", "none"])
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--stub-step-ms", type=float, default=0.0,
                    help="host-path rehearsal only: paced stub replicas emitting one token per stream every "
                         "STUB_STEP_MS instead of the model (router/bus/SSE/client at N GPUs' token rate)")
    args = ap.parse_args()

    from distributed_sse_for_llm_response_amd.engine import bench_harness

    # the SSE client process (rank 0 only: one client drives every replica through the router) must be
    # started before this process initialises the GPU
    sse = args.delivery == "sse"
    client = bench_harness.spawn_client() if sse and int(os.environ.get("RANK", "0")) == 0 else None

    import torch
    import torch.distributed as dist

    from distributed_sse_for_llm_response_amd.parallel.comm import init_distributed

    # bind this rank's GPU before the process group exists (RCCL communicators use the current device)
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # (local % count: a multi-rank rehearsal may put several ranks on one GPU, with DSSE_DIST_BACKEND=gloo)
    device = torch.device("cuda", local % torch.cuda.device_count()) if torch.cuda.is_available() else torch.device("cpu")
    if device.type == "cuda":
        torch.cuda.set_device(device)
    rank, local, world = init_distributed(device=device if device.type == "cuda" else None)
    if world != args.gpus and rank == 0:
        print(f"[bench] note: --gpus {args.gpus} but WORLD_SIZE {world}; using WORLD_SIZE", file=sys.stderr)
    n_gpus = world

    if sse:
        res = bench_harness.run_serving_bench(client, model=args.model, device=device, streams=args.streams,
                                              prompt_len=args.prompt_len, steps=args.steps, warmup=args.warmup,
                                              tp=args.tp, use_graphs=not args.no_graph, rank=rank, world=world,
                                              stub_step_ms=args.stub_step_ms)
    else:
        res = bench_harness.run_decode_bench(model=args.model, device=device, streams=args.streams,
                                             prompt_len=args.prompt_len, steps=args.steps, warmup=args.warmup,
                                             tp=args.tp, delivery=args.delivery, use_graphs=not args.no_graph,
                                             rank=rank, world=world)
    elapsed = res["elapsed_s"]
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        if not sse:  # frame/none: per-rank delivery gaps; sse: the rank-0 client saw every stream
            itl = torch.tensor([res["p50_itl_ms"]], dtype=torch.float64, device=device)
            dist.all_reduce(itl, op=dist.ReduceOp.MAX)
            res["p50_itl_ms"] = float(itl.item())
    replicas = world // args.tp
    total_streams = args.streams * replicas
    tokens = total_streams * args.steps
    value = tokens / elapsed
    if rank == 0:
        out = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "tokens/s (aggregate over concurrent SSE streams)",
            "n_gpus": n_gpus,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1000.0 * elapsed / args.steps, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16",
            "data": "synthetic prompts, random-init weights" if not args.stub_step_ms else
                    f"REHEARSAL: paced stub replicas at {args.stub_step_ms} ms/step, no model",
            "concurrent_streams": total_streams,
            "p50_itl_ms": round(res["p50_itl_ms"], 4),
            "p99_itl_ms": round(res.get("p99_itl_ms", 0.0), 4),
            "delivery": args.delivery,
            "tokens_delivered_in_window": res.get("delivered_in_window"),
            "client_errors": res.get("client_errors", []),
            "stalls": res.get("stalls", {}),
            "config": {"model": res.get("model", args.model), "global_batch": total_streams, "seq_len": res.get("max_context", args.prompt_len + args.steps + args.warmup),
                       "prompt_len": args.prompt_len,
                       "parallelism": f"dp{replicas}" + (f"xtp{args.tp}" if args.tp > 1 else "")},
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
