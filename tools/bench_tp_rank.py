"""One TP rank of Mistral-7B on one GPU (VERDICT r5 missing 2: BASELINE config 4's per-rank work, measured).

    python tools/bench_tp_rank.py --tp 8 [--streams 64] [--prompt-len 512] [--steps 50] [--prefill 8192]

Builds rank 0's shard of the real Mistral-7B-v0.3 dimensions at TP = t (random_engine_weights(tp_rank=0,
tp_size=t): qkv N = 6144 / t, o K = 4096 / t, gate_up N = 28672 / t, down K = 14336 / t, 8 / t KV heads, a 1 / t
vocab shard) and runs it through the production ModelRunner with a communicator that reports size t but keeps
every byte local (ShardComm below):

  * the decode step's two residual all-reduces per layer run the hand-written IPC all-reduce + RMSNorm kernel
    (allreduce.hip) of a one-rank IPC context -- the production kernel and launch sequence, minus the xGMI wait;
  * the sampling candidates' all-gather is a local replicate (copy kernel) instead of the IPC gather kernel;
  * prefill: the chunked TP path (>= 1024 rows: each row chunk's residual step -- reduce-scatter, add + RMSNorm of
    this rank's 1 / t of the rows, all-gather -- on a side stream) with the reduce-scatter a local copy of this
    rank's rows and the all-gather a no-op (its rows would come from the peers).

So the numbers are this rank's compute + the launch structure of a real TP group, not its communication: the xGMI
transfer time of the collectives comes on top (docs/operations.md, "TP = 8 budget").  Times: (a) the captured
decode step of `--streams` streams at ~`--prompt-len` context (graph replays, events), (b) an `--prefill`-token
prompt's prefill on this rank (eager, events).  One JSON line.  Random-init bf16 weights, synthetic prompts.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tp", type=int, default=8)
    ap.add_argument("--streams", type=int, default=64)
    ap.add_argument("--prompt-len", type=int, default=512)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--prefill", type=int, default=8192)
    ap.add_argument("--iters", type=int, default=3)
    ap.add_argument("--phase", default="both", choices=["both", "decode", "prefill"])
    ap.add_argument("--host-profile", action="store_true",
                    help="cProfile one timed prefill and print the top host functions (where the host time goes)")
    ap.add_argument("--split-any-rounds", action="store_true",
                    help="A/B: the flash key split's range length without the one-round rule (flash_split_plan)")
    ap.add_argument("--attn-wgs", type=int, default=0,
                    help="decode attention workgroup target of decode_partitioning (0 = the engine default, 512): "
                         "fewer flash-decoding partitions per sequence for an A/B")
    ap.add_argument("--profile-marker", action="store_true",
                    help="launch one bitwise_not kernel before the timed decode replays and one before the timed "
                         "prefills (tools/trace_sum.py --after-kernel bitwise_not keeps what follows)")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    from distributed_sse_for_llm_response_amd import ops
    from distributed_sse_for_llm_response_amd.engine.kv_cache import PAGE, blocks_needed
    from distributed_sse_for_llm_response_amd.engine.model_runner import ModelRunner, PrefillSeq
    from distributed_sse_for_llm_response_amd.engine.weights import random_engine_weights
    from distributed_sse_for_llm_response_amd.models.mistral import MISTRAL_7B_V03
    from distributed_sse_for_llm_response_amd.parallel.comm import IpcAllReduce, TPComm

    ops.load_library(required=True)
    import functools

    if args.split_any_rounds:
        from distributed_sse_for_llm_response_amd.engine import model_runner as mr

        mr.flash_split_plan = functools.partial(mr.flash_split_plan, one_round=False)
    if args.attn_wgs > 0:
        from distributed_sse_for_llm_response_amd.engine import model_runner as mr

        mr.decode_partitioning = functools.partial(mr.decode_partitioning, target_wgs=args.attn_wgs)
    device = torch.device("cuda", 0)
    torch.cuda.set_device(device)
    # a one-rank host group: the IPC context's handle exchange and self-test run over it
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(s.getsockname()[1]))
    s.close()
    dist.init_process_group("gloo", rank=0, world_size=1)

    class ShardComm(TPComm):
        """size = t for every sharding decision, collectives local (see the module docstring)."""

        def all_reduce(self, t):
            return None

        def all_gather_into(self, out, inp):
            flat = inp.contiguous().view(1, -1)
            out.view(self.size, -1).copy_(flat.expand(self.size, -1))

        def reduce_scatter_rows(self, out, inp):
            out.copy_(inp[: out.shape[0]])

        def all_gather_rows(self, out, own):
            return None  # the other ranks' rows would arrive over xGMI; own already sits in place

        def broadcast(self, t, src=0):
            return None

        def barrier(self):
            return None

        def enable_ipc_allreduce(self, device, rows, hidden):
            ctx, why = IpcAllReduce.create(TPComm(), device, rows, hidden)
            self.fast_ar = ctx
            return why

    comm = ShardComm(rank=0, size=args.tp)
    cfg = MISTRAL_7B_V03
    w = random_engine_weights(cfg, tp_rank=0, tp_size=args.tp, device=device, seed=7)
    B = args.streams
    max_len = max(args.prompt_len + args.steps + args.warmup + 2 * PAGE, args.prefill + 2 * PAGE)
    per_stream = blocks_needed(args.prompt_len + args.steps + args.warmup + 2 * PAGE)
    per_prefill = blocks_needed(args.prefill + PAGE)
    r = ModelRunner(w, num_blocks=B * per_stream + per_prefill + 8, max_batch=B, max_model_len=max_len,
                    device=device, comm=comm, max_prefill_tokens=max(args.prefill, 8192))
    r._collectives_capturable = lambda: (True, "")  # local no-op all-reduce: captures like RCCL would
    ipc = r.ipc_decode()
    r.capture([B])
    gen = torch.Generator().manual_seed(5)
    tables = [list(range(i * per_stream, (i + 1) * per_stream)) for i in range(B)]
    for i, bt in enumerate(tables):
        r.block_tables[i, : len(bt)] = torch.tensor(bt, dtype=torch.int32)
    # prompts in packed passes of <= 8192 rows
    prompts = [torch.randint(3, cfg.vocab_size, (args.prompt_len,), generator=gen).tolist() for _ in range(B)]
    per_pass = max(1, 8192 // args.prompt_len)
    for a in range(0, B, per_pass):
        r.prefill([PrefillSeq(i, prompts[i], 0, tables[i], True) for i in range(a, min(B, a + per_pass))], ring_row=0)
    r.active[:B] = 1
    r.temperature[:B] = 0.0
    torch.cuda.synchronize()
    step_ms = None
    if args.phase in ("both", "decode"):
        for _ in range(args.warmup):
            r.decode(B)
        torch.cuda.synchronize()
        if args.profile_marker:
            torch.bitwise_not(torch.zeros(1, dtype=torch.int32, device=device))
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.steps):
            r.decode(B)
        e1.record()
        torch.cuda.synchronize()
        step_ms = e0.elapsed_time(e1) / args.steps
    health = r.health.cpu().tolist()

    # an --prefill-token prompt on slot 0 of a free page range
    ptab = list(range(B * per_stream, B * per_stream + per_prefill))
    r.block_tables[0].zero_()
    r.block_tables[0, : len(ptab)] = torch.tensor(ptab, dtype=torch.int32)
    long_prompt = torch.randint(3, cfg.vocab_size, (args.prefill,), generator=gen).tolist()
    seq = PrefillSeq(0, long_prompt, 0, ptab, True)
    times = []
    if args.phase in ("both", "prefill"):
        r.prefill([seq], ring_row=0)  # warm
        torch.cuda.synchronize()
        if args.profile_marker:
            torch.bitwise_not(torch.zeros(1, dtype=torch.int32, device=device))
    for _ in range(args.iters if args.phase in ("both", "prefill") else 0):
        p0, p1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        p0.record()
        r.prefill([seq], ring_row=0)
        p1.record()
        torch.cuda.synchronize()
        times.append(p0.elapsed_time(p1))
    if args.host_profile and args.phase in ("both", "prefill"):
        import cProfile
        import pstats
        import time

        torch.cuda.synchronize()
        t0 = time.perf_counter()
        r.prefill([seq], ring_row=0)
        host_ms = (time.perf_counter() - t0) * 1e3  # enqueue time (the GPU may still be running)
        torch.cuda.synchronize()
        prof = cProfile.Profile()
        prof.enable()
        r.prefill([seq], ring_row=0)
        prof.disable()
        torch.cuda.synchronize()
        print(f"host enqueue of one prefill: {host_ms:.2f} ms (unprofiled)", flush=True)
        pstats.Stats(prof).sort_stats("tottime").print_stats(18)
    out = {
        "tp": args.tp, "rank": 0, "model": cfg.name, "streams": B, "prompt_len": args.prompt_len,
        "decode_step_ms": None if step_ms is None else round(step_ms, 4), "decode_collectives": "ipc kernel, 1-rank context" if ipc else "local",
        "attn_wgs": args.attn_wgs or 512, "prefill_tokens": args.prefill, "prefill_ms": [round(t, 3) for t in times],
        "prefill_ms_min": round(min(times), 3) if times else None, "health": health,
        "shard": {"qkv_N": (w.nh + 2 * w.nkv) * 128, "o_K": w.nh * 128, "gate_up_N": 2 * w.ffn, "down_K": w.ffn,
                  "kv_heads": w.nkv, "vocab_local": w.vocab_local},
        "note": "compute + launch structure of one rank; the xGMI collective time is not included",
    }
    print(json.dumps(out), flush=True)
    r.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
