"""Time to first token for long prompts (BASELINE config 4: 8k-token prompts, TTFT + ITL, TP=1/2/4/8).

    python tools/bench_ttft.py [--prompt-len 8192] [--prompts 1] [--iters 3] [--decode-steps 16]
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 tools/bench_ttft.py ...   # config 4 at TP=8 (one rank per GPU, RCCL)

Per iteration: prefill `--prompts` fresh random prompts of `--prompt-len` tokens in chunks of
`--chunk` tokens (one engine prefill call per chunk; the tiled-layout GEMMs + the flash-prefill kernel +
paged KV writes), sample the first token, copy it to the host: that wall time is the TTFT.  Then
`--decode-steps` graph-captured decode steps give the ITL at that context length.  Rank 0 prints one
JSON line.  Random-init Mistral-7B-v0.3 weights (bf16), synthetic prompts.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="mistral-7b-v0.3")
    ap.add_argument("--prompt-len", type=int, default=8192)
    ap.add_argument("--prompts", type=int, default=1)
    ap.add_argument("--chunk", type=int, default=8192)
    ap.add_argument("--iters", type=int, default=3)
    ap.add_argument("--decode-steps", type=int, default=16)
    ap.add_argument("--profile-marker", action="store_true",
                    help="launch one bitwise_not kernel after the warm-up iteration: tools/trace_sum.py --after-kernel "
                         "bitwise_not then keeps only the timed iterations of a rocprofv3 kernel trace")
    args = ap.parse_args()

    import numpy as np
    import torch
    import torch.distributed as dist

    from distributed_sse_for_llm_response_amd.engine.kv_cache import PAGE, blocks_needed
    from distributed_sse_for_llm_response_amd.engine.model_runner import ModelRunner, PrefillSeq
    from distributed_sse_for_llm_response_amd.engine.weights import random_engine_weights
    from distributed_sse_for_llm_response_amd.models.mistral import get_config
    from distributed_sse_for_llm_response_amd.parallel.comm import TPComm, init_distributed

    local = int(os.environ.get("LOCAL_RANK", "0"))
    device = torch.device("cuda", local)
    torch.cuda.set_device(device)
    rank, local, world = init_distributed(device=device)
    comm = TPComm(rank=rank, size=world) if world > 1 else TPComm()
    cfg = get_config(args.model)
    w = random_engine_weights(cfg, tp_rank=comm.rank, tp_size=comm.size, device=device, seed=7)
    max_len = args.prompt_len + args.decode_steps + 2 * PAGE
    per = blocks_needed(max_len)
    B = max(1, args.prompts)
    r = ModelRunner(w, num_blocks=B * per + 4, max_batch=B, max_model_len=max_len, device=device, comm=comm,
                    max_prefill_tokens=max(args.chunk, 8192))
    r.capture([B])
    gen = torch.Generator().manual_seed(5)

    # the slots' block tables and sampling parameters are set once, so a profiled iteration holds only the prefill
    # (and decode) kernels: no torch fill / copy kernels between the trace marker and the first prefill launch
    for s in range(B):
        r.block_tables[s, :per] = torch.tensor(list(range(s * per, (s + 1) * per)), dtype=torch.int32, device=device)
    r.temperature.fill_(1.0)
    r.top_p.fill_(1.0)
    r.active.zero_()

    def one_iter():
        seqs = []
        for s in range(B):
            blocks = list(range(s * per, (s + 1) * per))
            toks = torch.randint(3, cfg.vocab_size, (args.prompt_len,), generator=gen).tolist()
            seqs.append((s, toks, blocks))
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        t0 = time.perf_counter()
        for start in range(0, args.prompt_len, args.chunk):
            n = min(args.chunk, args.prompt_len - start)
            last = start + n == args.prompt_len
            r.prefill([PrefillSeq(s, toks[start:start + n], start, blocks, last) for s, toks, blocks in seqs],
                      ring_row=0)
        first = r.ids[:B].cpu()  # D2H: the first token is on the host
        ttft = time.perf_counter() - t0
        if args.decode_steps:
            r.active[:B] = 1
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for _ in range(args.decode_steps):
            r.decode(B)
        if args.decode_steps:
            r.active.zero_()
        torch.cuda.synchronize()
        itl = (time.perf_counter() - t1) / max(1, args.decode_steps)
        return ttft, itl, first

    one_iter()  # warm-up (allocator, first launches)
    if args.profile_marker:
        torch.ones(1, dtype=torch.int32, device=device).bitwise_not_()
        torch.cuda.synchronize()
    ttfts, itls = [], []
    for _ in range(args.iters):
        a, b, _ = one_iter()
        ttfts.append(a)
        itls.append(b)
    if world > 1:
        t = torch.tensor([max(ttfts), max(itls)], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    if rank == 0:
        flops = 2 * 7.25e9 * args.prompt_len * B
        p50 = float(np.median(ttfts))
        print(json.dumps({
            "metric": "p50 TTFT for long prompts (+ ITL at that context)", "model": cfg.name, "tp": world,
            "prompt_len": args.prompt_len, "prompts": B, "chunk": args.chunk, "p50_ttft_ms": round(1000 * p50, 3),
            "ttfts_ms": [round(1000 * x, 3) for x in ttfts], "prefill_tokens_per_s": round(args.prompt_len * B / p50, 1),
            "dense_gemm_tflops_equiv": round(flops / p50 / 1e12, 1), "p50_itl_ms": round(1000 * float(np.median(itls)), 4),
            "dtype": "bf16", "data": "synthetic prompts, random-init weights"}), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
