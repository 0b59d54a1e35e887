"""Mixed prefill + decode step cost: the captured decode step of bucket B alone vs the captured mixed step (B decode
rows + a C-row prompt chunk) for every captured chunk size -- the numbers the engine's PassCost fits at run time
(engine.PassCost.mixed_chunk), measured directly.

    python tools/bench_mixed.py [--streams 64,128] [--ctx 512] [--reps 20]

Random-init Mistral-7B weights, `--streams` decoding sequences at `--ctx` tokens of context (garbage KV), a prompt
filling the chunk in a slot outside the decode bucket.  One JSON line per (B, C): ms per step, extra over the decode
step, and us per prompt row.
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
    ap.add_argument("--streams", default="64,128")
    ap.add_argument("--ctx", type=int, default=512)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()

    import torch

    from distributed_sse_for_llm_response_amd.engine.kv_cache import PAGE, blocks_needed
    from distributed_sse_for_llm_response_amd.engine.model_runner import ModelRunner, PrefillSeq
    from distributed_sse_for_llm_response_amd.engine.weights import random_engine_weights
    from distributed_sse_for_llm_response_amd.models.mistral import get_config

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    cfg = get_config("mistral-7b-v0.3")
    w = random_engine_weights(cfg, device=dev, seed=7)
    bs = [int(b) for b in a.streams.split(",")]
    Bmax = max(bs)
    reps = a.reps
    max_len = a.ctx + 4 * (reps + 4) + 2 * PAGE + 512
    per = blocks_needed(max_len)
    r = ModelRunner(w, num_blocks=(Bmax + 1) * per + 4, max_batch=2 * Bmax, max_model_len=max_len, device=dev,
                    max_prefill_tokens=2048)
    for s in range(Bmax + 1):
        r.block_tables[s, :per] = torch.arange(s * per, (s + 1) * per, dtype=torch.int32, device=dev)
    r.temperature.fill_(1.0)
    r.top_p.fill_(1.0)
    r.capture(bs)
    torch.cuda.synchronize()
    gen = torch.Generator().manual_seed(3)

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        best = float("inf")
        for _ in range(3):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(reps):
                fn()
            e1.record()
            torch.cuda.synchronize()
            best = min(best, e0.elapsed_time(e1) / reps)
        return best

    for B in bs:
        r.active.zero_()
        r.active[:B] = 1
        r.positions[:B] = a.ctx
        step = timed(lambda: r.decode(B))
        print(json.dumps({"B": B, "C": 0, "ms": round(step, 3)}), flush=True)
        for C, _g in r.mx_graphs.get(B, []):
            toks = torch.randint(3, cfg.vocab_size, (C,), generator=gen).tolist()
            bt = list(range(B * per, (B + 1) * per))
            r.positions[:B] = a.ctx

            def one():
                r.mixed(B, [PrefillSeq(B, toks, 0, bt, True)], ring_row=0)
            ms = timed(one)
            print(json.dumps({"B": B, "C": C, "ms": round(ms, 3), "extra_ms": round(ms - step, 3),
                              "us_per_row": round(1000 * (ms - step) / C, 2), "x_step": round(ms / step, 3)}),
                  flush=True)


if __name__ == "__main__":
    main()
