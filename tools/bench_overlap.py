"""Design input for a concurrent prefill stream: a captured decode step and a prompt pass run one after the other (how the
engine runs them today) vs at the same time on two HIP streams.

    python tools/bench_overlap.py [--streams 128] [--ctx 512] [--prompt 512] [--steps 40]

Random-init Mistral-7B weights, `--streams` decoding sequences at `--ctx` tokens of context (garbage KV), one
`--prompt`-token prompt pass (the captured prefill graph of its row bucket) in a slot outside the decode bucket.
Prints the decode step alone, the pass alone, and, with the pass issued on a second stream while the decode
graph keeps replaying: every overlapped step's time and the pass's own duration.  Timing only: the two graphs
share scratch buffers (split-K slabs), so the overlapped run's values are not meaningful -- that sharing is what an
engine-level concurrent prefill has to split first.
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
    ap.add_argument("--streams", type=int, default=128)
    ap.add_argument("--ctx", type=int, default=512)
    ap.add_argument("--prompt", type=int, default=512)
    ap.add_argument("--steps", type=int, default=40)
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
    B = a.streams
    max_len = max(a.ctx + a.steps * 4 + 2 * PAGE, a.prompt + 2 * PAGE)
    per = blocks_needed(max_len)
    slot_p = B  # the prompt's slot: outside the decode bucket
    r = ModelRunner(w, num_blocks=(B + 1) * per + 4, max_batch=2 * B, max_model_len=max_len, device=dev,
                    max_prefill_tokens=max(512, a.prompt))
    for s in range(B + 1):
        r.block_tables[s, :per] = torch.arange(s * per, (s + 1) * per, dtype=torch.int32, device=dev)
    r.temperature.fill_(1.0)
    r.top_p.fill_(1.0)
    r.active.zero_()
    r.active[:B] = 1
    r.positions[:B] = a.ctx
    r.capture([B])
    torch.cuda.synchronize()

    gen = torch.Generator().manual_seed(3)
    toks = torch.randint(3, cfg.vocab_size, (a.prompt,), generator=gen).tolist()
    blocks = list(range(B * per, (B + 1) * per))
    seq = [PrefillSeq(slot_p, toks, 0, blocks, True)]

    def ev():
        return torch.cuda.Event(enable_timing=True)

    def decode_alone(n):
        es = [ev() for _ in range(n + 1)]
        es[0].record()
        for i in range(n):
            r.decode(B)
            es[i + 1].record()
        torch.cuda.synchronize()
        return [es[i].elapsed_time(es[i + 1]) for i in range(n)]

    def prefill_alone(n):
        out = []
        for _ in range(n):
            e0, e1 = ev(), ev()
            e0.record()
            r.prefill(seq, ring_row=1)
            e1.record()
            torch.cuda.synchronize()
            out.append(e0.elapsed_time(e1))
        return out

    side = torch.cuda.Stream(dev)

    def overlapped(n_steps):
        torch.cuda.synchronize()
        es = [ev() for _ in range(n_steps + 1)]
        p0, p1 = ev(), ev()
        main = torch.cuda.current_stream(dev)
        es[0].record()
        side.wait_stream(main)
        with torch.cuda.stream(side):
            p0.record()
            r.prefill(seq, ring_row=1)
            p1.record()
        for i in range(n_steps):
            r.decode(B)
            es[i + 1].record()
        torch.cuda.synchronize()
        return [es[i].elapsed_time(es[i + 1]) for i in range(n_steps)], p0.elapsed_time(p1), es[0].elapsed_time(p0)

    def med(x):
        x = sorted(x)
        return x[len(x) // 2]

    decode_alone(10)
    prefill_alone(3)
    d = decode_alone(a.steps)
    p = prefill_alone(5)
    runs = []
    for _ in range(5):
        steps, pass_ms, start_lag = overlapped(4)
        runs.append({"steps_ms": [round(x, 3) for x in steps], "pass_ms": round(pass_ms, 3),
                     "pass_start_lag_ms": round(start_lag, 3)})
    serial_gap = med(d) + med(p)
    worst_overlap = med([max(rn["steps_ms"]) for rn in runs])
    print(json.dumps({"tool": "bench_overlap", "streams": B, "ctx": a.ctx, "prompt": a.prompt,
                      "decode_step_ms": round(med(d), 3), "prefill_pass_ms": round(med(p), 3),
                      "serial_gap_ms": round(serial_gap, 3), "overlap_worst_step_ms": round(worst_overlap, 3),
                      "overlap_pass_ms": round(med([rn["pass_ms"] for rn in runs]), 3), "runs": runs}), flush=True)


if __name__ == "__main__":
    main()
