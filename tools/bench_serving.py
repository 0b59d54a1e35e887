#!/usr/bin/env python3
"""Serving under continuous arrivals: TTFT and in-flight inter-token latency while new prompts are prefilled.

The steady-state bench (bench.py) times decode once every stream is admitted.  Here requests arrive as a
Poisson process (the reference's producers start staggered and stream continuously: demo/load-generator/
main.go:166-184,204-240; its chat UI reports per-request TTFT: demo/chat-ui/index.html:580-588) through the
full path -- POST /chat on the native server -> engine (decode-priority chunked prefill, PREFILL_BUDGET prompt
tokens per step while streams decode) -> bus -> SSE sockets of the native load generator (-rate).

Per rate point: TTFT = first token received - request sent (short and long prompts separately), in-flight ITL
= gaps between consecutive tokens of a stream (its first token excluded), both p50 / p99, plus the mean number
of concurrent streams and the delivered token rate in the measurement window (the first `--skip-s` seconds,
while the system fills, are excluded from ITL).

    python tools/bench_serving.py --rates 40,70 --requests 600 --max-tokens 200 --prefill-budget 512,2048
    python tools/bench_serving.py --rates 70 --long-every 50 --long-words 8000   # some 8k-token prompts

Random-init Mistral-7B weights, synthetic prompts (one token per word).  Prints one JSON line per point.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def analyse(arrivals, n_req, long_every, skip_s, max_tokens):
    import numpy as np

    by = {}
    for s, seq, recv, _ts in arrivals:
        by.setdefault(int(s), []).append((int(seq), int(recv)))
    if not by:
        return {"error": "no arrivals"}
    t_first_send = min(min(r for q, r in v if q == 0) for v in by.values() if any(q == 0 for q, _ in v))
    w0 = t_first_send + int(skip_s * 1e9)
    ttft_s, ttft_l, gaps, spans, done, toks = [], [], [], [], 0, 0
    t_end = 0
    for s, v in by.items():
        v.sort(key=lambda x: x[1])
        send = [r for q, r in v if q == 0]
        tk = [r for q, r in v if q > 0]
        if not send or not tk:
            continue
        is_long = long_every > 0 and s % long_every == long_every - 1
        (ttft_l if is_long else ttft_s).append((tk[0] - send[0]) / 1e6)
        gaps += [(b - a) / 1e6 for a, b in zip(tk, tk[1:]) if a >= w0]
        spans.append((send[0], tk[-1]))
        toks += sum(1 for r in tk if r >= w0)
        t_end = max(t_end, tk[-1])
        done += 1
    q = lambda a, p: round(float(np.percentile(a, p)), 3) if len(a) else None  # noqa: E731
    win = max(1e-9, (t_end - w0) / 1e9)
    conc = sum(max(0, min(e, t_end) - max(b, w0)) for b, e in spans) / 1e9 / win
    return {"requests": n_req, "completed": done,
            "ttft_ms": {"p50": q(ttft_s, 50), "p99": q(ttft_s, 99), "n": len(ttft_s)},
            "ttft_long_ms": {"p50": q(ttft_l, 50), "p99": q(ttft_l, 99), "n": len(ttft_l)},
            "itl_ms": {"p50": q(gaps, 50), "p90": q(gaps, 90), "p99": q(gaps, 99), "max": q(gaps, 100)},
            "mean_concurrent_streams": round(conc, 1), "tokens_per_s": round(toks / win, 1), "window_s": round(win, 2)}


def ttft_split(trace):
    """p50 / p90 (ms) of the server-side parts of TTFT: arrival (HTTP request in the runtime) -> queued in the engine
    (polled + tokenized), queued -> first prompt chunk planned, planned -> first token drained, and the whole."""
    if not trace:
        return {}
    parts = {"poll_tokenize": [(q - a) / 1e6 for a, q, _, _ in trace],
             "queue": [(d - q) / 1e6 for _, q, d, _ in trace if d],
             "prefill_steps": [(t - d) / 1e6 for _, _, d, t in trace if d],
             "server_ttft": [(t - a) / 1e6 for a, _, _, t in trace]}
    out = {}
    for k, v in parts.items():
        if v:
            v = sorted(v)
            out[k] = {"p50": round(v[len(v) // 2], 2), "p90": round(v[int(len(v) * 0.9)], 2)}
    return out


def enq_split(trace):
    """p50 / p90 (ms) of the host time from a step's start to its enqueue, by step kind: the work the
    just-in-time margin has to cover."""
    out = {}
    for kind in sorted({e[0] for e in trace or ()}):
        v = sorted(e[1] * 1e3 for e in trace if e[0] == kind)
        out[kind] = {"n": len(v), "p50": round(v[len(v) // 2], 3), "p90": round(v[int(len(v) * 0.9)], 3)}
        phases = [e[2] for e in trace if e[0] == kind and len(e) > 2]
        if phases:  # engine.step: admit / compact, chunk plan, slot upload, the runner's enqueue
            for i, name in enumerate(("admit", "plan", "upload", "enqueue")):
                u = sorted(p[i] * 1e3 for p in phases)
                out[kind][name + "_p50"] = round(u[len(u) // 2], 3)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="mistral-7b-v0.3")
    ap.add_argument("--rates", default="70", help="comma list of request rates (req/s)")
    ap.add_argument("--requests", type=int, default=600)
    ap.add_argument("--max-tokens", type=int, default=200)
    ap.add_argument("--prompt-words", type=int, default=500, help="short prompt length (~1 token per word)")
    ap.add_argument("--long-every", type=int, default=0)
    ap.add_argument("--long-words", type=int, default=8000)
    ap.add_argument("--prefill-budget", default="",
                    help="comma list of PREFILL_BUDGET values (unset: the serving default)")
    ap.add_argument("--itl-ratios", default="",
                    help="comma list of DSSE_PREFILL_ITL_RATIO values (0 = fixed sizes; r > 1 = prompt work sized from "
                         "measured cost so a token gap stays <= r x the bucket's step; unset: the engine default)")
    ap.add_argument("--max-batch", type=int, default=256)
    ap.add_argument("--max-model-len", type=int, default=8448)
    ap.add_argument("--skip-s", type=float, default=2.0)
    ap.add_argument("--warmup-requests", type=int, default=48)
    ap.add_argument("--engine", default="gpu", help="gpu | cpu (the tiny CPU model: a functional check of the tool)")
    ap.add_argument("--no-queue-boost", action="store_true", help="mixed chunks stay at the ratio-sized cap when prompts queue")
    a = ap.parse_args()

    from distributed_sse_for_llm_response_amd.engine import bench_harness

    client = bench_harness.spawn_client()  # before this process touches the GPU

    import torch  # noqa: F401

    from distributed_sse_for_llm_response_amd.serving.app import ServingApp
    from distributed_sse_for_llm_response_amd.serving.config import ServeConfig

    cfg = ServeConfig(host="127.0.0.1", sse_port=0, origin_port=-1, metrics_port=-1, engine=a.engine, model=a.model,
                      max_batch=a.max_batch, max_model_len=a.max_model_len, max_tokens=a.max_tokens,
                      temperature=1.0, first_token_timeout_ms=300000)
    t0 = time.time()
    app = ServingApp(cfg).start()
    if a.no_queue_boost:
        app.engine.mixed_queue_boost = False
    print(f"[bench_serving] engine up in {time.time() - t0:.1f}s", file=sys.stderr, flush=True)
    port = app.port("edge")
    message = " ".join(f"w{i % 997}" for i in range(a.prompt_words))
    try:
        runs = 0
        budgets = [int(b) for b in a.prefill_budget.split(",")] if a.prefill_budget else [None]
        ratios = [float(q) for q in a.itl_ratios.split(",")] if a.itl_ratios else [None]
        for budget, ratio in [(b, q) for b in budgets for q in ratios]:
            if budget is not None:
                app.engine.prefill_budget = budget
            if ratio is not None:
                app.engine.set_itl_ratio(ratio)
            budget = app.engine.prefill_budget
            ratio = app.engine.cost.ratio if app.engine.cost is not None else 0.0
            for rate in [float(r) for r in a.rates.split(",")]:
                for warm, n in ((True, a.warmup_requests), (False, a.requests)):
                    if warm and runs > 0:
                        continue
                    runs += 1
                    req = {"host": "127.0.0.1", "port": port, "streams": n, "message": message,
                           "max_tokens": a.max_tokens, "prefix": f"srv{runs}-", "rate": rate, "seed": runs,
                           "duration_s": 1200}
                    if a.long_every and not warm:
                        req.update(long_every=a.long_every, long_words=a.long_words)
                    app.engine.ttft_trace = []
                    app.engine.enq_trace = []
                    app.engine.r.host_trace = []
                    client.stdin.write(json.dumps(req) + "\n")
                    client.stdin.flush()
                    res = json.loads(client.stdout.readline())
                    if warm:
                        continue
                    out = {"metric": "serving under Poisson arrivals", "rate_req_s": rate, "prefill_budget": budget,
                           "itl_ratio": ratio,
                           "max_tokens": a.max_tokens, "prompt_tokens": a.prompt_words + 6,
                           "long_prompt_every": a.long_every, "long_prompt_tokens": a.long_words + 6 if a.long_every else 0,
                           **analyse(res["arrivals"], n, a.long_every, a.skip_s, a.max_tokens),
                           "server_ttft_split_ms": ttft_split(app.engine.ttft_trace),
                           "host_enqueue_ms": enq_split(app.engine.enq_trace),
                           "mixed_host_ms": enq_split([(k, t) for row in app.engine.r.host_trace or ()
                                                       for k, t in zip(("upload", "replay", "sample"), row)]),
                           "client_errors": res.get("errors", [])[:3], "engine_stats_cumulative": {
                               k: app.engine.stats.get(k) for k in ("prefill_tokens", "decode_steps", "steps", "mixed_steps",
                                                                    "mixed_graph_rows", "preemptions", "compactions")},
                           # the engine's measured decode step per bucket (EMA, ms): ITL p99 is judged against the
                           # occupied bucket's value
                           "decode_step_ms": {b: round(v, 3) for b, v in sorted(
                               (app.engine.cost.step_ms if app.engine.cost is not None else {}).items())}}
                    print(json.dumps(out), flush=True)
    finally:
        client.stdin.close()
        app.stop()


if __name__ == "__main__":
    main()
