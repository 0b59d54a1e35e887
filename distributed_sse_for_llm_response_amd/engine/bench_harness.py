"""Decode-throughput harness behind bench.py (one engine replica per rank)."""
from __future__ import annotations

import math
import time

import numpy as np
import torch

from ..models.mistral import TINY, get_config
from ..parallel.comm import TPComm
from .kv_cache import PAGE, KVCache, blocks_needed
from .model_runner import RING_SIZE, ModelRunner, PrefillSeq
from .weights import random_engine_weights


class _Drain:
    """Side-stream device->host copy of one token-ring row per step into pinned memory."""

    def __init__(self, runner: ModelRunner):
        self.r = runner
        self.cuda = runner.device.type == "cuda"
        B = runner.max_batch
        if self.cuda:
            self.host = torch.zeros(RING_SIZE, B, dtype=torch.int32).pin_memory()
            self.stream = torch.cuda.Stream(runner.device)
            self.done = [torch.cuda.Event() for _ in range(RING_SIZE)]
        else:
            self.host = torch.zeros(RING_SIZE, B, dtype=torch.int32)

    def issue(self, row: int, B: int):
        if not self.cuda:
            self.host[row, :B] = self.r.ring[row, :B]
            return
        main = torch.cuda.current_stream(self.r.device)
        self.stream.wait_stream(main)
        with torch.cuda.stream(self.stream):
            self.host[row, :B].copy_(self.r.ring[row, :B], non_blocking=True)
            self.done[row].record(self.stream)

    def wait(self, row: int):
        if self.cuda:
            self.done[row].synchronize()
        return self.host[row]


class PacedStubEngine:
    """Host-path rehearsal engine: the LLMEngine surface the serving bench drives (add_request / step /
    slots / has_work), emitting one token per live stream every `step_ms`, like a GPU replica decoding
    at that step time.  Lets the N-replica router + bus + SSE server + client path be driven at the
    token rate of N real GPUs (N x streams / step_ms) on a host without them."""

    class _Seq:
        __slots__ = ("conversation_id", "state", "sequence", "max_tokens")

        def __init__(self, cid, max_tokens):
            self.conversation_id, self.state, self.sequence, self.max_tokens = cid, "decode", 0, max_tokens

    def __init__(self, streams: int, step_ms: float, vocab: int):
        from .engine import TokenEvent

        self.TokenEvent = TokenEvent
        self.slots: list = [None] * streams
        self.step_s = step_ms / 1000.0
        self.vocab = vocab
        self.next_t = 0.0
        self.started = False

    def next_rid(self) -> int:
        self._rid = getattr(self, "_rid", 0) + 1
        return self._rid

    def add_request(self, conversation_id, prompt, params, arrival_ns=0, rid=None):
        free = self.slots.index(None)
        self.slots[free] = self._Seq(conversation_id, params.max_tokens)

    def has_work(self) -> bool:
        return any(s is not None for s in self.slots)

    def step(self, block: bool = True) -> list:
        if not self.started:  # hold tokens until every stream is admitted (the stub has no prefill to bound skew)
            if any(s is None for s in self.slots):
                time.sleep(0.001)
                return []
            self.started = True
        now = time.perf_counter()
        if self.next_t > now:
            time.sleep(self.next_t - now)
        self.next_t = max(now, self.next_t) + self.step_s
        ev = []
        for i, s in enumerate(self.slots):
            if s is None:
                continue
            s.sequence += 1
            if s.sequence > s.max_tokens:
                ev.append(self.TokenEvent(s.conversation_id, 0, s.sequence, True, "[DONE]"))
                self.slots[i] = None
            else:
                ev.append(self.TokenEvent(s.conversation_id, 3 + (s.sequence * 7919 + i) % (self.vocab - 3),
                                          s.sequence, False))
        return ev


def _build_runner(model: str, device, streams: int, prompt_len: int, total_steps: int, tp: int, use_graphs: bool,
                  rank: int, world: int, comm: TPComm | None = None):
    # on CPU the 7B architecture is replaced by the tiny one (plumbing runs); named small configs are kept
    cfg = get_config(model) if device.type == "cuda" or not model.startswith("mistral-7b") else TINY
    if comm is None:
        comm = TPComm()
        if tp > 1:
            from ..parallel.comm import make_groups

            grp, _ = make_groups(world, tp)
            comm = TPComm(rank=rank % tp, size=tp, group=grp)
    w = random_engine_weights(cfg, tp_rank=comm.rank, tp_size=comm.size, device=device, seed=1234)
    max_len = prompt_len + total_steps + 2 * PAGE
    nblk = streams * (blocks_needed(max_len) + 1) + 4
    runner = ModelRunner(w, num_blocks=nblk, max_batch=streams, max_model_len=max_len, device=device, comm=comm,
                         use_graphs=use_graphs)
    return cfg, runner


def run_decode_bench(model="mistral-7b-v0.3", device=None, streams=64, prompt_len=512, steps=64, warmup=8, tp=1,
                     delivery="frame", use_graphs=True, rank=0, world=1, seed=0):
    device = device or torch.device("cuda" if torch.cuda.is_available() else "cpu")
    total = steps + warmup
    cfg, r = _build_runner(model, device, streams, prompt_len, total, tp, use_graphs, rank, world)
    gen = torch.Generator().manual_seed(seed + rank)
    V = cfg.vocab_size
    # ---- admit `streams` sequences: block tables, sampling params (vLLM defaults: T=1, top_p=1) ----
    per = blocks_needed(prompt_len + total + 1)
    bt = torch.zeros(streams, r.max_blocks, dtype=torch.int32)
    seqs = []
    for s in range(streams):
        blocks = list(range(s * per, (s + 1) * per))
        bt[s, :per] = torch.tensor(blocks, dtype=torch.int32)
        toks = torch.randint(3, V, (prompt_len,), generator=gen).tolist()
        seqs.append(PrefillSeq(slot=s, tokens=toks, start_pos=0, block_table=blocks, last_chunk=True))
    r.block_tables.copy_(bt.to(device))
    r.temperature.fill_(1.0)
    r.top_p.fill_(1.0)
    r.top_k.fill_(0)
    r.seeds.copy_(torch.randint(0, 2**31 - 1, (streams, 2), generator=gen, dtype=torch.int32).to(device))
    # ---- prefill in packed chunks of <= max_prefill_tokens ----
    chunk = max(1, r.max_prefill_tokens // max(1, prompt_len))
    for i in range(0, streams, chunk):
        r.prefill(seqs[i:i + chunk], ring_row=0)
    r.active.fill_(1)
    if use_graphs and device.type == "cuda":
        r.capture([streams])
    if device.type == "cuda":
        torch.cuda.synchronize(device)
    head = int(r.ring_counter.item())
    drain = _Drain(r)
    conv_ids = [f"bench-{rank}-{s}" for s in range(streams)]
    seq_no = [0] * streams
    frames_bytes = 0
    deliver_ts = []

    def deliver(row):
        nonlocal frames_bytes
        toks = drain.wait(row)[:streams].tolist()
        now = time.time_ns()
        if delivery != "none":
            for s, t in enumerate(toks):
                seq_no[s] += 1
                body = ('{"conversation_id":"%s","token":"%s","sequence":%d,"done":false,"timestamp":%d}'
                        % (conv_ids[s], "t%d" % t, seq_no[s], now))
                frame = "event: token\nid: %d\ndata: %s\n\n" % (seq_no[s], body)
                frames_bytes += len(frame)
        deliver_ts.append(time.perf_counter())

    def run(n):
        nonlocal head
        prev = None
        for _ in range(n):
            r.decode(streams)
            row = head % RING_SIZE
            head += 1
            drain.issue(row, streams)
            if prev is not None:
                deliver(prev)
            prev = row
        if prev is not None:
            deliver(prev)

    run(warmup)
    deliver_ts.clear()
    _sync(device, world)
    t0 = time.perf_counter()
    run(steps)
    _sync(device, world)
    elapsed = time.perf_counter() - t0
    itl = np.diff(np.array(deliver_ts)) * 1000.0 if len(deliver_ts) > 1 else np.array([elapsed * 1000.0])
    return {"elapsed_s": elapsed, "p50_itl_ms": float(np.percentile(itl, 50)),
            "p99_itl_ms": float(np.percentile(itl, 99)), "frames_bytes": frames_bytes, "model": cfg.name}


def spawn_client():
    """Start the SSE client process (call BEFORE the GPU is initialised in this process).  The package's parent
    directory goes on the child's PYTHONPATH, so the client starts whatever the working directory is (e.g.
    under rocprofv3 run from /tmp)."""
    import os
    import subprocess
    import sys
    from pathlib import Path

    env = dict(os.environ)
    root = str(Path(__file__).resolve().parents[2])
    env["PYTHONPATH"] = root + (os.pathsep + env["PYTHONPATH"] if env.get("PYTHONPATH") else "")
    return subprocess.Popen([sys.executable, "-m", "distributed_sse_for_llm_response_amd.engine.bench_client"],
                            stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True, env=env)


def run_serving_bench(client, model="mistral-7b-v0.3", device=None, streams=64, prompt_len=512, steps=64, warmup=8,
                      tp=1, use_graphs=True, rank=0, world=1, seed=0, stub_step_ms=0.0):
    """Full serving path: `streams` real POST /chat SSE connections per engine replica (one client process on
    rank 0) -> native runtime + data-parallel router on rank 0 -> shared-memory ring -> this rank's LLMEngine
    (scheduler, hipGraph decode, token-ring drain) -> ring -> router -> bus -> epoll writers -> sockets.

    Every TP group of `tp` ranks is one replica (tp == 1: every rank) and serves the `streams` conversations
    the router assigns it; inside a group the leader drives its followers with per-step plans
    (serving/tp.py), and the decode step's all-reduces / all-gather run over the group's communicator.
    Timed: exactly `steps` engine steps on every replica once all of its streams are decoding, bracketed by
    barrier + device synchronize.  The p50 inter-token latency is measured by the client (socket receive
    times of consecutive tokens of a stream) inside the timed window."""
    import json as _json
    import os

    from .. import runtime as rt_mod
    from ..models.tokenizer import SyntheticTokenizer, prompt_for_request
    from .engine import LLMEngine, SamplingParams

    from ..serving.tp import TPLeader, follower_loop, make_plan_channel, make_tp_groups

    device = device or torch.device("cuda" if torch.cuda.is_available() else "cpu")
    if world % tp:
        raise ValueError(f"world size {world} is not a multiple of tp={tp}")
    replicas, group, leader = world // tp, rank // tp, (rank // tp) * tp
    comm, plan_ch = TPComm(), None
    if tp > 1:
        import torch.distributed as dist

        tp_group, plan_group, group, leader = make_tp_groups(world, tp, dist.get_backend())
        comm = TPComm(rank=rank - leader, size=tp, group=tp_group)
        plan_ch = make_plan_channel(plan_group, leader, group, tp)
    # Admission prefills ~max_prefill_tokens of prompts per engine step while the already admitted streams
    # decode, so the first streams run ahead by up to `skew` steps.  Every stream must stay live through
    # the whole timed window (full batch on every timed step): budget the tokens and the KV for it.
    skew = math.ceil(streams * (prompt_len + 16) / 8192) + 4
    total = steps + warmup + skew
    if stub_step_ms > 0 and tp > 1:
        raise ValueError("the paced-stub rehearsal stands in for whole replicas (tp=1)")
    if stub_step_ms > 0:  # host-path rehearsal: paced stub replicas, no model
        cfg = get_config(model)
        tok = SyntheticTokenizer(cfg.vocab_size)
        engine = PacedStubEngine(streams, stub_step_ms, cfg.vocab_size)
    else:
        cfg, r = _build_runner(model, device, streams, prompt_len + 16, total + 4, tp, use_graphs, rank, world, comm)
        if use_graphs and device.type == "cuda":
            r.capture()
        tok = SyntheticTokenizer(cfg.vocab_size)
        engine = LLMEngine(r, eos_id=tok.eos_id, prefill_budget=r.max_prefill_tokens,
                           default_params=SamplingParams(temperature=1.0, top_p=1.0, max_tokens=total + 2))
    if rank != leader:  # a TP follower: mirror the leader's plans (its syncs included) until it stops
        follower_loop(engine, plan_ch, on_sync=lambda: _sync(device, world))
        _sync(device, world)
        return {"elapsed_s": 0.0, "p50_itl_ms": 0.0, "p99_itl_ms": 0.0, "delivered_in_window": None,
                "client_errors": [], "model": cfg.name, "max_context": prompt_len + 16 + total}
    drv = TPLeader(engine, plan_ch)

    def sync():
        drv.sync()
        _sync(device, world)
    mod = rt_mod.load()
    prefix = f"/dsse-bench-{os.environ.get('MASTER_PORT', '0')}-{os.getppid() if world > 1 else os.getpid()}"
    runtime = None
    if rank == 0:
        runtime = mod.Runtime({"host": "127.0.0.1", "sse_port": 0, "origin_port": -1, "metrics_port": -1,
                               "resp_port": -1, "io_threads": 4, "local_engine": True})
        runtime.set_vocab(tok.pieces())
        runtime.start_dp_router(prefix, replicas, 4, 600_000)  # 4 MiB rings: /dev/shm may be small in containers
        runtime.start()
    chan = mod.DpWorker(prefix, group, 600_000)
    chan.set_ready(True)
    if rank == 0:
        while sum(1 for i in runtime.dp_workers() if i["ready"]) < replicas:
            time.sleep(0.01)
        words = [f"w{i % 997}" for i in range(max(1, prompt_len - 8))]
        client.stdin.write(_json.dumps({"host": "127.0.0.1", "port": runtime.bound_port("edge"),
                                        "streams": streams * replicas, "message": " ".join(words),
                                        "max_tokens": total + 2, "prefix": "bench-"}) + "\n")
        client.stdin.flush()
        client.stdin.close()  # one run: the client exits after it

    def publish(events):
        if events:
            chan.publish_tokens([e.conversation_id for e in events], [e.token_id for e in events],
                                [e.sequence for e in events], [e.done for e in events], 0, [e.text for e in events])

    def pump(block_ms=0):
        for req in chan.poll_requests(1024, block_ms):
            p = SamplingParams(temperature=1.0, top_p=1.0, max_tokens=req["max_tokens"], ignore_eos=True)
            drv.add(req["conversation_id"], prompt_for_request(tok, req), p, req["arrival_ns"])

    def step():
        return drv.step(run=engine.has_work() or bool(drv.plan.adds))

    import gc

    gc.collect()
    gc.freeze()  # as in the serving loop (serving/app.py EngineLoop.run)
    # admission + prefill until every stream of this replica is decoding
    live = lambda: sum(1 for s in engine.slots if s is not None and s.state == "decode")  # noqa: E731
    t_admit = time.time()
    # the setup burst is prefilled in whole max_prefill_tokens passes, as the skew above assumes (mixed steps --
    # the serving default -- would absorb it in decode-sized chunks over ~100 steps; no prompt enters the timed
    # window, so the setting does not touch what is measured)
    boost = getattr(engine, "mixed_boost_steps", None)
    if boost is not None:
        engine.mixed_boost_steps = -1
    while sum(1 for s in engine.slots if s is not None and s.state == "decode") < streams:
        pump(20 if not engine.has_work() else 0)
        if engine.has_work() or drv.plan.adds:
            publish(step())
        if time.time() - t_admit > 900:
            raise RuntimeError("bench: streams did not all start decoding")
    if boost is not None:
        engine.mixed_boost_steps = boost
    sync()
    for _ in range(warmup):
        publish(step())
    sync()
    # stall attribution (timed window): per-step host / drain-wait time and start times, GC pauses
    trace, gc_ms = [], []
    gc_t = [0.0]

    def on_gc(phase, info):
        if phase == "start":
            gc_t[0] = time.perf_counter()
        else:
            gc_ms.append((time.perf_counter() - gc_t[0]) * 1000.0)

    gc.callbacks.append(on_gc)
    t0_ns = time.time_ns()
    t0 = time.perf_counter()
    for _ in range(steps):
        ts = time.perf_counter()
        publish(step())
        st = getattr(engine, "stats", {})
        trace.append((ts, time.perf_counter() - ts, st.get("host_s", 0.0), st.get("wait_s", 0.0)))
    sync()
    elapsed = time.perf_counter() - t0
    t1_ns = time.time_ns()
    gc.callbacks.remove(on_gc)
    if live() < streams:
        raise RuntimeError(f"bench: only {live()} of {streams} streams were still decoding at the end of the window")
    while engine.has_work():
        publish(step())
    drv.stop()
    res = {"arrivals": [], "errors": []}
    if rank == 0:
        out = client.stdout.readline()
        client.wait(timeout=300)
        res = _json.loads(out) if out.strip() else {"arrivals": [], "errors": ["client produced no output"]}
    _sync(device, world)  # the followers' last sync (after their loop's stop)
    if runtime is not None:
        runtime.stop()
    by_stream = {}
    for s, seq, t_ns, _ts in res["arrivals"]:
        by_stream.setdefault(s, []).append(t_ns)
    gaps = []
    for ts in by_stream.values():
        ts.sort()
        gaps += [(b - a) / 1e6 for a, b in zip(ts, ts[1:]) if t0_ns <= a and b <= t1_ns]
    delivered = sum(1 for _s, _q, t_ns, _ in res["arrivals"] if t0_ns <= t_ns <= t1_ns)
    itl = np.array(gaps) if gaps else np.array([elapsed * 1000.0 / max(1, steps)])
    return {"elapsed_s": elapsed, "p50_itl_ms": float(np.percentile(itl, 50)),
            "p99_itl_ms": float(np.percentile(itl, 99)), "delivered_in_window": delivered,
            "client_errors": res["errors"][:5], "model": cfg.name, "max_context": prompt_len + 16 + total,
            "stalls": _stall_report(trace, gc_ms, res["arrivals"], t0_ns, t1_ns) if rank == 0 else {}}


def _stall_report(trace, gc_ms, arrivals, t0_ns, t1_ns) -> dict:
    """Where inter-token time goes in the timed window: engine step cadence (host loop), its host vs
    drain-wait split, GC pauses, and the delivery delay (engine timestamp -> client socket receive)."""
    def pct(a, q):
        return round(float(np.percentile(a, q)), 4) if len(a) else 0.0

    starts = [t for t, *_ in trace]
    cadence = np.diff(starts) * 1000.0 if len(starts) > 1 else np.zeros(0)
    wall = np.array([w for _, w, _, _ in trace]) * 1000.0
    host = np.array([h for _, _, h, _ in trace]) * 1000.0
    wait = np.array([w for *_, w in trace]) * 1000.0
    deliv, eng = [], {}
    for s, _q, recv, ts in arrivals:
        if t0_ns <= recv <= t1_ns and ts > 0:
            deliv.append((recv - ts) / 1e6)
            eng.setdefault(s, []).append(ts)
    egaps = [(b - a) / 1e6 for v in eng.values() for a, b in zip(sorted(v), sorted(v)[1:])]
    return {"step_cadence_ms": {"p50": pct(cadence, 50), "max": pct(cadence, 100)},
            "step_wall_ms": {"p50": pct(wall, 50), "max": pct(wall, 100)},
            "host_ms": {"p50": pct(host, 50), "max": pct(host, 100)},
            "drain_wait_ms": {"p50": pct(wait, 50), "max": pct(wait, 100)},
            "gc": {"count": len(gc_ms), "max_ms": round(max(gc_ms), 4) if gc_ms else 0.0},
            "engine_token_gap_ms": {"p50": pct(egaps, 50), "p99": pct(egaps, 99)},
            "delivery_ms": {"p50": pct(deliv, 50), "p99": pct(deliv, 99), "max": pct(deliv, 100)}}


def _sync(device, world):
    if device.type == "cuda":
        torch.cuda.synchronize(device)
    if world > 1:
        import torch.distributed as dist

        dist.barrier()
