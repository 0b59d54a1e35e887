#!/usr/bin/env python3
"""Per-step host cost of the TP leader -> followers plan (serving/tp.py), CPU only.

Spawns T processes (gloo); the leader sends --steps plans (empty step plans, the steady decode case, and
every 16th step one admission of a --prompt-len prompt), each follower timestamps the arrival.  Reported:
the leader's send() time per plan and the send -> follower-receive latency (CLOCK_MONOTONIC, comparable across
processes of one host), for the shared-memory rings and the gloo fallback, plus the round-2 channel (a 64 Ki-word
gloo broadcast every step) for comparison.

    python tools/bench_plan_channel.py --tp 8 --steps 2000
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402

from distributed_sse_for_llm_response_amd.engine.engine import SamplingParams  # noqa: E402
from distributed_sse_for_llm_response_amd.serving.tp import GlooPlanChannel, Plan, ShmPlanChannel  # noqa: E402


class _Round2Channel:
    """The round-2 channel: the whole 65,536-word buffer broadcast over gloo every step."""

    def __init__(self, src):
        self.src, self.buf = src, torch.zeros(1 << 16, dtype=torch.int32)

    def send(self, plan):
        dist.broadcast(self.buf, src=self.src)

    def recv(self):
        dist.broadcast(self.buf, src=self.src)
        return Plan(step=True)


def _plans(steps, prompt_len):
    out = []
    for i in range(steps):
        p = Plan(step=True)
        if i % 16 == 0:
            p.adds.append((i, list(range(prompt_len)), SamplingParams(temperature=1.0, seed=i), time.time_ns()))
        out.append(p)
    return out + [Plan(stop=True)]


def _worker(rank, world, port, kind, steps, prompt_len, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        ranks = list(range(world))
        ch = {"shm": lambda: ShmPlanChannel(None, 0, rank, ranks, tag=f"bench-{port}"),
              "gloo": lambda: GlooPlanChannel(None, 0), "round2": lambda: _Round2Channel(0)}[kind]()
        plans = _plans(steps, prompt_len)
        dist.barrier()
        if rank == 0:
            sends, t_sent = [], []
            for p in plans:
                time.sleep(0.0002)  # the leader's GPU step between plans; followers are waiting, not racing
                t0 = time.perf_counter_ns()
                ch.send(p)
                t1 = time.perf_counter_ns()
                sends.append((t1 - t0) / 1e3)
                t_sent.append(t0)
            out[0] = (sends, t_sent)
        else:
            t_recv = []
            for _ in plans:
                ch.recv()
                t_recv.append(time.perf_counter_ns())
            out[rank] = t_recv
        dist.barrier()
    finally:
        dist.destroy_process_group()


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def run(kind, tp, steps, prompt_len):
    with mp.Manager() as m:
        out = m.dict()
        mp.spawn(_worker, args=(tp, _port(), kind, steps, prompt_len, out), nprocs=tp, join=True)
        sends, t_sent = out[0]
        lat = [max(out[r][i] for r in range(1, tp)) - t_sent[i] for i in range(len(t_sent))]
    sends, lat = sends[:-1], [x / 1e3 for x in lat[:-1]]
    q = lambda v, f: sorted(v)[min(len(v) - 1, int(f * len(v)))]  # noqa: E731
    return {"channel": kind, "tp": tp, "steps": steps,
            "leader_send_us": {"p50": round(statistics.median(sends), 2), "p99": round(q(sends, 0.99), 2)},
            "send_to_last_follower_us": {"p50": round(statistics.median(lat), 2), "p99": round(q(lat, 0.99), 2)}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tp", type=int, default=8)
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--prompt-len", type=int, default=512)
    ap.add_argument("--kinds", default="shm,gloo,round2")
    a = ap.parse_args()
    for kind in a.kinds.split(","):
        print(json.dumps(run(kind, a.tp, a.steps, a.prompt_len)), flush=True)


if __name__ == "__main__":
    main()
