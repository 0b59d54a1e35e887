"""Tensor-parallel serving: one TP group per engine replica, its leader mirrored by the followers.

A TP group of T ranks (T GPUs, one process each) runs ONE engine: every rank holds a 1/T Megatron shard of
the weights and executes the identical scheduler, and the decode step's collectives (two all-reduces per
layer, the sampling-candidate all-gather; ``parallel/comm.py``) run over RCCL inside the captured graph.
Only the group's leader talks to the outside world (the runtime, or a data-parallel router's ring); before
each engine step it broadcasts a **plan** -- the step's admissions, aborts and flow-control changes -- to
the followers, which apply it to their own engine and step too.  Every scheduling decision is then made
from identical inputs on every rank: the engine runs with ``deterministic=True`` (drained steps are
consumed by count, never by whether an event happens to have completed on this rank).

The plan is a fixed-size int32 message broadcast over a CPU (gloo) group of the TP ranks -- no pickling,
no GPU sync -- split over several broadcasts when a step admits more prompt tokens than one holds.
Followers know sequences by the leader's request id (``Sequence.rid``, which also seeds their sampling),
so no conversation-id strings cross ranks.

Reference: the reference configures TP only as a vLLM flag (kubernetes/base/llm/deployment.yaml:88-89).
"""
from __future__ import annotations

import struct
from dataclasses import dataclass, field

import torch
import torch.distributed as dist

from ..engine.engine import SamplingParams

MAGIC = 0x54505031  # "TPP1"
F_STEP, F_STOP, F_MORE, F_SYNC = 1, 2, 4, 8


def _f2i(x: float) -> int:
    return struct.unpack("<i", struct.pack("<f", float(x)))[0]


def _i2f(x: int) -> float:
    return struct.unpack("<f", struct.pack("<i", int(x)))[0]


@dataclass
class Plan:
    step: bool = False
    stop: bool = False
    sync: bool = False  # followers run the caller's sync hook after the step (e.g. a timing barrier)
    adds: list = field(default_factory=list)    # (rid, prompt ids, SamplingParams, arrival_ns)
    aborts: list = field(default_factory=list)  # rid
    flow: list = field(default_factory=list)    # (rid, paused)

    def empty(self) -> bool:
        return not (self.step or self.stop or self.sync or self.adds or self.aborts or self.flow)

    # ---- int32 wire form ----------------------------------------------------------------------
    def encode(self) -> list:
        w = []
        for rid, prompt, p, arrival in self.adds:
            seed = -1 if p.seed is None else int(p.seed) & 0x7FFFFFFF
            w += [rid, arrival & 0x7FFFFFFF, (arrival >> 31) & 0x7FFFFFFF, int(p.max_tokens), int(p.top_k), seed,
                  int(bool(p.ignore_eos)), _f2i(p.temperature), _f2i(p.top_p), len(prompt)]
            w += [int(t) for t in prompt]
        for rid in self.aborts:
            w.append(rid)
        for rid, paused in self.flow:
            w += [rid, int(bool(paused))]
        return w

    @staticmethod
    def decode(flags: int, n_add: int, n_abort: int, n_flow: int, w: list) -> "Plan":
        p = Plan(step=bool(flags & F_STEP), stop=bool(flags & F_STOP), sync=bool(flags & F_SYNC))
        o = 0
        for _ in range(n_add):
            rid, a_lo, a_hi, mt, tk, seed, ie, temp, top_p, n = w[o:o + 10]
            o += 10
            prompt = w[o:o + n]
            o += n
            sp = SamplingParams(temperature=_i2f(temp), top_p=_i2f(top_p), top_k=tk, max_tokens=mt,
                                seed=None if seed < 0 else seed, ignore_eos=bool(ie))
            p.adds.append((rid, prompt, sp, a_lo | (a_hi << 31)))
        for _ in range(n_abort):
            p.aborts.append(w[o])
            o += 1
        for _ in range(n_flow):
            p.flow.append((w[o], bool(w[o + 1])))
            o += 2
        return p


class PlanChannel:
    """Leader -> followers plan broadcast over a gloo group of one TP group (``src`` = leader's global rank)."""

    HEADER = 6  # magic, flags, n_add, n_abort, n_flow, payload words in this message

    def __init__(self, group, src: int, capacity: int = 1 << 16):
        self.group, self.src, self.cap = group, src, capacity
        self.buf = torch.zeros(capacity, dtype=torch.int32)

    def send(self, plan: Plan) -> None:
        words = plan.encode()
        room = self.cap - self.HEADER
        chunks = [words[i:i + room] for i in range(0, len(words), room)] or [[]]
        for k, chunk in enumerate(chunks):
            last = k == len(chunks) - 1
            flags = ((F_STEP if plan.step else 0) | (F_STOP if plan.stop else 0) | (F_SYNC if plan.sync else 0) |
                     (0 if last else F_MORE))
            self.buf[: self.HEADER] = torch.tensor([MAGIC, flags, len(plan.adds), len(plan.aborts), len(plan.flow),
                                                    len(chunk)], dtype=torch.int32)
            if chunk:
                self.buf[self.HEADER:self.HEADER + len(chunk)] = torch.tensor(chunk, dtype=torch.int32)
            dist.broadcast(self.buf, src=self.src, group=self.group)

    def recv(self) -> Plan:
        words = []
        while True:
            dist.broadcast(self.buf, src=self.src, group=self.group)
            magic, flags, n_add, n_abort, n_flow, n = self.buf[: self.HEADER].tolist()
            if magic != MAGIC:
                raise RuntimeError(f"TP plan channel: bad message (magic {magic:#x})")
            words += self.buf[self.HEADER:self.HEADER + n].tolist()
            if not flags & F_MORE:
                return Plan.decode(flags, n_add, n_abort, n_flow, words)


def follower_conv(rid: int) -> str:
    return f"tp-rid-{rid}"


def apply_plan(engine, plan: Plan, conv_of=follower_conv) -> None:
    """Apply a plan's admissions, aborts and flow changes to an engine, in that order (leader and followers)."""
    for rid, prompt, params, arrival in plan.adds:
        engine.add_request(conv_of(rid), prompt, params, arrival_ns=arrival, rid=rid)
    for rid in plan.aborts:
        engine.abort(conv_of(rid))
    for rid, paused in plan.flow:
        engine.set_paused(conv_of(rid), paused)


class TPLeader:
    """The leader's side: collects the step's inputs, broadcasts them, applies them locally and steps."""

    def __init__(self, engine, channel: PlanChannel | None):
        self.engine, self.ch = engine, channel
        self.plan = Plan()
        self._conv = {}   # rid -> conversation id (leader's real ids)
        self._rid = {}    # conversation id -> rid

    def add(self, conversation_id: str, prompt: list, params: SamplingParams, arrival_ns: int) -> None:
        rid = self.engine.next_rid()
        self._conv[rid], self._rid[conversation_id] = conversation_id, rid
        self.plan.adds.append((rid, list(prompt), params, arrival_ns))

    def abort(self, conversation_id: str) -> None:
        rid = self._rid.get(conversation_id)
        if rid is not None:
            self.plan.aborts.append(rid)

    def set_paused(self, conversation_id: str, paused: bool) -> None:
        rid = self._rid.get(conversation_id)
        if rid is not None:
            self.plan.flow.append((rid, paused))

    def step(self, run: bool = True) -> list:
        """Broadcast and apply the pending plan; with `run`, step the engine (returns its events)."""
        plan, self.plan = self.plan, Plan()
        plan.step = run
        if self.ch is not None:
            self.ch.send(plan)
        apply_plan(self.engine, plan, self._conv.__getitem__)
        events = self.engine.step() if run else []
        for e in events:  # forget finished conversations
            if e.done:
                rid = self._rid.pop(e.conversation_id, None)
                if rid is not None:
                    self._conv.pop(rid, None)
        return events

    def sync(self) -> None:
        """Ask the followers to run their sync hook now (the leader runs its own right after)."""
        if self.ch is not None:
            self.ch.send(Plan(sync=True))

    def stop(self) -> None:
        if self.ch is not None:
            self.ch.send(Plan(stop=True))


def follower_loop(engine, channel: PlanChannel, on_sync=None) -> None:
    """A follower rank: mirror the leader's plans until it sends stop."""
    while True:
        plan = channel.recv()
        if plan.stop:
            return
        apply_plan(engine, plan)
        if plan.step:
            engine.step()
        if plan.sync and on_sync is not None:
            on_sync()


def make_tp_groups(world: int, tp: int, backend: str):
    """(tp_group, plan_group, group_index, leader_global_rank) of this rank.  Every rank must call it (group
    creation is collective); TP groups are contiguous ranks [g*tp, (g+1)*tp)."""
    rank = dist.get_rank()
    mine = (None, None, rank // tp, (rank // tp) * tp)
    for g in range(world // tp):
        ranks = list(range(g * tp, (g + 1) * tp))
        tg = dist.new_group(ranks, backend=backend) if tp > 1 else None
        pg = dist.new_group(ranks, backend="gloo") if tp > 1 else None
        if rank in ranks:
            mine = (tg, pg, g, g * tp)
    return mine
