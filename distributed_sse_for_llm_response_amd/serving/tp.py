"""Tensor-parallel serving: one TP group per engine replica, its leader mirrored by the followers.

A TP group of T ranks (T GPUs, one process each) runs ONE engine: every rank holds a 1/T Megatron shard of
the weights and executes the identical scheduler, and the decode step's collectives (two all-reduces per
layer, the sampling-candidate all-gather; ``parallel/comm.py``) run over RCCL inside the captured graph.
Only the group's leader talks to the outside world (the runtime, or a data-parallel router's ring); before
each engine step it broadcasts a **plan** -- the step's admissions, aborts and flow-control changes -- to
the followers, which apply it to their own engine and step too.  Every scheduling decision is then made
from identical inputs on every rank: the engine runs with ``deterministic=True`` (drained steps are
consumed by count, never by whether an event happens to have completed on this rank).

The plan is a small int32 message (a 6-word header plus only the words the step needs -- an empty step is 24
bytes).  Between ranks of one node it travels through POSIX shared-memory rings (``ShmPlanChannel``: one SPSC
ring per follower, the follower polls for 2 ms -- longer than a TP decode step -- before it sleeps, so the per-step host cost is a few
microseconds -- ``tools/bench_plan_channel.py``, ``profiles/r3/plan_channel.md``); ``GlooPlanChannel`` (header
broadcast, then the payload only when there is one) is the fallback when the ranks do not share a node.  The
leader applies the DECODED plan, exactly what the followers apply, so every rank admits the same parameters
(seed, float32 temperature / top-p).  Followers know sequences by the leader's request id (``Sequence.rid``,
which also seeds their sampling), so no conversation-id strings cross ranks.

Reference: the reference configures TP only as a vLLM flag (kubernetes/base/llm/deployment.yaml:88-89).
"""
from __future__ import annotations

import struct
from array import array
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
            # seeds travel whole: two 31-bit words (the server accepts seeds up to 2^53 - 1); -1 = no seed
            if p.seed is None:
                s_lo, s_hi = -1, -1
            else:
                sd = int(p.seed)
                if not 0 <= sd < (1 << 62):
                    raise ValueError(f"TP plan: seed {sd} outside [0, 2^62)")
                s_lo, s_hi = sd & 0x7FFFFFFF, (sd >> 31) & 0x7FFFFFFF
            w += [rid, arrival & 0x7FFFFFFF, (arrival >> 31) & 0x7FFFFFFF, int(p.max_tokens), int(p.top_k), s_lo, s_hi,
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
            rid, a_lo, a_hi, mt, tk, s_lo, s_hi, ie, temp, top_p, n = w[o:o + 11]
            o += 11
            prompt = w[o:o + n]
            o += n
            sp = SamplingParams(temperature=_i2f(temp), top_p=_i2f(top_p), top_k=tk, max_tokens=mt,
                                seed=None if s_lo < 0 else s_lo | (s_hi << 31), ignore_eos=bool(ie))
            p.adds.append((rid, prompt, sp, a_lo | (a_hi << 31)))
        for _ in range(n_abort):
            p.aborts.append(w[o])
            o += 1
        for _ in range(n_flow):
            p.flow.append((w[o], bool(w[o + 1])))
            o += 2
        return p

    def flags(self) -> int:
        return (F_STEP if self.step else 0) | (F_STOP if self.stop else 0) | (F_SYNC if self.sync else 0)

    def roundtrip(self) -> "Plan":
        """The plan exactly as a follower decodes it (the leader applies this, so every rank agrees bit for bit)."""
        if not (self.adds or self.aborts or self.flow):
            return self
        return Plan.decode(self.flags(), len(self.adds), len(self.aborts), len(self.flow), self.encode())


def _messages(plan: Plan, room: int):
    """The plan's wire messages: [header(6) + payload chunk] int32 arrays, F_MORE on all but the last."""
    words = plan.encode()
    chunks = [words[i:i + room] for i in range(0, len(words), room)] or [[]]
    out = []
    for k, chunk in enumerate(chunks):
        flags = plan.flags() | (0 if k == len(chunks) - 1 else F_MORE)
        out.append(array("i", [MAGIC, flags, len(plan.adds), len(plan.aborts), len(plan.flow), len(chunk)] + chunk))
    return out


class _Reassembly:
    def __init__(self):
        self.words = []

    def feed(self, msg) -> "Plan | None":
        magic, flags, n_add, n_abort, n_flow, n = msg[:6]
        if magic != MAGIC:
            raise RuntimeError(f"TP plan channel: bad message (magic {magic:#x})")
        self.words += list(msg[6:6 + n])
        if flags & F_MORE:
            return None
        words, self.words = self.words, []
        return Plan.decode(flags, n_add, n_abort, n_flow, words)


class ShmPlanChannel:
    """Leader -> followers plans through one shared-memory SPSC ring per follower (same node).

    The leader creates the rings (``/dsse-tp-<pid>-<group>-<k>``) and sends their prefix over the gloo plan group
    once; a follower polls its ring for ``spin_us`` before it sleeps on the ring's futex, so a step plan arriving
    right after the previous step is picked up without a wake-up syscall."""

    ROOM = 1 << 18  # payload words per message (1 MiB: a ring holds at least two)

    def __init__(self, group, src: int, rank: int, group_ranks: list, tag: str = "", spin_us: int | None = None):
        import os

        from .. import runtime

        self.src, self.rank = src, rank
        self.spin_us = int(os.environ.get("DSSE_TP_PLAN_SPIN_US", "2000")) if spin_us is None else spin_us
        rt = runtime.load()
        obj = [None]
        if rank == src:
            prefix = f"/dsse-tp-{os.getpid()}-{tag or src}"
            self.out = rt.ShmFanout([f"{prefix}-{k}" for k in range(1, len(group_ranks))], 4 << 20)
            obj[0] = prefix
        dist.broadcast_object_list(obj, src=src, group=group)
        if rank != src:
            k = group_ranks.index(rank)
            self.inp = rt.ShmChannel(f"{obj[0]}-{k}", False, 0, 60000)
        dist.barrier(group=group)  # every follower attached before the leader may close anything
        self._re = _Reassembly()
        self._hdr = {}

    def send(self, plan: Plan) -> None:
        if plan.empty() or not (plan.adds or plan.aborts or plan.flow):  # the steady decode step: cached bytes
            b = self._hdr.get(plan.flags())
            if b is None:
                b = self._hdr[plan.flags()] = _messages(plan, self.ROOM)[0].tobytes()
            msgs = (b,)
        else:
            msgs = [m.tobytes() for m in _messages(plan, self.ROOM)]
        for b in msgs:
            if not self.out.push(b, 60000):
                raise RuntimeError("TP plan channel: follower ring full or closed")

    def recv(self) -> Plan:
        while True:
            b = self.inp.pop(60000, self.spin_us)
            if b is None:
                if self.inp.closed():
                    raise RuntimeError("TP plan channel closed by the leader")
                continue
            plan = self._re.feed(array("i", b))
            if plan is not None:
                return plan


class GlooPlanChannel:
    """Leader -> followers plans over a gloo group (ranks on different nodes): a 6-word header broadcast, then the
    payload words only when the message has any (an empty step plan is one 24-byte broadcast)."""

    HEADER = 6
    ROOM = 1 << 16

    def __init__(self, group, src: int):
        self.group, self.src = group, src
        self.hdr = torch.zeros(self.HEADER, dtype=torch.int32)
        self._re = _Reassembly()

    def send(self, plan: Plan) -> None:
        for msg in _messages(plan, self.ROOM):
            t = torch.frombuffer(bytearray(msg.tobytes()), dtype=torch.int32)
            self.hdr.copy_(t[: self.HEADER])
            dist.broadcast(self.hdr, src=self.src, group=self.group)
            if len(msg) > self.HEADER:
                dist.broadcast(t[self.HEADER:].clone(), src=self.src, group=self.group)

    def recv(self) -> Plan:
        while True:
            dist.broadcast(self.hdr, src=self.src, group=self.group)
            hdr = self.hdr.tolist()
            payload = []
            if hdr[5] > 0:
                buf = torch.zeros(hdr[5], dtype=torch.int32)
                dist.broadcast(buf, src=self.src, group=self.group)
                payload = buf.tolist()
            plan = self._re.feed(hdr + payload)
            if plan is not None:
                return plan


def make_plan_channel(plan_group, leader: int, group_index: int, tp: int):
    """Shared-memory plan rings when every rank of the TP group runs on this node, gloo otherwise
    (``DSSE_TP_PLAN=gloo`` forces it).  Co-location is decided from the ranks' host names, gathered over the plan
    group, so every rank takes the same branch; a shared-memory open that still fails (e.g. /dev/shm not shared
    between containers of one host) is voted on by the whole group, which then falls back to gloo together."""
    import os
    import socket

    rank = dist.get_rank()
    ranks = list(range(leader, leader + tp))
    hosts = [None] * tp
    dist.all_gather_object(hosts, socket.gethostname(), group=plan_group)
    if os.environ.get("DSSE_TP_PLAN", "shm") == "gloo" or len(set(hosts)) > 1:
        return GlooPlanChannel(plan_group, leader)
    ch, err = None, ""
    try:
        ch = ShmPlanChannel(plan_group, leader, rank, ranks, tag=f"{os.environ.get('MASTER_PORT', '0')}-{group_index}")
    except Exception as e:  # noqa: BLE001 - voted on below, every rank falls back together
        err = f"{type(e).__name__}: {e}"
    ok = [None] * tp
    dist.all_gather_object(ok, err, group=plan_group)
    if any(ok):
        if rank == leader:
            print(f"[serve] TP plan rings unavailable ({'; '.join(x for x in ok if x)}); using gloo", flush=True)
        return GlooPlanChannel(plan_group, leader)
    return ch


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

    def __init__(self, engine, channel):
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
        apply_plan(self.engine, plan.roundtrip(), self._conv.__getitem__)
        events = self.engine.step() if run else []
        self.forget(events)
        return events

    def forget(self, events) -> None:
        """Drop the rid mappings of conversations that finished in `events` (every event path calls this: the
        step's return value and the events the engine flushes mid-step through on_flush)."""
        for e in events:
            if e.done:
                rid = self._rid.pop(e.conversation_id, None)
                if rid is not None:
                    self._conv.pop(rid, None)

    def sync(self) -> None:
        """Ask the followers to run their sync hook now (the leader runs its own right after)."""
        if self.ch is not None:
            self.ch.send(Plan(sync=True))

    def stop(self) -> None:
        if self.ch is not None:
            self.ch.send(Plan(stop=True))


def follower_loop(engine, channel, on_sync=None, faults=None) -> None:
    """A follower rank: mirror the leader's plans until it sends stop.  `faults` (serving/faults.py FaultPlan, e.g.
    ``DSSE_FAULTS=stall_after_steps=N:MS DSSE_FAULTS_RANKS=1``) drills a stalled or crashed TP follower: the
    leader's IPC all-reduce then times out, its health word fails the step, and its streams end with [ERROR]."""
    while True:
        plan = channel.recv()
        if plan.stop:
            return
        apply_plan(engine, plan)
        if plan.step:
            engine.step()
            if faults is not None and faults.active:
                faults.after_step(engine)
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
