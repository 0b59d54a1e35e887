"""Fault injection, engine watchdog and step tracing for the serving loop.

The reference has no fault injection and no tracing (reconnect loops, probes and
a first-token timeout only).  Here:

* ``DSSE_FAULTS`` — comma-separated faults applied by the engine loop, for tests and drills:
    ``drop_token=P``           drop each non-final token event with probability P (clients see a
                               sequence gap; Last-Event-ID replay cannot recover it — it never reached
                               the bus — which is what a lossy producer looks like)
    ``delay_ms=D``             sleep D ms before publishing each step's events (slow producer)
    ``crash_after_steps=N``    hard-exit the process after N engine steps (no goodbye: the DP router
                               must detect it by heartbeat and requeue / terminate its conversations)
    ``error_after_steps=N``    raise inside the loop after N steps (readiness drops, /readyz -> 503)
    ``stall_after_steps=N:MS`` block the loop for MS ms once after N steps (trips the watchdog; on a TP
                               follower: the leader's IPC all-reduce times out instead)
    ``health_after_steps=N``   set the runner's device health word after N steps, as a timed-out in-kernel wait
                               does (the next drained step raises EngineFault: every stream ends with [ERROR])
    ``seed=S``                 RNG seed for drop_token
  ``DSSE_FAULTS_RANKS=1,3`` restricts the faults to those ranks (e.g. crash one DP replica of eight).
* ``Watchdog`` — marks the replica not-ready while it has work but no step completed for ``timeout_s``
  (default ``DSSE_WATCHDOG_S``=30), and ready again when steps resume.  A stall past ``DSSE_STEP_FAIL_S`` (120 s;
  0 = never) is a device or peer hang the loop cannot leave by itself (a TP peer gone while this rank waits inside
  an RCCL collective): every live stream gets the reference's [ERROR] token and the process exits with status 3
  (``DSSE_STEP_FAIL_EXIT=0``: readiness stays down instead, for tests).
* ``StepTracer`` — ``DSSE_TRACE=/path.jsonl`` writes one JSON line per engine step (wall time, step
  latency, batch, queue, tokens out); ``DSSE_ROCTX=1`` wraps each step in a roctx range (visible in
  ``rocprofv3 --marker-trace`` timelines next to the kernels).
"""
from __future__ import annotations

import json
import os
import random
import threading
import time


class FaultPlan:
    def __init__(self, spec: str = ""):
        self.drop_token = 0.0
        self.delay_ms = 0.0
        self.crash_after_steps = 0
        self.error_after_steps = 0
        self.stall_after_steps = 0
        self.stall_ms = 0
        self.health_after_steps = 0
        seed = 0
        for item in filter(None, (x.strip() for x in spec.split(","))):
            k, _, v = item.partition("=")
            if k == "drop_token":
                self.drop_token = float(v)
            elif k == "delay_ms":
                self.delay_ms = float(v)
            elif k == "crash_after_steps":
                self.crash_after_steps = int(v)
            elif k == "error_after_steps":
                self.error_after_steps = int(v)
            elif k == "stall_after_steps":
                n, _, ms = v.partition(":")
                self.stall_after_steps, self.stall_ms = int(n), int(ms or 1000)
            elif k == "health_after_steps":
                self.health_after_steps = int(v)
            elif k == "seed":
                seed = int(v)
            else:
                raise ValueError(f"unknown fault {k!r} in DSSE_FAULTS")
        self.rng = random.Random(seed)
        self.steps = 0
        self._stalled = False
        self.active = bool(spec.strip())

    @classmethod
    def from_env(cls, follower: bool = False) -> "FaultPlan":
        """DSSE_FAULTS, optionally restricted to some ranks with DSSE_FAULTS_RANKS="1,3".  A TP follower takes the
        faults only when DSSE_FAULTS_RANKS names it explicitly (an unrestricted drill targets the serving ranks)."""
        ranks = os.environ.get("DSSE_FAULTS_RANKS", "")
        if ranks and os.environ.get("RANK", "0") not in ranks.split(","):
            return cls("")
        if follower and not ranks:
            return cls("")
        return cls(os.environ.get("DSSE_FAULTS", ""))

    def filter_events(self, events):
        if self.delay_ms > 0 and events:
            time.sleep(self.delay_ms / 1000.0)
        if self.drop_token <= 0:
            return events
        return [e for e in events if e.done or self.rng.random() >= self.drop_token]

    def after_step(self, engine=None):
        self.steps += 1
        if self.health_after_steps and self.steps == self.health_after_steps and engine is not None:
            engine.r.health[0] = 1  # what a bounded device wait does on timeout (model_runner.HEALTH_WORDS)
        if self.crash_after_steps and self.steps >= self.crash_after_steps:
            os._exit(17)  # simulated process death: no cleanup, no goodbye to the router
        if self.error_after_steps and self.steps >= self.error_after_steps:
            raise RuntimeError(f"injected engine fault after {self.steps} steps")
        if self.stall_after_steps and self.steps >= self.stall_after_steps and not self._stalled:
            self._stalled = True
            time.sleep(self.stall_ms / 1000.0)


class Watchdog(threading.Thread):
    """Readiness follows engine progress: not ready while work is pending and no step finished recently."""

    def __init__(self, loop, set_ready, timeout_s: float | None = None, period_s: float = 0.2,
                 fail_s: float | None = None):
        super().__init__(daemon=True, name="engine-watchdog")
        self.loop, self.set_ready = loop, set_ready
        self.timeout_s = float(os.environ.get("DSSE_WATCHDOG_S", "30")) if timeout_s is None else timeout_s
        self.fail_s = float(os.environ.get("DSSE_STEP_FAIL_S", "120")) if fail_s is None else fail_s
        self.period_s = period_s
        self.stalled = False
        self.failed = False
        self.trips = 0
        self._stop = threading.Event()

    def _fail(self, idle_for: float) -> None:
        """The loop is stuck inside a device or collective wait: end every live stream with [ERROR], then exit.
        The loop is halted first (on waking it publishes nothing and leaves its loop) and the [ERROR] events are built
        from a read-only view: only the loop thread ever mutates the engine, even if its wait completes later."""
        self.failed = True
        with self.loop.pub_lock:  # wait out a publish() the loop thread is inside of; after this, none of its frames
            self.loop.halted = True
        print(json.dumps({"level": "ERROR", "msg": "engine hung; failing every stream", "seconds": round(idle_for, 3)}),
              flush=True)
        try:
            self.loop.publish(self.loop.engine.error_events(), final=True)
        finally:
            self.set_ready(False)
            if os.environ.get("DSSE_STEP_FAIL_EXIT", "1") != "0":
                time.sleep(0.5)  # the I/O threads write the [ERROR] frames
                os._exit(3)

    def run(self):
        while not self._stop.wait(self.period_s):
            if self.loop.error is not None:
                return  # the loop itself dropped readiness
            busy = self.loop.engine.runnable()  # streams paused by flow control are not a stall
            idle_for = time.monotonic() - self.loop.last_progress
            stalled = busy and idle_for > self.timeout_s
            if stalled and self.fail_s > 0 and idle_for > self.fail_s and not self.failed:
                self._fail(idle_for)
                return
            if stalled and not self.stalled:
                self.trips += 1
                print(json.dumps({"level": "WARN", "msg": "engine stalled", "seconds": round(idle_for, 3)}), flush=True)
                self.set_ready(False)
            elif not stalled and self.stalled:
                self.set_ready(True)
            self.stalled = stalled

    def stop(self):
        self._stop.set()


class StepTracer:
    def __init__(self, path: str | None = None, roctx: bool | None = None):
        path = os.environ.get("DSSE_TRACE", "") if path is None else path
        self.f = open(path, "a", buffering=1) if path else None
        self.roctx = (os.environ.get("DSSE_ROCTX", "0") == "1") if roctx is None else roctx
        self._nvtx = None
        if self.roctx:
            try:
                import torch

                self._nvtx = torch.cuda.nvtx  # roctx on ROCm builds of PyTorch
            except Exception:  # noqa: BLE001 - tracing is best effort
                self._nvtx = None

    def begin(self, step: int):
        if self._nvtx is not None:
            self._nvtx.range_push(f"engine.step {step}")

    def end(self, step: int, engine, events, dt_s: float):
        if self._nvtx is not None:
            self._nvtx.range_pop()
        if self.f is not None:
            self.f.write(json.dumps({"t_ns": time.time_ns(), "step": step, "step_ms": round(dt_s * 1000, 4),
                                     "running": engine.num_running(), "waiting": len(engine.waiting),
                                     "tokens_out": len(events), "kv_free": engine.alloc.num_free,
                                     "host_ms": round(engine.stats.get("host_s", 0.0) * 1000, 4),
                                     "wait_ms": round(engine.stats.get("wait_s", 0.0) * 1000, 4),
                                     "preemptions": engine.stats.get("preemptions", 0),
                                     "prefill_tokens": engine.stats["prefill_tokens"]}) + "\n")

    def close(self):
        if self.f is not None:
            self.f.close()
            self.f = None
