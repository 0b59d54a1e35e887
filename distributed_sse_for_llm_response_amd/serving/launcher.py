"""Process launcher for the serving stack.

* single process (WORLD_SIZE unset / 1): runtime + one engine replica on cuda:0 (or CPU / stub);
  ``serve --dp N`` spawns N replica processes itself (``serving/dp.py``);
* under torchrun with WORLD_SIZE = DP x TP (``--tp T``; DP = WORLD_SIZE / T): contiguous groups of T ranks
  are tensor-parallel replicas.  Each group's leader (its first rank) is the replica's only connection to
  the outside -- the in-process runtime when DP = 1, else a data-parallel router ring -- and drives its
  followers with per-step plans (``serving/tp.py``); the decode step's all-reduces / all-gather run over
  the group's RCCL communicator, captured in the decode graphs after a startup self-check.  Rank 0 also
  hosts the front door (runtime + DP router).  TP = 1: every rank is a replica (``serving/dp.py``).
"""
from __future__ import annotations

import os
import time

import torch
import torch.distributed as dist

from .. import runtime as rt_mod
from ..parallel.comm import TPComm, init_distributed
from ..engine.engine import EngineFault
from .app import EngineLoop, ServingApp, build_engine
from .config import ServeConfig
from .faults import FaultPlan, Watchdog
from .tp import TPLeader, follower_loop, make_plan_channel, make_tp_groups


class TPLeaderLoop(EngineLoop):
    """The first rank of a TP group: the normal engine loop, every step preceded by a plan broadcast."""

    def __init__(self, runtime, engine, tokenizer, cfg, channel):
        super().__init__(runtime, engine, tokenizer, cfg)
        self.drv = TPLeader(engine, channel)

    def _flush(self, events):
        """Mid-step events (engine.on_flush) go through the same rid bookkeeping as the step's own events."""
        self.drv.forget(events)
        super()._flush(events)

    def run(self):
        import gc

        gc.collect()
        gc.freeze()
        try:
            while not self.stop_flag.is_set() and not self._shutdown():
                busy = self.engine.runnable()
                wait = 0 if busy else (2 if self.engine.has_work() else 20)
                for req in self.rt.poll_requests(256, wait):
                    prompt = self.tokenize(req)
                    if prompt is not None:
                        self.drv.add(req["conversation_id"], prompt, self._params(req), req["arrival_ns"])
                for conv in self.rt.pop_cancellations():
                    self.drv.abort(conv)
                for conv, paused in self.flow_events():  # pause timeouts are decided here, so all ranks agree
                    self.drv.set_paused(conv, paused)
                run = bool(self.drv.plan.adds) or self.engine.runnable()
                if self.drv.plan.empty() and not run:
                    self.last_progress = time.monotonic()
                    continue
                self.tracer.begin(self.steps)
                t0 = time.perf_counter()
                events = self.drv.step(run)
                self.publish(events)
                self.tracer.end(self.steps, self.engine, events, time.perf_counter() - t0)
                self.steps += 1
                self.last_progress = time.monotonic()
                self._observe()
        except EngineFault as e:
            self.error = e
            self.rt.set_ready(False)
            print(f"[engine] TP leader FAULT: {e}", flush=True)
            self.publish(self.engine.fail_all())
            raise
        except Exception as e:  # noqa: BLE001 - surfaced to the operator, readiness drops
            self.error = e
            self.rt.set_ready(False)
            raise
        finally:
            self.drv.stop()
            self.tracer.close()


def serve_tp(cfg: ServeConfig, rank: int, local: int, world: int, tp: int, device) -> int:
    """One rank of a DP x TP launch (WORLD_SIZE = dp * tp, TP groups of contiguous ranks)."""
    backend = dist.get_backend()
    tp_group, plan_group, g, leader = make_tp_groups(world, tp, backend)
    comm = TPComm(rank=rank - leader, size=tp, group=tp_group)
    channel = make_plan_channel(plan_group, leader, g, tp)
    dp = world // tp
    if rank != leader:
        engine, _ = build_engine(cfg, device=device, comm=comm)
        try:
            follower_loop(engine, channel, faults=FaultPlan.from_env(follower=True))
        finally:
            engine.r.close()
        return 0
    if dp == 1:  # one replica: the leader owns the sockets
        app = ServingApp(cfg, device=device, comm=comm)
        app.rt.start()
        app.loop = TPLeaderLoop(app.rt, app.engine, app.tok, cfg, channel)
        app.loop.start()
        app.rt.set_ready(True)
        app.watchdog = Watchdog(app.loop, app.rt.set_ready)
        app.watchdog.start()
        print(f"[serve] TP={tp} listening on :{app.port('edge')} (edge) :{app.port('origin')} (origin)", flush=True)
        app.serve_forever()
        return 0
    from .dp import dp_prefix, start_router

    rt = start_router(cfg, dp) if rank == 0 else None
    if rt is not None:
        print(f"[serve] DP={dp} x TP={tp} router listening on :{rt.bound_port('edge')} (edge) "
              f":{rt.bound_port('origin')} (origin) :{rt.bound_port('metrics')} (metrics)", flush=True)
    engine, tok = build_engine(cfg, device=device, comm=comm)
    chan = rt_mod.load().DpWorker(dp_prefix(cfg), g, 600_000)
    loop = TPLeaderLoop(chan, engine, tok, cfg, channel)
    loop.start()
    chan.set_ready(True)
    Watchdog(loop, chan.set_ready).start()
    try:
        while loop.is_alive():
            loop.join(0.5)
        if loop.error is not None:
            raise RuntimeError(f"TP group {g} leader died: {loop.error!r}")
    except KeyboardInterrupt:
        pass
    finally:
        loop.stop_flag.set()
        if rt is not None:
            rt.stop()
    return 0


def serve_main(cfg: ServeConfig) -> int:
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world == 1:
        if cfg.dp > 1:
            if cfg.tp > 1:
                raise ValueError("DP x TP needs one process per GPU: launch with torchrun --nproc-per-node DP*TP")
            from .dp import spawn_dp

            return spawn_dp(cfg, cfg.dp)
        app = ServingApp(cfg).start()
        print(f"[serve] engine={cfg.engine} model={cfg.model} listening on :{app.port('edge')} (edge) "
              f":{app.port('origin')} (origin) :{app.port('metrics')} (metrics)"
              + (f" :{app.port('resp')} (resp)" if cfg.resp_port >= 0 else ""), flush=True)
        app.serve_forever()
        return 0
    tp = max(1, cfg.tp)
    if world % tp:
        raise ValueError(f"WORLD_SIZE={world} is not a multiple of TP={tp}")
    if cfg.dp > 1 and cfg.dp * tp != world:
        raise ValueError(f"DP={cfg.dp} x TP={tp} != WORLD_SIZE={world}")
    rank, local = int(os.environ.get("RANK", "0")), int(os.environ.get("LOCAL_RANK", os.environ.get("RANK", "0")))
    if tp == 1:  # data-parallel replicas share nothing on the token path: no process group needed
        from .dp import serve_dp

        if cfg.engine == "gpu":
            torch.cuda.set_device(local)
        return serve_dp(cfg, rank, local, world)
    device = None
    if cfg.engine == "gpu":
        device = torch.device("cuda", local % torch.cuda.device_count())
        torch.cuda.set_device(device)
    rank, local, world = init_distributed(backend=None if cfg.engine == "gpu" else "gloo", device=device)
    return serve_tp(cfg, rank, local, world, tp, device)
