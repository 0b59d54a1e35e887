"""Process launcher for the serving stack.

* single process (WORLD_SIZE unset / 1): runtime + one engine replica on cuda:0 (or CPU / stub);
* tensor parallel (torchrun --nproc-per-node T, TP=T): every rank holds a 1/T shard of the weights
  and runs the identical scheduler; rank 0 owns the runtime (sockets + bus) and broadcasts each step's
  admissions and aborts over the process group, so all ranks take the same decisions.  Collectives
  inside the step (two all-reduces per layer + the sampling-candidate all-gather) run over RCCL;
* data parallel replicas (DP > 1) are served by ``serving/dp.py`` (router + shared-memory rings).
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist

from ..parallel.comm import TPComm, init_distributed
from .app import EngineLoop, ServingApp, build_engine
from .config import ServeConfig


class TPFollowerLoop:
    """Non-zero TP ranks: mirror rank 0's engine step by step."""

    def __init__(self, engine, tok, cfg):
        self.engine, self.tok, self.cfg = engine, tok, cfg

    def run(self):
        while True:
            obj = [None]
            dist.broadcast_object_list(obj, src=0)
            plan = obj[0]
            if plan is None:
                return
            for conv, prompt, params, arrival in plan["add"]:
                self.engine.add_request(conv, prompt, params, arrival_ns=arrival)
            for conv in plan["abort"]:
                self.engine.abort(conv)
            for conv, paused in plan["flow"]:
                self.engine.set_paused(conv, paused)
            if plan["step"]:
                self.engine.step()


class TPLeaderLoop(EngineLoop):
    """Rank 0 of a TP group: the normal engine loop + a per-step plan broadcast."""

    def run(self):
        try:
            while not self.stop_flag.is_set():
                busy = self.engine.runnable()
                adds, aborts = [], []
                wait = 0 if busy else (2 if self.engine.has_work() else 20)
                for req in self.rt.poll_requests(256, wait):
                    prompt = self.tokenize(req)
                    if prompt is not None:
                        adds.append((req["conversation_id"], prompt, self._params(req), req["arrival_ns"]))
                aborts = list(self.rt.pop_cancellations())
                flow = self.flow_events()  # pause timeouts are decided here, so all ranks agree
                for conv, paused in flow:
                    self.engine.set_paused(conv, paused)
                step = bool(adds) or self.engine.runnable()
                if not (adds or aborts or flow or step):
                    continue
                dist.broadcast_object_list([{"add": adds, "abort": aborts, "flow": flow, "step": step}], src=0)
                for conv, prompt, p, arrival in adds:
                    self.engine.add_request(conv, prompt, p, arrival_ns=arrival)
                for conv in aborts:
                    self.engine.abort(conv)
                if step:
                    self.publish(self.engine.step())
        finally:
            dist.broadcast_object_list([None], src=0)


def serve_main(cfg: ServeConfig) -> int:
    if cfg.dp > 1 and int(os.environ.get("WORLD_SIZE", "1")) == 1:
        from .dp import spawn_dp

        return spawn_dp(cfg, cfg.dp)
    if cfg.dp > 1:
        # DP replicas share nothing on the token path: no process group is needed
        from .dp import serve_dp

        rank, local, world = (int(os.environ.get(k, d)) for k, d in (("RANK", "0"), ("LOCAL_RANK", "0"),
                                                                     ("WORLD_SIZE", "1")))
        if cfg.engine == "gpu":
            torch.cuda.set_device(local)
        return serve_dp(cfg, rank, local, world)
    local = int(os.environ.get("LOCAL_RANK", os.environ.get("RANK", "0")))
    device = None
    if cfg.engine == "gpu":
        device = torch.device("cuda", local)
        torch.cuda.set_device(device)
    rank, local, world = init_distributed(backend="nccl" if cfg.engine == "gpu" else "gloo", device=device)
    if world > 1:
        if cfg.tp not in (1, world):
            raise ValueError(f"TP={cfg.tp} but WORLD_SIZE={world}: one TP group spans the whole launch (use DP for replicas)")
        comm = TPComm(rank=rank, size=world, group=None)
        if rank == 0:
            app = ServingApp(cfg, device=device, comm=comm)
            app.rt.start()
            app.loop = TPLeaderLoop(app.rt, app.engine, app.tok, cfg)
            app.loop.start()
            app.rt.set_ready(True)
            print(f"[serve] TP={world} listening on :{app.port('edge')} (edge) :{app.port('origin')} (origin)",
                  flush=True)
            app.serve_forever()
        else:
            engine, tok = build_engine(cfg, device=device, comm=comm)
            TPFollowerLoop(engine, tok, cfg).run()
        return 0
    app = ServingApp(cfg).start()
    print(f"[serve] engine={cfg.engine} model={cfg.model} listening on :{app.port('edge')} (edge) "
          f":{app.port('origin')} (origin) :{app.port('metrics')} (metrics)"
          + (f" :{app.port('resp')} (resp)" if cfg.resp_port >= 0 else ""), flush=True)
    app.serve_forever()
    return 0
