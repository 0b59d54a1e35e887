"""Data-parallel serving: one engine replica per GPU behind a single front door (BASELINE config 3).

Launched as ``torchrun --nproc-per-node N -m distributed_sse_for_llm_response_amd serve`` with ``DP=N``
(or ``serve --dp N`` which spawns the N processes itself, see :func:`spawn_dp`):

* rank 0 owns the sockets: the native runtime (edge SSE, origin API, RESP ingest, metrics) plus the
  C++ ``DpRouter`` (csrc/runtime/dp.h), which routes each chat to the live worker with the fewest
  outstanding conversations and drains every worker's token ring into the bus;
* every rank (rank 0 included) is an engine worker on its own GPU: a ``DpWorker`` channel (two POSIX
  shared-memory SPSC rings) replaces the in-process runtime in the unchanged ``EngineLoop``.

No collective runs on the token path: replicas never talk to each other (weights are random-init
from a shared seed or loaded per process), so the only cross-GPU traffic is host memory.  Compare the
reference, where scaling the LLM means adding vLLM pods behind Redis and NATS
(docs/architecture.md:235, kubernetes/base/llm/deployment.yaml:56).
"""
from __future__ import annotations

import os
import time

import torch

from .. import runtime as rt_mod
from ..models.mistral import TINY, get_config
from ..models.tokenizer import get_tokenizer
from .app import EngineLoop, build_engine
from .config import ServeConfig
from .faults import Watchdog


def dp_prefix(cfg: ServeConfig) -> str:
    if cfg.dp_prefix:
        return cfg.dp_prefix
    return f"/dsse-dp-{os.environ.get('MASTER_PORT', '0')}"


def start_router(cfg: ServeConfig, workers: int):
    """Rank 0: the front-door runtime in router mode (returns the started Runtime)."""
    mod = rt_mod.load()
    rd = cfg.runtime_dict()
    rd["local_engine"] = True
    rt = mod.Runtime(rd)
    mcfg = TINY if (cfg.engine == "cpu" and cfg.model.startswith("mistral-7b")) else get_config(cfg.model)
    rt.set_vocab(get_tokenizer(mcfg.vocab_size, cfg.tokenizer_path or None).pieces())
    rt.start_dp_router(dp_prefix(cfg), workers, 8, cfg.dp_worker_timeout_ms)
    rt.start()
    return rt


def run_worker(cfg: ServeConfig, rank: int, device=None):
    """Build this rank's engine and serve the router's requests until it shuts the group down."""
    engine, tok = build_engine(cfg, device=device)
    chan = rt_mod.load().DpWorker(dp_prefix(cfg), rank, 600_000)
    loop = EngineLoop(chan, engine, tok, cfg)
    loop.start()
    chan.set_ready(True)
    # a stalled replica says goodbye (the router stops routing to it) and hello again when it recovers
    Watchdog(loop, chan.set_ready).start()
    return loop


def serve_dp(cfg: ServeConfig, rank: int, local: int, world: int) -> int:
    device = torch.device("cuda", local) if cfg.engine == "gpu" else None
    rt = start_router(cfg, world) if rank == 0 else None
    if rt is not None:
        print(f"[serve] DP={world} router listening on :{rt.bound_port('edge')} (edge) :{rt.bound_port('origin')} "
              f"(origin) :{rt.bound_port('metrics')} (metrics)", flush=True)
    loop = run_worker(cfg, rank, device)
    try:
        while loop.is_alive():
            loop.join(0.5)
            if loop.error is not None:
                raise RuntimeError(f"dp worker {rank} engine loop died: {loop.error!r}")
    except KeyboardInterrupt:
        pass
    finally:
        loop.stop_flag.set()
        if rt is not None:
            rt.stop()
    return 0


def spawn_dp(cfg: ServeConfig, world: int) -> int:
    """``serve --dp N`` without torchrun: start N-1 worker processes, run rank 0 here."""
    import subprocess
    import sys

    env = dict(os.environ)
    env.setdefault("MASTER_PORT", str(29500 + os.getpid() % 1000))
    env["DP"] = str(world)
    env["WORLD_SIZE"] = str(world)
    env["DSSE_SERVE_CONFIG"] = cfg.to_json()
    procs = []
    for r in range(1, world):
        e = dict(env, RANK=str(r), LOCAL_RANK=str(r))
        procs.append(subprocess.Popen([sys.executable, "-m", "distributed_sse_for_llm_response_amd", "serve",
                                       "--dp-worker-only"], env=e))
    os.environ.update({"MASTER_PORT": env["MASTER_PORT"], "RANK": "0", "LOCAL_RANK": "0"})
    # SIGTERM (an orchestrator's stop, a test's terminate()) ends this process through the finally below, so the
    # worker processes are stopped with it instead of outliving it; they also watch for this process's death
    import signal

    def _term(signum, frame):
        raise KeyboardInterrupt

    signal.signal(signal.SIGTERM, _term)
    try:
        if cfg.engine == "gpu":
            torch.cuda.set_device(0)
        return serve_dp(cfg, 0, 0, world)
    finally:
        for p in procs:
            p.terminate()
        for p in procs:
            try:
                p.wait(timeout=30)
            except Exception:  # noqa: BLE001
                p.kill()


def worker_only_main(cfg: ServeConfig) -> int:
    """Entry of a worker process started by :func:`spawn_dp`."""
    rank = int(os.environ.get("RANK", "1"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    device = None
    if cfg.engine == "gpu":
        torch.cuda.set_device(local)
        device = torch.device("cuda", local)
    parent = os.getppid()
    loop = run_worker(cfg, rank, device)
    while loop.is_alive():
        loop.join(0.5)
        if os.getppid() != parent:  # the launching process died without stopping us: do not outlive it
            print(f"[serve] dp worker {rank}: launcher {parent} is gone, exiting", flush=True)
            loop.stop_flag.set()
            loop.join(5)
            break
    time.sleep(0.1)
    return 0
