"""The serving process: native runtime (HTTP/SSE/bus) + one engine loop per GPU replica.

Data path of one token (compare reference README.md:59-68, six network hops and four JSON
round trips): sampled on the GPU into the HBM token ring -> side-stream copy into pinned host memory
-> engine loop publishes the step's tokens in one call -> C++ bus formats one SSE frame per token
and fans it out to the subscribed connections' I/O threads -> epoll writer.  No network hop inside
the node.

Engine kinds:
* ``gpu``  Mistral on the gfx950 kernels (TP group of this process, captured hipGraphs);
* ``cpu``  the same engine on the fp32 reference ops with a tiny model (plumbing tests, no GPU);
* ``stub`` the C++ stub token generator (BASELINE config 1: delivery plumbing only).
"""
from __future__ import annotations

import threading
import os
import time

import torch

from .. import runtime as rt_mod
from ..engine.engine import FINISH_CODES, EngineFault, LLMEngine, SamplingParams, TokenEvent
from ..engine.kv_cache import KVCache
from ..engine.model_runner import ModelRunner
from ..models.mistral import TINY, get_config, init_standard_weights
from ..models.tokenizer import get_tokenizer, prompt_for_request
from .config import ServeConfig
from .faults import FaultPlan, StepTracer, Watchdog


def build_engine(cfg: ServeConfig, device=None, comm=None):
    """Weights + KV cache + runner + engine for this process (one DP replica / TP rank)."""
    from ..engine.weights import convert_standard, load_safetensors, random_engine_weights

    if cfg.engine == "cpu":
        mcfg = TINY if cfg.model.startswith("mistral-7b") else get_config(cfg.model)
        tp_rank, tp = (comm.rank, comm.size) if comm is not None else (0, 1)
        w = convert_standard(mcfg, init_standard_weights(mcfg, seed=cfg.seed), tp_rank=tp_rank, tp_size=tp)
        runner = ModelRunner(w, num_blocks=256, max_batch=min(cfg.max_batch, 8),
                             max_model_len=min(cfg.max_model_len, 1024), device="cpu", comm=comm, use_graphs=False)
    else:
        device = device or torch.device("cuda", torch.cuda.current_device())
        mcfg = get_config(cfg.model)
        tp_rank, tp = (comm.rank, comm.size) if comm is not None else (0, 1)
        if cfg.weights_path:
            w = load_safetensors(mcfg, cfg.weights_path, tp_rank, tp, device)
        else:
            w = random_engine_weights(mcfg, tp_rank=tp_rank, tp_size=tp, device=device, seed=cfg.seed)
        free, total = torch.cuda.mem_get_info(device)
        budget = int(total * cfg.gpu_memory_utilization) - (total - free) - (2 << 30)
        nkv = mcfg.num_kv_heads // tp
        nblk = max(64, min(KVCache.blocks_for_budget(budget, mcfg.num_layers, nkv),
                           cfg.max_batch * (cfg.max_model_len // 32 + 2) * 4))
        runner = ModelRunner(w, num_blocks=nblk, max_batch=cfg.max_batch, max_model_len=cfg.max_model_len,
                             device=device, comm=comm)
        runner.capture()
    tok = get_tokenizer(mcfg.vocab_size, cfg.tokenizer_path or None)
    engine = LLMEngine(runner, eos_id=tok.eos_id, prefill_budget=cfg.prefill_budget, max_pause_s=cfg.max_pause_s,
                       default_params=SamplingParams(temperature=cfg.temperature, max_tokens=cfg.max_tokens))
    return engine, tok


class EngineLoop(threading.Thread):
    """Pulls chat requests from the runtime, steps the engine, publishes token events.

    `runtime` is either the in-process ``Runtime`` (single replica, TP leader) or a ``DpWorker`` channel
    to a data-parallel router (``serving/dp.py``); both expose poll_requests / pop_cancellations /
    publish_tokens / set_ready.  A DP worker ships its engine metrics to the router (``observe``).
    """

    halted = False
    pub_lock = threading.Lock()  # class default (a loop built without __init__); each loop sets its own

    def __init__(self, runtime, engine: LLMEngine, tokenizer, cfg: ServeConfig):
        super().__init__(daemon=True, name="engine-loop")
        self.rt, self.engine, self.tok, self.cfg = runtime, engine, tokenizer, cfg
        self.stop_flag = threading.Event()
        self.error = None
        self.halted = False  # set by the watchdog after it failed every stream: the loop must not touch the engine
        # publish() and the watchdog's halt + [ERROR] publish serialise on this lock, so no token frame of the loop
        # thread can follow a stream's terminal [ERROR] (the loop may be inside publish() when the watchdog fires)
        self.pub_lock = threading.Lock()
        rt = rt_mod.load()
        self._rt = rt
        self._remote = hasattr(runtime, "observe")
        self._ttft, self._itl, self._host = [], [], []
        self._last_obs = 0.0
        self.faults = FaultPlan.from_env()
        self.tracer = StepTracer()
        self.last_progress = time.monotonic()
        self.steps = 0
        self.tokenize_errors = 0
        # just-in-time enqueue (LLMEngine.jit_delay): the host work that must fit between polling the requests and
        # the in-flight step's end; DSSE_JIT_MARGIN_MS=0 enqueues every step at once (one queued ahead)
        self.jit_margin_s = float(os.environ.get("DSSE_JIT_MARGIN_MS", "1.5")) / 1e3
        if self._remote:
            engine.on_ttft = self._ttft.append
            engine.on_itl = self._itl.append
        else:
            engine.on_ttft = rt.observe_ttft
            engine.on_itl = rt.observe_itl
        if isinstance(engine, LLMEngine):  # (a TP leader post-processes the events of its step itself)
            engine.on_flush = self._flush

    def _params(self, req) -> SamplingParams:
        d = self.engine.default_params
        return SamplingParams(
            temperature=req["temperature"] if req["temperature"] >= 0 else d.temperature,
            top_p=req["top_p"] if 0 < req["top_p"] <= 1 else d.top_p,
            top_k=req["top_k"] if req["top_k"] > 0 else d.top_k,
            max_tokens=req["max_tokens"] if req["max_tokens"] > 0 else d.max_tokens,
            seed=req["seed"] if req["seed"] >= 0 else None, ignore_eos=bool(req.get("ignore_eos", False)))

    def flow_events(self) -> list:
        """Flow-control transitions from the runtime plus pauses that outlived ``max_pause_s``."""
        ev = list(self.rt.pop_flow_events())
        return ev + [(c, False) for c in self.engine.expired_pauses()]

    def _flush(self, events):
        """Events the engine hands over before it blocks on a drain (LLMEngine.on_flush)."""
        if self.faults.active:
            events = self.faults.filter_events(events)
        self.publish(events)

    def publish(self, events, final: bool = False):
        """Hand events to the runtime.  After the watchdog halted the loop only its own `final` batch goes out."""
        if not events:
            return
        with self.pub_lock:
            if self.halted and not final:
                return
            self._publish(events)

    def _publish(self, events):
        self.rt.publish_tokens([e.conversation_id for e in events], [e.token_id for e in events],
                               [e.sequence for e in events], [e.done for e in events], 0,
                               [e.text for e in events], [FINISH_CODES.get(e.finish, 0) for e in events],
                               [e.prompt_tokens for e in events])

    def tokenize(self, req):
        """Prompt ids of a queued request, or None after publishing a terminal [ERROR] event for it: a
        conversation the tokenizer / chat template rejects must fail alone, not stop the loop (every other
        live stream of this replica depends on it)."""
        try:
            return prompt_for_request(self.tok, req)
        except Exception as e:  # noqa: BLE001 - any tokenizer / template failure is this request's error
            self.tokenize_errors += 1
            self.publish([TokenEvent(req["conversation_id"], -1, 1, True, text="[ERROR]", timestamp_ns=time.time_ns(),
                                     finish="abort", prompt_tokens=0)])
            print(f"[engine] request {req['conversation_id']} rejected by the tokenizer: {e!r}", flush=True)
            return None

    def _take(self, reqs):
        for req in reqs:
            prompt = self.tokenize(req)
            if prompt is not None:
                self.engine.add_request(req["conversation_id"], prompt, self._params(req), arrival_ns=req["arrival_ns"])

    def _jit_wait(self):
        """Wait until the just-in-time deadline (LLMEngine.jit_delay), taking in the requests that arrive meanwhile
        -- tokenized and queued as they come, so the host work left at the deadline is the step's plan and enqueue
        and a prompt that arrives during the wait still rides in the next step."""
        if self.jit_margin_s <= 0:
            return
        t_end = time.perf_counter() + min(self.engine.jit_delay(self.jit_margin_s), 0.05)
        while True:
            left = t_end - time.perf_counter()
            if left < 1e-3:  # the poll's timeout has millisecond granularity
                if left > 0:
                    time.sleep(left)
                return
            self._take(self.rt.poll_requests(256, int(left * 1e3)))

    def _observe(self):
        e = self.engine
        running, free = float(e.num_running()), float(e.alloc.num_free)
        host = e.stats.get("host_s", -1.0)
        if not self._remote:
            self._rt.engine_observe(e.stats["last_step_s"], running, free, host)
            self._rt.set_active_chats(running + len(e.waiting))
            return
        if host >= 0:
            self._host.append(host)
        now = time.monotonic()
        if now - self._last_obs < 0.05 and len(self._itl) < 4096 and len(self._host) < 4096:
            return  # batch the observations: one stats message per ~50 ms
        self._last_obs = now
        ttft, itl, hs = self._ttft[:], self._itl[:], self._host[:]
        self._ttft.clear()
        self._itl.clear()
        self._host.clear()
        self.rt.observe(e.stats["last_step_s"], running, free, running + len(e.waiting), ttft, itl, hs)

    def _shutdown(self) -> bool:
        f = getattr(self.rt, "shutdown_requested", None)
        return bool(f and f())

    def run(self):
        # Everything allocated so far (weights, graphs, runtime objects) moves to the permanent generation:
        # the per-step objects of the loop then never make a full collection walk the whole heap (those
        # pauses showed up as 0.5 ms gaps between decode graphs at 256 streams).
        import gc

        gc.collect()
        gc.freeze()
        try:
            while not self.stop_flag.is_set() and not self._shutdown() and not self.halted:
                busy = self.engine.runnable()
                # only paused streams left: wait briefly so their resume events get through
                wait = 0 if busy else (2 if self.engine.has_work() else 20)
                self._take(self.rt.poll_requests(256, wait))
                for conv in self.rt.pop_cancellations():
                    self.engine.abort(conv)
                for conv, paused in self.flow_events():
                    self.engine.set_paused(conv, paused)
                if not self.engine.runnable():
                    self.last_progress = time.monotonic()
                    continue
                self.tracer.begin(self.steps)
                t0 = time.perf_counter()
                events = self.engine.step()
                if self.halted:  # the watchdog ended every stream while this step was blocked
                    break
                if self.faults.active:
                    events = self.faults.filter_events(events)
                self.publish(events)
                self.tracer.end(self.steps, self.engine, events, time.perf_counter() - t0)
                self.steps += 1
                self.last_progress = time.monotonic()
                self._observe()
                if self.faults.active:
                    self.faults.after_step(self.engine)
                # just-in-time enqueue: plan the next step as late as the in-flight step allows (TTFT)
                self._jit_wait()
        except EngineFault as e:
            # untrusted device state: every live stream ends with [ERROR] now, readiness drops, the process exits
            # non-zero through serve_forever (the orchestrator restarts it; nothing re-execs in this process)
            self.error = e
            self.rt.set_ready(False)
            print(f"[engine] FAULT: {e}; ending {self.engine.num_running() + len(self.engine.waiting)} streams",
                  flush=True)
            self.publish(self.engine.fail_all())
            raise
        except Exception as e:  # noqa: BLE001 - surfaced to the operator, readiness drops
            self.error = e
            self.rt.set_ready(False)
            raise
        finally:
            self.tracer.close()


class ServingApp:
    def __init__(self, cfg: ServeConfig, device=None, comm=None):
        self.cfg = cfg
        mod = rt_mod.load()
        rd = cfg.runtime_dict()
        rd["local_engine"] = cfg.engine in ("gpu", "cpu", "stub")
        self.rt = mod.Runtime(rd)
        self.loop = None
        self.watchdog = None
        self.engine = None
        self.tok = None
        if cfg.engine in ("gpu", "cpu"):
            self.rt.set_ready(False)
            self.engine, self.tok = build_engine(cfg, device=device, comm=comm)
            self.rt.set_vocab(self.tok.pieces())

    def start(self):
        self.rt.start()
        if self.cfg.engine == "stub":
            self.rt.start_stub(self.cfg.stub_tokens, self.cfg.stub_token_delay_ms, 2)
        elif self.engine is not None:
            self.loop = EngineLoop(self.rt, self.engine, self.tok, self.cfg)
            self.loop.start()
            self.rt.set_ready(True)
            self.watchdog = Watchdog(self.loop, self.rt.set_ready)
            self.watchdog.start()
        return self

    def port(self, role: str) -> int:
        return self.rt.bound_port(role)

    def stop(self):
        if self.watchdog is not None:
            self.watchdog.stop()
        if self.loop is not None:
            self.loop.stop_flag.set()
            self.loop.join(timeout=10)
        self.rt.stop()
        if self.engine is not None and (self.loop is None or not self.loop.is_alive()):
            self.engine.r.close()  # TP: unmap the IPC all-reduce peers' buffers

    def serve_forever(self):
        try:
            while True:
                time.sleep(0.5)
                if self.loop is not None and not self.loop.is_alive():
                    if isinstance(self.loop.error, EngineFault):
                        time.sleep(0.5)  # let the I/O threads write the [ERROR] frames already on the bus
                    raise RuntimeError(f"engine loop died: {self.loop.error!r}")
        except KeyboardInterrupt:
            pass
        finally:
            self.stop()
