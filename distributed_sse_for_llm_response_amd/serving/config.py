"""Typed configuration honouring the reference's environment variables.

Reference keys (same names, same defaults where they apply here):
  SSE_PORT=8080 METRICS_PORT=9090 (sse-adapter, src/sse-adapter/main.go:29-40), PORT / ORIGIN_PORT
  (llm-stream-proxy, src/llm-stream-proxy/main.go:70-96; the origin gets its own port because both
  services default to 8080 and they now share a process), LLM_PROXY_URL, INSPECTION_MODE,
  INSPECTION_BUFFER_MS, LOG_LEVEL, MODEL_NAME, REDIS_ADDR (the RESP ingest port, e.g. ":6379").
Topology keys (new): UPSTREAM_URL (edge: relay conversations from the origin), UI_PATH.
Flow control (new): FLOW_HIGH_WATER (bytes queued for every subscriber of a conversation before its decode
  pauses; 0 = off), MAX_PAUSE_S (a paused stream resumes after this long regardless).
Engine keys (new): TP, DP, DP_PREFIX, DP_WORKER_TIMEOUT_MS, MAX_MODEL_LEN, MAX_BATCH, KV_BLOCK (fixed 32), GPU_MEMORY_UTILIZATION,
  SEED, MAX_TOKENS, PREFILL_BUDGET, TOKENIZER_PATH, WEIGHTS_PATH.
"""
from __future__ import annotations

import argparse
import os
from dataclasses import asdict, dataclass, fields


def _env(name, default, cast=str):
    v = os.environ.get(name)
    if v is None or v == "":
        return default
    if cast is bool:
        return v.lower() in ("1", "true", "yes", "on")
    return cast(v)


@dataclass
class ServeConfig:
    # delivery (reference sse-adapter / proxy)
    host: str = "0.0.0.0"
    sse_port: int = 8080
    origin_port: int = 8081
    metrics_port: int = 9090
    resp_port: int = -1
    io_threads: int = 4
    llm_proxy_url: str = ""
    upstream_url: str = ""       # edge: origin SSE endpoint to relay conversations from (csrc/runtime/relay.h)
    ui_path: str = ""            # chat page served at GET / ("" = the built-in page, "none" = off)
    inspection_mode: str = "disabled"
    inspection_buffer_ms: int = 150
    inspection_endpoint: str = ""  # remote inspector URL (POST /inspect of the reference's Spin function)
    inspection_timeout_ms: int = 250
    inspection_fail_open: int = 0  # 1: a failed / overloaded inline inspector delivers uninspected (default: [ERROR])
    dedupe_window_s: int = 30      # bus duplicate window (the bridge's DEDUPE_WINDOW_SEC; 0 = off)
    log_level: str = "info"
    model_name: str = "mistralai/Mistral-7B-Instruct-v0.3"
    keepalive_ms: int = 15000
    first_token_timeout_ms: int = 30000
    flow_high_water: int = 256 << 10   # per-conversation backpressure (csrc/runtime/server.h)
    max_pause_s: float = 30.0
    # engine
    engine: str = "gpu"          # gpu | cpu (tiny reference-op model) | stub (C++ token generator)
    model: str = "mistral-7b-v0.3"
    tp: int = 1
    dp: int = 1
    max_model_len: int = 4096
    max_batch: int = 256  # decode slots (captured buckets 1..64 by powers of two, then every 64); KV pages are lazy
    gpu_memory_utilization: float = 0.85
    seed: int = 0
    max_tokens: int = 256
    temperature: float = 1.0
    prefill_budget: int = 512
    tokenizer_path: str = ""
    weights_path: str = ""
    stub_tokens: int = 50
    stub_token_delay_ms: int = 50
    dp_prefix: str = ""          # shared-memory ring name prefix of a DP group (default from MASTER_PORT)
    dp_worker_timeout_ms: int = 10000

    @classmethod
    def from_env(cls) -> "ServeConfig":
        c = cls()
        c.sse_port = _env("SSE_PORT", c.sse_port, int)
        c.metrics_port = _env("METRICS_PORT", c.metrics_port, int)
        c.origin_port = _env("ORIGIN_PORT", _env("PORT", c.origin_port, int), int)
        redis = _env("REDIS_ADDR", "")
        if redis and ":" in redis and redis.rsplit(":", 1)[0] in ("", "0.0.0.0", "localhost", "127.0.0.1"):
            c.resp_port = int(redis.rsplit(":", 1)[1])
        c.resp_port = _env("RESP_PORT", c.resp_port, int)
        c.io_threads = _env("IO_THREADS", c.io_threads, int)
        c.llm_proxy_url = _env("LLM_PROXY_URL", c.llm_proxy_url)
        c.upstream_url = _env("UPSTREAM_URL", c.upstream_url)
        c.ui_path = _env("UI_PATH", c.ui_path)
        c.flow_high_water = _env("FLOW_HIGH_WATER", c.flow_high_water, int)
        c.max_pause_s = _env("MAX_PAUSE_S", c.max_pause_s, float)
        c.inspection_mode = _env("INSPECTION_MODE", c.inspection_mode)
        c.inspection_buffer_ms = _env("INSPECTION_BUFFER_MS", c.inspection_buffer_ms, int)
        c.inspection_endpoint = _env("INSPECTION_ENDPOINT", c.inspection_endpoint)
        c.inspection_timeout_ms = _env("INSPECTION_TIMEOUT_MS", c.inspection_timeout_ms, int)
        c.inspection_fail_open = _env("INSPECTION_FAIL_OPEN", c.inspection_fail_open, int)
        c.dedupe_window_s = _env("DEDUPE_WINDOW_SEC", c.dedupe_window_s, int)
        c.log_level = _env("LOG_LEVEL", c.log_level)
        c.model_name = _env("MODEL_NAME", c.model_name)
        c.engine = _env("ENGINE", c.engine)
        c.model = _env("MODEL", c.model)
        c.tp = _env("TP", c.tp, int)
        c.dp = _env("DP", c.dp, int)
        c.max_model_len = _env("MAX_MODEL_LEN", c.max_model_len, int)
        c.max_batch = _env("MAX_BATCH", c.max_batch, int)
        c.gpu_memory_utilization = _env("GPU_MEMORY_UTILIZATION", c.gpu_memory_utilization, float)
        c.seed = _env("SEED", c.seed, int)
        c.max_tokens = _env("MAX_TOKENS", c.max_tokens, int)
        c.temperature = _env("TEMPERATURE", c.temperature, float)
        c.prefill_budget = _env("PREFILL_BUDGET", c.prefill_budget, int)
        c.tokenizer_path = _env("TOKENIZER_PATH", c.tokenizer_path)
        c.weights_path = _env("WEIGHTS_PATH", c.weights_path)
        c.stub_tokens = _env("STUB_TOKENS", c.stub_tokens, int)
        c.stub_token_delay_ms = _env("STUB_TOKEN_DELAY_MS", c.stub_token_delay_ms, int)
        c.dp_prefix = _env("DP_PREFIX", c.dp_prefix)
        c.dp_worker_timeout_ms = _env("DP_WORKER_TIMEOUT_MS", c.dp_worker_timeout_ms, int)
        return c

    @classmethod
    def add_args(cls, ap: argparse.ArgumentParser):
        for f in fields(cls):
            ap.add_argument("--" + f.name.replace("_", "-"), type=type(f.default) if f.default is not None else str,
                            default=None)

    def update_from_args(self, ns: argparse.Namespace) -> "ServeConfig":
        for f in fields(self):
            v = getattr(ns, f.name, None)
            if v is not None:
                setattr(self, f.name, v)
        return self

    def to_json(self) -> str:
        import json

        return json.dumps(asdict(self))

    @classmethod
    def from_json(cls, s: str) -> "ServeConfig":
        import json

        return cls(**json.loads(s))

    def runtime_dict(self) -> dict:
        d = asdict(self)
        keys = ("host", "sse_port", "origin_port", "metrics_port", "resp_port", "io_threads", "llm_proxy_url",
                "upstream_url", "inspection_mode", "inspection_buffer_ms", "inspection_endpoint",
                "inspection_timeout_ms", "inspection_fail_open", "dedupe_window_s", "model_name", "keepalive_ms",
                "first_token_timeout_ms", "flow_high_water")
        out = {k: d[k] for k in keys}
        if self.ui_path != "none":
            from pathlib import Path

            p = Path(self.ui_path) if self.ui_path else Path(__file__).with_name("static") / "chat.html"
            if p.exists():
                out["ui_html"] = p.read_text()
        return out
