"""SSE client process for bench.py --delivery sse.

Started BEFORE the parent touches the GPU (plain subprocess).  Reads JSON config lines from stdin, one run each
({"host", "port", "streams", "message", "max_tokens", "prefix"}, optional "rate" / "seed" / "long_every" /
"long_words" for Poisson arrivals), opens `streams` POST /chat
SSE streams and records the arrival time of every token event, then prints one JSON object
{"arrivals": [[stream, sequence, recv_ns, msg_timestamp_ns], ...], "errors": [...]}.

The streams are driven by the native load generator (``_lib/dsse-loadgen -chat``, epoll, one thread
per 128 streams) so that the client is never the bottleneck at 8 GPUs x 64 streams; the asyncio
client in ``utils/sse_client.py`` is the fallback when the binary is missing.
"""
from __future__ import annotations

import asyncio
import json
import os
import subprocess
import sys
import tempfile
import time

import numpy as np

from ..utils.sse_client import astream

_REC = np.dtype([("stream", "<i4"), ("seq", "<i4"), ("recv", "<i8"), ("ts", "<i8")])


def _native(cfg):
    from .. import runtime as rt_mod

    exe = rt_mod.loadgen_binary()
    if not exe.exists():
        return None
    with tempfile.TemporaryDirectory() as d:
        arr = os.path.join(d, "arrivals.bin")
        threads = max(1, min(8, (cfg["streams"] + 127) // 128))
        cmd = [str(exe), "-chat", "-sse", f"http://{cfg['host']}:{cfg['port']}", "-conversations", str(cfg["streams"]),
               "-message", cfg["message"], "-max-tokens", str(cfg["max_tokens"]), "-ignore-eos",
               "-id-prefix", cfg.get("prefix", "bench-"), "-duration", str(cfg.get("duration_s", 900)) + "s",
               "-threads", str(threads), "-arrivals", arr, "-json"]
        if cfg.get("rate"):  # serving under continuous arrivals (tools/bench_serving.py): Poisson starts, send records
            cmd += ["-rate", str(cfg["rate"]), "-seed", str(cfg.get("seed", 42))]
        if cfg.get("long_every") and cfg.get("long_words"):
            cmd += ["-long-every", str(cfg["long_every"]), "-long-words", str(cfg["long_words"])]
        out = subprocess.run(cmd, capture_output=True, text=True)
        summary = json.loads(out.stdout.strip().splitlines()[-1]) if out.stdout.strip() else {}
        rec = np.fromfile(arr, dtype=_REC) if os.path.exists(arr) else np.zeros(0, dtype=_REC)
    errors = [] if summary.get("errors", 1) == 0 else [f"loadgen: {summary} {out.stderr[-500:]}"]
    return {"arrivals": np.stack([rec["stream"], rec["seq"], rec["recv"], rec["ts"]], axis=1).tolist(),
            "errors": errors, "summary": summary}


async def _one(cfg, i, out):
    def on_event(ev):
        if ev.event != "token":
            return True
        d = json.loads(ev.data)
        out.append((i, d["sequence"], time.time_ns(), d["timestamp"]))
        return not d["done"]

    body = {"message": cfg["message"], "conversation_id": f"{cfg.get('prefix', 'bench-')}{i}",
            "max_tokens": cfg["max_tokens"], "ignore_eos": True}
    return await astream(cfg["host"], cfg["port"], "POST", "/chat", body=body, on_event=on_event, timeout=900)


async def _asyncio_main(cfg):
    out = []
    res = await asyncio.gather(*[_one(cfg, i, out) for i in range(cfg["streams"])], return_exceptions=True)
    errors = [repr(r) for r in res if isinstance(r, BaseException) or (isinstance(r, tuple) and r[0] != 200)]
    return {"arrivals": out, "errors": errors}


def main():
    # one JSON config line per run, until stdin closes (tools/bench_serving.py sends several rate points)
    for line in sys.stdin:
        if not line.strip():
            break
        cfg = json.loads(line)
        result = None if cfg.get("python_client") else _native(cfg)
        if result is None:
            result = asyncio.run(_asyncio_main(cfg))
        sys.stdout.write(json.dumps(result) + "\n")
        sys.stdout.flush()
    return 0


if __name__ == "__main__":
    sys.exit(main())
