"""SSE client process for bench.py --delivery sse.

Started BEFORE the parent touches the GPU (plain subprocess).  Reads one JSON config line from stdin
({"host", "port", "streams", "message", "max_tokens"}), opens `streams` concurrent POST /chat SSE
streams, records the arrival time of every token event, and prints one JSON object with
[[stream, sequence, t_ns], ...] when every stream has finished.
"""
from __future__ import annotations

import asyncio
import json
import sys
import time

from ..utils.sse_client import astream


async def _one(cfg, i, out):
    def on_event(ev):
        if ev.event != "token":
            return True
        d = json.loads(ev.data)
        out.append((i, d["sequence"], time.time_ns(), d["timestamp"]))
        return not d["done"]

    body = {"message": cfg["message"], "conversation_id": f"bench-{cfg.get('rank', 0)}-{i}",
            "max_tokens": cfg["max_tokens"], "ignore_eos": True}
    return await astream(cfg["host"], cfg["port"], "POST", "/chat", body=body, on_event=on_event, timeout=600)


async def _main(cfg):
    out = []
    res = await asyncio.gather(*[_one(cfg, i, out) for i in range(cfg["streams"])], return_exceptions=True)
    errors = [repr(r) for r in res if isinstance(r, BaseException) or (isinstance(r, tuple) and r[0] != 200)]
    return {"arrivals": out, "errors": errors}


def main():
    line = sys.stdin.readline()
    if not line.strip():
        return 0
    cfg = json.loads(line)
    result = asyncio.run(_main(cfg))
    sys.stdout.write(json.dumps(result) + "\n")
    sys.stdout.flush()
    return 0


if __name__ == "__main__":
    sys.exit(main())
