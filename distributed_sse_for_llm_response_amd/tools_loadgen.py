"""Python twin of the reference load generator (reference ``demo/load-generator/main.go``; Go is not
installed here, the Go original still works unchanged against this server's RESP + SSE ports).

Same flags and semantics: ``-mode producer|consumer|both -redis host:port -sse URL -conversations N
-tokens T -token-delay MS -duration 30s``; conversation ids ``loadtest-<unixnano>-<i>``; consumers
connect first (``GET /stream/<id>``) and wait 500 ms; producers ``PUBLISH llm:tokens:<id>`` one
TokenMessage per token with ``delay + U[0, delay/2)`` ms sleeps; latency = receive time - the
message's nanosecond timestamp.  Additions: ``-chat`` (drive POST /chat through the engine instead
of publishing), ``-procs`` (spread conversations over processes), p50/p99 latency and inter-token
gaps, and ``-json`` output.  ``-token-delay 1`` does not panic here (the Go one does,
``rand.Intn(0)``).
"""
from __future__ import annotations

import argparse
import asyncio
import json
import multiprocessing as mp
import os
import random
import sys
import time
from urllib.parse import urlparse

from .utils.sse_client import astream

SAMPLE = ("Streaming tokens travel from the sampler through the in-node bus to every subscribed browser as "
          "server-sent events each carrying a sequence number and a nanosecond timestamp").split(" ")


def _parse_duration(s: str) -> float:
    s = s.strip()
    for suf, mul in (("ms", 1e-3), ("s", 1.0), ("m", 60.0), ("h", 3600.0)):
        if s.endswith(suf) and s[: -len(suf)].replace(".", "", 1).isdigit():
            return float(s[: -len(suf)]) * mul
    return float(s)


class Stats:
    def __init__(self):
        self.published = self.received = self.opened = self.closed = self.errors = 0
        self.lat = []
        self.gaps = []

    def merge(self, d):
        self.published += d["published"]
        self.received += d["received"]
        self.opened += d["opened"]
        self.closed += d["closed"]
        self.errors += d["errors"]
        self.lat += d["lat"]
        self.gaps += d["gaps"]

    def as_dict(self):
        return {"published": self.published, "received": self.received, "opened": self.opened,
                "closed": self.closed, "errors": self.errors, "lat": self.lat, "gaps": self.gaps}

    def summary(self):
        def pct(v, p):
            if not v:
                return None
            v = sorted(v)
            return v[min(len(v) - 1, int(p / 100 * len(v)))]
        s = {"tokens_published": self.published, "tokens_received": self.received,
             "connections_opened": self.opened, "connections_closed": self.closed, "errors": self.errors}
        if self.lat:
            s.update({"avg_latency_ms": sum(self.lat) / len(self.lat), "min_latency_ms": min(self.lat),
                      "max_latency_ms": max(self.lat), "p50_latency_ms": pct(self.lat, 50),
                      "p99_latency_ms": pct(self.lat, 99)})
        if self.gaps:
            s.update({"p50_inter_token_ms": pct(self.gaps, 50), "p99_inter_token_ms": pct(self.gaps, 99)})
        return s

    def print(self):
        s = self.summary()
        print("\n=== Load Test Statistics ===")
        print(f"Tokens Published:    {self.published}")
        print(f"Tokens Received:     {self.received}")
        print(f"Connections Opened:  {self.opened}")
        print(f"Connections Closed:  {self.closed}")
        print(f"Errors:              {self.errors}")
        if self.lat:
            print(f"Avg Latency:         {s['avg_latency_ms']:.2f} ms")
            print(f"Min Latency:         {s['min_latency_ms']:.2f} ms")
            print(f"Max Latency:         {s['max_latency_ms']:.2f} ms")
            print(f"P50 / P99 Latency:   {s['p50_latency_ms']:.2f} / {s['p99_latency_ms']:.2f} ms")
        if self.gaps:
            print(f"P50 / P99 ITL:       {s['p50_inter_token_ms']:.2f} / {s['p99_inter_token_ms']:.2f} ms")
        print("============================")


class RespPool:
    """A few RESP2 connections shared by all producers (go-redis keeps a pool too)."""

    def __init__(self, host, port, size):
        self.host, self.port, self.size = host, port, size
        self.conns = []
        self.i = 0

    async def connect(self):
        for _ in range(self.size):
            r, w = await asyncio.open_connection(self.host, self.port)
            self.conns.append((r, w, asyncio.Lock()))
        r, w, _ = self.conns[0]
        w.write(b"*1\r\n$4\r\nPING\r\n")
        await w.drain()
        line = await r.readline()
        if not line.startswith(b"+PONG"):
            raise RuntimeError(f"PING failed: {line!r}")

    async def publish(self, channel: str, payload: str) -> int:
        r, w, lock = self.conns[self.i % len(self.conns)]
        self.i += 1
        c, p = channel.encode(), payload.encode()
        msg = b"*3\r\n$7\r\nPUBLISH\r\n$%d\r\n%s\r\n$%d\r\n%s\r\n" % (len(c), c, len(p), p)
        async with lock:
            w.write(msg)
            await w.drain()
            line = await r.readline()
        if not line.startswith(b":"):
            raise RuntimeError(line.decode(errors="replace"))
        return int(line[1:])

    def close(self):
        for _, w, _ in self.conns:
            w.close()


async def _consumer(host, port, conv, stats, deadline, chat_message=None):
    last = [None]

    def on_event(ev):
        if ev.event == "comment" or not ev.data:
            return True
        try:
            tok = json.loads(ev.data)
        except ValueError:
            return True
        if "token" not in tok:
            return True  # event: connected
        now = time.time_ns()
        ts = tok.get("timestamp", 0)
        if ts > 0:
            stats.lat.append((now - ts) / 1e6)
        if last[0] is not None:
            stats.gaps.append((now - last[0]) / 1e6)
        last[0] = now
        stats.received += 1
        if tok.get("done"):
            return False
        return time.time() < deadline

    try:
        if chat_message is None:
            st, _ = await astream(host, port, "GET", f"/stream/{conv}",
                                  headers={"Accept": "text/event-stream", "Cache-Control": "no-cache"},
                                  on_event=on_event, timeout=max(5.0, deadline - time.time() + 5))
        else:
            st, _ = await astream(host, port, "POST", "/chat", body={"message": chat_message, "conversation_id": conv},
                                  on_event=on_event, timeout=max(5.0, deadline - time.time() + 5))
        if st != 200:
            stats.errors += 1
            return
        stats.opened += 1
        stats.closed += 1
    except Exception:  # noqa: BLE001 - counted like the Go harness
        if time.time() < deadline:
            stats.errors += 1


async def _producer(pool, conv, tokens, delay_ms, stats, deadline):
    ch = f"llm:tokens:{conv}"
    for i in range(tokens):
        if time.time() > deadline:
            return
        msg = json.dumps({"conversation_id": conv, "token": SAMPLE[i % len(SAMPLE)], "sequence": i + 1,
                          "done": i == tokens - 1, "timestamp": time.time_ns()}, separators=(",", ":"))
        try:
            await pool.publish(ch, msg)
            stats.published += 1
        except Exception:  # noqa: BLE001
            stats.errors += 1
            continue
        if delay_ms > 0:
            jitter = random.randrange(delay_ms // 2) if delay_ms >= 2 else 0
            await asyncio.sleep((delay_ms + jitter) / 1000.0)


async def _run_part(args, conv_ids):
    stats = Stats()
    deadline = time.time() + (args.duration if args.duration > 0 else 1e9)
    u = urlparse(args.sse)
    host, port = u.hostname or "localhost", u.port or 80
    tasks = []
    if args.chat:
        tasks = [asyncio.create_task(_consumer(host, port, c, stats, deadline, chat_message=args.message))
                 for c in conv_ids]
    else:
        if args.mode in ("consumer", "both"):
            tasks += [asyncio.create_task(_consumer(host, port, c, stats, deadline)) for c in conv_ids]
            await asyncio.sleep(0.5)  # give consumers time to connect (main.go:162)
        if args.mode in ("producer", "both"):
            rh, _, rp = args.redis.rpartition(":")
            pool = RespPool(rh or "localhost", int(rp), max(1, min(args.pool, len(conv_ids))))
            await pool.connect()
            tasks += [asyncio.create_task(_producer(pool, c, args.tokens, args.token_delay, stats, deadline))
                      for c in conv_ids]
    if tasks:
        await asyncio.wait(tasks, timeout=max(1.0, deadline - time.time() + 2))
    for t in tasks:
        t.cancel()
    return stats


def _worker(args, conv_ids, q):
    q.put(asyncio.run(_run_part(args, conv_ids)).as_dict())


def parse_args(argv):
    ap = argparse.ArgumentParser(prog="loadgen", description=__doc__.split("\n")[0])
    ap.add_argument("-mode", "--mode", default="both", choices=["producer", "consumer", "both"])
    ap.add_argument("-redis", "--redis", default="localhost:6379")
    ap.add_argument("-sse", "--sse", default="http://localhost:8080")
    ap.add_argument("-conversations", "--conversations", type=int, default=5)
    ap.add_argument("-tokens", "--tokens", type=int, default=50)
    ap.add_argument("-token-delay", "--token-delay", type=int, default=50)
    ap.add_argument("-duration", "--duration", type=_parse_duration, default=30.0)
    ap.add_argument("-chat", "--chat", action="store_true", help="POST /chat (engine-generated tokens)")
    ap.add_argument("-message", "--message", default="Tell me about streaming token delivery.")
    ap.add_argument("-procs", "--procs", type=int, default=1)
    ap.add_argument("-pool", "--pool", type=int, default=16)
    ap.add_argument("-json", "--json", action="store_true")
    return ap.parse_args(argv)


def run(args) -> Stats:
    ids = [f"loadtest-{time.time_ns()}-{i}" for i in range(args.conversations)]
    if args.procs <= 1:
        return asyncio.run(_run_part(args, ids))
    q = mp.get_context("fork").Queue()
    ps = [mp.get_context("fork").Process(target=_worker, args=(args, ids[k::args.procs], q))
          for k in range(args.procs)]
    for p in ps:
        p.start()
    total = Stats()
    for _ in ps:
        total.merge(q.get())
    for p in ps:
        p.join()
    return total


def main(argv=None):
    args = parse_args(sys.argv[1:] if argv is None else argv)
    stats = run(args)
    if args.json:
        print(json.dumps(stats.summary()))
    else:
        stats.print()
    return 0


if __name__ == "__main__":
    sys.exit(main())
