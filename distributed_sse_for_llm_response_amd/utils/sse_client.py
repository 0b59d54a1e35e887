"""Minimal HTTP/1.1 + SSE client (blocking and asyncio) used by tests, the load generator twin and
bench.py.  It speaks exactly what browsers / Go's net/http client see: chunked transfer encoding,
`event:`/`id:`/`data:` fields, comment lines (`: keep-alive`), blank-line event terminators.
"""
from __future__ import annotations

import asyncio
import json
import socket
from dataclasses import dataclass, field


@dataclass
class SSEEvent:
    event: str = "message"
    data: str = ""
    id: str | None = None
    comment: str | None = None

    def json(self):
        return json.loads(self.data)


class SSEParser:
    """Incremental parser: feed() decoded body bytes, get complete events (comments included)."""

    def __init__(self):
        self.buf = ""
        self.cur = SSEEvent()
        self._has = False

    def feed(self, text: str):
        self.buf += text
        out = []
        while "\n" in self.buf:
            line, self.buf = self.buf.split("\n", 1)
            if line.endswith("\r"):
                line = line[:-1]
            if line == "":
                if self._has:
                    out.append(self.cur)
                self.cur, self._has = SSEEvent(), False
                continue
            if line.startswith(":"):
                out.append(SSEEvent(event="comment", comment=line[1:].strip()))
                continue
            k, _, v = line.partition(":")
            v = v[1:] if v.startswith(" ") else v
            if k == "event":
                self.cur.event = v
            elif k == "data":
                self.cur.data = v if not self._has or not self.cur.data else self.cur.data + "\n" + v
            elif k == "id":
                self.cur.id = v
            self._has = True
        return out


class ChunkedDecoder:
    def __init__(self):
        self.buf = b""
        self.done = False
        self._need = None

    def feed(self, data: bytes) -> bytes:
        self.buf += data
        out = b""
        while not self.done:
            if self._need is None:
                i = self.buf.find(b"\r\n")
                if i < 0:
                    break
                n = int(self.buf[:i].split(b";")[0], 16)
                self.buf = self.buf[i + 2:]
                if n == 0:
                    self.done = True
                    break
                self._need = n
            if len(self.buf) < self._need + 2:
                break
            out += self.buf[: self._need]
            self.buf = self.buf[self._need + 2:]
            self._need = None
        return out


@dataclass
class Response:
    status: int
    headers: dict
    body: bytes = b""
    events: list = field(default_factory=list)


def _request_bytes(method, path, body=None, headers=None, host="localhost"):
    h = {"Host": host, "User-Agent": "dsse-client/1", "Accept": "*/*"}
    if headers:
        h.update(headers)
    data = b""
    if body is not None:
        data = body if isinstance(body, bytes) else json.dumps(body).encode()
        h.setdefault("Content-Type", "application/json")
        h["Content-Length"] = str(len(data))
    lines = [f"{method} {path} HTTP/1.1"] + [f"{k}: {v}" for k, v in h.items()]
    return ("\r\n".join(lines) + "\r\n\r\n").encode() + data


def _parse_head(raw: bytes):
    head, _, rest = raw.partition(b"\r\n\r\n")
    lines = head.decode("latin-1").split("\r\n")
    status = int(lines[0].split()[1])
    headers = {}
    for ln in lines[1:]:
        k, _, v = ln.partition(":")
        headers[k.strip().lower()] = v.strip()
    return status, headers, rest


def request(host, port, method, path, body=None, headers=None, timeout=10.0, max_events=None,
            stop_on_done=True) -> Response:
    """Blocking request.  For event-stream responses, collects SSE events until the chunked body ends
    (or a done=true token / max_events)."""
    s = socket.create_connection((host, port), timeout=timeout)
    try:
        s.sendall(_request_bytes(method, path, body, headers))
        raw = b""
        while b"\r\n\r\n" not in raw:
            chunk = s.recv(65536)
            if not chunk:
                break
            raw += chunk
        status, hdrs, rest = _parse_head(raw)
        resp = Response(status, hdrs)
        if hdrs.get("transfer-encoding", "").lower() == "chunked":
            dec, parser = ChunkedDecoder(), SSEParser()
            data = dec.feed(rest)
            while True:
                if data:
                    resp.body += data
                    for ev in parser.feed(data.decode("utf-8", "replace")):
                        resp.events.append(ev)
                        if max_events and len(resp.events) >= max_events:
                            return resp
                if dec.done:
                    break
                chunk = s.recv(65536)
                if not chunk:
                    break
                data = dec.feed(chunk)
        else:
            n = int(hdrs.get("content-length", "0"))
            body_b = rest
            while len(body_b) < n:
                chunk = s.recv(65536)
                if not chunk:
                    break
                body_b += chunk
            resp.body = body_b[:n]
        return resp
    finally:
        s.close()


async def astream(host, port, method, path, body=None, headers=None, on_event=None, timeout=60.0):
    """asyncio SSE stream; calls on_event(ev) for each event; returns (status, n_events)."""
    reader, writer = await asyncio.wait_for(asyncio.open_connection(host, port), timeout)
    try:
        writer.write(_request_bytes(method, path, body, headers))
        await writer.drain()
        raw = b""
        while b"\r\n\r\n" not in raw:
            chunk = await asyncio.wait_for(reader.read(65536), timeout)
            if not chunk:
                return 0, 0
            raw += chunk
        status, hdrs, rest = _parse_head(raw)
        if status != 200:
            return status, 0
        dec, parser = ChunkedDecoder(), SSEParser()
        n = 0
        data = dec.feed(rest)
        while True:
            if data:
                for ev in parser.feed(data.decode("utf-8", "replace")):
                    n += 1
                    if on_event is not None and on_event(ev) is False:
                        return status, n
            if dec.done:
                return status, n
            chunk = await asyncio.wait_for(reader.read(65536), timeout)
            if not chunk:
                return status, n
            data = dec.feed(chunk)
    finally:
        writer.close()
        try:
            await writer.wait_closed()
        except Exception:  # noqa: BLE001
            pass


class RespClient:
    """Tiny RESP2 client (the load generator's Redis producer side)."""

    def __init__(self, host, port, timeout=5.0):
        self.s = socket.create_connection((host, port), timeout=timeout)
        self.f = self.s.makefile("rb")

    def cmd(self, *args):
        out = f"*{len(args)}\r\n".encode()
        for a in args:
            b = a if isinstance(a, bytes) else str(a).encode()
            out += f"${len(b)}\r\n".encode() + b + b"\r\n"
        self.s.sendall(out)
        return self.read()

    def read(self):
        line = self.f.readline()
        t, rest = line[:1], line[1:-2]
        if t == b"+":
            return rest.decode()
        if t == b"-":
            raise RuntimeError(rest.decode())
        if t == b":":
            return int(rest)
        if t == b"$":
            n = int(rest)
            if n < 0:
                return None
            data = self.f.read(n + 2)[:-2]
            return data
        if t == b"*":
            return [self.read() for _ in range(int(rest))]
        raise RuntimeError(f"bad RESP reply {line!r}")

    def close(self):
        self.s.close()
