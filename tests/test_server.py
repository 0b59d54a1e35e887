"""HTTP / SSE / RESP behaviour of the native server against the reference's contract
(src/sse-adapter/sse_handler.go, src/llm-stream-proxy/main.go, demo/load-generator/main.go)."""
import json
import socket
import threading
import time

import pytest

from distributed_sse_for_llm_response_amd import runtime as rtmod
from distributed_sse_for_llm_response_amd.utils.sse_client import RespClient, request

H = "127.0.0.1"


def make_rt(**kw):
    cfg = {"sse_port": 0, "origin_port": 0, "metrics_port": 0, "resp_port": 0, "io_threads": 2, "host": H}
    cfg.update(kw)
    r = rtmod.load().Runtime(cfg)
    r.start()
    return r


@pytest.fixture
def stub_rt():
    r = make_rt()
    r.start_stub(6, 2, 1)
    yield r
    r.stop()


@pytest.fixture
def bare_rt():
    r = make_rt()
    yield r
    r.stop()


def _metric(rt, name):
    text = request(H, rt.bound_port("metrics"), "GET", "/metrics").body.decode()
    return float(next(ln.split()[1] for ln in text.splitlines() if ln.startswith(name + " ")))


def tokens_of(resp):
    return [e.json() for e in resp.events if e.event == "token"]


def test_chat_sse_stream(stub_rt):
    p = stub_rt.bound_port("edge")
    resp = request(H, p, "POST", "/chat", {"message": "hello"})
    assert resp.status == 200
    assert resp.headers["content-type"] == "text/event-stream"
    assert resp.headers["cache-control"] == "no-cache"
    assert resp.headers["access-control-allow-origin"] == "*"
    assert resp.headers["x-accel-buffering"] == "no"
    assert resp.events[0].event == "connected"
    conv = json.loads(resp.events[0].data)["conversation_id"]
    toks = tokens_of(resp)
    assert [t["sequence"] for t in toks] == [1, 2, 3, 4, 5, 6, 7]
    assert all(t["conversation_id"] == conv for t in toks)
    assert toks[-1] == {**toks[-1], "token": "[DONE]", "done": True}
    assert [e.id for e in resp.events if e.event == "token"] == [str(i) for i in range(1, 8)]
    assert all(t["timestamp"] > 1_600_000_000_000_000_000 for t in toks)  # nanoseconds


def test_chat_with_given_conversation_id_and_keepalive_reuse(stub_rt):
    p = stub_rt.bound_port("edge")
    s = socket.create_connection((H, p))
    try:
        for i in range(2):  # two requests on one keep-alive connection
            body = json.dumps({"message": "x", "conversation_id": f"my-conv-{i}"}).encode()
            s.sendall(b"POST /chat HTTP/1.1\r\nHost: h\r\nContent-Length: %d\r\n\r\n%s" % (len(body), body))
            buf = b""
            while not buf.endswith(b"0\r\n\r\n"):
                buf += s.recv(65536)
            assert b'"conversation_id":"my-conv-%d"' % i in buf
            assert b'"done":true' in buf
    finally:
        s.close()


def test_chat_errors(bare_rt):
    p = bare_rt.bound_port("edge")
    r = request(H, p, "POST", "/chat", {"message": "hi"})
    assert r.status == 503 and r.body == b"LLM proxy not configured\n"
    bare_rt.set_local_engine(True)
    r = request(H, p, "POST", "/chat", b"{not json")
    assert r.status == 400 and r.body == b"Invalid JSON body\n"
    r = request(H, p, "POST", "/chat", {"message": ""})
    assert r.status == 400 and r.body == b"message is required\n"
    r = request(H, p, "GET", "/chat")
    assert r.status == 405 and r.body == b"Method not allowed\n"
    r = request(H, p, "OPTIONS", "/chat")
    assert r.status == 200
    assert r.headers["access-control-allow-methods"] == "POST, OPTIONS"
    assert r.headers["access-control-allow-headers"] == "Content-Type"
    assert r.headers["access-control-allow-origin"] == "*"
    r = request(H, p, "GET", "/nope")
    assert r.status == 404


def test_first_token_timeout():
    r = make_rt(first_token_timeout_ms=200)
    try:
        r.set_local_engine(True)  # requests queue up but nothing generates
        resp = request(H, r.bound_port("edge"), "POST", "/chat", {"message": "hi"}, timeout=5)
        assert resp.events[0].event == "connected"
        assert resp.events[-1].event == "error"
        assert json.loads(resp.events[-1].data) == {"error": "timeout waiting for response"}
        assert len(r.poll_requests(10, 0)) == 1
    finally:
        r.stop()


def test_keepalive_comments():
    r = make_rt(keepalive_ms=100)
    try:
        resp = request(H, r.bound_port("edge"), "GET", "/stream/ka-test", timeout=5, max_events=4)
        assert resp.events[0].comment == "connected to ka-test"
        assert [e.comment for e in resp.events[1:4]] == ["keep-alive"] * 3
    finally:
        r.stop()


def test_stream_publish_and_last_event_id_replay(bare_rt):
    p = bare_rt.bound_port("edge")
    conv = "replay-1"
    for i in range(1, 6):
        bare_rt.publish(conv, f"t{i}", i, False, 0)
    # reconnect with Last-Event-ID: 2 -> frames 3, 4, 5 (no off-by-one loss), then live frames
    got = []

    def reader():
        got.append(request(H, p, "GET", f"/stream/{conv}", headers={"Last-Event-ID": "2"}, timeout=5))

    th = threading.Thread(target=reader)
    th.start()
    time.sleep(0.3)
    bare_rt.publish(conv, "t6", 6, False, 0)
    bare_rt.publish(conv, "[DONE]", 7, True, 0)
    th.join(5)
    toks = tokens_of(got[0])
    assert [t["sequence"] for t in toks] == [3, 4, 5, 6, 7]
    assert got[0].events[0].comment == f"connected to {conv}"


def test_stream_requires_id(bare_rt):
    r = request(H, bare_rt.bound_port("edge"), "GET", "/stream/")
    assert r.status == 400 and r.body == b"conversation_id required\n"


def test_publish_endpoint_and_inspect(bare_rt):
    p = bare_rt.bound_port("edge")
    r = request(H, p, "POST", "/publish/chat.pub-1.tokens", {"token": "x", "sequence": 1})
    assert r.status == 200 and json.loads(r.body) == {"status": "published"}
    assert bare_rt.last_sequence("pub-1") == 1
    r = request(H, p, "POST", "/inspect", {"subject": "chat.a.tokens", "data": "the password"})
    assert json.loads(r.body)["action"] == "redact"


def test_health_ready_metrics(stub_rt):
    p = stub_rt.bound_port("edge")
    assert request(H, p, "GET", "/healthz").body == b"ok"
    assert request(H, p, "GET", "/readyz").body == b"ready"
    stub_rt.set_ready(False)
    assert request(H, p, "GET", "/readyz").status == 503
    stub_rt.set_ready(True)
    request(H, p, "POST", "/chat", {"message": "m"})
    m = request(H, stub_rt.bound_port("metrics"), "GET", "/metrics").body.decode()
    for name in ("sse_active_connections", "sse_total_connections", "sse_messages_delivered_total",
                 'sse_connection_duration_seconds_bucket{le="600"}', "bus_published_total"):
        assert name in m
    # every delivered token frame carries a fresh ns timestamp: the delivery-latency histogram saw them
    assert _metric(stub_rt, "sse_delivery_latency_seconds_count") >= 7
    assert _metric(stub_rt, 'sse_delivery_latency_seconds_bucket{le="0.5"}') >= 7


def test_origin_api(stub_rt):
    p = stub_rt.bound_port("origin")
    r = request(H, p, "POST", "/chat", {"message": "hi", "conversation_id": "orig-1"})
    assert r.status == 200 and r.headers["content-type"] == "application/json"
    assert r.body == b'{"conversation_id":"orig-1","status":"streaming"}\n'
    r = request(H, p, "POST", "/chat", {"message": "hi"})
    assert len(json.loads(r.body)["conversation_id"]) == 36
    assert request(H, p, "POST", "/chat", {"message": ""}).body == b"Message is required\n"
    assert request(H, p, "POST", "/chat", b"[").body == b"Invalid request body\n"
    assert request(H, p, "GET", "/chat").status == 405
    assert request(H, p, "GET", "/health").body == b"ok"
    assert request(H, p, "GET", "/metrics").body.startswith(b"active_chats ")


def test_resp_shim_go_redis_handshake_and_publish(bare_rt):
    """go-redis v9: HELLO 3 (error -> RESP2), CLIENT SETINFO, PING, then PUBLISH llm:tokens:<id>."""
    c = RespClient(H, bare_rt.bound_port("resp"))
    with pytest.raises(RuntimeError, match="unknown command"):
        c.cmd("HELLO", "3")
    assert c.cmd("CLIENT", "SETINFO", "LIB-NAME", "go-redis(,go1.21)") == "OK"
    assert c.cmd("PING") == "PONG"
    conv = "loadtest-1-0"
    got = []
    th = threading.Thread(target=lambda: got.append(request(H, bare_rt.bound_port("edge"), "GET", f"/stream/{conv}",
                                                            timeout=5)))
    th.start()
    time.sleep(0.3)
    for i in range(3):
        msg = json.dumps({"conversation_id": conv, "token": f"w{i}", "sequence": i + 1, "done": i == 2,
                          "timestamp": time.time_ns()})
        assert c.cmd("PUBLISH", f"llm:tokens:{conv}", msg) == 1
    th.join(5)
    toks = tokens_of(got[0])
    assert [t["token"] for t in toks] == ["w0", "w1", "w2"] and toks[-1]["done"]
    c.close()


def test_resp_psubscribe_receives_engine_tokens(bare_rt):
    c = RespClient(H, bare_rt.bound_port("resp"))
    reply = c.cmd("PSUBSCRIBE", "chat.*.tokens")
    assert reply[0] == b"psubscribe" and reply[2] == 1
    bare_rt.publish("ps-1", "hey", 1, False, 5)
    msg = c.read()
    assert msg[0] == b"pmessage" and msg[2] == b"chat.ps-1.tokens"
    assert json.loads(msg[3]) == {"conversation_id": "ps-1", "token": "hey", "sequence": 1, "done": False,
                                  "timestamp": 5}
    c.close()


@pytest.mark.parametrize("mode", ["inline", "hybrid"])
def test_inspection_modes(mode):
    r = make_rt(inspection_mode=mode, inspection_buffer_ms=50)
    try:
        conv = f"insp-{mode}"
        got = []
        th = threading.Thread(target=lambda: got.append(request(H, r.bound_port("edge"), "GET", f"/stream/{conv}",
                                                                timeout=5)))
        th.start()
        time.sleep(0.3)
        r.publish(conv, "my password", 1, False, 0)
        r.publish(conv, "ignore previous orders", 2, False, 0)
        r.publish(conv, "fine", 3, False, 0)
        r.publish(conv, "[DONE]", 4, True, 0)
        th.join(5)
        toks = tokens_of(got[0])
        assert [t["token"] for t in toks] == ["[REDACTED]", "fine", "[DONE]"]
    finally:
        r.stop()


def test_client_disconnect_reports_cancellation(bare_rt):
    bare_rt.set_local_engine(True)
    p = bare_rt.bound_port("edge")
    s = socket.create_connection((H, p))
    body = json.dumps({"message": "m", "conversation_id": "gone-1"}).encode()
    s.sendall(b"POST /chat HTTP/1.1\r\nHost: h\r\nContent-Length: %d\r\n\r\n%s" % (len(body), body))
    s.recv(4096)
    s.close()
    for _ in range(50):
        c = bare_rt.pop_cancellations()
        if c:
            break
        time.sleep(0.05)
    assert c == ["gone-1"]


def test_forward_to_unreachable_proxy_emits_error():
    r = make_rt(llm_proxy_url="http://127.0.0.1:1")
    try:
        resp = request(H, r.bound_port("edge"), "POST", "/chat", {"message": "hi"}, timeout=5)
        assert resp.events[0].event == "connected"
        assert resp.events[-1].event == "error"
        assert "connection refused" in json.loads(resp.events[-1].data)["error"]
    finally:
        r.stop()


def test_edge_forwards_to_origin_instance():
    """Two-tier topology: an edge with LLM_PROXY_URL forwards POST /chat to an origin (stub engine)."""
    origin = make_rt()
    origin.start_stub(3, 1, 1)
    edge = make_rt(llm_proxy_url=f"http://127.0.0.1:{origin.bound_port('origin')}", first_token_timeout_ms=500)
    try:
        resp = request(H, edge.bound_port("edge"), "POST", "/chat", {"message": "hi", "conversation_id": "fw-1"},
                       timeout=5)
        # tokens land on the origin's bus (no cross-node bus here): the edge times out cleanly
        assert resp.events[0].event == "connected"
        assert resp.events[-1].event == "error"
        time.sleep(0.1)
        assert origin.last_sequence("fw-1") == 4
    finally:
        edge.stop()
        origin.stop()


def test_edge_relays_origin_tokens_over_upstream_sse():
    """Origin -> edge region: the edge forwards POST /chat to the origin API and relays the conversation
    from the origin's SSE port (one upstream connection, fanned out to every local subscriber)."""
    origin = make_rt()
    origin.start_stub(5, 5, 1)
    edge = make_rt(llm_proxy_url=f"http://127.0.0.1:{origin.bound_port('origin')}",
                   upstream_url=f"http://127.0.0.1:{origin.bound_port('edge')}")
    frames0 = _metric(edge, "relay_frames_total")
    try:
        ep = edge.bound_port("edge")
        side = {}

        def watcher():
            side["r"] = request(H, ep, "GET", "/stream/relay-1", timeout=10)

        t = threading.Thread(target=watcher)
        t.start()
        time.sleep(0.2)
        resp = request(H, ep, "POST", "/chat", {"message": "hi", "conversation_id": "relay-1"}, timeout=10)
        t.join(10)
        toks = tokens_of(resp)
        assert [x["sequence"] for x in toks] == [1, 2, 3, 4, 5, 6]
        assert toks[-1]["token"] == "[DONE]" and toks[-1]["done"]
        assert [x["sequence"] for x in tokens_of(side["r"])] == [1, 2, 3, 4, 5, 6]
        # the origin served the conversation exactly once over its SSE port (the relay)
        assert _metric(edge, "relay_frames_total") == frames0 + 6
    finally:
        edge.stop()
        origin.stop()


def test_edge_relay_resumes_with_last_event_id_from_origin_ring(bare_rt):
    """A conversation already (partly) produced on the origin is replayed to a late edge subscriber."""
    origin = bare_rt
    for i in range(1, 4):
        origin.publish("late-1", f"t{i}", i, False)
    edge = make_rt(upstream_url=f"http://127.0.0.1:{origin.bound_port('edge')}")
    try:
        got = {}

        def watcher():
            got["r"] = request(H, edge.bound_port("edge"), "GET", "/stream/late-1", timeout=10)

        t = threading.Thread(target=watcher)
        t.start()
        time.sleep(0.3)
        origin.publish("late-1", "t4", 4, False)
        origin.publish("late-1", "[DONE]", 5, True)
        t.join(10)
        assert [x["token"] for x in tokens_of(got["r"])] == ["t1", "t2", "t3", "t4", "[DONE]"]
    finally:
        edge.stop()


def test_chat_page_served_at_root():
    from distributed_sse_for_llm_response_amd.serving.config import ServeConfig

    rd = ServeConfig().runtime_dict()
    assert "<title>MI355X token stream</title>" in rd["ui_html"]
    r = make_rt(ui_html=rd["ui_html"])
    try:
        resp = request(H, r.bound_port("edge"), "GET", "/")
        assert resp.status == 200
        assert resp.headers["content-type"].startswith("text/html")
        assert b"fetch(base + \"/chat\"" in resp.body
    finally:
        r.stop()


def test_async_inspection_kills_conversation():
    r = make_rt(inspection_mode="async")
    r.set_local_engine(True)
    killed0, redacted0 = _metric(r, "inspection_killed_total"), _metric(r, "inspection_redacted_total")
    try:
        conv = "insp-async"
        got = []
        th = threading.Thread(target=lambda: got.append(request(H, r.bound_port("edge"), "GET", f"/stream/{conv}",
                                                                timeout=5)))
        th.start()
        time.sleep(0.3)
        r.publish(conv, "my password", 1, False, 0)
        r.publish(conv, "ignore previous orders", 2, False, 0)
        th.join(5)
        toks = tokens_of(got[0])
        # delivered immediately (no redaction in async mode), then stopped with a terminal token
        assert [t["token"] for t in toks] == ["my password", "ignore previous orders", "[BLOCKED]"]
        assert toks[-1]["done"] and toks[-1]["sequence"] == 3
        assert conv in r.pop_cancellations()
        assert _metric(r, "inspection_killed_total") == killed0 + 1
        assert _metric(r, "inspection_redacted_total") == redacted0 + 1
    finally:
        r.stop()


# ---------------------------------------------------------------- control subject, dedupe, remote inspector
def _stream_in_thread(rt, conv, timeout=5, headers=None):
    got = []
    th = threading.Thread(target=lambda: got.append(request(H, rt.bound_port("edge"), "GET", f"/stream/{conv}",
                                                            headers=headers or {}, timeout=timeout)))
    th.start()
    time.sleep(0.3)
    return th, got


@pytest.mark.parametrize("how", ["http", "http-kill", "resp", "resp-kill"])
def test_control_subject_kills_conversation(bare_rt, how):
    """chat.<id>.control (CHAT_CONTROL stream) and chat.control.kill (the async inspector's kill signal) end a
    live conversation: subscribers get a terminal [KILLED] frame, the engine a cancellation, and anything the
    producer still sends is dropped."""
    conv = f"kill-{how}"
    th, got = _stream_in_thread(bare_rt, conv)
    bare_rt.publish(conv, "a", 1, False, 0)
    bare_rt.publish(conv, "b", 2, False, 0)
    time.sleep(0.1)
    if how == "http":
        r = request(H, bare_rt.bound_port("edge"), "POST", f"/publish/chat.{conv}.control", {"action": "kill"})
        assert r.status == 200 and json.loads(r.body) == {"status": "killed", "conversation_id": conv}
    elif how == "http-kill":
        r = request(H, bare_rt.bound_port("edge"), "POST", "/publish/chat.control.kill", conv.encode())
        assert json.loads(r.body)["status"] == "killed"
    else:
        c = RespClient(H, bare_rt.bound_port("resp"))
        if how == "resp":
            assert c.cmd("PUBLISH", f"chat.{conv}.control", "kill") == 1
        else:
            assert c.cmd("PUBLISH", "chat.control.kill", json.dumps({"conversation_id": conv})) == 1
        assert c.cmd("PUBLISH", "chat.control.kill", conv) == 0  # already ended
        c.close()
    bare_rt.publish(conv, "late", 3, False, 0)  # the producer had not seen the kill yet
    th.join(5)
    toks = tokens_of(got[0])
    assert [(t["token"], t["sequence"], t["done"]) for t in toks] == [("a", 1, False), ("b", 2, False),
                                                                     ("[KILLED]", 3, True)]
    assert conv in bare_rt.pop_cancellations()
    assert _metric(bare_rt, "control_kills_total") >= 1


def test_dedupe_window_and_post_terminal_frames(bare_rt):
    """A (conversation, sequence) seen within the window is delivered once (at-least-once producers retry);
    frames after the terminal one are dropped; a new stream restarting at sequence 1 reopens the conversation."""
    conv = "dup-1"
    th, got = _stream_in_thread(bare_rt, conv)
    c = RespClient(H, bare_rt.bound_port("resp"))
    before = _metric(bare_rt, "bus_duplicates_dropped_total")
    for seq, tok, done in [(1, "x", False), (1, "x", False), (2, "y", False), (2, "y", False), (3, "[DONE]", True),
                           (3, "[DONE]", True), (4, "after", False)]:
        c.cmd("PUBLISH", f"llm:tokens:{conv}", json.dumps({"conversation_id": conv, "token": tok, "sequence": seq,
                                                           "done": done, "timestamp": time.time_ns()}))
    th.join(5)
    assert [(t["token"], t["sequence"]) for t in tokens_of(got[0])] == [("x", 1), ("y", 2), ("[DONE]", 3)]
    assert _metric(bare_rt, "bus_duplicates_dropped_total") - before == 4
    # next turn of the same conversation id
    th, got = _stream_in_thread(bare_rt, conv)
    bare_rt.publish(conv, "new", 1, False, 0)
    bare_rt.publish(conv, "[DONE]", 2, True, 0)
    th.join(5)
    assert [t["token"] for t in tokens_of(got[0])] == ["new", "[DONE]"]
    c.close()


def test_dedupe_window_can_be_disabled():
    r = make_rt(dedupe_window_s=0)
    try:
        th, got = _stream_in_thread(r, "nodup")
        r.publish("nodup", "x", 1, False, 0)
        r.publish("nodup", "x", 1, False, 0)
        r.publish("nodup", "[DONE]", 2, True, 0)
        th.join(5)
        assert [t["token"] for t in tokens_of(got[0])] == ["x", "x", "[DONE]"]
    finally:
        r.stop()


class _Inspector:
    """A stand-in for the reference's Spin inspector (POST /inspect, NatsMessage -> InspectionResult):
    "evil" -> drop, "pw" -> redact, else allow; records every call."""

    def __init__(self, fail=False):
        import http.server

        calls = self.calls = []

        class Handler(http.server.BaseHTTPRequestHandler):
            protocol_version = "HTTP/1.1"

            def log_message(self, *a):
                pass

            def do_POST(self):
                body = json.loads(self.rfile.read(int(self.headers["Content-Length"])))
                calls.append(body)
                if fail:
                    self.send_response(500)
                    self.send_header("Content-Length", "0")
                    self.end_headers()
                    return
                data = body["data"].lower()
                if "evil" in data:
                    res = {"action": "drop", "reason": "evil", "redacted_content": None}
                elif "pw" in data:
                    res = {"action": "redact", "reason": "pw", "redacted_content": "[REDACTED]"}
                else:
                    res = {"action": "allow", "reason": None, "redacted_content": None}
                out = json.dumps(res).encode()
                self.send_response(200)
                self.send_header("Content-Type", "application/json")
                self.send_header("Content-Length", str(len(out)))
                self.end_headers()
                self.wfile.write(out)

        self.srv = http.server.ThreadingHTTPServer((H, 0), Handler)
        self.url = f"http://{H}:{self.srv.server_address[1]}/inspect"
        threading.Thread(target=self.srv.serve_forever, daemon=True).start()

    def close(self):
        self.srv.shutdown()


def test_inspection_endpoint_inline_one_call_per_token_for_all_subscribers():
    insp = _Inspector()
    r = make_rt(inspection_mode="inline", inspection_endpoint=insp.url)
    try:
        d0, r0 = _metric(r, "inspection_dropped_total"), _metric(r, "inspection_redacted_total")
        conv = "remote-inline"
        a = _stream_in_thread(r, conv)
        b = _stream_in_thread(r, conv)
        for i, tok in enumerate(["hello", "my pw is x", "evil plan", "bye"]):
            r.publish(conv, tok, i + 1, False, 0)
        r.publish(conv, "[DONE]", 5, True, 0)
        for th, got in (a, b):
            th.join(5)
            assert [t["token"] for t in tokens_of(got[0])] == ["hello", "[REDACTED]", "bye", "[DONE]"]
        # one remote call per token (not per subscriber), the reference's NatsMessage shape
        assert len(insp.calls) == 4
        assert insp.calls[0] == {"subject": f"chat.{conv}.tokens", "data": "hello", "sequence": 1,
                                 "timestamp": insp.calls[0]["timestamp"]}
        assert _metric(r, "inspection_dropped_total") - d0 == 1 and _metric(r, "inspection_redacted_total") - r0 == 1
    finally:
        r.stop()
        insp.close()


def test_inspection_endpoint_hybrid_inspects_the_buffered_text_and_kills():
    insp = _Inspector()
    r = make_rt(inspection_mode="hybrid", inspection_endpoint=insp.url, inspection_buffer_ms=200)
    r.set_local_engine(True)
    try:
        th, got = _stream_in_thread(r, "hyb-ok")
        th2, got2 = _stream_in_thread(r, "hyb-bad")
        for i, tok in enumerate(["all ", "good ", "here"]):
            r.publish("hyb-ok", tok, i + 1, False, 0)
            r.publish("hyb-bad", ["ev", "il ", "scheme"][i], i + 1, False, 0)
        time.sleep(0.5)  # the buffer window passes: one verdict per conversation on the joined text
        r.publish("hyb-ok", "after", 4, False, 0)
        r.publish("hyb-ok", "[DONE]", 5, True, 0)
        th.join(5)
        th2.join(5)
        assert [t["token"] for t in tokens_of(got[0])] == ["all ", "good ", "here", "after", "[DONE]"]
        bad = tokens_of(got2[0])
        assert [(t["token"], t["done"]) for t in bad] == [("[BLOCKED]", True)]  # nothing of it reached clients
        assert "hyb-bad" in r.pop_cancellations()
        assert sorted(c["data"] for c in insp.calls) == ["all good here", "evil scheme"]
    finally:
        r.stop()
        insp.close()


def test_inspection_endpoint_failure_fails_closed_by_default_and_async_uses_it():
    """inline inspection is fail-closed like the reference ("inspector down = streaming stops",
    docs/security-inspection-patterns.md:38): the stream ends with [ERROR] and the unchecked token never reaches the
    client.  INSPECTION_FAIL_OPEN=1 delivers it instead, counted in inspection_fail_open_total."""
    insp = _Inspector(fail=True)
    r = make_rt(inspection_mode="inline", inspection_endpoint=insp.url)
    try:
        e0, c0 = _metric(r, "inspection_remote_errors_total"), _metric(r, "inspection_fail_closed_total")
        th, got = _stream_in_thread(r, "failclosed")
        r.publish("failclosed", "evil but unchecked", 1, False, 0)
        r.publish("failclosed", "more", 2, False, 0)
        r.publish("failclosed", "[DONE]", 3, True, 0)
        th.join(5)
        assert [(t["token"], t["done"]) for t in tokens_of(got[0])] == [("[ERROR]", True)]
        assert _metric(r, "inspection_remote_errors_total") - e0 == 1  # later frames are not re-inspected
        assert _metric(r, "inspection_fail_closed_total") - c0 == 1
    finally:
        r.stop()
        insp.close()
    insp = _Inspector(fail=True)
    r = make_rt(inspection_mode="inline", inspection_endpoint=insp.url, inspection_fail_open=1)
    try:
        o0 = _metric(r, "inspection_fail_open_total")
        th, got = _stream_in_thread(r, "failopen")
        r.publish("failopen", "evil but unchecked", 1, False, 0)
        r.publish("failopen", "[DONE]", 2, True, 0)
        th.join(5)
        assert [t["token"] for t in tokens_of(got[0])] == ["evil but unchecked", "[DONE]"]
        assert _metric(r, "inspection_fail_open_total") - o0 == 1
    finally:
        r.stop()
        insp.close()
    insp = _Inspector()
    r = make_rt(inspection_mode="async", inspection_endpoint=insp.url)
    r.set_local_engine(True)
    try:
        th, got = _stream_in_thread(r, "async-remote")
        r.publish("async-remote", "fine", 1, False, 0)
        r.publish("async-remote", "evil", 2, False, 0)
        th.join(5)
        toks = tokens_of(got[0])
        assert toks[-1]["token"] == "[BLOCKED]" and toks[-1]["done"]
        assert "async-remote" in r.pop_cancellations()
    finally:
        r.stop()
        insp.close()


def test_redelivered_first_token_after_done_is_a_duplicate(bare_rt):
    """a redelivered seq-1 frame of a finished stream (its old timestamp, inside the dedupe window) must
    not reopen the conversation: it is dropped and the replay ring survives for Last-Event-ID reconnects."""
    conv = "redeliver-1"
    c = RespClient(H, bare_rt.bound_port("resp"))
    ts0 = time.time_ns()
    msgs = [(1, "a", False, ts0), (2, "b", False, ts0 + 1), (3, "[DONE]", True, ts0 + 2)]
    for seq, tok, done, ts in msgs + [(1, "a", False, ts0)]:  # the last one is an at-least-once redelivery
        c.cmd("PUBLISH", f"llm:tokens:{conv}", json.dumps({"conversation_id": conv, "token": tok, "sequence": seq,
                                                           "done": done, "timestamp": ts}))
    c.close()
    time.sleep(0.1)
    resp = request(H, bare_rt.bound_port("edge"), "GET", f"/stream/{conv}", headers={"Last-Event-ID": "1"}, timeout=5)
    assert [(t["token"], t["sequence"]) for t in tokens_of(resp)] == [("b", 2), ("[DONE]", 3)]
    assert bare_rt.last_sequence(conv) == 3


@pytest.mark.parametrize("fail_open", [0, 1])
def test_black_holed_inspection_endpoint_fails_quickly(fail_open):
    """an INSPECTION_ENDPOINT that accepts TCP but never answers must not stall every token for the
    timeout: the first failure opens the circuit.  Fail-closed (default) the stream ends at once with [ERROR];
    with INSPECTION_FAIL_OPEN=1 it is delivered, uninspected, at once."""
    hole = socket.socket()
    hole.bind((H, 0))
    hole.listen(1)  # the kernel completes the handshake; nobody ever reads or answers
    r = make_rt(inspection_mode="inline", inspection_endpoint=f"http://{H}:{hole.getsockname()[1]}/inspect",
                inspection_timeout_ms=300, inspection_fail_open=fail_open)
    try:
        th, got = _stream_in_thread(r, "hole")
        t0 = time.monotonic()
        for i in range(40):
            r.publish("hole", f"t{i}", i + 1, False, 0)
        r.publish("hole", "[DONE]", 41, True, 0)
        th.join(10)
        want = [f"t{i}" for i in range(40)] + ["[DONE]"] if fail_open else ["[ERROR]"]
        assert [t["token"] for t in tokens_of(got[0])] == want
        assert time.monotonic() - t0 < 3.0  # 40 tokens x 2 attempts x 300 ms without the circuit breaker
    finally:
        r.stop()
        hole.close()


@pytest.mark.parametrize("role", ["edge", "origin"])
@pytest.mark.parametrize("body, err", [
    ({"max_tokens": 1e20}, b"max_tokens must be an integer in [1, 1048576]\n"),
    ({"max_tokens": 0}, b"max_tokens must be an integer in [1, 1048576]\n"),
    ({"top_k": 2.5}, b"top_k must be an integer in [-1, 1048576]\n"),
    ({"seed": -5}, b"seed must be an integer in [0, 9007199254740991]\n"),
    ({"seed": 2 ** 60}, b"seed must be an integer in [0, 9007199254740991]\n"),
    (b'{"message":"hi","temperature":1e400}', b"temperature and top_p must be finite\n"),
])
def test_chat_rejects_bad_sampling_fields(bare_rt, role, body, err):
    """/chat's optional integer fields are range- and integrality-checked before any cast (a
    400 before the SSE response starts), on the edge and on the origin API alike."""
    bare_rt.set_local_engine(True)
    raw = body if isinstance(body, bytes) else json.dumps({"message": "hi", **body}).encode()
    r = request(H, bare_rt.bound_port(role), "POST", "/chat", raw)
    assert r.status == 400 and r.body == err
    assert bare_rt.poll_requests(10, 0) == []


def test_chat_accepts_valid_sampling_fields(bare_rt):
    bare_rt.set_local_engine(True)
    r = request(H, bare_rt.bound_port("origin"), "POST", "/chat",
                {"message": "hi", "max_tokens": 7, "top_k": 3, "seed": 2 ** 40, "temperature": 0.5, "top_p": 0.9})
    assert r.status == 200
    (q,) = bare_rt.poll_requests(10, 0)
    assert (q["max_tokens"], q["top_k"], q["seed"]) == (7, 3, 2 ** 40)
