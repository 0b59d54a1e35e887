"""Per-conversation flow control: a stream whose subscribers stop reading is paused at its producer
(stub generator or engine decode slot) instead of losing frames, and resumes exactly where it stopped
once they drain.  The reference dropped frames once a subscriber's 100-slot channel was full
(src/sse-adapter/sse_handler.go:147-156); SURVEY.md §7.2 step 8 asks for a per-sequence pause."""
import json
import re
import socket
import time

from distributed_sse_for_llm_response_amd import runtime as rtmod
from distributed_sse_for_llm_response_amd.engine.engine import SamplingParams
from distributed_sse_for_llm_response_amd.serving.app import EngineLoop, build_engine
from distributed_sse_for_llm_response_amd.serving.config import ServeConfig
from distributed_sse_for_llm_response_amd.utils.sse_client import request

H = "127.0.0.1"


def _metric(rt, name):
    text = request(H, rt.bound_port("metrics"), "GET", "/metrics").body.decode()
    return float(next(ln.split()[1] for ln in text.splitlines() if ln.startswith(name + " ")))


def _wait(pred, timeout=20.0):
    t0 = time.monotonic()
    while time.monotonic() - t0 < timeout:
        if pred():
            return True
        time.sleep(0.02)
    return False


def test_slow_reader_pauses_stream_without_loss():
    rt = rtmod.load().Runtime({"sse_port": 0, "origin_port": 0, "metrics_port": 0, "io_threads": 2, "host": H,
                               "flow_high_water": 8192, "max_pending_bytes": 64 << 20,
                               "socket_sndbuf": 8192})
    rt.start()
    rt.start_stub(50, 1, 1)
    try:
        pauses0 = _metric(rt, "bus_backpressure_pauses_total")
        dropped0 = _metric(rt, "bus_dropped_tokens_total")
        n = 3000
        s = socket.socket()
        s.setsockopt(socket.SOL_SOCKET, socket.SO_RCVBUF, 4096)  # small window: the server queue fills fast
        s.connect((H, rt.bound_port("edge")))
        body = json.dumps({"message": "x", "conversation_id": "slow-1", "max_tokens": n}).encode()
        s.sendall(b"POST /chat HTTP/1.1\r\nHost: h\r\nContent-Length: %d\r\n\r\n%s" % (len(body), body))
        # never read: the stream must pause rather than run to completion
        assert _wait(lambda: _metric(rt, "bus_paused_conversations") == 1), "stream never paused"
        assert _metric(rt, "bus_backpressure_pauses_total") == pauses0 + 1
        held = rt.last_sequence("slow-1")
        time.sleep(0.3)
        assert rt.last_sequence("slow-1") == held < n  # the producer is holding this stream
        # drain: it resumes and every frame arrives exactly once, in order
        s.settimeout(30)
        buf = b""
        while not buf.endswith(b"0\r\n\r\n"):
            chunk = s.recv(1 << 16)
            assert chunk, "connection closed early"
            buf += chunk
        s.close()
        seqs = [int(x) for x in re.findall(rb'"sequence":(\d+)', buf)]
        assert seqs == list(range(1, n + 2))
        assert b'"token":"[DONE]"' in buf
        assert _metric(rt, "bus_dropped_tokens_total") == dropped0
        assert _metric(rt, "bus_paused_conversations") == 0
        ev = rt.pop_flow_events()
        assert ("slow-1", True) in ev and ev[-1] == ("slow-1", False)
    finally:
        rt.stop()


def test_second_reader_resumes_paused_stream():
    """Pause needs *every* subscriber to be behind: a healthy second reader un-pauses the stream."""
    rt = rtmod.load().Runtime({"sse_port": 0, "origin_port": 0, "metrics_port": 0, "io_threads": 2, "host": H,
                               "flow_high_water": 8192, "max_pending_bytes": 64 << 20,
                               "socket_sndbuf": 8192})
    rt.start()
    rt.start_stub(50, 1, 1)
    try:
        s = socket.socket()
        s.setsockopt(socket.SOL_SOCKET, socket.SO_RCVBUF, 4096)
        s.connect((H, rt.bound_port("edge")))
        body = json.dumps({"message": "x", "conversation_id": "slow-2", "max_tokens": 3000}).encode()
        s.sendall(b"POST /chat HTTP/1.1\r\nHost: h\r\nContent-Length: %d\r\n\r\n%s" % (len(body), body))
        assert _wait(lambda: _metric(rt, "bus_paused_conversations") == 1)
        # a fast consumer joins with GET /stream: the conversation resumes and it reads to the end
        r = request(H, rt.bound_port("edge"), "GET", "/stream/slow-2", timeout=60)
        toks = [e.json() for e in r.events if e.event == "token"]
        assert toks[-1]["done"] and toks[-1]["sequence"] == 3001
        s.close()
        assert _wait(lambda: _metric(rt, "bus_paused_conversations") == 0)
    finally:
        rt.stop()


def test_engine_pause_resume_is_exact():
    """A paused sequence keeps its slot, KV and position: pause/resume yields the very same tokens."""
    engine, tok = build_engine(ServeConfig(engine="cpu", max_batch=4))
    pa, pb = tok.chat_prompt("first prompt"), tok.chat_prompt("second, longer prompt here")

    def run(pause: bool):
        engine.add_request("a", pa, SamplingParams(temperature=1.0, max_tokens=14, seed=7, ignore_eos=True))
        engine.add_request("b", pb, SamplingParams(temperature=1.0, max_tokens=14, seed=9, ignore_eos=True))
        out, frozen, step = {"a": [], "b": []}, [], 0
        while engine.has_work():
            if pause and step == 3:
                assert engine.set_paused("a", True)
            if pause and step in (6, 10):
                frozen.append(len(out["a"]))
            if pause and step == 10:
                assert engine.set_paused("a", False)
            for e in engine.step():
                if not e.done:
                    out[e.conversation_id].append(e.token_id)
            step += 1
        return out, frozen

    ref, _ = run(False)
    got, frozen = run(True)
    assert len(ref["a"]) == len(ref["b"]) == 14
    assert got == ref
    assert frozen[0] == frozen[1]            # no progress while paused
    assert engine.stats["pauses"] >= 1
    assert not engine.set_paused("a", True)  # finished conversations are unknown


def test_pause_timeout_resumes():
    engine, tok = build_engine(ServeConfig(engine="cpu", max_batch=2, max_pause_s=0.0))
    engine.add_request("t", tok.chat_prompt("x"), SamplingParams(max_tokens=4, ignore_eos=True))
    engine.step()
    engine.set_paused("t", True)
    time.sleep(0.01)
    assert not engine.runnable() or engine.inflight
    assert engine.expired_pauses() == ["t"]

    class _Rt:  # the parts of the runtime interface EngineLoop.flow_events touches
        def pop_flow_events(self):
            return [("t", True)]

    loop = EngineLoop.__new__(EngineLoop)
    loop.rt, loop.engine = _Rt(), engine
    assert loop.flow_events() == [("t", True), ("t", False)]
    engine.set_paused("t", False)
    out = engine.run_until_idle()
    assert [e.sequence for e in out if e.conversation_id == "t"][-1] == 5


def test_dp_router_forwards_flow_control_to_the_owning_worker():
    """With data parallelism the pause travels over the router's shared-memory ring to the worker
    process that owns the conversation (csrc/runtime/dp.cpp kFlow)."""
    import threading
    import uuid

    mod = rtmod.load()
    rt = mod.Runtime({"sse_port": 0, "origin_port": 0, "metrics_port": 0, "resp_port": -1, "io_threads": 2,
                      "host": H, "local_engine": True, "flow_high_water": 8192, "max_pending_bytes": 64 << 20,
                      "socket_sndbuf": 8192})
    rt.set_vocab([f"tok{i}" for i in range(100)])
    prefix = f"/dsse-flow-{uuid.uuid4().hex[:8]}"
    rt.start_dp_router(prefix, 1, 1, 10000)
    rt.start()
    n, seen, stop = 4000, [], threading.Event()

    def worker():
        chan = mod.DpWorker(prefix, 0, 5000)
        chan.set_ready(True)
        conv, sent, paused = None, 0, False
        while not stop.is_set() and sent <= n:
            for req in chan.poll_requests(16, 0 if conv else 50):
                conv = req["conversation_id"]
            for ev in chan.pop_flow_events():
                seen.append(ev)
                paused = ev[1]
            if conv is None or paused:
                time.sleep(0.002)
                continue
            k = min(20, n - sent)
            if k > 0:
                chan.publish_tokens([conv] * k, [10] * k, list(range(sent + 1, sent + k + 1)), [False] * k, 0, [])
            else:
                chan.publish_tokens([conv], [-1], [n + 1], [True], 0, ["[DONE]"])
            sent += max(k, 1)
            time.sleep(0.001)

    t = threading.Thread(target=worker, daemon=True)
    t.start()
    try:
        assert _wait(lambda: all(i["ready"] for i in rt.dp_workers()), 10)
        s = socket.socket()
        s.setsockopt(socket.SOL_SOCKET, socket.SO_RCVBUF, 4096)
        s.connect((H, rt.bound_port("edge")))
        body = json.dumps({"message": "x", "conversation_id": "dp-slow"}).encode()
        s.sendall(b"POST /chat HTTP/1.1\r\nHost: h\r\nContent-Length: %d\r\n\r\n%s" % (len(body), body))
        assert _wait(lambda: ("dp-slow", True) in seen), "worker never saw the pause"
        s.settimeout(30)
        buf = b""
        while not buf.endswith(b"0\r\n\r\n"):
            chunk = s.recv(1 << 16)
            assert chunk, "connection closed early"
            buf += chunk
        s.close()
        assert [int(x) for x in re.findall(rb'"sequence":(\d+)', buf)] == list(range(1, n + 2))
        assert ("dp-slow", False) in seen
    finally:
        stop.set()
        t.join(5)
        rt.stop()
