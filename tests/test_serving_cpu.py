"""End-to-end on CPU: POST /chat -> engine (tiny Mistral on the reference ops) -> bus -> SSE, and the
load-generator twin against the RESP + SSE ports (BASELINE config 1 plumbing)."""
import concurrent.futures as cf
import json

import pytest

from distributed_sse_for_llm_response_amd.serving.app import ServingApp
from distributed_sse_for_llm_response_amd.serving.config import ServeConfig
from distributed_sse_for_llm_response_amd.tools_loadgen import parse_args, run
from distributed_sse_for_llm_response_amd.utils.sse_client import request

H = "127.0.0.1"


def _cfg(**kw):
    c = ServeConfig(host=H, sse_port=0, origin_port=0, metrics_port=0, resp_port=0, io_threads=2)
    for k, v in kw.items():
        setattr(c, k, v)
    return c


@pytest.fixture(scope="module")
def cpu_app():
    app = ServingApp(_cfg(engine="cpu", max_tokens=8, temperature=0.0)).start()
    yield app
    app.stop()


def test_chat_through_cpu_engine(cpu_app):
    resp = request(H, cpu_app.port("edge"), "POST", "/chat", {"message": "Why stream tokens?", "max_tokens": 6},
                   timeout=60)
    assert resp.status == 200
    toks = [e.json() for e in resp.events if e.event == "token"]
    assert toks[-1]["done"] and toks[-1]["token"] == "[DONE]"
    body = toks[:-1]
    assert 1 <= len(body) <= 6
    assert [t["sequence"] for t in toks] == list(range(1, len(toks) + 1))
    # the delta text is the tokenizer piece of the sampled id
    pieces = set(cpu_app.tok.pieces())
    assert all(t["token"] in pieces for t in body)


def test_concurrent_chats_greedy_deterministic(cpu_app):
    def one(i):
        r = request(H, cpu_app.port("edge"), "POST", "/chat",
                    {"message": "same prompt", "conversation_id": f"c-{i}", "max_tokens": 5}, timeout=60)
        return [e.json()["token"] for e in r.events if e.event == "token"]

    with cf.ThreadPoolExecutor(4) as ex:
        outs = list(ex.map(one, range(4)))
    assert all(o == outs[0] for o in outs), outs  # greedy + same prompt -> same stream


def test_origin_then_stream(cpu_app):
    r = request(H, cpu_app.port("origin"), "POST", "/chat", {"message": "hi", "conversation_id": "o-s-1"})
    assert json.loads(r.body)["status"] == "streaming"
    s = request(H, cpu_app.port("edge"), "GET", "/stream/o-s-1?replay=1", timeout=60)
    toks = [e.json() for e in s.events if e.event == "token"]
    assert toks and toks[-1]["done"] and toks[0]["sequence"] == 1


def test_loadgen_twin_resp_producer_sse_consumer():
    app = ServingApp(_cfg(engine="stub")).start()
    try:
        args = parse_args(["-mode", "both", "-redis", f"{H}:{app.port('resp')}", "-sse", f"http://{H}:{app.port('edge')}",
                           "-conversations", "40", "-tokens", "10", "-token-delay", "2", "-duration", "20s"])
        st = run(args)
        assert st.published == 400 and st.received == 400 and st.errors == 0
        assert st.opened == 40
        assert 0 < st.summary()["p50_latency_ms"] < 1000
    finally:
        app.stop()


def test_loadgen_twin_chat_mode_against_stub():
    app = ServingApp(_cfg(engine="stub", stub_tokens=5, stub_token_delay_ms=1)).start()
    try:
        args = parse_args(["-chat", "-sse", f"http://{H}:{app.port('edge')}", "-conversations", "50",
                           "-duration", "20s"])
        st = run(args)
        assert st.errors == 0 and st.received == 50 * 6
    finally:
        app.stop()
