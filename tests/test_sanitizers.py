"""Race detection / memory-safety / undefined-behaviour runs of the native host runtime: the
ASan, TSan and UBSan builds of dsse-server (``_build runtime-address`` / ``runtime-thread`` /
``runtime-undefined``) serve a concurrent workload from the native load generator — RESP producers, SSE
consumers, POST /chat streams through the stub engine, client disconnects, control-subject kills, duplicate
publishes, inline inspection — and must exit without a sanitizer report."""
import os
import signal
import socket
import subprocess
import time

import pytest

from distributed_sse_for_llm_response_amd import _build
from distributed_sse_for_llm_response_amd.runtime import loadgen_binary

H = "127.0.0.1"


def _port():
    s = socket.socket()
    s.bind((H, 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _kills_and_duplicates(sse, resp):
    """Control-subject kills racing live publishes, duplicate publishes, and the dedupe / post-terminal paths."""
    import json
    import threading

    from distributed_sse_for_llm_response_amd.utils.sse_client import RespClient, request

    c = RespClient(H, resp)
    readers = [threading.Thread(target=request, args=(H, sse, "GET", f"/stream/san-{i}"), kwargs={"timeout": 5})
               for i in range(20)]
    for t in readers:
        t.start()
    time.sleep(0.3)
    for seq in range(1, 6):
        for i in range(20):
            msg = json.dumps({"conversation_id": f"san-{i}", "token": "t", "sequence": seq, "done": False,
                              "timestamp": time.time_ns()})
            c.cmd("PUBLISH", f"llm:tokens:san-{i}", msg)
            c.cmd("PUBLISH", f"llm:tokens:san-{i}", msg)  # duplicate
        if seq == 3:
            for i in range(0, 20, 2):
                c.cmd("PUBLISH", "chat.control.kill", f"san-{i}")
    for i in range(1, 20, 2):
        c.cmd("PUBLISH", f"chat.san-{i}.control", "kill")
    for t in readers:
        t.join(10)
    c.close()


@pytest.mark.timeout(900)
@pytest.mark.parametrize("san", ["address", "thread", "undefined"])
def test_server_under_load_is_sanitizer_clean(san, tmp_path):
    _build.build_runtime(sanitize=san)
    exe = _build.LIB_DIR / f"dsse-server-{san}"
    sse, resp, met = _port(), _port(), _port()
    env = dict(os.environ, SSE_PORT=str(sse), RESP_PORT=str(resp), METRICS_PORT=str(met), ORIGIN_PORT="-1",
               STUB_TOKENS="12", STUB_TOKEN_DELAY_MS="2", IO_THREADS="3", INSPECTION_MODE="inline",
               ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", TSAN_OPTIONS="halt_on_error=0:second_deadlock_stack=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=0")
    log = tmp_path / "server.log"
    with open(log, "w") as lf:
        srv = subprocess.Popen([str(exe)], env=env, stdout=lf, stderr=subprocess.STDOUT)
    try:
        deadline = time.time() + 30
        while time.time() < deadline:
            try:
                socket.create_connection((H, sse), timeout=1).close()
                break
            except OSError:
                time.sleep(0.1)
        lg = str(loadgen_binary())
        runs = [
            [lg, "-mode", "both", "-redis", f"{H}:{resp}", "-sse", f"http://{H}:{sse}", "-conversations", "150",
             "-tokens", "10", "-token-delay", "3", "-duration", "30s", "-threads", "3", "-json"],
            [lg, "-chat", "-sse", f"http://{H}:{sse}", "-conversations", "80", "-duration", "30s", "-threads", "2",
             "-json"],
            # consumers that give up early: server-side disconnect + cancellation paths
            [lg, "-mode", "consumer", "-sse", f"http://{H}:{sse}", "-conversations", "50", "-duration", "1s", "-json"],
        ]
        for cmd in runs:
            out = subprocess.run(cmd, capture_output=True, text=True, timeout=120)
            assert out.returncode == 0, out.stderr
        _kills_and_duplicates(sse, resp)
    finally:
        srv.send_signal(signal.SIGTERM)
        try:
            srv.wait(timeout=60)
        except subprocess.TimeoutExpired:
            srv.kill()
            srv.wait()
    text = log.read_text()
    assert "ERROR: AddressSanitizer" not in text, text[-4000:]
    assert "ERROR: LeakSanitizer" not in text, text[-4000:]
    assert "WARNING: ThreadSanitizer" not in text, text[-6000:]
    assert "runtime error:" not in text, text[-4000:]  # UBSan
    assert srv.returncode == 0, text[-2000:]
