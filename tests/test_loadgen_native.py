"""The native load generator (csrc/tools/loadgen.cpp) against the native server: the reference's
producer/consumer workload (demo/load-generator/main.go) and the POST /chat bench-client mode."""
import json
import subprocess

import numpy as np

from distributed_sse_for_llm_response_amd import runtime as rtmod

H = "127.0.0.1"


def _rt(**kw):
    cfg = {"sse_port": 0, "origin_port": -1, "metrics_port": -1, "resp_port": 0, "io_threads": 2, "host": H}
    cfg.update(kw)
    r = rtmod.load().Runtime(cfg)
    r.start()
    return r


def _run(args):
    out = subprocess.run([str(rtmod.loadgen_binary()), *args, "-json"], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    return json.loads(out.stdout.strip().splitlines()[-1])


def test_producer_consumer_both_modes():
    r = _rt()
    try:
        s = _run(["-mode", "both", "-redis", f"{H}:{r.bound_port('resp')}", "-sse", f"http://{H}:{r.bound_port('edge')}",
                  "-conversations", "300", "-tokens", "12", "-token-delay", "5", "-duration", "20s", "-threads", "2"])
    finally:
        r.stop()
    assert s["errors"] == 0
    assert s["tokens_published"] == 300 * 12
    assert s["tokens_received"] == 300 * 12
    assert s["connections_opened"] == s["connections_closed"] == 300
    assert 0 < s["p50_latency_ms"] < 1000


def test_chat_mode_records_arrivals(tmp_path):
    r = _rt(local_engine=True)
    r.start_stub(9, 1, 2)
    arr = tmp_path / "arr.bin"
    try:
        s = _run(["-chat", "-sse", f"http://{H}:{r.bound_port('edge')}", "-conversations", "40", "-duration", "20s",
                  "-arrivals", str(arr), "-id-prefix", "t-"])
    finally:
        r.stop()
    assert s["errors"] == 0 and s["connections_closed"] == 40
    assert s["tokens_received"] == 40 * 10  # 9 tokens + [DONE]
    rec = np.fromfile(arr, dtype=np.dtype([("stream", "<i4"), ("seq", "<i4"), ("recv", "<i8"), ("ts", "<i8")]))
    assert len(rec) == 400
    for i in range(40):
        seqs = np.sort(rec["seq"][rec["stream"] == i])
        assert seqs.tolist() == list(range(1, 11))
