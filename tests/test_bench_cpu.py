"""bench.py contract on CPU (tiny model): one JSON line with the driver's fields, for 1 rank and for 2
ranks under torchrun (gloo), through the full serving path (client -> router -> replicas -> SSE)."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
        "vs_baseline", "dtype", "data", "config"}


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _json_line(out):
    lines = [ln for ln in out.splitlines() if ln.startswith("{\"metric\"")]
    assert len(lines) == 1, out[-2000:]
    return json.loads(lines[0])


@pytest.mark.timeout(600)
@pytest.mark.parametrize("world", [1, 2])
def test_bench_contract(world):
    args = ["bench.py", "--gpus", str(world), "--steps", "3", "--warmup", "1", "--streams", "3", "--prompt-len", "24"]
    env = dict(os.environ)
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    if world == 1:
        cmd = [sys.executable, *args]
    else:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
               "--master-addr", "127.0.0.1", "--master-port", str(_port()), *args]
    out = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=540)
    assert out.returncode == 0, out.stderr[-3000:]
    d = _json_line(out.stdout)
    assert KEYS <= set(d)
    assert d["n_gpus"] == world and d["steps"] == 3 and d["warmup"] == 1
    assert d["scaling"] == "weak" and d["higher_is_better"] is True
    assert d["config"]["global_batch"] == 3 * world and d["config"]["parallelism"] == f"dp{world}"
    assert d["value"] > 0 and d["client_errors"] == []
    assert d["tokens_delivered_in_window"] >= 3 * world * 2


@pytest.mark.timeout(600)
def test_bench_host_path_rehearsal_with_paced_stubs():
    """--stub-step-ms: 4 stub replicas at 5 ms/step through router + bus + SSE + native client; the measured
    step time tracks the stub pace and every stream's tokens arrive (profiles/host_path_rehearsal_r1.md)."""
    args = ["bench.py", "--gpus", "4", "--steps", "32", "--warmup", "4", "--streams", "16", "--stub-step-ms", "5"]
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR",
                                                            "MASTER_PORT")}
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=4",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), *args]
    out = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=540)
    assert out.returncode == 0, out.stderr[-3000:]
    d = _json_line(out.stdout)
    assert d["data"].startswith("REHEARSAL")
    assert d["config"]["global_batch"] == 64 and d["client_errors"] == []
    assert 4.5 < d["ms_per_step"] < 8.0, d
    assert d["tokens_delivered_in_window"] >= 0.9 * 64 * 32, d


@pytest.mark.timeout(900)
@pytest.mark.parametrize("world,tp", [(2, 2), (8, 8), (8, 4)])
def test_bench_tensor_parallel_serving_path(world, tp):
    """bench.py with --tp over the serving path: `world / tp` replicas of `tp` ranks each (TP=8 is config 4's
    degree; 8 = DP2 x TP4), leaders driving followers by plan broadcasts, collectives over gloo; one valid
    JSON line with every token of every stream delivered through the router, bus and SSE."""
    args = ["bench.py", "--gpus", str(world), "--tp", str(tp), "--steps", "3", "--warmup", "1", "--streams", "3",
            "--prompt-len", "24", "--model", "mistral-tiny-kv8"]
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR",
                                                            "MASTER_PORT")}
    env["OMP_NUM_THREADS"] = "1"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), *args]
    out = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=840)
    assert out.returncode == 0, out.stderr[-3000:]
    d = _json_line(out.stdout)
    replicas = world // tp
    assert d["n_gpus"] == world and d["config"]["parallelism"] == f"dp{replicas}xtp{tp}"
    assert d["config"]["global_batch"] == 3 * replicas and d["client_errors"] == []
    assert d["tokens_delivered_in_window"] >= 3 * replicas * 2
