"""Deployment assets stay consistent with the code: manifests parse, every metric the dashboard, alerts
and HPA reference is exported by the server, and env keys in the manifests are ones the code reads."""
import glob
import json
import os
import re

import yaml

from distributed_sse_for_llm_response_amd import runtime as rtmod
from distributed_sse_for_llm_response_amd.utils.sse_client import request

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DEPLOY = os.path.join(ROOT, "deploy", "kubernetes")


def _docs():
    out = []
    for f in sorted(glob.glob(os.path.join(DEPLOY, "**", "*.yaml"), recursive=True)):
        with open(f) as fh:
            out += [(f, d) for d in yaml.safe_load_all(fh) if d]
    return out


def _exported_metrics():
    r = rtmod.load().Runtime({"sse_port": -1, "origin_port": -1, "metrics_port": 0, "resp_port": -1, "host": "127.0.0.1"})
    r.start()
    try:
        text = request("127.0.0.1", r.bound_port("metrics"), "GET", "/metrics").body.decode()
    finally:
        r.stop()
    return {ln.split()[2] for ln in text.splitlines() if ln.startswith("# TYPE")}


def test_manifests_parse_and_reference_known_kinds():
    kinds = {d["kind"] for _, d in _docs()}
    assert {"Deployment", "Service", "ConfigMap", "HorizontalPodAutoscaler", "PodDisruptionBudget"} <= kinds


def test_dashboard_alerts_and_hpa_use_exported_metrics():
    exported = _exported_metrics()
    assert {"sse_active_connections", "sse_total_connections", "sse_messages_delivered_total",
            "sse_connection_duration_seconds"} <= exported
    exprs = []
    dash = json.load(open(os.path.join(DEPLOY, "base", "monitoring", "dashboards", "dsse.json")))
    for p in dash["panels"]:
        exprs += [t["expr"] for t in p["targets"]]
    for f, d in _docs():
        if d["kind"] == "ConfigMap" and "rules.yml" in d.get("data", {}):
            exprs += re.findall(r"expr: (.*)", d["data"]["rules.yml"])
        if d["kind"] == "HorizontalPodAutoscaler":
            exprs += [m["pods"]["metric"]["name"] for m in d["spec"]["metrics"] if m["type"] == "Pods"]
    names = set()
    for e in exprs:
        names |= {n for n in re.findall(r"[a-z_][a-z0-9_]*", e) if n.endswith(("_total", "_seconds_bucket", "_connections",
                                                                                "_size", "_free", "_alive", "_chats"))}
    missing = {n for n in names if n.removesuffix("_bucket") not in exported}
    assert not missing, missing


def test_configmap_env_keys_are_read_by_the_code():
    code = ""
    for f in glob.glob(os.path.join(ROOT, "csrc", "runtime", "*.cpp")) + glob.glob(
            os.path.join(ROOT, "distributed_sse_for_llm_response_amd", "serving", "*.py")):
        code += open(f).read()
    for f, d in _docs():
        if d["kind"] == "ConfigMap" and d["metadata"]["name"].startswith("dsse-"):
            for k in d["data"]:
                if k == "HSA_ENABLE_IPC_MODE_LEGACY":
                    continue  # consumed by the ROCm runtime
                assert f'"{k}"' in code, f"{os.path.relpath(f, ROOT)}: {k} is not read anywhere"


def test_run_loadtest_renders_the_job():
    import subprocess

    out = subprocess.run(["bash", os.path.join(ROOT, "scripts", "run-loadtest.sh"), "--k8s", "-conversations", "100",
                          "-tokens", "200", "-duration", "5m", "-chat"], env={**os.environ, "DRY_RUN": "1"},
                         capture_output=True, text=True, check=True).stdout
    job = yaml.safe_load(out)
    assert job["kind"] == "Job"
    args = job["spec"]["template"]["spec"]["containers"][0]["args"]
    assert args[args.index("-conversations") + 1] == "100" and args[args.index("-tokens") + 1] == "200"
    assert "-chat" in args and args[-1] == "-json" and args[args.index("-sse") + 1] == "http://dsse-edge:80"


def test_run_loadtest_local_against_a_stub_server():
    """The wrapper's local mode drives the native load generator (RESP producers + SSE consumers)."""
    import subprocess

    r = rtmod.load().Runtime({"sse_port": 0, "origin_port": -1, "metrics_port": -1, "resp_port": 0,
                              "host": "127.0.0.1", "io_threads": 2})
    r.start()
    try:
        out = subprocess.run(["bash", os.path.join(ROOT, "scripts", "run-loadtest.sh"),
                              "-sse", f"http://127.0.0.1:{r.bound_port('edge')}",
                              "-redis", f"127.0.0.1:{r.bound_port('resp')}", "-conversations", "4", "-tokens", "6",
                              "-token-delay", "5", "-duration", "10s", "-json"],
                             capture_output=True, text=True, timeout=60)
    finally:
        r.stop()
    assert out.returncode == 0, out.stderr
    stats = json.loads(out.stdout.strip().splitlines()[-1])
    assert stats["tokens_received"] == stats["tokens_published"] == 4 * 6, stats
