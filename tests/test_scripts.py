"""Operator scripts and images (reference scripts/deploy-origin.sh, deploy-edge.sh, build-push-images.sh,
run-demo.sh and the per-service Dockerfiles): every script parses, the Dockerfiles only COPY paths that exist,
and deploy.sh / build-images.sh issue the expected kubectl / docker commands (stubbed on PATH, nothing runs)."""
import glob
import os
import re
import stat
import subprocess

import yaml

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SCRIPTS = sorted(glob.glob(os.path.join(ROOT, "scripts", "*.sh")))


def _stub(tmp_path, name, body):
    d = tmp_path / "bin"
    d.mkdir(exist_ok=True)
    p = d / name
    p.write_text("#!/usr/bin/env bash\n" + body)
    p.chmod(p.stat().st_mode | stat.S_IEXEC)
    return str(d)


def test_every_script_parses():
    assert len(SCRIPTS) >= 4
    for s in SCRIPTS:
        r = subprocess.run(["bash", "-n", s], capture_output=True, text=True)
        assert r.returncode == 0, (s, r.stderr)


def test_dockerfiles_copy_existing_paths():
    for df in glob.glob(os.path.join(ROOT, "deploy", "docker", "Dockerfile*")):
        for line in open(df):
            m = re.match(r"COPY\s+(?!--from)(.+)\s+\S+\s*$", line.strip())
            if not m:
                continue
            for src in m.group(1).split():
                assert os.path.exists(os.path.join(ROOT, src)), (os.path.basename(df), src)


def test_build_images_builds_and_pushes_both_images(tmp_path):
    log = tmp_path / "docker.log"
    path = _stub(tmp_path, "docker", f'echo "$@" >> {log}\n')
    subprocess.run(["bash", os.path.join(ROOT, "scripts", "build-images.sh"), "reg.local/x", "v1", "--push"],
                   env={**os.environ, "PATH": path + os.pathsep + os.environ["PATH"]}, check=True,
                   capture_output=True)
    cmds = log.read_text().splitlines()
    assert cmds[0].startswith("build -f deploy/docker/Dockerfile -t reg.local/x/origin:v1")
    assert cmds[1].startswith("build -f deploy/docker/Dockerfile.edge -t reg.local/x/edge:v1")
    assert cmds[2:] == ["push reg.local/x/origin:v1", "push reg.local/x/edge:v1"]


def test_deploy_edge_renders_the_overlay_with_the_origin_address(tmp_path):
    cap = tmp_path / "overlay"
    log = tmp_path / "kubectl.log"
    # `apply -k DIR` snapshots the rendered overlay before deploy.sh deletes its temp dir
    path = _stub(tmp_path, "kubectl",
                 f'echo "$@" >> {log}\nif [ "$1" = apply ]; then cp -r "$3" {cap}; fi\n')
    subprocess.run(["bash", os.path.join(ROOT, "scripts", "deploy.sh"), "edge", "/dev/null", "origin.example.net"],
                   env={**os.environ, "PATH": path + os.pathsep + os.environ["PATH"]}, check=True,
                   capture_output=True)
    cmds = log.read_text().splitlines()
    assert cmds[0].startswith("apply -k ") and "rollout status deploy/dsse-edge" in cmds[1]
    patch = yaml.safe_load((cap / "origin-address.yaml").read_text())
    assert patch["data"] == {"LLM_PROXY_URL": "http://origin.example.net:8081",
                             "UPSTREAM_URL": "http://origin.example.net:80"}
    kust = yaml.safe_load((cap / "kustomization.yaml").read_text())
    for res in kust["resources"]:
        assert os.path.isabs(res) and os.path.isdir(res), res
    # the patch targets a ConfigMap the edge base actually defines
    base = [d for f in glob.glob(os.path.join(ROOT, "deploy", "kubernetes", "base", "edge", "*.yaml"))
            for d in yaml.safe_load_all(open(f)) if d]
    assert any(d["kind"] == "ConfigMap" and d["metadata"]["name"] == patch["metadata"]["name"] for d in base)


def test_deploy_origin_applies_the_origin_overlay(tmp_path):
    log = tmp_path / "kubectl.log"
    path = _stub(tmp_path, "kubectl", f'echo "$@" >> {log}\n')
    subprocess.run(["bash", os.path.join(ROOT, "scripts", "deploy.sh"), "origin", "/dev/null"],
                   env={**os.environ, "PATH": path + os.pathsep + os.environ["PATH"]}, check=True,
                   capture_output=True)
    cmds = log.read_text().splitlines()
    assert cmds[0] == "apply -k deploy/kubernetes/overlays/origin"
    assert "rollout status deploy/dsse-origin" in cmds[1]
    r = subprocess.run(["bash", os.path.join(ROOT, "scripts", "deploy.sh"), "bogus", "/dev/null"],
                       env={**os.environ, "PATH": path + os.pathsep + os.environ["PATH"]}, capture_output=True)
    assert r.returncode == 2
