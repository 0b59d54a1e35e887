"""Command line: ``python -m distributed_sse_for_llm_response_amd <command>``.

  serve     serving process (runtime + engine); env/flags per serving/config.py
            e.g. ``serve --engine gpu --model mistral-7b-v0.3`` (one MI355X), ``--engine stub`` (CPU),
            ``serve --dp 8`` (eight engine replicas behind one router; or torchrun with DP=8),
            ``torchrun --nproc-per-node 8 -m distributed_sse_for_llm_response_amd serve --tp 8``
  loadgen   Python twin of the reference demo/load-generator (producer via RESP, consumer via SSE);
            the native one is ``_lib/dsse-loadgen`` (same flags, epoll, 10k+ connections)
  build     compile the HIP kernels + native runtime in-tree
"""
from __future__ import annotations

import argparse
import sys


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    if not argv or argv[0] in ("-h", "--help"):
        print(__doc__)
        return 0
    cmd, rest = argv[0], argv[1:]
    if cmd == "serve":
        from .serving.config import ServeConfig
        from .serving.launcher import serve_main

        ap = argparse.ArgumentParser(prog="serve")
        ServeConfig.add_args(ap)
        ap.add_argument("--dp-worker-only", action="store_true", help=argparse.SUPPRESS)
        ns = ap.parse_args(rest)
        cfg = ServeConfig.from_env().update_from_args(ns)
        if ns.dp_worker_only:
            import os

            from .serving.dp import worker_only_main

            if os.environ.get("DSSE_SERVE_CONFIG"):
                cfg = ServeConfig.from_json(os.environ["DSSE_SERVE_CONFIG"])
            return worker_only_main(cfg)
        return serve_main(cfg)
    if cmd == "loadgen":
        from .tools_loadgen import main as lg_main

        return lg_main(rest)
    if cmd == "build":
        from . import _build

        _build.build_all(verbose=True, force="--force" in rest)
        return 0
    print(f"unknown command {cmd!r}\n{__doc__}")
    return 2


if __name__ == "__main__":
    sys.exit(main())
