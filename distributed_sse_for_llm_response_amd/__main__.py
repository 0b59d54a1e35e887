"""Command line: ``python -m distributed_sse_for_llm_response_amd <command>``.

  serve     serving process (runtime + engine); env/flags per serving/config.py
            e.g. ``serve --engine gpu --model mistral-7b-v0.3`` (one MI355X), ``--engine stub`` (CPU)
  loadgen   Python twin of the reference demo/load-generator (producer via RESP, consumer via SSE)
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
        ns = ap.parse_args(rest)
        cfg = ServeConfig.from_env().update_from_args(ns)
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
