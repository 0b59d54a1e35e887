"""Loader for the native host runtime (``_lib/_dsse_runtime*.so``, C++ sources in ``csrc/runtime``).

Exposes ``Runtime`` (bus + epoll SSE/HTTP server + RESP ingest + metrics) and the wire helpers
(``encode_token_message``, ``sse_frame``, ``inspect``).  The module is built in-tree by
``_build.build_runtime`` (g++, no GPU needed) and rebuilt on demand when missing.
"""
from __future__ import annotations

import importlib
import os
import sys
from pathlib import Path

_LIB_DIR = Path(__file__).resolve().parent.parent / "_lib"
_mod = None


def load(sanitizer: str | None = None):
    """Import the runtime extension (optionally an ASan/TSan/UBSan build: ``runtime-address`` etc.)."""
    global _mod
    if _mod is not None and sanitizer is None:
        return _mod
    name = "_dsse_runtime" if not sanitizer else f"_dsse_runtime_{sanitizer}"
    if not any(_LIB_DIR.glob(name + "*.so")) and os.environ.get("DSSE_AUTOBUILD", "1") == "1":
        from .._build import build_runtime

        build_runtime(sanitize=sanitizer)
    if str(_LIB_DIR) not in sys.path:
        sys.path.insert(0, str(_LIB_DIR))
    mod = importlib.import_module(name)
    if sanitizer is None:
        _mod = mod
    return mod


def server_binary() -> Path:
    """The standalone server (csrc/runtime/server_main.cpp), built on demand."""
    p = _LIB_DIR / "dsse-server"
    if not p.exists() and os.environ.get("DSSE_AUTOBUILD", "1") == "1":
        from .._build import build_runtime

        build_runtime()
    return p


def loadgen_binary() -> Path:
    """The native load generator / bench client (csrc/tools/loadgen.cpp), built on demand."""
    p = _LIB_DIR / "dsse-loadgen"
    if not p.exists() and os.environ.get("DSSE_AUTOBUILD", "1") == "1":
        from .._build import build_runtime

        build_runtime()
    return p


def __getattr__(name):
    return getattr(load(), name)
