"""In-tree native build: HIP kernels for gfx950 and the C++ host runtime.

Everything is compiled with explicit ``hipcc`` / ``g++`` command lines (no hipify, no JIT cache) and
the resulting shared objects are written next to the Python package in ``_lib/`` so they travel
with the repository snapshot to the GPU box.

* ``_lib/libdsse_kernels.so`` — every ``csrc/kernels/*.hip`` file plus ``bindings.cpp`` (torch op
  registrations, namespace ``torch.ops.dsse``), built with ``--offload-arch=gfx950``.
* ``_lib/_dsse_runtime*.so`` — the C++ host runtime (bus, SSE/HTTP server, RESP ingest, inspector,
  metrics, shared-memory rings) as a CPython extension (pybind11), plus the standalone
  ``_lib/dsse-server`` binary (CPU plumbing mode, BASELINE config 1).

Rebuilds are incremental on file mtimes (sources and headers of their directory).
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import shutil
import subprocess
import sys
import sysconfig
from pathlib import Path

PKG_DIR = Path(__file__).resolve().parent
REPO = PKG_DIR.parent
CSRC = REPO / "csrc"
LIB_DIR = PKG_DIR / "_lib"
BUILD_DIR = REPO / "build" / "native"
ARCH = os.environ.get("DSSE_OFFLOAD_ARCH", "gfx950")
HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"

KERNELS_SO = LIB_DIR / "libdsse_kernels.so"


def _torch_paths():
    import torch  # noqa: WPS433  (only needed for the kernel extension)

    root = Path(torch.__file__).resolve().parent
    return root / "include", root / "include" / "torch" / "csrc" / "api" / "include", root / "lib", int(
        torch._C._GLIBCXX_USE_CXX11_ABI
    )


def _stale(out: Path, deps) -> bool:
    if not out.exists():
        return True
    t = out.stat().st_mtime
    return any(Path(d).stat().st_mtime > t for d in deps)


def _run(cmd, verbose):
    if verbose:
        print("[build]", " ".join(str(c) for c in cmd), flush=True)
    res = subprocess.run([str(c) for c in cmd], capture_output=True, text=True)
    if res.returncode != 0:
        raise RuntimeError(f"command failed ({res.returncode}): {' '.join(map(str, cmd))}\n{res.stdout}\n{res.stderr}")
    return res


def _parallel(jobs, verbose):
    if not jobs:
        return
    workers = max(1, min(len(jobs), int(os.environ.get("MAX_JOBS", os.cpu_count() or 4)), 16))
    with cf.ThreadPoolExecutor(workers) as ex:
        futs = [ex.submit(_run, cmd, verbose) for cmd in jobs]
        for f in futs:
            f.result()


KERNEL_VARIANTS = {
    "checked": ["-DDSSE_KERNEL_CHECKS=1"],  # device index-check debug build (tools/check_kernels.py)
    "burst": ["-DDSSE_TILED_BURST=1"],  # A/B build: gemm_tiled issues each stage's DMA in one burst
    "stamps": ["-DDSSE_PIPE_STAMPS=1"],  # diagnostic build: gemm_pipe FIX phase stamps (tools/pipe_stamps.py)
}  # libdsse_kernels_<variant>.so, selected at import with DSSE_KERNELS_VARIANT


def kernels_so(variant: str | None = None) -> Path:
    return LIB_DIR / (f"libdsse_kernels_{variant}.so" if variant else "libdsse_kernels.so")


def build_kernels(verbose: bool = False, force: bool = False, variant: str | None = None) -> Path:
    """Compile csrc/kernels into _lib/libdsse_kernels.so (gfx950 code objects + torch ops)."""
    inc, api_inc, torch_lib, abi = _torch_paths()
    kdir = CSRC / "kernels"
    obj_dir = BUILD_DIR / ("kernels" + (f"_{variant}" if variant else ""))
    obj_dir.mkdir(parents=True, exist_ok=True)
    LIB_DIR.mkdir(parents=True, exist_ok=True)
    headers = sorted(kdir.glob("*.h"))
    common = ["-O3", "-std=c++17", "-fPIC", f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-Wno-unused-result"]
    common += KERNEL_VARIANTS.get(variant, [])
    out_so = kernels_so(variant)
    jobs, objs = [], []
    for src in sorted(kdir.glob("*.hip")):
        obj = obj_dir / (src.stem + ".o")
        objs.append(obj)
        if force or _stale(obj, [src, *headers]):
            jobs.append([HIPCC, f"--offload-arch={ARCH}", *common, "-munsafe-fp-atomics", "-c", src, "-o", obj])
    bsrc = kdir / "bindings.cpp"
    bobj = obj_dir / "bindings.o"
    objs.append(bobj)
    if force or _stale(bobj, [bsrc, *headers]):
        jobs.append([
            HIPCC, *common, "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1", "-x", "hip", "--offload-host-only",
            "-I", inc, "-I", api_inc, "-c", bsrc, "-o", bobj,
        ])
    _parallel(jobs, verbose)
    if force or _stale(out_so, objs):
        tmp = out_so.with_name(out_so.name + ".tmp")
        _run([
            HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", *objs, "-o", tmp,
            "-L", torch_lib, "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip",
            f"-Wl,-rpath,{torch_lib}",
        ], verbose)
        os.replace(tmp, out_so)  # atomic: a concurrent reader (or a tree snapshot) never sees a half-written library
    return out_so


def _py_ext_suffix() -> str:
    return sysconfig.get_config_var("EXT_SUFFIX") or ".so"


RUNTIME_SO = LIB_DIR / f"_dsse_runtime{_py_ext_suffix()}"
SERVER_BIN = LIB_DIR / "dsse-server"


def build_runtime(verbose: bool = False, force: bool = False, sanitize: str | None = None) -> Path:
    """Compile the C++ host runtime (csrc/runtime) into a pybind11 module and a standalone server."""
    import pybind11

    rdir = CSRC / "runtime"
    if not rdir.exists():
        return RUNTIME_SO
    tag = f"-{sanitize}" if sanitize else ""
    obj_dir = BUILD_DIR / f"runtime{tag}"
    obj_dir.mkdir(parents=True, exist_ok=True)
    LIB_DIR.mkdir(parents=True, exist_ok=True)
    headers = sorted(rdir.glob("*.h"))
    cxx = os.environ.get("CXX", "g++")
    flags = ["-O2", "-g", "-std=c++17", "-fPIC", "-Wall", "-Wextra", "-Wno-unused-parameter", "-pthread"]
    if sanitize:
        flags += [f"-fsanitize={sanitize}", "-fno-omit-frame-pointer", "-O1"]
    lib_srcs = [s for s in sorted(rdir.glob("*.cpp")) if s.name not in ("pybind_module.cpp", "server_main.cpp")]
    jobs, objs = [], []
    for src in lib_srcs:
        obj = obj_dir / (src.stem + ".o")
        objs.append(obj)
        if force or _stale(obj, [src, *headers]):
            jobs.append([cxx, *flags, "-c", src, "-o", obj])
    py_inc = sysconfig.get_paths()["include"]
    mod_src = rdir / "pybind_module.cpp"
    mod_obj = obj_dir / "pybind_module.o"
    if force or _stale(mod_obj, [mod_src, *headers]):
        jobs.append([cxx, *flags, "-fvisibility=hidden", "-I", pybind11.get_include(), "-I", py_inc, "-c", mod_src,
                     "-o", mod_obj])
    main_src = rdir / "server_main.cpp"
    main_obj = obj_dir / "server_main.o"
    if main_src.exists() and (force or _stale(main_obj, [main_src, *headers])):
        jobs.append([cxx, *flags, "-c", main_src, "-o", main_obj])
    _parallel(jobs, verbose)
    if sanitize:
        out_so = LIB_DIR / f"_dsse_runtime_{sanitize}{_py_ext_suffix()}"
        out_bin = LIB_DIR / f"dsse-server-{sanitize}"
    else:
        out_so, out_bin = RUNTIME_SO, SERVER_BIN
    if force or _stale(out_so, objs + [mod_obj]):
        _run([cxx, *flags, "-shared", *objs, mod_obj, "-o", out_so], verbose)
    if main_src.exists() and (force or _stale(out_bin, objs + [main_obj])):
        _run([cxx, *flags, *objs, main_obj, "-o", out_bin], verbose)
    # standalone tools (no runtime library): the native load generator / bench client
    lg_src = CSRC / "tools" / "loadgen.cpp"
    lg_bin = LIB_DIR / (f"dsse-loadgen-{sanitize}" if sanitize else "dsse-loadgen")
    if lg_src.exists() and (force or _stale(lg_bin, [lg_src])):
        _run([cxx, *flags, lg_src, "-o", lg_bin], verbose)
    return out_so


def build_all(verbose: bool = False, force: bool = False) -> None:
    with cf.ThreadPoolExecutor(2) as ex:
        fk = ex.submit(build_kernels, verbose, force)
        fr = ex.submit(build_runtime, verbose, force)
        fk.result()
        fr.result()


if __name__ == "__main__":
    what = sys.argv[1] if len(sys.argv) > 1 else "all"
    force = "--force" in sys.argv
    if what == "kernels":
        build_kernels(True, force)
    elif what.startswith("kernels-"):
        build_kernels(True, force, variant=what.split("-", 1)[1])
    elif what == "runtime":
        build_runtime(True, force)
    elif what.startswith("runtime-"):
        build_runtime(True, force, sanitize=what.split("-", 1)[1])
    else:
        build_all(True, force)
