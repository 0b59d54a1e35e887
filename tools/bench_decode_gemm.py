"""Decode-shape GEMM variants timed the way the decode step runs them: captured in a hipGraph, back to back, over
enough distinct weight copies (> the 256 MB Infinity Cache) that every call streams its weights from HBM.

    python tools/bench_decode_gemm.py --shape o,down --M 64 --variants split_norm,resid:gemm_impl=0 ...

A variant is OP[:key=value,...] with the keys of DSSE_KERNEL_CFG; OP is
    split_norm  gemm_resid_split + rmsnorm (slabs reduced in the norm: the TP = 1 decode path)
    resid       gemm_resid (resid += x·wᵀ, no norm)
    out         gemm_out (bf16 out)       silu   gemm_silu
    lib         torch.matmul on a row-major copy (hipBLASLt: a yardstick only, the engine never calls it)
Prints one line per (shape, variant): us per call (graph replay, events), effective weight bandwidth.
"""
import argparse
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from distributed_sse_for_llm_response_amd import ops  # noqa: E402
from distributed_sse_for_llm_response_amd.ops import reference as R  # noqa: E402

SHAPES = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336),
          # one rank's shard at TP = 8 (tools/bench_tp_rank.py): column-parallel N / 8, row-parallel K / 8
          "qkv_tp8": (768, 4096), "o_tp8": (4096, 512), "gate_up_tp8": (3584, 4096), "down_tp8": (4096, 1792),
          "lm_tp8": (4096, 4096)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="o,down")
    ap.add_argument("--M", default="64")
    ap.add_argument("--variants", default="split_norm")
    ap.add_argument("--bytes", type=float, default=1.2e9, help="weight bytes cycled through per replay")
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    ops.load_library(required=True)
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(0)
    base_cfg = os.environ.get("DSSE_KERNEL_CFG", "")
    for shape in a.shape.split(","):
        N, K = SHAPES[shape]
        ncopy = max(2, math.ceil(a.bytes / (N * K * 2)))
        w0 = R.tile_weight(((torch.rand(N, K, generator=g) * 2 - 1) / math.sqrt(K)).bfloat16().to(dev))
        ws = [w0.clone() for _ in range(ncopy)]
        libw = None
        for M in [int(m) for m in a.M.split(",")]:
            x = (torch.rand(M, K, generator=g) * 2 - 1).bfloat16().to(dev)
            resid = torch.randn(M, N, generator=g).to(dev)
            nw = torch.ones(N, device=dev, dtype=torch.bfloat16)
            y = torch.zeros(M, N, device=dev, dtype=torch.bfloat16)
            part = torch.zeros(32 * max(M, 64) * N, device=dev)
            outb = torch.zeros(M, N, device=dev, dtype=torch.bfloat16)
            outh = torch.zeros(M, N // 2, device=dev, dtype=torch.bfloat16)
            for var in a.variants.split(","):
                op, _, cfg = var.partition(":")
                if op == "lib" and libw is None:
                    libw = [R.untile_weight(w) for w in ws]
                    idx = {id(w): i for i, w in enumerate(ws)}
                os.environ["DSSE_KERNEL_CFG"] = ",".join(c for c in (base_cfg, cfg.replace(";", ",")) if c)
                ops.refresh_env()

                def one(w):
                    if op == "split_norm":
                        ns = ops.gemm_resid_split(x, w, resid, part)
                        ops.rmsnorm(resid, nw, y, 1e-5, part=part, nsplit=ns)
                    elif op == "resid":
                        ops.gemm_resid(x, w, resid)
                    elif op == "out":
                        ops.gemm_out(x, w, outb)
                    elif op == "silu":
                        ops.gemm_silu(x, w, outh)
                    elif op == "lib":
                        torch.matmul(x, libw[idx[id(w)]].t(), out=outb)
                    else:
                        raise SystemExit(f"unknown op {op}")

                try:
                    for w in ws[:2]:
                        one(w)
                    torch.cuda.synchronize()
                    s = torch.cuda.Stream()
                    with torch.cuda.stream(s):
                        graph = torch.cuda.CUDAGraph()
                        with torch.cuda.graph(graph, stream=s):
                            for w in ws:
                                one(w)
                    torch.cuda.synchronize()
                    graph.replay()
                    torch.cuda.synchronize()
                    best = float("inf")
                    for _ in range(a.reps):
                        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                        e0.record()
                        graph.replay()
                        e1.record()
                        torch.cuda.synchronize()
                        best = min(best, e0.elapsed_time(e1) * 1e3 / ncopy)
                    impl, cfg_, S_, fix_, est = torch.ops.dsse.gemm_plan(M, N, K, op == "split_norm")
                    plan = f"impl {impl} cfg {cfg_} S {S_}{' fix' if fix_ else ''} est {est:6.1f}" if impl == 4 else \
                        f"impl {impl}"
                    print(f"{shape:8s} M={M:4d} {var:40s} {best:8.2f} us/call  {N * K * 2 / best / 1e6:6.2f} TB/s "
                          f"{2 * M * N * K / best / 1e6:7.1f} TF/s  [{plan}]", flush=True)
                    del graph
                except Exception as e:  # noqa: BLE001 - report and go on with the next variant
                    print(f"{shape:8s} M={M:4d} {var:40s} FAILED {type(e).__name__}: {str(e)[:200]}", flush=True)
    os.environ["DSSE_KERNEL_CFG"] = base_cfg


if __name__ == "__main__":
    main()
