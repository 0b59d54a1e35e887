"""Phase stamps of gemm_pipe's in-launch split-K fix-up (round 6): build the diagnostic library
(python -m distributed_sse_for_llm_response_amd._build kernels-stamps, or _build.build_kernels(variant="stamps")),
then on the GPU box

    DSSE_KERNELS_VARIANT=stamps python tools/pipe_stamps.py --shape gate_up --M 256 --cfg 8 --split 2

Every workgroup's thread 0 stamps s_memrealtime (100 MHz, one clock for the whole chip) at: 0 start, 1 K loop done,
2 ticket drawn, 3 writer: slot stored + drained / reader: every writer counted, 4 writer: released + counted /
reader: slots read, 5 reader: epilogue stored.  Prints the phase durations (us; median and max over workgroups) and
the launch span."""
import argparse
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from distributed_sse_for_llm_response_amd import ops  # noqa: E402
from distributed_sse_for_llm_response_amd.ops import reference as R  # noqa: E402

SHAPES = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="gate_up")
    ap.add_argument("--M", type=int, default=256)
    ap.add_argument("--cfg", default="8")
    ap.add_argument("--split", default="2")
    a = ap.parse_args()
    os.environ["DSSE_KERNEL_CFG"] = f"t_cfg={a.cfg},t_split={a.split},t_fix=1"
    ops.load_library(required=True)
    ops.refresh_env()
    dev = torch.device("cuda", 0)
    N, K = SHAPES[a.shape]
    g = torch.Generator().manual_seed(0)
    x = (torch.rand(a.M, K, generator=g) * 2 - 1).bfloat16().to(dev)
    w = R.tile_weight(((torch.rand(N, K, generator=g) * 2 - 1) / math.sqrt(K)).bfloat16().to(dev))
    out = torch.empty(a.M, N, device=dev, dtype=torch.bfloat16)
    for _ in range(20):
        ops.gemm_out(x, w, out)
    torch.cuda.synchronize()
    st = torch.ops.dsse.gemm_fix_stamps(0)
    S = int(a.split)
    bm = {"8": 256, "9": 192, "10": 128}[a.cfg]
    wgs = (a.M + bm - 1) // bm * (N // 256) * S
    st = st[:wgs].double()
    t0 = st[:, 0].min()
    ticket = (st[:, 6].long() >> 32)
    last = ticket == S - 1
    us = lambda v: v / 100.0  # noqa: E731 - 100 MHz ticks -> us

    def phase(sel, i, j, name):
        d = us(st[sel, j] - st[sel, i])
        print(f"  {name:34s} median {d.median().item():7.2f}  max {d.max().item():7.2f}  (n={int(sel.sum())})")

    print(f"{a.shape} M={a.M} cfg {a.cfg} S {S}: {wgs} workgroups, span {us(st[last, 5].max() - t0).item():.2f} us")
    print(f"  start spread                       {us(st[:, 0].max() - t0).item():7.2f}")
    phase(torch.ones_like(last), 0, 1, "K loop")
    phase(torch.ones_like(last), 1, 2, "ticket")
    phase(~last, 2, 3, "writer: slot stores + drain")
    phase(~last, 3, 4, "writer: release + count")
    phase(last, 2, 3, "reader: wait for the writers")
    phase(last, 3, 4, "reader: slot reads")
    phase(last, 4, 5, "reader: epilogue")
    print(f"  K loop end: first {us(st[:, 1].min() - t0).item():.2f}, last {us(st[:, 1].max() - t0).item():.2f}")
    xcc = st[:, 6].long() & 0xF
    print(f"  XCCs seen: {sorted(set(xcc.tolist()))}")


if __name__ == "__main__":
    main()
