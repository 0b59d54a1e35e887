"""A/B of the decode MLP block at M rows: the launch-per-op chain (gemm_ring o -> rmsnorm<3> -> gate_up -> down ->
rmsnorm<3>) vs the persistent kernel (decode_mega.hip), both captured as hipGraphs of 32 blocks over 8 distinct
weight sets (3 GB, far past the 256 MB Infinity Cache), replayed alternately in one process (guide §5.4 rule 24).

    python tools/bench_mega.py [--M 64] [--rounds 10] [--qkv] [--stamps]

--qkv adds the next layer's QKV projection phase to the persistent kernel (and a gemm_qkv_slabs launch to the
unfused chain).  --stamps re-runs a few persistent launches with per-workgroup phase timestamps (s_memrealtime,
10 ns) and prints when each phase's dependency was met and when it finished, across the 256 workgroups: where the
weight stream waits on a seam.
"""
import argparse
import math
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_sse_for_llm_response_amd import ops  # noqa: E402
from distributed_sse_for_llm_response_amd.ops import reference as R  # noqa: E402

H, F = 4096, 14336


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, default=64)
    ap.add_argument("--rounds", type=int, default=10)
    ap.add_argument("--sets", type=int, default=8)
    ap.add_argument("--blocks", type=int, default=32)
    ap.add_argument("--qkv", action="store_true")
    ap.add_argument("--stamps", action="store_true")
    ap.add_argument("--pf", default="4", help="seam prefetch steps to A/B (comma list, each a persistent arm)")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    ops.load_library(required=True)
    torch.manual_seed(0)

    def w(n, k):  # random bf16 directly on the device (tiled layout is a permutation: random stays random)
        return (torch.randn(n, k, device=dev) / math.sqrt(k)).bfloat16()

    sets = [dict(wo=w(H, H), wgu=w(2 * F, H), wd=w(H, F), wqkv=w(6144, H) if a.qkv else None,
                 w_ffn=torch.ones(H, device=dev).bfloat16(), w_next=torch.ones(H, device=dev).bfloat16())
            for _ in range(a.sets)]
    M = a.M
    attn = torch.randn(M, H, device=dev).bfloat16()
    resid = torch.randn(M, H, device=dev)
    xm = torch.zeros(M, H, device=dev, dtype=torch.bfloat16)
    x = torch.zeros_like(xm)
    h = torch.zeros(M, F, device=dev, dtype=torch.bfloat16)
    part = torch.zeros(32 * 64 * H, device=dev)
    sync = ops.mega_sync(dev)
    err = torch.zeros(1, dtype=torch.int32, device=dev)
    qkv_slabs = torch.zeros(4 * M * 6144, device=dev) if a.qkv else None

    def unfused():
        for i in range(a.blocks):
            s = sets[i % a.sets]
            ns = ops.gemm_resid_split(attn, s["wo"], resid, part)
            ops.rmsnorm(resid, s["w_ffn"], xm, 1e-5, part=part, nsplit=ns)
            ops.gemm_silu(xm, s["wgu"], h)
            ns = ops.gemm_resid_split(h, s["wd"], resid, part)
            ops.rmsnorm(resid, s["w_next"], x, 1e-5, part=part, nsplit=ns)
            if a.qkv:
                ops.gemm_qkv_slabs(x, s["wqkv"], qkv_slabs)

    pfs = [int(v) for v in a.pf.split(",")]

    def fused(stamps=None, i0=0, n=None, pf=pfs[0]):
        for i in range(i0, i0 + (n or a.blocks)):
            s = sets[i % a.sets]
            ops.mega_mlp(attn, s["wo"], s["wgu"], s["wd"], resid, s["w_ffn"], s["w_next"], xm, h, x, part, sync, err,
                         1e-5, wqkv=s["wqkv"], qkv_slabs=qkv_slabs,
                         stamps=None if stamps is None else stamps[i - i0], pf_steps=pf)

    graphs = {}
    arms = [("unfused", unfused)] + [(f"mega_pf{v}", (lambda v=v: fused(pf=v))) for v in pfs]
    for name, fn in arms:
        st = torch.cuda.Stream()
        st.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(st):
            fn()
        torch.cuda.current_stream().wait_stream(st)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            fn()
        graphs[name] = g
    times = {k: [] for k in graphs}
    for _ in range(a.rounds):
        for name, g in graphs.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            g.replay()
            e1.record()
            e1.synchronize()
            times[name].append(e0.elapsed_time(e1) * 1000 / a.blocks)
    assert int(err.item()) == 0, "mega kernel: a bounded wait timed out"
    byts = (H * H + 2 * F * H + H * F + (6144 * H if a.qkv else 0)) * 2
    for name, t in times.items():
        t = sorted(t)
        med = t[len(t) // 2]
        print(f"{name:8s} M={M}: per block median {med:7.2f} us  min {t[0]:7.2f} us  "
              f"({byts / med / 1e6:.2f} TB/s weight stream)", flush=True)
    if a.stamps:
        n = 6
        st = torch.zeros(n, 256, 16, dtype=torch.int64, device=dev)
        fused(st, 0, n, pf=pfs[-1])
        torch.cuda.synchronize()
        assert int(err.item()) == 0, "mega kernel: a bounded wait timed out"
        names = ["start", "attention done", "O dep met", "O done", "N1 dep met", "N1 done", "gate_up dep met",
                 "gate_up done", "down dep met", "down done", "N2 dep met", "N2 done", "QKV dep met", "QKV done", "end", "gate_up pre-fence"]
        for k in (3, 4, 5):  # launches whose weight sets are cold (rotating 8 sets)
            s = st[k].cpu().double()
            t0 = s[:, 0].min()
            print(f"\nlaunch {k}: phase stamps in us from the first workgroup's start (over the workgroups that record it)")
            print(f"{'phase':18s} {'n':>4s} {'min':>8s} {'median':>8s} {'max':>8s}")
            for i, nm in enumerate(names):
                col = s[:, i]
                col = col[col > 0]
                if col.numel() == 0:
                    continue
                us = ((col - t0) / 100.0).sort().values  # 100 MHz
                print(f"{nm:18s} {us.numel():4d} {us[0]:8.2f} {us[us.numel() // 2]:8.2f} {us[-1]:8.2f}")


if __name__ == "__main__":
    main()
