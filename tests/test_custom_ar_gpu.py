"""Fused TP all-reduce + residual + RMSNorm over IPC peer buffers (csrc/kernels/allreduce.hip), several processes
sharing the one GPU of the test box through IPC handles (the 8-GPU node runs the same code over xGMI).

Every rank's result must equal torch.sum of all ranks' partial rows (+ residual, then the fp32 reference norm),
bit-identical across ranks, over many back-to-back calls with varying row counts (both buffer parities, rows
that sit out some calls), and no peer wait may time out."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, iters, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0")
    from distributed_sse_for_llm_response_amd.ops import reference as R
    from distributed_sse_for_llm_response_amd.parallel.comm import TPComm

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        comm = TPComm(rank=rank, size=world, group=None)
        H, rows = 4096, 64
        why = comm.enable_ipc_allreduce(dev, rows, H)
        res = {"why": why, "bad": [], "uncached": None, "digest": []}
        if why:
            out[rank] = res
            return
        ar = comm.fast_ar
        res["uncached"] = ar.uncached
        g = torch.Generator().manual_seed(99)  # same stream on every rank: shared resid / norm weight
        gl = torch.Generator().manual_seed(1000 + rank)  # this rank's partials
        w = (1 + 0.1 * torch.randn(H, generator=g)).bfloat16()
        for it in range(iters):
            M = [64, 1, 33, 64, 5][it % 5]
            resid0 = torch.randn(M, H, generator=g)
            mine = (torch.randn(M, H, generator=gl) * (1 + it % 3)).bfloat16()
            r = resid0.to(dev)
            y = torch.zeros(M, H, dtype=torch.bfloat16, device=dev)
            comm.all_reduce_rmsnorm(mine.to(dev), r, w.to(dev), y, 1e-5)
            allp = [torch.zeros(M, H, dtype=torch.bfloat16) for _ in range(world)]
            dist.all_gather(allp, mine)
            tot = torch.stack([p.float() for p in allp]).sum(0)
            r_ref = resid0 + tot
            y_ref = torch.zeros(M, H, dtype=torch.bfloat16)
            R.rmsnorm(r_ref.clone(), w, y_ref, 1e-5)
            rc, yc = r.cpu(), y.cpu()
            er, ey = float((rc - r_ref).abs().max()), float((yc.float() - y_ref.float()).abs().max())
            if er > 1e-4 or ey > 3e-2:
                res["bad"].append((it, M, er, ey))
            res["digest"].append(float(rc.double().sum()) + float(yc.double().sum()))
        torch.cuda.synchronize(dev)
        res["err"] = int(ar.err.item())
        out[rank] = res
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world", [2, 4])
def test_ipc_allreduce_rmsnorm_multiprocess_one_gpu(gpu, world):
    with mp.Manager() as m:
        out = m.dict()
        ctx = mp.get_context("spawn")
        port = _port()
        procs = [ctx.Process(target=_worker, args=(r, world, port, 40, out)) for r in range(world)]
        for p in procs:
            p.start()
        for p in procs:
            p.join(240)
        for p in procs:  # never leave a rank behind on the GPU
            if p.is_alive():
                p.kill()
                p.join(10)
        codes = [p.exitcode for p in procs]
        res = [out.get(r) for r in range(world)]
    assert codes == [0] * world, codes
    assert all(r is not None for r in res)
    assert res[0]["why"] == "", res[0]["why"]
    for r in res:
        assert r["err"] == 0, "a peer wait timed out"
        assert r["bad"] == [], r["bad"][:5]
    # identical bits on every rank (rank-order fp32 sum): the TP ranks' residual streams never drift apart
    assert all(r["digest"] == res[0]["digest"] for r in res)



def _replay_worker(rank, world, port, buckets, iters, out):
    """One TP rank: all_reduce_rmsnorm captured into one hipGraph per bucket, replayed `iters` times in a seeded mixed
    bucket order (the same on every rank), every result checked against torch fp32 on the device."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0")
    import random

    from distributed_sse_for_llm_response_amd.parallel.comm import TPComm

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    res = {"why": "", "bad": [], "digest": [], "err": -1}
    try:
        comm = TPComm(rank=rank, size=world, group=None)
        H, rows = 4096, max(buckets)
        res["why"] = comm.enable_ipc_allreduce(dev, rows, H)
        if res["why"]:
            out[rank] = res
            return
        w = (1 + 0.1 * torch.sin(torch.arange(H, device=dev, dtype=torch.float32))).bfloat16()
        st = {b: dict(tmp=torch.zeros(b, H, dtype=torch.bfloat16, device=dev), r=torch.zeros(b, H, device=dev),
                      y=torch.zeros(b, H, dtype=torch.bfloat16, device=dev)) for b in buckets}
        graphs = {}
        s = torch.cuda.Stream(dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        for b in buckets:  # capture only (no eager warm-up: the kernel needs no library init)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=s):
                comm.all_reduce_rmsnorm(st[b]["tmp"], st[b]["r"], w, st[b]["y"], 1e-5)
            graphs[b] = g
        torch.cuda.current_stream(dev).wait_stream(s)
        torch.cuda.synchronize(dev)
        n = torch.arange(H, device=dev, dtype=torch.float32)
        order = random.Random(5).choices(buckets, k=iters)

        def partial(q, it, b):  # rank q's partial rows of iteration it (every rank can rebuild every partial)
            m = torch.arange(b, device=dev, dtype=torch.float32)[:, None]
            return torch.sin(0.37 * q + 0.011 * it + 0.13 * m + 0.007 * n[None, :] * (q + 1)).bfloat16()

        for it, b in enumerate(order):
            t = st[b]
            r0 = torch.cos(0.05 * it + 0.21 * torch.arange(b, device=dev)[:, None] + 0.003 * n[None, :])
            t["tmp"].copy_(partial(rank, it, b))
            t["r"].copy_(r0)
            graphs[b].replay()
            tot = torch.zeros(b, H, device=dev)
            for q in range(world):
                tot += partial(q, it, b).float()
            r_ref = r0 + tot
            y_ref = (r_ref * torch.rsqrt(r_ref.pow(2).mean(-1, keepdim=True) + 1e-5) * w.float()).bfloat16()
            er = float((t["r"] - r_ref).abs().max())
            ey = float((t["y"].float() - y_ref.float()).abs().max())
            if er > 1e-4 or ey > 3e-2:
                res["bad"].append((it, b, er, ey))
            res["digest"].append(float(t["r"].double().sum()) + float(t["y"].double().sum()))
        torch.cuda.synchronize(dev)
        res["err"] = int(comm.fast_ar.err.item())
        dist.barrier()
        comm.close()  # IPC handles closed, buffer freed (ar_close)
        res["closed"] = comm.fast_ar is None
        out[rank] = res
        dist.barrier()
    finally:
        dist.destroy_process_group()


# 8 ranks at 1 and 64 rows; 256 rows with 2 ranks.  On the one-GPU box all ranks' workgroups share its CUs: 8 ranks x
# 256 rows = 2048 workgroups of 512 threads against ~1024 resident slots, and ranks replay asynchronously, so half the
# ranks' grids could fill the GPU while waiting for the other half's rows.  On the 8-GPU node each rank's grid has
# its own device.
@pytest.mark.timeout(600)
@pytest.mark.parametrize("world,buckets", [(8, (1, 64)), (2, (1, 64, 256))])
def test_ipc_allreduce_graph_replay_multiprocess(gpu, world, buckets):
    """The decode path's form of the IPC all-reduce: captured into hipGraphs per bucket and replayed 200 times in
    mixed bucket order (the per-row epoch counters live in device memory across replays); every replay equals the
    fp32 sum of all ranks' partials + residual and its norm, identical bits on every rank, no peer wait timed out,
    and the context is torn down with ar_close."""
    with mp.Manager() as m:
        out = m.dict()
        ctx = mp.get_context("spawn")
        port = _port()
        procs = [ctx.Process(target=_replay_worker, args=(r, world, port, list(buckets), 200, out))
                 for r in range(world)]
        for p in procs:
            p.start()
        for p in procs:
            p.join(540)
        for p in procs:
            if p.is_alive():
                p.kill()
                p.join(10)
        codes = [p.exitcode for p in procs]
        res = [out.get(r) for r in range(world)]
    assert codes == [0] * world, codes
    assert all(r is not None for r in res)
    assert res[0]["why"] == "", res[0]["why"]
    for r in res:
        assert r["err"] == 0, "a peer wait timed out"
        assert r["bad"] == [], r["bad"][:5]
        assert r["closed"]
    assert all(r["digest"] == res[0]["digest"] for r in res)


@pytest.mark.parametrize("M,S", [(1, 2), (37, 2), (64, 4), (64, 7)])
def test_ar_rmsnorm_sums_split_k_slabs(gpu, M, S):
    """Round 6: the IPC all-reduce + RMSNorm kernel takes the O / down GEMM's fp32 split-K slabs directly (part /
    nsplit) -- bit for bit what the splitk_reduce_kernel -> bf16 tmp -> ar_rmsnorm chain gives (one rank, its own
    buffer as the only peer: the kernel, the flags and the epochs run as in a TP group)."""
    from distributed_sse_for_llm_response_amd import ops

    ops.load_library(required=True)
    rows, H = 64, 4096
    _, ptr, _ = torch.ops.dsse.ar_alloc(rows, H)
    try:
        peers = torch.tensor([ptr], dtype=torch.int64, device=gpu)
        epoch = torch.zeros(rows, dtype=torch.int32, device=gpu)
        err = torch.zeros(1, dtype=torch.int32, device=gpu)
        g = torch.Generator().manual_seed(M * 10 + S)
        slabs = torch.randn(S, M, H, generator=g).to(gpu)
        acc = torch.zeros(M, H, device=gpu)
        for s in range(S):  # the kernel's summation order
            acc += slabs[s]
        tmp = acc.bfloat16()
        resid = torch.randn(M, H, generator=g).to(gpu)
        w = (1 + 0.1 * torch.randn(H, generator=g)).bfloat16().to(gpu)
        r1, r2 = resid.clone(), resid.clone()
        y1 = torch.empty(M, H, device=gpu, dtype=torch.bfloat16)
        y2 = torch.empty_like(y1)
        torch.ops.dsse.ar_rmsnorm(tmp, r1, w, y1, 1e-5, peers, 0, rows, epoch, err)
        torch.ops.dsse.ar_rmsnorm(torch.zeros_like(tmp), r2, w, y2, 1e-5, peers, 0, rows, epoch, err,
                                  slabs.view(-1), S)
        torch.cuda.synchronize()
        assert int(err.item()) == 0
        assert torch.equal(r1, r2) and torch.equal(y1, y2)
        assert torch.allclose(r1, resid + tmp.float(), atol=0, rtol=0)
    finally:
        torch.cuda.synchronize()
        torch.ops.dsse.ar_close(int(ptr), False)
