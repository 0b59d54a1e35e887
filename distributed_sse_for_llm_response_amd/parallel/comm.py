"""Collectives for tensor-parallel decode: one process per GPU, RCCL over xGMI.

``torch.distributed`` with backend ``"nccl"`` is RCCL on ROCm.  Per decode step a TP group runs
exactly two bf16 all-reduces per layer (after the row-parallel O and down projections; SURVEY.md
§2.4 C1/C2) and one all-gather of per-rank sampling candidates (C3: 8 bytes per sequence instead of
the vocab-sized logits).  All of them are issued on torch's current stream, so they are captured
into the decode hipGraph together with the kernels.

The same code runs on CPU tensors with the ``gloo`` backend for the multi-process tests.

Decode collectives on GPUs go through ``IpcAllReduce`` when it is available: one hand-written kernel per
all-reduce (``csrc/kernels/allreduce.hip``) that exchanges the rows of the O / down partial products through
IPC-mapped peer buffers over xGMI and folds the residual add + RMSNorm in, and one for the candidate all-gather
(same buffers, flags and parity scheme).  With both, the TP decode step holds no RCCL call at all and is captured
into one hipGraph per bucket even where RCCL cannot be captured (ranks sharing a GPU over gloo).  It is set up once
per TP group (handles exchanged over the group, a self-test against ``dist.all_reduce`` / ``all_gather`` decided by
all ranks together) and RCCL stays the fallback (``DSSE_CUSTOM_AR=0`` forces it).
"""
from __future__ import annotations

import os
from dataclasses import dataclass

import torch
import torch.distributed as dist


@dataclass
class TPComm:
    """Tensor-parallel communicator (size 1 = no-op)."""

    rank: int = 0
    size: int = 1
    group: object = None

    def _host_staged(self, t: torch.Tensor) -> bool:
        # gloo with GPU tensors (several TP ranks sharing one GPU in a rehearsal, DSSE_DIST_BACKEND=gloo):
        # run the collective on a host copy; never taken on the RCCL path
        return t.is_cuda and dist.get_backend(self.group) == "gloo"

    def all_reduce(self, t: torch.Tensor) -> None:
        if self.size > 1:
            if self._host_staged(t):
                h = t.cpu()
                dist.all_reduce(h, group=self.group)
                t.copy_(h)
            else:
                dist.all_reduce(t, group=self.group)

    def all_gather_into(self, out: torch.Tensor, inp: torch.Tensor) -> None:
        """out: [size * numel(inp)] contiguous.  Sampling candidates ([rows, 16, 2] fp32) take the IPC gather
        kernel when the IPC context is up."""
        if self.size > 1 and self.fast_ar is not None and self.fast_ar.can_gather(inp, out):
            self.fast_ar.gather(inp, out)
            return
        if self.size > 1:
            if self._host_staged(out):
                h = torch.empty(out.numel(), dtype=out.dtype)
                dist.all_gather_into_tensor(h, inp.contiguous().view(-1).cpu(), group=self.group)
                out.view(-1).copy_(h)
                return
            # flat views: RCCL accepts stacked outputs, gloo only the dim-0 concatenation
            dist.all_gather_into_tensor(out.view(-1), inp.contiguous().view(-1), group=self.group)
        else:
            out.copy_(inp.view(-1)[: out.numel()].view_as(out))

    def reduce_scatter_rows(self, out: torch.Tensor, inp: torch.Tensor) -> None:
        """out = rows [rank * n, (rank + 1) * n) of the sum over ranks of inp ([size * n, ...] -> [n, ...]): the
        first half of a ring all-reduce, so the caller can normalise only its own rows (TP prefill)."""
        if self.size == 1:
            out.copy_(inp)
            return
        if self._host_staged(inp):
            h = torch.empty(out.shape, dtype=out.dtype)
            dist.reduce_scatter_tensor(h, inp.contiguous().cpu(), group=self.group)
            out.copy_(h)
            return
        dist.reduce_scatter_tensor(out, inp.contiguous(), group=self.group)

    def all_gather_rows(self, out: torch.Tensor, own: torch.Tensor) -> None:
        """out ([size * n, ...], contiguous) = every rank's `own` rows in rank order; `own` may be this rank's slice
        of `out` itself (in place)."""
        if self.size == 1:
            if own.data_ptr() != out.data_ptr():
                out.copy_(own)
            return
        if self._host_staged(out):
            h = torch.empty(out.shape, dtype=out.dtype)
            dist.all_gather_into_tensor(h, own.contiguous().cpu(), group=self.group)
            out.copy_(h)
            return
        dist.all_gather_into_tensor(out, own.contiguous(), group=self.group)

    def broadcast(self, t: torch.Tensor, src: int = 0) -> None:
        if self.size > 1:
            dist.broadcast(t, src=src, group=self.group)

    def barrier(self) -> None:
        if self.size > 1:
            dist.barrier(group=self.group)

    def close(self) -> None:
        """Tear down the IPC all-reduce context (IPC handles closed, buffer freed); RCCL stays usable."""
        if self.fast_ar is not None:
            self.fast_ar.close()
            self.fast_ar = None

    # ---- fused all-reduce + residual + RMSNorm (decode) ------------------------------------------------------
    fast_ar: object = None  # IpcAllReduce once enable_ipc_allreduce succeeded on every rank

    def enable_ipc_allreduce(self, device, rows: int, hidden: int) -> str:
        """Set up the IPC all-reduce for up to `rows` rows of width `hidden` (collective over the TP group).
        Returns "" when enabled, else the reason RCCL stays in use (identical on every rank)."""
        if self.size <= 1:
            return "tp=1"
        why = ""
        if os.environ.get("DSSE_CUSTOM_AR", "1") == "0":
            why = "DSSE_CUSTOM_AR=0"
        elif torch.device(device).type != "cuda":
            why = "not on a GPU"
        elif self.size > IpcAllReduce.MAX_RANKS:
            why = f"more than {IpcAllReduce.MAX_RANKS} ranks"
        # every rank takes the same branch: the reasons above depend only on the environment and the TP size
        if why:
            return why
        ar, why = IpcAllReduce.create(self, torch.device(device), rows, hidden)
        self.fast_ar = ar
        return why

    def all_reduce_rmsnorm(self, tmp, resid, norm_w, y, eps: float, part=None, nsplit: int = 0) -> None:
        """resid += all_reduce(tmp); y = rmsnorm(resid) * norm_w (the TP decode residual step).  part / nsplit: this
        rank's partial product is still `nsplit` fp32 split-K slabs (gemm_out_split), summed by the IPC kernel
        itself; only valid when the IPC context serves these rows (ipc_rows)."""
        from .. import ops

        if self.fast_ar is not None and tmp.shape[0] <= self.fast_ar.rows:
            self.fast_ar(tmp, resid, norm_w, y, eps, part, nsplit)
            return
        assert nsplit == 0, "split-K slabs need the IPC all-reduce"
        self.all_reduce(tmp)
        ops.rmsnorm(resid, norm_w, y, eps, delta=tmp)

    def ipc_rows(self, rows: int) -> bool:
        """The IPC all-reduce serves `rows` rows (so the O / down GEMM may leave its split-K slabs to it)."""
        return self.size > 1 and self.fast_ar is not None and rows <= self.fast_ar.rows


class IpcAllReduce:
    """Per-rank context of the fused IPC all-reduce (allreduce.hip ar_rmsnorm_kernel).

    Every rank allocates one buffer (flags + two parities of [rows, H] bf16), exports its IPC handle, and opens
    the handles of the other ranks of its TP group; ``peers`` holds the T buffer pointers as this process sees
    them.  ``epoch`` counts calls per row (the kernel's flag values) and must advance identically on every rank,
    which it does because every rank runs the same decode steps.  ``err`` is set by a timed-out peer wait."""

    MAX_RANKS = 8

    def __init__(self, comm, device, rows, hidden, own_ptr, peer_ptrs, uncached):
        self.comm, self.device, self.rows, self.hidden = comm, device, rows, hidden
        self.own_ptr, self.peer_ptrs, self.uncached = own_ptr, peer_ptrs, uncached
        self.peers = torch.tensor(peer_ptrs, dtype=torch.int64, device=device)
        self.epoch = torch.zeros(rows, dtype=torch.int32, device=device)
        self.gepoch = torch.zeros(rows, dtype=torch.int32, device=device)  # the candidate gather's own counters
        self.err = torch.zeros(1, dtype=torch.int32, device=device)

    @classmethod
    def create(cls, comm, device, rows: int, hidden: int):
        """(context or None, reason).  Collective: handle exchange + self-test + a MIN vote over the group."""
        from .. import ops

        ok, why, ctx = True, "", None
        try:
            ops.load_library(required=True)
            handle, ptr, uncached = torch.ops.dsse.ar_alloc(rows, hidden)
            payload = [bytes(handle.tolist())]
        except Exception as e:  # noqa: BLE001 - the vote below makes every rank fall back together
            ok, why, payload, ptr, uncached = False, f"alloc: {type(e).__name__}: {e}", [b""], 0, 0
        handles = [None] * comm.size
        dist.all_gather_object(handles, payload[0], group=comm.group)
        if ok and all(handles):
            try:
                ptrs = []
                for q, h in enumerate(handles):
                    if q == comm.rank:
                        ptrs.append(ptr)
                    else:
                        ptrs.append(int(torch.ops.dsse.ar_open(torch.tensor(list(h), dtype=torch.uint8))))
                ctx = cls(comm, device, rows, hidden, ptr, ptrs, bool(uncached))
            except Exception as e:  # noqa: BLE001
                ok, why = False, f"open: {type(e).__name__}: {e}"
        elif ok:
            ok, why = False, "a peer could not allocate its buffer"

        def vote(mine: bool) -> bool:
            flag = torch.tensor([1 if mine else 0], dtype=torch.int32, device=device)
            if dist.get_backend(comm.group) == "gloo":
                flag = flag.cpu()
            dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=comm.group)
            return int(flag.item()) == 1

        # every rank opened every peer before any rank starts the self-test's kernels and collectives
        if not vote(ok):
            if ctx is not None:
                ctx.close()
            return None, why or "another rank of the TP group could not open the IPC buffers"
        why = ctx.self_test()  # votes after every check: all ranks return from it at the same point
        ok = not why
        if not vote(ok):
            ctx.close()
            return None, why or "another rank of the TP group failed the IPC all-reduce self-test"
        return ctx, ""

    def close(self) -> None:
        """Unmap the peers' buffers and free this rank's (idempotent; the caller has synchronised the device, and
        no graph that captured this context may be replayed afterwards)."""
        if not self.peer_ptrs:
            return
        for q, ptr in enumerate(self.peer_ptrs):
            if q != self.comm.rank and ptr:
                torch.ops.dsse.ar_close(int(ptr), True)
        if self.own_ptr:
            torch.ops.dsse.ar_close(int(self.own_ptr), False)
        self.peer_ptrs, self.own_ptr = [], 0

    def __call__(self, tmp, resid, norm_w, y, eps: float, part=None, nsplit: int = 0) -> None:
        torch.ops.dsse.ar_rmsnorm(tmp, resid, norm_w, y, eps, self.peers, self.comm.rank, self.rows, self.epoch,
                                  self.err, part if nsplit > 0 else None, nsplit)

    GATHER_ROW_FLOATS = 32  # allreduce.hip kGatherRowBytes / 4: 16 vocab chunks x (score, index)

    def can_gather(self, inp, out) -> bool:
        return (inp.is_cuda and inp.dtype == torch.float32 and out.dtype == torch.float32 and inp.is_contiguous()
                and out.is_contiguous() and inp.dim() >= 1 and 0 < inp.shape[0] <= self.rows
                and inp.numel() == inp.shape[0] * self.GATHER_ROW_FLOATS
                and out.numel() == self.comm.size * inp.numel())

    def gather(self, inp, out) -> None:
        """out[q] = rank q's inp rows (rank-major, the layout of dist.all_gather_into_tensor)."""
        torch.ops.dsse.ar_gather(inp, out, self.peers, self.comm.rank, self.rows, self.hidden, self.gepoch, self.err)

    def self_test(self) -> str:
        """Fused all-reduce of random partials vs RCCL/gloo sum + reference norm, and the candidate gather vs
        all_gather, at a few row counts; ""=ok.  Every rank runs the same sequence of collectives whatever its own
        checks find: after each check the ranks vote (MIN of an ok flag) and all stop together at the first failure
        anywhere, so a rank that fails cannot leave its peers inside an IPC kernel or a collective it skipped."""
        from ..ops import reference as R

        gen = torch.Generator().manual_seed(1234 + self.comm.rank)
        H = self.hidden
        gloo = dist.get_backend(self.comm.group) == "gloo"

        def vote(why: str) -> bool:
            flag = torch.tensor([0 if why else 1], dtype=torch.int32, device="cpu" if gloo else self.device)
            dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=self.comm.group)
            return int(flag.item()) == 1

        for M in sorted({1, min(7, self.rows), self.rows}):
            for _ in range(3):  # both buffer parities, twice
                why = ""
                tmp = (torch.randn(M, H, generator=gen) * 0.5).bfloat16().to(self.device)
                resid0 = torch.randn(M, H, generator=torch.Generator().manual_seed(M)).to(self.device)
                w = (1 + 0.1 * torch.randn(H, generator=torch.Generator().manual_seed(7))).bfloat16().to(self.device)
                r = resid0.clone()
                y = torch.zeros(M, H, dtype=torch.bfloat16, device=self.device)
                self(tmp, r, w, y, 1e-5)
                ref = tmp.float().clone()
                self.comm.all_reduce(ref)
                r_ref = resid0.cpu() + ref.cpu()
                y_ref = torch.zeros(M, H, dtype=torch.bfloat16)
                R.rmsnorm(r_ref.clone(), w.cpu(), y_ref, 1e-5)
                torch.cuda.synchronize(self.device)
                if int(self.err.item()) != 0:
                    why = "self-test: a peer wait timed out"
                else:
                    err_r = float((r.cpu() - r_ref).abs().max())
                    err_y = float((y.cpu().float() - y_ref.float()).abs().max())
                    if err_r > 1e-3 or err_y > 5e-2:
                        why = f"self-test: M={M} max |resid err| {err_r:.3g}, |y err| {err_y:.3g}"
                if not vote(why):
                    return why or "self-test: another rank's all-reduce check failed"
                # the candidate gather: exact copies of every rank's rows, rank-major
                cand = torch.randn(M, 16, 2, generator=gen).to(self.device)
                got = torch.zeros(self.comm.size, M, 16, 2, device=self.device)
                self.gather(cand, got)
                if gloo:
                    ref_all = torch.zeros(self.comm.size * cand.numel())
                    dist.all_gather_into_tensor(ref_all, cand.cpu().view(-1), group=self.comm.group)
                else:
                    ref_dev = torch.zeros(self.comm.size * cand.numel(), device=self.device)
                    dist.all_gather_into_tensor(ref_dev, cand.view(-1), group=self.comm.group)
                    ref_all = ref_dev.cpu()
                torch.cuda.synchronize(self.device)
                if int(self.err.item()) != 0:
                    why = "self-test: a peer gather wait timed out"
                elif not torch.equal(got.cpu().view(-1), ref_all):
                    why = f"self-test: M={M} candidate gather differs from all_gather"
                if not vote(why):
                    return why or "self-test: another rank's gather check failed"
        return ""


def env_rank_info():
    """(rank, local_rank, world_size) from torchrun-style environment variables."""
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    return rank, local, world


def init_distributed(backend: str | None = None, device: torch.device | None = None):
    """Initialise the default process group from the environment if WORLD_SIZE > 1.

    Defaults MASTER_ADDR to 127.0.0.1 (the container hostname may not resolve).
    """
    rank, local, world = env_rank_info()
    if world <= 1 or dist.is_initialized():
        return rank, local, world
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29511")
    if backend is None:  # DSSE_DIST_BACKEND=gloo: several ranks sharing one GPU (RCCL rejects duplicate devices)
        backend = os.environ.get("DSSE_DIST_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
    kwargs = {}
    if backend == "nccl" and device is not None:
        kwargs["device_id"] = device
    dist.init_process_group(backend=backend, rank=rank, world_size=world, **kwargs)
    return rank, local, world


def make_groups(world: int, tp: int):
    """Split ranks into contiguous TP groups (DP replicas = world // tp). Returns (tp_group, dp_index)."""
    assert world % tp == 0, "world size must be a multiple of the TP degree"
    rank = dist.get_rank() if dist.is_initialized() else 0
    my_group = None
    for g in range(world // tp):
        ranks = list(range(g * tp, (g + 1) * tp))
        grp = dist.new_group(ranks) if (dist.is_initialized() and tp > 1) else None
        if rank in ranks:
            my_group = grp
    return my_group, rank // tp
