"""Collectives for tensor-parallel decode: one process per GPU, RCCL over xGMI.

``torch.distributed`` with backend ``"nccl"`` is RCCL on ROCm.  Per decode step a TP group runs
exactly two bf16 all-reduces per layer (after the row-parallel O and down projections; SURVEY.md
§2.4 C1/C2) and one all-gather of per-rank sampling candidates (C3: 8 bytes per sequence instead of
the vocab-sized logits).  All of them are issued on torch's current stream, so they are captured
into the decode hipGraph together with the kernels.

The same code runs on CPU tensors with the ``gloo`` backend for the multi-process tests.
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
        """out: [size * numel(inp)] contiguous."""
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

    def broadcast(self, t: torch.Tensor, src: int = 0) -> None:
        if self.size > 1:
            dist.broadcast(t, src=src, group=self.group)

    def barrier(self) -> None:
        if self.size > 1:
            dist.barrier(group=self.group)


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
