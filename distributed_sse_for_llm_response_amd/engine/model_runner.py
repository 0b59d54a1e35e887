"""Mistral forward passes on the engine's kernels: hipGraph-captured decode step + chunked prefill.

Decode step for a batch bucket of B slots (all device-resident, no host round trip):

    decode_prep          slots / ctx_len / q_len from positions + block tables
    embed+rmsnorm        resid = E[ids]; x = norm(resid)
    per layer:
      qkv GEMM           x·Wqkvᵀ as fp32 split-K slabs
      paged_attention    sums the slabs, RoPE, writes this token's K/V into the paged cache, then
                         flash-decoding over the pages (+ partition combine)
      gemm_resid         resid += attn·Woᵀ          (TP>1: gemm_out + one fused IPC all-reduce + add + norm kernel)
      rmsnorm            x = norm(resid)
      gemm_silu          h = silu(x·Wgᵀ)·(x·Wuᵀ)
      gemm_resid         resid += h·Wdᵀ             (TP>1: gemm_out + all-reduce + add)
      rmsnorm            x = norm(resid) with the next layer's (or the final) weight
    gemm_out (fp32)      logits = x·Wlmᵀ (vocab shard)

    sample               Gumbel-max / greedy; ids[b] <- token, ring[head][b] <- token, positions += 1
    ring_advance         head += 1

The sampled token becomes the next step's input in place, so consecutive steps need no host sync;
the host drains the token ring asynchronously (engine.py).  The whole step is captured once per
batch bucket into a torch.cuda.CUDAGraph (a hipGraph on ROCm).
"""
from __future__ import annotations

import contextlib
import gc
import math
import os
import time
from dataclasses import dataclass

import numpy as np
import torch

from .. import ops
from ..ops.reference import rope_table
from ..parallel.comm import TPComm
from .kv_cache import PAGE, KVCache
from .weights import EngineWeights

RING_SIZE = 64
SAMPLE_CHUNKS = 16  # vocab chunks per row in the candidate pass (B x 16 workgroups)
@contextlib.contextmanager
def _capture(graph, **kw):
    """torch.cuda.graph with the garbage collector off for the capture: a collection inside it could run a finaliser
    that destroys another object's graph or event (a HIP call that stream capture forbids: the process aborts)."""
    enabled = gc.isenabled()
    gc.collect()
    gc.disable()
    try:
        with torch.cuda.graph(graph, **kw):
            yield
    finally:
        if enabled:
            gc.enable()


PREFILL_TILE = 64   # query tokens per flash-prefill workgroup (attention_prefill.hip)
# Prefill batches of up to 2048 tokens replay a captured graph per row bucket (padded rows: slot -1, no K/V write,
# no attention work); larger batches (long prompts at an idle budget) run eagerly.  DSSE_PREFILL_GRAPHS=0 disables.
PREFILL_GRAPH_BUCKETS = (128, 256, 512, 1024, 2048)
PREFILL_GRAPH_SEQS = 16  # sequences per captured prefill batch (more: eager)
# Largest decode bucket on the fused-norm decode step (gemm_skinny / gemm_stream, split-K slabs reduced in the
# norms); larger buckets take the wide path (_decode_layers_wide), whose projections the kernel library routes to
# gemm_wide / gemm_tiled by row count (bindings.cpp gemm_impl).  Round 1 measured the split at 128 rows
# (profiles/bucket_ab_r1.md).
DECODE_GEMM_MAX_M = 128
# Health words (runner.health, int32 on the device, copied to the host with every drained step; nonzero = the step's
# outputs cannot be trusted and the engine fails: engine.py EngineFault).
HEALTH_TP_PEER = 0      # a TP peer's all-reduce row did not arrive in time (allreduce.hip)
HEALTH_WORDS = ("TP peer all-reduce wait timed out",)


# TP prefill: the row-independent post-attention half of each layer (O -> all-reduce -> norm -> gate_up -> down ->
# all-reduce -> norm) runs in row chunks so that each chunk's all-reduce (RCCL, a side stream) overlaps the next chunk's
# GEMMs (64 MiB all-reduces at 8k tokens, VERDICT r3 missing 1).  Chunked from
# DSSE_TP_PREFILL_OVERLAP_MIN rows, in DSSE_TP_PREFILL_CHUNKS chunks of whole 64-row tiles.
def flash_split_plan(tiles: list, hkv: int, min_blocks: int = 32, fill: int = 256, min_target: int = 16,
                     one_round: bool = True):
    """Key split of the flash prefill for an under-filled grid (round 6).  `tiles`: [(seq, tile, key blocks)]
    heaviest first.  With fewer than `fill` (tile, kv head) workgroups and a tile of >= `min_blocks` 64-key blocks (a
    TP = 8 rank has ONE kv head: an 8k prompt is 128 workgroups for 256 CUs, and the last tile walks 128 blocks
    alone), every tile longer than `target` blocks is cut into even key ranges: target = max(16, blocks x Hkv / fill),
    raised (one_round) until the ranges fit one round of `fill` workgroups.  Each range leaves partial O in its own
    slot and flash_combine_kernel merges a tile's slots.  Returns None (no split)
    or (work int32 [seq | tile | (kb0, kb1) pairs | slot], comb int32 [(seq, tile, first slot, slots)], slots), the
    work list heaviest range first."""
    if not tiles or len(tiles) * hkv >= fill or max(n for _, _, n in tiles) < min_blocks:
        return None
    # the smallest range length whose parts still fit one round of `fill` workgroups (one flash workgroup per CU):
    # a second round of leftover ranges would cost a whole range's time again
    nmax = max(n for _, _, n in tiles)
    target = max(min_target, -(-sum(n for _, _, n in tiles) * hkv // fill))
    if one_round:  # the smallest fitting length (the part count falls as the length grows): binary search
        ns = [n for _, _, n in tiles]
        lo, hi = target, max(target, nmax)
        while lo < hi:
            mid = (lo + hi) // 2
            if sum(-(-n // mid) for n in ns) * hkv > fill:
                lo = mid + 1
            else:
                hi = mid
        target = lo
    work, comb, nslots = [], [], 0
    for b, t, n in tiles:
        parts = -(-n // target)
        if parts == 1:
            work.append((n, b, t, 0, n, -1))
            continue
        per = -(-n // parts)
        comb.append((b, t, nslots, parts))
        for k in range(parts):
            work.append((min(n, (k + 1) * per) - k * per, b, t, k * per, min(n, (k + 1) * per), nslots + k))
        nslots += parts
    if not comb:
        return None
    work.sort(key=lambda x: -x[0])
    cols = list(zip(*work))
    kb = [v for a, e in zip(cols[3], cols[4]) for v in (a, e)]
    w = np.asarray(list(cols[1]) + list(cols[2]) + kb + list(cols[5]), dtype=np.int32)
    return w, np.asarray([v for c in comb for v in c], dtype=np.int32), nslots


def prefill_row_chunks(T: int, tp: int) -> list:
    """[(row0, row1)] of the overlapped TP prefill (one chunk when it does not apply)."""
    lo = int(os.environ.get("DSSE_TP_PREFILL_OVERLAP_MIN", "1024"))
    n = int(os.environ.get("DSSE_TP_PREFILL_CHUNKS", "4")) if tp > 1 and T >= lo else 1
    step = max(64, -(-T // max(1, n) // 64) * 64)
    return [(a, min(T, a + step)) for a in range(0, T, step)]


# prompt passes up to this many rows send the residual projections' split-K slabs to the norm (_prefill_resid)
PREFILL_SLAB_ROWS = 512


# Prompt-chunk sizes of the captured mixed steps: one graph per (decode bucket, C).  The engine sizes each step's
# chunk from the measured step costs (engine.PassCost.mixed_chunk); a prompt longer than the chunk is split evenly.
# B + C stays within MIXED_MAX_ROWS.  Round 5 set 512 because of a GEMM cliff at 576 rows; the round-6 cost-model
# dispatch removed that cliff (profiles/r6/gemm_model_r6.md), and 768 was re-measured with the serving bench at
# 40 req/s: TTFT p50 29.5 vs 29.8 ms, ITL p99 13.4 vs 10.7 ms (profiles/r6/serving_r6.md).  The bigger chunks buy no
# TTFT and cost ITL, so 512 stays.
MIXED_CHUNKS = (128, 256, 384, 512)
MIXED_MAX_ROWS = 512


def mixed_mode() -> str:
    """DSSE_MIXED: "1" (default) = prompt chunks ride in the decode step whenever streams decode (mixed prefill +
    decode steps, chunk sized per step from measured cost), "0" = separate prefill passes.  Separate passes keep
    TTFT lower but every pass is a whole extra weight stream between two decode tokens: ITL p99 ~3x the step
    (profiles/r4/serving_r4.md, profiles/r5/serving_r5.md)."""
    return os.environ.get("DSSE_MIXED", "1")


def batch_buckets(max_batch: int):
    """Captured decode batch sizes: powers of two up to 64, then every 64 (less padding at 65-256 streams)."""
    out, b = [], 1
    while b < max_batch:
        out.append(b)
        b = b * 2 if b < 64 else b + 64
    out.append(max_batch)
    return sorted(set(out))


def decode_partitioning(B: int, nkv: int, max_ctx: int, target_wgs: int = 512, max_parts: int = 32):
    """(part, nparts) for flash-decoding so that B·Hkv·nparts workgroups fill the chip.

    512 = two 256-thread workgroups per CU; at B·Hkv >= 512 (e.g. 64 streams x 8 KV heads) there is a
    single partition and the combine kernel is skipped.
    """
    want = max(1, min(max_parts, math.ceil(target_wgs / max(1, B * nkv))))
    part = max(128, math.ceil(max_ctx / want / 128) * 128)
    nparts = math.ceil(max_ctx / part)
    # several partitions: part 0 = each sequence's keys split evenly over them (attention.hip part_keys), so the
    # partitions stay busy at the served contexts, not only at max_ctx (TP = 8, 64 streams: 19 -> ~? us per layer,
    # profiles/r6/tp8_rank_decode_kernels_r6.md)
    return (0 if nparts > 1 else part), nparts


@dataclass
class PrefillSeq:
    slot: int               # decode slot the sequence occupies
    tokens: list            # token ids of this chunk
    start_pos: int          # absolute position of tokens[0]
    block_table: list       # the sequence's full block table
    last_chunk: bool        # sample a token after this chunk


class ModelRunner:
    def __init__(self, w: EngineWeights, num_blocks: int, max_batch: int = 64, max_model_len: int = 4096,
                 max_prefill_tokens: int = 8192, device="cuda", comm: TPComm | None = None, use_graphs=None):
        self.w, self.cfg = w, w.cfg
        self.device = torch.device(device)
        self.comm = comm or TPComm()
        self.max_batch = max_batch
        self.max_model_len = max_model_len
        self.max_blocks = math.ceil(max_model_len / PAGE) + 1
        self.max_prefill_tokens = max_prefill_tokens
        self.use_graphs = (self.device.type == "cuda") if use_graphs is None else use_graphs
        cfg, dev = self.cfg, self.device
        H = cfg.hidden_size
        nh, nkv, F, V = w.nh, w.nkv, w.ffn, w.vocab_local
        self.kv = KVCache(cfg.num_layers, num_blocks, nkv, dev)
        self.rope = rope_table(max(cfg.max_position, max_model_len + 1), cfg.rope_theta, dev)
        Bm = max_batch
        i32 = dict(device=dev, dtype=torch.int32)
        # ---- decode state (slot-indexed, device resident) ----
        self.ids = torch.zeros(Bm, **i32)
        self.positions = torch.zeros(Bm, **i32)
        # per-slot sampling state in ONE int32 buffer [active | temperature | top_k | top_p | seeds (Bm x 2)] (the
        # float fields are views of their words): the engine uploads a changed slot set with one pinned copy
        # (LLMEngine._upload)
        self.slot_meta = torch.zeros(6 * Bm, **i32)
        self.active = self.slot_meta[:Bm]
        self.block_tables = torch.zeros(Bm, self.max_blocks, **i32)
        self.slots = torch.full((Bm,), -1, **i32)
        self.ctx_len = torch.zeros(Bm, **i32)
        self.q_len = torch.zeros(Bm, **i32)
        self.q_start = torch.arange(Bm, **i32)
        self.work_seq = torch.arange(Bm, **i32)
        self.work_tile = torch.zeros(Bm, **i32)
        self.temperature = self.slot_meta[Bm:2 * Bm].view(torch.float32)
        self.top_k = self.slot_meta[2 * Bm:3 * Bm]
        self.top_p = self.slot_meta[3 * Bm:4 * Bm].view(torch.float32)
        self.top_p.fill_(1.0)
        self.seeds = self.slot_meta[4 * Bm:].view(Bm, 2)
        self.ring = torch.zeros(RING_SIZE, Bm, **i32)
        self.ring_counter = torch.zeros(1, **i32)
        # ---- decode activations ----
        bf = dict(device=dev, dtype=torch.bfloat16)
        self.resid = torch.zeros(Bm, H, device=dev, dtype=torch.float32)
        self.x = torch.zeros(Bm, H, **bf)
        self.q = torch.zeros(Bm, nh * 128, **bf)
        self.attn = torch.zeros(Bm, nh * 128, **bf)
        self.h = torch.zeros(Bm, F, **bf)
        self.tmp = torch.zeros(Bm, H, **bf)
        # fp32 split-K slabs of the residual projections (reduced inside the next RMSNorm)
        # (on a GPU also large enough for the 8 slabs of a PREFILL_SLAB_ROWS-row prompt pass: _prefill_resid)
        slab_floats = 32 * Bm * H
        if torch.device(dev).type == "cuda":
            slab_floats = max(slab_floats, 8 * min(PREFILL_SLAB_ROWS, max_prefill_tokens) * H)
        self.split_part = torch.zeros(slab_floats, device=dev, dtype=torch.float32)
        self.health = torch.zeros(4, device=dev, dtype=torch.int32)
        self.logits = torch.zeros(Bm, V, device=dev, dtype=torch.float32)
        nch = SAMPLE_CHUNKS if dev.type == "cuda" else 1
        self._cand = {b: torch.zeros(b, nch, 2, device=dev, dtype=torch.float32) for b in batch_buckets(Bm)}
        self._cand_all = {b: torch.zeros(self.comm.size, b, nch, 2, device=dev, dtype=torch.float32)
                          for b in batch_buckets(Bm)}
        part, nparts = decode_partitioning(1, nkv, max_model_len)
        ws = max(decode_partitioning(b, nkv, max_model_len)[1] * b for b in batch_buckets(Bm))
        self.part_o = torch.zeros(max(1, ws) * nkv * 16 * 128, device=dev, dtype=torch.float32)
        self.part_ml = torch.zeros(max(1, ws) * nkv * 16 * 2, device=dev, dtype=torch.float32)
        # TP decode: the residual all-reduces on the fused IPC kernel (parallel/comm.py IpcAllReduce), RCCL otherwise
        self.fast_ar_reason = self.comm.enable_ipc_allreduce(dev, Bm, H) if self.comm.size > 1 else "tp=1"
        if self.comm.fast_ar is not None:
            # a timed-out peer wait now marks this runner's health word (checked at every drained step)
            self.comm.fast_ar.err = self.health[HEALTH_TP_PEER:HEALTH_TP_PEER + 1]
        if self.comm.size > 1 and self.comm.rank == 0:
            print(f"[engine] TP={self.comm.size} decode all-reduce + candidate all-gather: "
                  f"{'IPC kernels' if not self.fast_ar_reason else 'RCCL (' + self.fast_ar_reason + ')'}", flush=True)
        self.graphs = {}
        self.graph_pool = None
        self.pf_graphs = {}   # row bucket -> captured prefill graph
        self.pf = None        # static prefill buffers (allocated by capture)
        self.mx_graphs = {}   # decode bucket B -> [(chunk rows C, captured mixed prefill + decode graph)], C ascending
        self.host_trace = None  # a list: host seconds of each graph-replayed mixed step (upload, replay, sampling)

    # ------------------------------------------------------------------ decode
    def decode_forward(self, B: int) -> None:
        """One decode step over slots [0, B) (graph-capturable: fixed shapes, no host sync)."""
        w, cfg, comm = self.w, self.cfg, self.comm
        nh, nkv = w.nh, w.nkv
        r = slice(0, B)
        eps = cfg.rms_eps
        ops.decode_prep(self.active[r], self.positions[r], self.block_tables[r], self.slots[r], self.ctx_len[r],
                        self.q_len[r], self.kv.num_blocks)
        resid, x = self.resid[r], self.x[r]
        ops.rmsnorm(resid, w.layers[0].attn_norm, x, eps, embed=w.embed, ids=self.ids[r])
        part, nparts = decode_partitioning(B, nkv, self.max_model_len)
        nl = len(w.layers)
        if B > DECODE_GEMM_MAX_M:
            self._decode_layers_wide(B, resid, x, part, nparts)
            return
        for li, L in enumerate(w.layers):
            self._qkv_attention(li, L, B, x, part, nparts)
            self._resid_proj(self.attn[r], L.wo_t, resid, L.ffn_norm, x, self.tmp[r])
            ops.gemm_silu(x, L.wgu_t, self.h[r])
            w_next = w.layers[li + 1].attn_norm if li + 1 < nl else w.final_norm
            self._resid_proj(self.h[r], L.wd_t, resid, w_next, x, self.tmp[r])
        ops.gemm_out(x, w.lm_head_t, self.logits[r])
        self._sample_commit(B)
        ops.ring_advance(self.ring_counter)

    def _decode_layers_wide(self, B: int, resid, x, part: int, nparts: int) -> None:
        """Decode step for buckets above DECODE_GEMM_MAX_M sequences (256 streams per GPU, BASELINE config 3).

        At B > 128 a weight byte feeds > 128 rows and the projections become compute-heavy skinny GEMMs; they run
        on the engine's tiled-layout GEMMs with fused epilogues (QKV + RoPE + KV write, residual + split-K norm,
        SiLU·mul) -- gemm_wide or the register-blocked gemm_tiled, chosen per shape by the kernel library.  The
        LM head stays on the fp32-output GEMM in 256-row blocks (sampling wants fp32 logits).  One captured graph
        per bucket.
        """
        w, cfg, comm = self.w, self.cfg, self.comm
        nh, nkv = w.nh, w.nkv
        r = slice(0, B)
        eps = cfg.rms_eps
        nl = len(w.layers)
        for li, L in enumerate(w.layers):
            self._qkv_attention(li, L, B, x, part, nparts)
            self._resid_proj(self.attn[r], L.wo_t, resid, L.ffn_norm, x, self.tmp[r])
            self._gate_up(x, L, self.h[r])
            w_next = w.layers[li + 1].attn_norm if li + 1 < nl else w.final_norm
            self._resid_proj(self.h[r], L.wd_t, resid, w_next, x, self.tmp[r])
        step = 256 if DECODE_GEMM_MAX_M > 2 else DECODE_GEMM_MAX_M  # one 256-row call streams the head once
        for b0 in range(0, B, step):
            b1 = min(B, b0 + step)
            ops.gemm_out(x[b0:b1], w.lm_head_t, self.logits[b0:b1])
        self._sample_commit(B)
        ops.ring_advance(self.ring_counter)

    def _qkv_attention(self, li: int, L, B: int, x, part: int, nparts: int) -> None:
        """QKV projection + RoPE + KV write + decode attention of layer li.  The projection's split-K slabs go
        to split_part (free here: the previous norm consumed it) and the attention kernel folds their reduction,
        RoPE and the K/V write in (ops.qkv_attention_decode)."""
        r = slice(0, B)
        nh, nkv = self.w.nh, self.w.nkv
        ops.qkv_attention_decode(x, L.wqkv_t, self.positions[r], self.slots[r], self.rope, self.q[r], self.kv.k[li],
                                 self.kv.v[li], nh, nkv, self.split_part, self.block_tables[r], self.q_start[r],
                                 self.q_len[r], self.ctx_len[r], self.work_seq[r], self.work_tile[r], self.attn[r],
                                 self.part_o, self.part_ml, part, nparts)

    def _resid_proj(self, a, wt, resid, norm_w, x, tmp) -> None:
        """resid += a·wᵀ (TP: all-reduced), then x = RMSNorm(resid)·norm_w.  TP = 1: split-K slabs (if the GEMM
        splits) are reduced inside the norm; TP > 1: the bf16 partial product is all-reduced first."""
        eps = self.cfg.rms_eps
        if self.comm.size == 1:
            ns = ops.gemm_resid_split(a, wt, resid, self.split_part)
            ops.rmsnorm(resid, norm_w, x, eps, part=self.split_part, nsplit=ns)
        elif self.comm.ipc_rows(a.shape[0]) and a.is_cuda:
            # the IPC all-reduce kernel sums the GEMM's split-K slabs itself (no splitk_reduce launch)
            ns = ops.gemm_out_split(a, wt, tmp, self.split_part)
            self.comm.all_reduce_rmsnorm(tmp, resid, norm_w, x, eps, part=self.split_part, nsplit=ns)
        else:
            ops.gemm_out(a, wt, tmp)
            self.comm.all_reduce_rmsnorm(tmp, resid, norm_w, x, eps)

    def _sample_commit(self, B: int) -> None:
        """Candidates per (row, vocab chunk) on each rank -> (TP: all-gather, 8 B per candidate) -> pick."""
        r = slice(0, B)
        cand = self._cand[B]
        ops.sample_candidates(self.logits[r], self.temperature[r], self.top_k[r], self.top_p[r], self.seeds[r],
                              self.positions[r], self.active[r], cand, self.w.vocab_offset)
        if self.comm.size == 1:
            cand_all = cand.unsqueeze(0)
        else:
            cand_all = self._cand_all[B]
            self.comm.all_gather_into(cand_all, cand)
        ops.sample_pick(cand_all, self.active[r], self.ids[r], self.ring, self.ring_counter, self.positions[r],
                        vocab=self.cfg.vocab_size)

    def health_faults(self, words) -> list:
        """Descriptions of the nonzero health words in `words` (a host copy of self.health)."""
        return [HEALTH_WORDS[i] for i in range(min(len(HEALTH_WORDS), len(words))) if int(words[i]) != 0]

    def close(self) -> None:
        """Release the TP all-reduce's IPC mappings and buffer.  Collective over the TP group: the device is
        synchronised, then every rank passes a barrier, so no peer's kernel can still be reading this rank's buffer
        (the IPC kernels pull peer rows) when it is unmapped and freed."""
        if self.comm.fast_ar is not None:
            if self.device.type == "cuda":
                torch.cuda.synchronize(self.device)
            try:
                self.comm.barrier()
            except Exception as e:  # noqa: BLE001 - a dead peer cannot be reading any more either
                print(f"[engine] TP rank {self.comm.rank}: barrier before the IPC teardown failed ({e})", flush=True)
            self.comm.fast_ar.close()
            self.comm.fast_ar = None

    def bucket_for(self, n_active_max_slot: int) -> int:
        for b in batch_buckets(self.max_batch):
            if b >= n_active_max_slot:
                return b
        return self.max_batch

    def _collectives_capturable(self) -> tuple:
        """TP>1 startup self-check: an all-reduce captured into a graph and replayed must produce the sum on
        every rank.  Decided by all ranks together (an eager MIN of the local verdicts), so either every rank
        captures its decode step or every rank runs it eagerly -- the collectives stay matched."""
        import torch.distributed as dist

        ok, why = True, ""
        if dist.get_backend(self.comm.group) == "gloo":
            ok, why = False, "gloo backend (host-staged collectives cannot be captured)"
        try:
            if not ok:
                raise StopIteration
            t = torch.ones(8, device=self.device, dtype=torch.float32)
            s = torch.cuda.Stream(self.device)
            s.wait_stream(torch.cuda.current_stream(self.device))
            with torch.cuda.stream(s):
                self.comm.all_reduce(t)  # warm the communicator outside capture
            torch.cuda.current_stream(self.device).wait_stream(s)
            torch.cuda.synchronize(self.device)
            g = torch.cuda.CUDAGraph()
            with _capture(g):
                self.comm.all_reduce(t)
            t.fill_(1.0)
            g.replay()
            torch.cuda.synchronize(self.device)
            if not torch.all(t == float(self.comm.size)):
                ok, why = False, f"replayed all-reduce gave {t.tolist()}"
        except StopIteration:
            pass
        except Exception as e:  # noqa: BLE001 - the reason is logged, decode then runs eagerly
            ok, why = False, f"{type(e).__name__}: {e}"
        flag = torch.tensor([1 if ok else 0], dtype=torch.int32, device=self.device)
        if dist.get_backend(self.comm.group) == "gloo":
            flag = flag.cpu()
        dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=self.comm.group)
        if ok and int(flag.item()) == 0:
            why = "another rank of the TP group cannot capture its collectives"
        return int(flag.item()) == 1, why

    def ipc_decode(self) -> bool:
        """TP > 1 with the IPC context up for every decode row: the decode step's collectives are the hand-written
        IPC all-reduce (both per layer) and candidate all-gather kernels only -- no RCCL call in the step."""
        ar = self.comm.fast_ar
        return self.comm.size > 1 and ar is not None and ar.rows >= self.max_batch

    def capture(self, buckets=None) -> None:
        """Capture the decode step of each batch bucket into its own graph (shared memory pool).  TP > 1: the decode
        graphs hold the IPC collective kernels when that context is up (ipc_decode), else the RCCL collectives after
        a capture self-check; the prefill / mixed graphs (their all-reduces are RCCL) only when RCCL captures.
        Neither: eager decode (reason logged)."""
        if not self.use_graphs:
            return
        prefill_graphs = True
        if self.comm.size > 1:
            ipc = self.ipc_decode()
            rccl_ok, why = self._collectives_capturable()
            if not ipc and not rccl_ok:
                print(f"[engine] TP rank {self.comm.rank}: decode graphs disabled, collectives not capturable "
                      f"({why}); decoding eagerly", flush=True)
                self.use_graphs = False
                return
            prefill_graphs = rccl_ok
            if self.comm.rank == 0:
                print(f"[engine] TP={self.comm.size} decode graphs captured with "
                      f"{'the IPC all-reduce + all-gather kernels (no RCCL in the step)' if ipc else 'RCCL collectives'}"
                      f"; prefill graphs {'captured' if rccl_ok else 'off (' + why + ')'}", flush=True)
        buckets = buckets or batch_buckets(self.max_batch)
        # Warm up on a side stream (allocator + library init) before capture.
        s = torch.cuda.Stream(self.device)
        s.wait_stream(torch.cuda.current_stream(self.device))
        saved = self._snapshot_state()
        with torch.cuda.stream(s):
            for B in buckets:
                self.decode_forward(B)
        torch.cuda.current_stream(self.device).wait_stream(s)
        torch.cuda.synchronize(self.device)
        for B in sorted(buckets, reverse=True):
            g = torch.cuda.CUDAGraph()
            with _capture(g, pool=self.graph_pool):
                self.decode_forward(B)
            if self.graph_pool is None:
                self.graph_pool = g.pool()
            self.graphs[B] = g
        torch.cuda.synchronize(self.device)
        self._restore_state(saved)
        if prefill_graphs:
            self._capture_prefill(buckets)

    def _capture_prefill(self, decode_buckets) -> None:
        """One graph per prefill row bucket over static buffers (_PrefillStatic); the metadata of a batch is
        uploaded into them before the replay.  Captured with all-padding metadata (every row slot -1: no K/V
        write; every work item on the empty sequence)."""
        if os.environ.get("DSSE_PREFILL_GRAPHS", "1") == "0":
            return
        buckets = [t for t in PREFILL_GRAPH_BUCKETS if t <= self.max_prefill_tokens]
        if not buckets:
            return
        self.pf = _PrefillStatic(self, max(buckets))
        self.pf.upload_padding()
        s = torch.cuda.Stream(self.device)
        s.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(s):
            for tb in buckets:
                self._prefill_layers(tb, self.pf.views(tb))
                self._graph_sample()  # padding metadata: no prompt finishes, nothing is committed
        torch.cuda.current_stream(self.device).wait_stream(s)
        torch.cuda.synchronize(self.device)
        for tb in sorted(buckets, reverse=True):
            g = torch.cuda.CUDAGraph()
            with _capture(g, pool=self.graph_pool):
                self._prefill_layers(tb, self.pf.views(tb))
                self._graph_sample()
            if self.graph_pool is None:
                self.graph_pool = g.pool()
            self.pf_graphs[tb] = g
        torch.cuda.synchronize(self.device)
        if mixed_mode() != "0" and os.environ.get("DSSE_MIXED_GRAPHS", "1") != "0":
            self._capture_mixed(list(decode_buckets))

    def mixed_chunk(self, B: int) -> int:
        """The prompt rows of a mixed step before its cost is measured: DSSE_MIXED_CHUNK when set (then the only
        captured chunk size), else 256; whole 64-row flash-prefill tiles."""
        fixed = int(os.environ.get("DSSE_MIXED_CHUNK", "0"))
        return -(-fixed // PREFILL_TILE) * PREFILL_TILE if fixed > 0 else 256

    def mixed_chunks(self, B: int) -> list:
        """The chunk sizes C captured for decode bucket B (B + C rows fit the static prefill buffers)."""
        fixed = int(os.environ.get("DSSE_MIXED_CHUNK", "0"))
        tmax = self.pf.tmax if self.pf is not None else 0
        if fixed > 0:
            return [c for c in [self.mixed_chunk(B)] if B + c <= tmax]
        top = (MIXED_MAX_ROWS - B) // PREFILL_TILE * PREFILL_TILE
        sizes = sorted({c for c in MIXED_CHUNKS if c <= top} | ({top} if top >= MIXED_CHUNKS[0] else set()))
        return [c for c in sizes if B + c <= tmax]

    def _capture_mixed(self, decode_buckets) -> None:
        """One graph per (decode bucket B, chunk size C in mixed_chunks(B)) for the mixed step (ModelRunner.mixed;
        captured like the decode step: the decode state restored afterwards).  mx_graphs[B] = [(C, graph), ...]
        by ascending C."""
        pairs = [(B, C) for B in decode_buckets for C in self.mixed_chunks(B)]
        if not pairs:
            return
        saved = self._snapshot_state()
        self.pf.upload_padding()
        s = torch.cuda.Stream(self.device)
        s.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(s):
            for B, C in pairs:  # eager warm-up of every shape (kernel attributes, library state)
                self._mixed_layers(B, C)
                self._graph_sample()
        torch.cuda.current_stream(self.device).wait_stream(s)
        torch.cuda.synchronize(self.device)
        for B, C in sorted(pairs, reverse=True):
            g = torch.cuda.CUDAGraph()
            with _capture(g, pool=self.graph_pool):
                self._mixed_layers(B, C)
                self._graph_sample()
            self.mx_graphs.setdefault(B, []).insert(0, (C, g))
        torch.cuda.synchronize(self.device)
        self._restore_state(saved)

    def mixed_graph_rows(self, B: int, T: int):
        """C of the captured mixed graph that a step of bucket B with T prompt rows replays (the smallest C >= T),
        or None (the step runs eagerly)."""
        return next((c for c, _ in self.mx_graphs.get(B, ()) if c >= T), None)

    def _snapshot_state(self):
        return [t.clone() for t in (self.ids, self.positions, self.ring, self.ring_counter)]

    def _restore_state(self, saved):
        for t, s in zip((self.ids, self.positions, self.ring, self.ring_counter), saved):
            t.copy_(s)

    def move_slots(self, src: list, dst: list) -> None:
        """Slot compaction: decode state (last token, position) of slot src[i] -> dst[i], gathered before it
        is scattered so swaps work; stream-ordered after every decode step already enqueued."""
        idx = torch.tensor([src, dst], dtype=torch.long)
        if self.device.type == "cuda":  # pinned + non_blocking: no host wait for the decode steps already queued
            idx = idx.pin_memory().to(self.device, non_blocking=True)
        si, di = idx[0], idx[1]
        for t in (self.ids, self.positions):
            t.index_copy_(0, di, t.index_select(0, si))

    def decode(self, B: int) -> None:
        g = self.graphs.get(B)
        if g is not None:
            g.replay()
        else:
            self.decode_forward(B)

    # ------------------------------------------------------------------ prefill
    def _proj(self, a, wt, out) -> None:
        """out = a·wᵀ in bf16 on the engine's tiled-layout GEMMs (every row count: no library GEMM)."""
        ops.gemm_out(a, wt, out)

    def _gate_up(self, x, L, h) -> None:
        """h = SiLU(x·W_gateᵀ)·(x·W_upᵀ) with the fused SiLU·mul epilogue (gate / up rows interleaved by 8)."""
        ops.gemm_silu(x, L.wgu_t, h)

    def _seq_sharded_norm(self, tmp, resid, norm_w, x) -> None:
        """TP prefill residual step in its sequence-sharded form: reduce-scatter the partial products over the rows
        (rank r gets the summed rows [r n, (r + 1) n)), add + RMSNorm those n = T / t rows only, all-gather the normed
        bf16 rows.  Same bytes on the wire as the all-reduce it replaces (a ring all-reduce IS reduce-scatter +
        all-gather), 1 / t of the norm work, and each rank's residual stream is authoritative for its own rows only
        (the next residual step adds into the same rows; nothing else reads resid)."""
        t, r = self.comm.size, self.comm.rank
        n = tmp.shape[0] // t
        own = slice(r * n, (r + 1) * n)
        # one reduce-scatter target per shape, reused: every use of it is ordered on one stream (the side stream in
        # the chunked path, the current one otherwise, and the two paths are ordered against each other by the
        # chunked path's events); no allocation on the host's per-chunk path
        key = (n, tmp.shape[1], tmp.dtype, tmp.device)
        cache = self.__dict__.setdefault("_rs_bufs", {})
        summed = cache.get(key)
        if summed is None:
            summed = cache[key] = torch.empty(n, tmp.shape[1], device=tmp.device, dtype=tmp.dtype)
        self.comm.reduce_scatter_rows(summed, tmp)
        ops.rmsnorm(resid[own], norm_w, x[own], self.cfg.rms_eps, delta=summed)
        self.comm.all_gather_rows(x, x[own])

    def _resid_async(self, tmp, resid, norm_w, x):
        """Residual step of one row chunk on the communication side stream, ordered after everything queued on the
        current stream: the sequence-sharded reduce-scatter -> add + RMSNorm of this rank's rows -> all-gather when
        the chunk's rows divide by the TP degree, else all-reduce -> replicated norm.  Returns the event the consumer
        of x waits for (None: done synchronously, CPU / gloo)."""
        sharded = tmp.shape[0] % self.comm.size == 0
        if not tmp.is_cuda:
            if sharded:
                self._seq_sharded_norm(tmp, resid, norm_w, x)
            else:
                self.comm.all_reduce(tmp)
                ops.rmsnorm(resid, norm_w, x, self.cfg.rms_eps, delta=tmp)
            return None
        main = torch.cuda.current_stream(self.device)
        if getattr(self, "_side", None) is None:
            self._side = torch.cuda.Stream(self.device)
            # a ring of event pairs, reused: every wait on an event is enqueued before the event is recorded again
            # (the ring outlasts a layer's 2 x chunks residual steps)
            self._side_evs = [(torch.cuda.Event(), torch.cuda.Event()) for _ in range(32)]
            self._side_ev_i = 0
        ready, done = self._side_evs[self._side_ev_i]
        self._side_ev_i = (self._side_ev_i + 1) % len(self._side_evs)
        ready.record(main)
        self._side.wait_event(ready)
        with torch.cuda.stream(self._side):
            if sharded:
                self._seq_sharded_norm(tmp, resid, norm_w, x)
            else:
                self.comm.all_reduce(tmp)
                ops.rmsnorm(resid, norm_w, x, self.cfg.rms_eps, delta=tmp)
        done.record(self._side)
        return done

    def _prefill_post_attention(self, T: int, attn, L, w_next, resid, x, h, tmp) -> None:
        """resid += all_reduce(attn·Woᵀ); x = norm(resid); resid += all_reduce(silu-mlp(x)); x = norm(resid)·w_next.

        TP: whenever the rows divide by the TP degree, each all-reduce + replicated norm is the sequence-sharded
        reduce-scatter -> norm on T / t rows -> all-gather (_seq_sharded_norm; VERDICT r5 missing 3): the same bytes
        on the wire as the all-reduce (a ring all-reduce is reduce-scatter + all-gather), 1 / t of the norm work.

        TP prefill of >= DSSE_TP_PREFILL_OVERLAP_MIN rows: these ops are row-independent, so they run in row chunks and
        every chunk's residual step (collectives + its 1 / t of the norm) is issued on a side stream the moment its
        GEMM is done -- the O steps of chunk i under the O GEMM of chunk i + 1 and the MLP of chunk i - 1, the down
        steps under the next chunks' MLP; only the last chunk's second step is exposed (1 / 2n of the layer's
        communication, n chunks).  Each rank's residual rows are then updated on the side stream only (nothing on the
        main stream reads resid).  Every rank issues the collectives in the same order.  TP = 1 or short prompts: the
        unchunked chain."""
        chunks = prefill_row_chunks(T, self.comm.size)
        if len(chunks) == 1:
            self._prefill_resid(attn, L.wo_t, resid, L.ffn_norm, x, tmp)
            self._gate_up(x, L, h)
            self._prefill_resid(h, L.wd_t, resid, w_next, x, tmp)
            return
        main = torch.cuda.current_stream(self.device) if tmp.is_cuda else None
        ev1 = []
        for a, b in chunks:
            self._proj(attn[a:b], L.wo_t, tmp[a:b])
            ev1.append(self._resid_async(tmp[a:b], resid[a:b], L.ffn_norm, x[a:b]))
        ev2 = []
        for (a, b), ev in zip(chunks, ev1):
            if ev is not None:
                main.wait_event(ev)
            self._gate_up(x[a:b], L, h[a:b])
            self._proj(h[a:b], L.wd_t, tmp[a:b])  # tmp rows [a, b) are free: their O step was waited for
            ev2.append(self._resid_async(tmp[a:b], resid[a:b], w_next, x[a:b]))
        for ev in ev2:
            if ev is not None:
                main.wait_event(ev)

    def _prefill_resid(self, a, wt, resid, norm_w, x, tmp) -> None:
        """resid += a·wᵀ, x = RMSNorm(resid).  Thousands of rows: the product goes out as a bf16 tile (row-contiguous
        stores) and the norm kernel adds it -- the fused fp32 read-modify-write epilogue measured +120 us per
        8192-row projection (profiles/r2/prefill_kernels_8k.md).  Up to PREFILL_SLAB_ROWS rows on the tiled kernels
        (split K) the norm reduces the fp32 split-K slabs itself, as in decode: no reduce launch, no bf16 round trip."""
        rows = a.shape[0]
        if self.comm.size == 1 and rows <= PREFILL_SLAB_ROWS and self.split_part.numel() >= 8 * rows * wt.shape[0]:
            ns = ops.gemm_resid_split(a, wt, resid, self.split_part)
            ops.rmsnorm(resid, norm_w, x, self.cfg.rms_eps, part=self.split_part, nsplit=ns)
            return
        self._proj(a, wt, tmp)
        if self.comm.size > 1 and rows % self.comm.size == 0:
            self._seq_sharded_norm(tmp, resid, norm_w, x)
            return
        self.comm.all_reduce(tmp)
        ops.rmsnorm(resid, norm_w, x, self.cfg.rms_eps, delta=tmp)

    def _prefill_meta(self, seqs: list, row0: int = 0, split: bool = False):
        """Packed metadata of prefill chunks whose rows start at `row0` of the activations (0 for a prefill-only
        batch, B for the prefill rows of a mixed step): host lists + device tensors (one pinned upload).  split: add
        the flash key-split plan when the grid is under-filled (flash_split_plan: d["fw"], d["fc"], d["fslots"])."""
        dev = self.device
        n = len(seqs)
        # vectorised per sequence (an 8k-token chunk was ~25k Python list appends on the TTFT path)
        ids_l, pos_l, slots_l = [], [], []
        q_start, q_len, ctx_len, items = [], [], [], []
        bt = torch.zeros(n, self.max_blocks, dtype=torch.int32)
        row = 0
        for i, s in enumerate(seqs):
            m = len(s.tokens)
            q_start.append(row0 + row)
            p = s.start_pos + np.arange(m, dtype=np.int64)
            table = np.asarray(s.block_table, dtype=np.int64)
            ids_l.append(np.asarray(s.tokens, dtype=np.int64))
            pos_l.append(p)
            slots_l.append(table[p // PAGE] * PAGE + p % PAGE)
            q_len.append(m)
            ctx_len.append(s.start_pos + m)
            bt[i, : len(s.block_table)] = torch.from_numpy(table.astype(np.int32))
            # flash prefill: heaviest (most keys) 64-query tiles first, so the causal tail balances over the CUs
            items += [(-(s.start_pos + min(m, (t + 1) * PREFILL_TILE)), i, t) for t in range(math.ceil(m / PREFILL_TILE))]
            row += m
        items.sort()
        work_seq = [i for _, i, _ in items]
        work_tile = [t for _, _, t in items]
        T = row
        plan = None
        if split:
            plan = flash_split_plan([(i, t, -(-(-k) // PREFILL_TILE)) for k, i, t in items], self.w.nkv)
        fw, fc = (plan[0], plan[1]) if plan else (np.zeros(0, np.int32), np.zeros(0, np.int32))
        empty = np.zeros(0, dtype=np.int64)
        meta = torch.from_numpy(np.concatenate(
            [np.concatenate(ids_l) if ids_l else empty, np.concatenate(pos_l) if pos_l else empty,
             np.concatenate(slots_l) if slots_l else empty,
             np.asarray(q_start + q_len + ctx_len + work_seq + work_tile, dtype=np.int64),
             fw.astype(np.int64), fc.astype(np.int64)]).astype(np.int32))
        if dev.type == "cuda":
            meta = meta.pin_memory().to(dev, non_blocking=True)
            bt = bt.pin_memory().to(dev, non_blocking=True)
        d, o = {}, 0
        for name, k in (("ids", T), ("pos", T), ("slots", T), ("qs", n), ("ql", n), ("ctx", n),
                        ("ws", len(work_seq)), ("wt", len(work_seq)), ("fw", len(fw)), ("fc", len(fc))):
            d[name], o = meta[o:o + k], o + k
        d["bt"] = bt
        d["fslots"] = plan[2] if plan else 0
        return T, q_start, q_len, ctx_len, d

    def _prefill_sample(self, seqs: list, x, q_start: list, q_len: list, ring_row: int) -> None:
        """Sequences whose last chunk this is sample their first token (rows q_start + q_len - 1 of `x`) into
        ids[slot] and ring[ring_row, slot]; positions[slot] is set on the device."""
        w, cfg, comm, dev = self.w, self.cfg, self.comm, self.device
        last = [i for i, s in enumerate(seqs) if s.last_chunk]
        if not last:
            return
        f32 = dict(device=dev, dtype=torch.float32)
        nL = len(last)
        # one pinned, non-blocking upload of the three index vectors: a pageable torch.tensor(..., device=dev) is a
        # synchronous copy that waits for every step already queued (the prefill graph and the pipelined decode
        # steps) -- 27-30 ms of host stall per prompt at ~120 streams (profiles/r3/serving_trace.md)
        idx = torch.tensor([q_start[i] + q_len[i] - 1 for i in last] + [seqs[i].slot for i in last] +
                           [seqs[i].start_pos + len(seqs[i].tokens) - 1 for i in last], dtype=torch.long)
        if dev.type == "cuda":
            idx = idx.pin_memory().to(dev, non_blocking=True)
        rows, slot_idx, last_pos = idx[:nL], idx[nL:2 * nL], idx[2 * nL:].to(torch.int32)
        xl = x.index_select(0, rows)
        logits = torch.empty(nL, w.vocab_local, **f32)
        ops.gemm_out(xl, w.lm_head_t, logits)
        new_ids = torch.zeros(nL, dtype=torch.int32, device=dev)
        temp = self.temperature.index_select(0, slot_idx)
        tk = self.top_k.index_select(0, slot_idx)
        tp = self.top_p.index_select(0, slot_idx)
        sd = self.seeds.index_select(0, slot_idx).contiguous()
        nch = SAMPLE_CHUNKS if dev.type == "cuda" else 1
        cand = torch.zeros(nL, nch, 2, **f32)
        ops.sample_candidates(logits, temp, tk, tp, sd, last_pos, None, cand, w.vocab_offset)
        if comm.size == 1:
            cand_all = cand.unsqueeze(0)
        else:
            cand_all = torch.zeros(comm.size, nL, nch, 2, **f32)
            comm.all_gather_into(cand_all, cand)
        ops.sample_pick(cand_all, None, new_ids, vocab=cfg.vocab_size)
        self.ids.index_copy_(0, slot_idx, new_ids)
        self.ring[ring_row].index_copy_(0, slot_idx, new_ids)
        self.positions.index_copy_(0, slot_idx, last_pos + 1)

    def prefill(self, seqs: list, ring_row: int) -> None:
        """Run one packed prefill batch: a captured graph of the smallest row bucket that holds it (metadata
        uploaded into the static buffers first), else eagerly.  Sequences whose last chunk this is sample their
        first token into ids[slot] and ring[ring_row, slot] and get positions[slot] set on device."""
        if not seqs:
            return
        T = sum(len(s.tokens) for s in seqs)
        tb = next((t for t in sorted(self.pf_graphs) if t >= T), None) if len(seqs) <= PREFILL_GRAPH_SEQS else None
        if tb is not None:
            self.pf.upload(seqs, tb, ring_row=ring_row)
            self.pf_graphs[tb].replay()  # first tokens sampled inside the graph (_graph_sample)
            return
        w, dev = self.w, self.device
        nh, nkv, F, H = w.nh, w.nkv, w.ffn, self.cfg.hidden_size
        T, q_start, q_len, ctx_len, d = self._prefill_meta(seqs, split=True)
        f32 = dict(device=dev, dtype=torch.float32)
        bf = dict(device=dev, dtype=torch.bfloat16)
        if d["fslots"]:  # partial slots of the flash key split: [slots][Hkv][G][64 queries] x (128 dims | (m, l))
            d.update(fpo=torch.empty(d["fslots"] * nh * PREFILL_TILE * 128, **f32),
                     fpm=torch.empty(d["fslots"] * nh * PREFILL_TILE * 2, **f32))
        d.update(resid=torch.empty(T, H, **f32), x=torch.empty(T, H, **bf), q=torch.empty(T, nh, 128, **bf),
                 attn=torch.empty(T, nh, 128, **bf), h=torch.empty(T, F, **bf), tmp=torch.empty(T, H, **bf),
                 qkv=torch.empty(T, (nh + 2 * nkv) * 128, **bf), part=math.ceil(max(ctx_len) / 32) * 32)
        self._prefill_layers(T, d)
        self._prefill_sample(seqs, d["x"], q_start, q_len, ring_row)

    def _prefill_layers(self, T: int, d: dict) -> None:
        """Embedding + every layer over T packed prompt rows (buffers and metadata in `d`; graph-capturable)."""
        w, eps = self.w, self.cfg.rms_eps
        nh, nkv = w.nh, w.nkv
        resid, x, q, attn, h, tmp, qkv = (d[k] for k in ("resid", "x", "q", "attn", "h", "tmp", "qkv"))
        ops.rmsnorm(resid, w.layers[0].attn_norm, x, eps, embed=w.embed, ids=d["ids"])
        nl = len(w.layers)
        # projections on the engine's tiled-layout GEMMs (gemm_pipe.hip / gemm_tiled.hip for T > 128 rows; gate_up with
        # its fused SiLU·mul epilogue): no library GEMM
        for li, L in enumerate(w.layers):
            # QKV out as a plain bf16 tile, then the vectorised RoPE + paged-KV-write kernel: the fused
            # per-element RoPE epilogue measured +200 us per 8192-row layer (profiles/r2/prefill_kernels_8k.md), and
            # at 512 rows (gemm_qkv_rope, one launch fewer) 9.21-9.37 vs 9.15-9.33 ms TTFT, alternating
            # (profiles/r6/ttft512_qkv_fused_ab_r6.log)
            self._proj(x, L.wqkv_t, qkv)
            ops.rope_kv_write(qkv, d["pos"], d["slots"], self.rope, q, self.kv.k[li], self.kv.v[li], nh, nkv)
            if d.get("fslots"):
                ops.flash_prefill_split(q, self.kv.k[li], self.kv.v[li], d["bt"], d["qs"], d["ql"], d["ctx"],
                                        d["fw"], d["fc"], attn, d["fpo"], d["fpm"], d["fslots"])
            else:
                ops.paged_attention(2, q, self.kv.k[li], self.kv.v[li], d["bt"], d["qs"], d["ql"], d["ctx"], d["ws"],
                                    d["wt"], attn, self.part_o, self.part_ml, d["part"], 1)
            w_next = w.layers[li + 1].attn_norm if li + 1 < nl else w.final_norm
            self._prefill_post_attention(T, attn.view(T, nh * 128), L, w_next, resid, x, h, tmp)

    # ------------------------------------------------------------------ mixed prefill + decode
    def _graph_sample(self) -> None:
        """The first-token sampling of the prompts a captured prefill / mixed batch finishes, inside the graph
        (VERDICT r5 item 5): gather their last rows of the static x and their slots' sampling parameters
        (prefill_sample_gather), LM head, candidates (TP: all-gathered), pick, commit ids / ring row / positions
        (prefill_sample_commit) -- static shapes of PREFILL_GRAPH_SEQS rows, rows past the batch's count inactive.
        Replaces _prefill_sample's torch index kernels and per-call index upload on the graph paths."""
        pf, w, cfg, comm = self.pf, self.w, self.cfg, self.comm
        ns = pf.ns
        meta, sm = pf.samp_meta(), pf.s_meta
        ops.prefill_sample_gather(pf.x, meta, self.slot_meta, pf.s_xl, sm)
        ops.gemm_out(pf.s_xl, w.lm_head_t, pf.s_logits)
        active = sm[:ns]
        ops.sample_candidates(pf.s_logits, sm[ns:2 * ns].view(torch.float32), sm[2 * ns:3 * ns],
                              sm[3 * ns:4 * ns].view(torch.float32), sm[4 * ns:6 * ns].view(ns, 2), sm[6 * ns:7 * ns],
                              active, pf.s_cand, w.vocab_offset)
        if comm.size == 1:
            cand_all = pf.s_cand.unsqueeze(0)
        else:
            cand_all = pf.s_cand_all
            comm.all_gather_into(cand_all, pf.s_cand)
        ops.sample_pick(cand_all, active, pf.s_new, vocab=cfg.vocab_size)
        ops.prefill_sample_commit(meta, pf.s_new, self.ids, self.ring, self.positions)

    def mixed(self, B: int, seqs: list, ring_row: int) -> None:
        """ONE forward over the decode slots [0, B) and the prefill chunks `seqs` (rows B .. B+T-1): every weight
        byte streams once for both, so prompt tokens absorbed while streams decode cost the in-flight streams a
        bigger GEMM (M = B + T rows) instead of a whole extra prefill pass (decode-priority
        chunked prefill).  The captured graph of bucket B with the smallest chunk size C >= the chunks' rows (metadata
        uploaded into the static prefill buffers first), else eagerly.  Decode rows: QKV as a bf16 tile ->
        vectorised RoPE + K/V write for all rows -> decode attention (partitioned flash-decoding) for the B decode
        rows and flash prefill for the chunk rows -> shared o / gate_up / down / norms -> the B decode rows sample
        and commit exactly as the captured decode step does (ids, ring row, positions), the chunks that finish a
        prompt sample their first token as prefill() does.  Same tokens as prefill() + decode() (greedy:
        tests/test_mixed_step.py)."""
        T = sum(len(s.tokens) for s in seqs)
        entry = next(((c, g) for c, g in self.mx_graphs.get(B, ()) if c >= T), None)
        if entry is not None and len(seqs) <= PREFILL_GRAPH_SEQS:
            t0 = time.perf_counter()
            self.pf.upload(seqs, entry[0], row0=B, ring_row=ring_row)
            t1 = time.perf_counter()
            entry[1].replay()  # the finishing prompts' first tokens are sampled inside (_graph_sample)
            t2 = time.perf_counter()
            if self.host_trace is not None:  # host seconds: metadata upload, graph launch, (in-graph sampling: 0)
                self.host_trace.append((t1 - t0, t2 - t1, time.perf_counter() - t2))
            return
        w, dev = self.w, self.device
        nh, nkv, F, H = w.nh, w.nkv, w.ffn, self.cfg.hidden_size
        T, q_start, q_len, ctx_len, d = self._prefill_meta(seqs, row0=B)
        M = B + T
        f32 = dict(device=dev, dtype=torch.float32)
        bf = dict(device=dev, dtype=torch.bfloat16)
        d.update(resid=torch.empty(M, H, **f32), x=torch.empty(M, H, **bf), q=torch.empty(M, nh, 128, **bf),
                 attn=torch.empty(M, nh, 128, **bf), h=torch.empty(M, F, **bf), tmp=torch.empty(M, H, **bf),
                 qkv=torch.empty(M, (nh + 2 * nkv) * 128, **bf), part=math.ceil(max(ctx_len) / 32) * 32,
                 mx_ids=torch.empty(M, dtype=torch.int32, device=dev),
                 mx_pos=torch.empty(M, dtype=torch.int32, device=dev),
                 mx_slots=torch.empty(M, dtype=torch.int32, device=dev))
        self._mixed_body(B, T, d)
        self._prefill_sample(seqs, d["x"], q_start, q_len, ring_row)

    def _mixed_layers(self, B: int, C: int) -> None:
        """The graph body of a mixed step: bucket B decode rows + C static prompt rows (_PrefillStatic)."""
        d = self.pf.views(C)
        M = B + C
        for k in ("resid", "x", "q", "attn", "h", "tmp", "qkv"):
            d[k] = getattr(self.pf, k)[:M]
        d.update(mx_ids=self.pf.mx_ids[:M], mx_pos=self.pf.mx_pos[:M], mx_slots=self.pf.mx_slots[:M])
        self._mixed_body(B, C, d)

    def _mixed_body(self, B: int, T: int, d: dict) -> None:
        """Decode prep, the forward over B + T rows, the decode rows' sampling and the ring advance (graph-capturable
        when `d` holds static buffers)."""
        w, cfg = self.w, self.cfg
        nh, nkv = w.nh, w.nkv
        eps = cfg.rms_eps
        r = slice(0, B)
        M = B + T
        ops.decode_prep(self.active[r], self.positions[r], self.block_tables[r], self.slots[r], self.ctx_len[r],
                        self.q_len[r], self.kv.num_blocks)
        ids, pos, slots = d["mx_ids"], d["mx_pos"], d["mx_slots"]
        ids[:B].copy_(self.ids[r])
        ids[B:].copy_(d["ids"][:T])
        pos[:B].copy_(self.positions[r])
        pos[B:].copy_(d["pos"][:T])
        slots[:B].copy_(self.slots[r])
        slots[B:].copy_(d["slots"][:T])
        resid, x, q, attn, h, tmp, qkv = (d[k] for k in ("resid", "x", "q", "attn", "h", "tmp", "qkv"))
        ops.rmsnorm(resid, w.layers[0].attn_norm, x, eps, embed=w.embed, ids=ids)
        dpart, dnparts = decode_partitioning(B, nkv, self.max_model_len)
        nl = len(w.layers)
        for li, L in enumerate(w.layers):
            kc, vc = self.kv.k[li], self.kv.v[li]
            self._proj(x, L.wqkv_t, qkv)
            ops.rope_kv_write(qkv, pos, slots, self.rope, q, kc, vc, nh, nkv)
            ops.paged_attention(0, q[r], kc, vc, self.block_tables[r], self.q_start[r], self.q_len[r],
                                self.ctx_len[r], self.work_seq[r], self.work_tile[r], attn[r], self.part_o,
                                self.part_ml, dpart, dnparts)
            ops.paged_attention(2, q, kc, vc, d["bt"], d["qs"], d["ql"], d["ctx"], d["ws"], d["wt"], attn,
                                self.part_o, self.part_ml, d["part"], 1)
            self._resid_proj(attn.view(M, nh * 128), L.wo_t, resid, L.ffn_norm, x, tmp)
            self._gate_up(x, L, h)
            w_next = w.layers[li + 1].attn_norm if li + 1 < nl else w.final_norm
            self._resid_proj(h, L.wd_t, resid, w_next, x, tmp)
        ops.gemm_out(x[r], w.lm_head_t, self.logits[r])
        self._sample_commit(B)
        ops.ring_advance(self.ring_counter)


class _PrefillStatic:
    """Static buffers of the captured prefill graphs (sized for the largest bucket Tmax; a bucket's graph uses
    the first tb rows) and their metadata upload: one int32 image [ids | pos | slots | q_start | q_len | ctx_len |
    work_seq | work_tile | block tables] filled on the host (two pinned buffers, alternating; an event guards
    reuse) and copied with one non-blocking H2D before the replay.  Padding: rows >= T have slot -1 (no K/V
    write) and token 0; sequence index NS is the empty sequence (q_len 0) that padded work items point at."""

    def __init__(self, runner: ModelRunner, tmax: int):
        # no back-reference to the runner: a runner <-> buffers cycle kept captured graphs alive until a garbage
        # collection, which could then run inside ANOTHER runner's capture and free a graph pool mid-capture (abort)
        self.tmax = tmax
        w, cfg, dev = runner.w, runner.cfg, runner.device
        nh, nkv, F, H = w.nh, w.nkv, w.ffn, cfg.hidden_size
        self.ns = PREFILL_GRAPH_SEQS
        self.nw = tmax // PREFILL_TILE + self.ns  # work items: sum of ceil(q_len / 64) <= T / 64 + seqs
        self.mb = runner.max_blocks
        n1 = self.ns + 1
        self.off = {}
        o = 0
        for name, k in (("ids", tmax), ("pos", tmax), ("slots", tmax), ("qs", n1), ("ql", n1), ("ctx", n1),
                        ("ws", self.nw), ("wt", self.nw), ("bt", n1 * self.mb), ("samp", 3 * self.ns + 2)):
            self.off[name] = (o, k)
            o += k
        self.words = o
        self.dev_meta = torch.zeros(o, dtype=torch.int32, device=dev)
        pin = dev.type == "cuda"
        self.host = [torch.zeros(o, dtype=torch.int32).pin_memory() if pin else torch.zeros(o, dtype=torch.int32)
                     for _ in range(2)]
        self.events = [None, None]
        self.flip = 0
        f32 = dict(device=dev, dtype=torch.float32)
        bf = dict(device=dev, dtype=torch.bfloat16)
        self.resid = torch.zeros(tmax, H, **f32)
        self.x = torch.zeros(tmax, H, **bf)
        self.q = torch.zeros(tmax, nh, 128, **bf)
        self.attn = torch.zeros(tmax, nh, 128, **bf)
        self.h = torch.zeros(tmax, F, **bf)
        self.tmp = torch.zeros(tmax, H, **bf)
        self.qkv = torch.zeros(tmax, (nh + 2 * nkv) * 128, **bf)
        self.part = math.ceil(runner.max_model_len / 32) * 32
        # mixed steps: ids / positions / slots of the B decode rows followed by the chunk rows
        i32 = dict(device=dev, dtype=torch.int32)
        self.mx_ids, self.mx_pos, self.mx_slots = (torch.zeros(tmax, **i32) for _ in range(3))
        # first-token sampling inside the graph (ModelRunner._graph_sample): the finishing prompts' last rows, their
        # sampling parameters, logits, candidates and picks, ns rows each
        ns, V = self.ns, w.vocab_local
        nch = SAMPLE_CHUNKS if dev.type == "cuda" else 1
        self.s_xl = torch.zeros(ns, H, **bf)
        self.s_meta = torch.zeros(7 * ns, **i32)
        self.s_logits = torch.zeros(ns, V, **f32)
        self.s_cand = torch.zeros(ns, nch, 2, **f32)
        self.s_cand_all = torch.zeros(runner.comm.size, ns, nch, 2, **f32)
        self.s_new = torch.zeros(ns, **i32)

    def _meta(self, name):
        o, k = self.off[name]
        return self.dev_meta[o:o + k]

    def samp_meta(self):
        """[rows | slots | last_pos (ns each) | n | ring_row] of the prompts the uploaded batch finishes."""
        return self._meta("samp")

    def views(self, tb: int) -> dict:
        nwb = tb // PREFILL_TILE + self.ns
        d = {"ids": self._meta("ids")[:tb], "pos": self._meta("pos")[:tb], "slots": self._meta("slots")[:tb],
             "qs": self._meta("qs"), "ql": self._meta("ql"), "ctx": self._meta("ctx"),
             "ws": self._meta("ws")[:nwb], "wt": self._meta("wt")[:nwb],
             "bt": self._meta("bt").view(self.ns + 1, self.mb), "part": self.part}
        d.update(resid=self.resid[:tb], x=self.x[:tb], q=self.q[:tb], attn=self.attn[:tb], h=self.h[:tb],
                 tmp=self.tmp[:tb], qkv=self.qkv[:tb])
        return d

    def _fill(self, buf: torch.Tensor, seqs: list, tb: int, row0: int = 0, ring_row: int = 0):
        a = buf.numpy()
        a[:] = 0
        o = self.off
        sm = a[o["samp"][0]:o["samp"][0] + o["samp"][1]]
        ns, row = self.ns, row0
        n = 0
        for s in seqs:
            row += len(s.tokens)
            if s.last_chunk:  # the chunk's last row samples the prompt's first token (as _prefill_sample)
                sm[n], sm[ns + n], sm[2 * ns + n] = row - 1, s.slot, s.start_pos + len(s.tokens) - 1
                n += 1
        sm[3 * ns], sm[3 * ns + 1] = n, ring_row
        ids, pos, slots = (a[o[k][0]:o[k][0] + o[k][1]] for k in ("ids", "pos", "slots"))
        qs, ql, ctx = (a[o[k][0]:o[k][0] + o[k][1]] for k in ("qs", "ql", "ctx"))
        ws, wt = (a[o[k][0]:o[k][0] + o[k][1]] for k in ("ws", "wt"))
        bt = a[o["bt"][0]:o["bt"][0] + o["bt"][1]].reshape(self.ns + 1, self.mb)
        slots[:] = -1
        q_start, q_len, items = [], [], []
        row = 0
        for i, s in enumerate(seqs):
            n = len(s.tokens)
            q_start.append(row0 + row)
            q_len.append(n)
            p = s.start_pos + np.arange(n)
            ids[row:row + n] = s.tokens
            pos[row:row + n] = p
            table = np.asarray(s.block_table, dtype=np.int64)
            slots[row:row + n] = table[p // PAGE] * PAGE + p % PAGE
            bt[i, :len(s.block_table)] = s.block_table
            qs[i], ql[i], ctx[i] = row0 + row, n, s.start_pos + n
            # flash prefill: heaviest (most keys) 64-query tiles first (as _prefill_meta)
            items += [(-(s.start_pos + min(n, (t + 1) * PREFILL_TILE)), i, t)
                      for t in range(math.ceil(n / PREFILL_TILE))]
            row += n
        items.sort()
        ws[:] = self.ns  # padded items -> the empty sequence
        for k, (_key, i, t) in enumerate(items):
            ws[k], wt[k] = i, t
        return q_start, q_len

    def upload(self, seqs: list, tb: int, row0: int = 0, ring_row: int = 0):
        """Metadata of `seqs` into the static buffers (stream-ordered before the replay that follows); the rows of
        the chunks start at `row0` of the activations (a mixed step: after the B decode rows); the prompts finishing
        in this batch commit their first token to ring row `ring_row` inside the graph."""
        k = self.flip
        self.flip ^= 1
        if self.events[k] is not None:
            self.events[k].synchronize()  # that pinned buffer's previous copy has been consumed
        q_start, q_len = self._fill(self.host[k], seqs, tb, row0, ring_row)
        self.dev_meta.copy_(self.host[k], non_blocking=True)
        if self.dev_meta.is_cuda:
            ev = torch.cuda.Event()
            ev.record()
            self.events[k] = ev
        return q_start, q_len

    def upload_padding(self):
        self.upload([], self.tmax)
