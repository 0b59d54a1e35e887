"""Plain-PyTorch fp32 reference implementations of every engine op.

These define the exact semantics (including the engine's permuted weight/cache layouts) that the
gfx950 HIP kernels in ``csrc/kernels`` implement.  They serve two purposes:

* numerics oracle: every GPU kernel test compares the HIP op against the function here;
* CPU execution: the engine, scheduler and server run end-to-end on CPU tensors for the
  plumbing tests (no GPU in the build container).  On a GPU tensor the HIP op always runs — there
  is no silent fallback (see ``ops/__init__.py``).
"""
from __future__ import annotations

import math

import numpy as np
import torch

PAGE = 32  # KV-cache page size in tokens (kBS in csrc/kernels/api.h)
HEAD_DIM = 128


# ---------------------------------------------------------------- layouts
def rotary_perm() -> torch.Tensor:
    """perm[c] = head dim stored in permuted column c of a 128-wide head unit.

    Inside each 16-column tile j: columns 0..7 hold dims 8j..8j+7 and columns 8..15 hold dims
    64+8j..64+8j+7, so the rotary partners (d, d+64) are 8 lanes apart in the MFMA output tile.
    """
    c = torch.arange(HEAD_DIM)
    j, rr = c // 16, c % 16
    return torch.where(rr < 8, 8 * j + rr, 64 + 8 * j + (rr - 8))


def gate_up_perm(F: int) -> torch.Tensor:
    """Row order of the fused gate/up weight: tile t = [gate 8t..8t+7, up 8t..8t+7] (up at +F)."""
    c = torch.arange(2 * F)
    t, rr = c // 16, c % 16
    return torch.where(rr < 8, 8 * t + rr, F + 8 * t + (rr - 8))


def vperm(off: torch.Tensor) -> torch.Tensor:
    """Position of token `off` (0..31) inside a transposed V page row."""
    return ((off & 15) >> 2) * 8 + ((off >> 4) & 1) * 4 + (off & 3)


def tile_weight(w: torch.Tensor) -> torch.Tensor:
    """Row-major [N, K] weight -> the decode GEMMs' tiled layout (same shape, permuted storage).

    Blocks of (16-row tile T, 128-column chunk c) are stored contiguously in (T, c) order; inside a
    block, element [s][lane][j] with lane = r + 16 g holds W[16T + r][128c + 32g + 8s + j], i.e. the
    MFMA B fragment of k-step s (csrc/kernels/api.h kTileChunk), so every weight load instruction of
    the decode GEMM reads 1 KiB contiguous.
    """
    N, K = w.shape
    assert N % 16 == 0 and K % 128 == 0, (N, K)
    return w.reshape(N // 16, 16, K // 128, 4, 4, 8).permute(0, 2, 4, 3, 1, 5).contiguous().view(N, K)


def untile_weight(wt: torch.Tensor) -> torch.Tensor:
    """Inverse of :func:`tile_weight`."""
    N, K = wt.shape
    return wt.reshape(N // 16, K // 128, 4, 4, 16, 8).permute(0, 4, 1, 3, 2, 5).reshape(N, K)


def rope_table(max_pos: int, theta: float, device=None) -> torch.Tensor:
    """[max_pos, 64, 2] fp32 (cos, sin) for the rotate-half convention, head_dim 128."""
    inv = theta ** (-torch.arange(0, HEAD_DIM, 2, dtype=torch.float64) / HEAD_DIM)
    ang = torch.arange(max_pos, dtype=torch.float64)[:, None] * inv[None, :]
    return torch.stack([ang.cos(), ang.sin()], dim=-1).float().to(device)


def _unpermute_units(y: torch.Tensor, n_units: int) -> torch.Tensor:
    """[M, n_units*128] permuted columns -> [M, n_units, 128] in natural head-dim order."""
    perm = rotary_perm().to(y.device)
    yu = y.view(y.shape[0], n_units, HEAD_DIM)
    out = torch.empty_like(yu)
    out[:, :, perm] = yu
    return out


def _rope(x: torch.Tensor, positions: torch.Tensor, rope: torch.Tensor) -> torch.Tensor:
    """x [M, U, 128] natural order -> rotated (rotate-half)."""
    cs = rope[positions.long()]  # [M, 64, 2]
    cos, sin = cs[..., 0][:, None, :], cs[..., 1][:, None, :]
    x1, x2 = x[..., :64], x[..., 64:]
    return torch.cat([x1 * cos - x2 * sin, x2 * cos + x1 * sin], dim=-1)


def _write_kv(k: torch.Tensor, v: torch.Tensor, slots: torch.Tensor, k_cache, v_cache):
    """k, v: [M, Hkv, 128] (natural order) -> paged caches at `slots` (skip slot < 0)."""
    for m in range(k.shape[0]):
        s = int(slots[m])
        if s < 0:
            continue
        blk, off = s // PAGE, s % PAGE
        k_cache[blk, :, off, :] = k[m].to(k_cache.dtype)
        v_cache[blk, :, :, int(vperm(torch.tensor(off)))] = v[m].to(v_cache.dtype)


# ---------------------------------------------------------------- GEMMs
# The decode GEMMs take their weight in the tiled layout (tile_weight), like the HIP kernels.
def gemm_out(x, w, out):
    out.copy_((x.float() @ untile_weight(w).float().t()).to(out.dtype))


def gemm_resid(x, w, resid):
    resid.add_(x.float() @ untile_weight(w).float().t())


def gemm_silu(x, w, out):
    y = (x.float() @ untile_weight(w).float().t()).view(x.shape[0], -1, 2, 8)
    g, u = y[:, :, 0, :], y[:, :, 1, :]
    out.copy_((torch.nn.functional.silu(g) * u).reshape(x.shape[0], -1).to(out.dtype))


def gemm_qkv_rope(x, w, positions, slots, rope, q_out, k_cache, v_cache, nh, nkv):
    M = x.shape[0]
    y = x.float() @ untile_weight(w).float().t()
    qkv = _unpermute_units(y, nh + 2 * nkv)
    rot = _rope(qkv[:, : nh + nkv], positions[:M], rope)
    q_out.view(-1)[: M * nh * HEAD_DIM].copy_(rot[:, :nh].reshape(-1).to(q_out.dtype))
    _write_kv(rot[:, nh:], qkv[:, nh + nkv:], slots[:M], k_cache, v_cache)


def rope_kv_write(qkv, positions, slots, rope, q_out, k_cache, v_cache, nh, nkv):
    T = qkv.shape[0]
    u = _unpermute_units(qkv.float(), nh + 2 * nkv)
    rot = _rope(u[:, : nh + nkv], positions[:T], rope)
    q_out.view(-1)[: T * nh * HEAD_DIM].copy_(rot[:, :nh].reshape(-1).to(q_out.dtype))
    _write_kv(rot[:, nh:], u[:, nh + nkv:], slots[:T], k_cache, v_cache)


def silu_mul(gu, h):
    y = gu.float().view(gu.shape[0], -1, 2, 8)
    h.copy_((torch.nn.functional.silu(y[:, :, 0]) * y[:, :, 1]).reshape(gu.shape[0], -1).to(h.dtype))


# ---------------------------------------------------------------- norms
def rmsnorm(resid, w, y, eps, delta=None, embed=None, ids=None, part=None, nsplit=0):
    M = y.shape[0]
    H = y.shape[1]
    if embed is not None:
        resid[:M] = embed[ids[:M].long()].float()
    elif delta is not None:
        resid[:M] += delta[:M].float()
    elif part is not None and nsplit > 0:
        resid[:M] += part.view(-1)[: nsplit * M * H].view(nsplit, M, H).sum(0)
    r = resid[:M]
    y.copy_((r * torch.rsqrt(r.pow(2).mean(-1, keepdim=True) + eps) * w.float()).to(y.dtype))


def decode_prep(active, positions, block_tables, slots, ctx_len, q_len, num_blocks: int = 2**31 - 1):
    B = active.numel()
    for b in range(B):
        if int(active[b]):
            pos = int(positions[b])
            slots[b] = int(block_tables[b, pos // PAGE]) * PAGE + pos % PAGE
            ctx_len[b] = pos + 1
            q_len[b] = 1
        else:
            slots[b] = -1
            ctx_len[b] = 0
            q_len[b] = 0


def ring_advance(counter):
    counter += 1


# ---------------------------------------------------------------- attention
def gather_kv(k_cache, v_cache, block_table, n):
    """Keys/values 0..n-1 of one sequence in natural order: ([n, Hkv, 128], [n, Hkv, 128])."""
    ks, vs = [], []
    pos_of_tok = vperm(torch.arange(PAGE)).to(v_cache.device)  # natural token t lives at pos_of_tok[t]
    for p in range((n + PAGE - 1) // PAGE):
        blk = int(block_table[p])
        ks.append(k_cache[blk].permute(1, 0, 2).float())               # [32, Hkv, 128]
        vs.append(v_cache[blk][:, :, pos_of_tok].permute(2, 0, 1).float())  # [32, Hkv, 128]
    return torch.cat(ks)[:n], torch.cat(vs)[:n]


def paged_attention(mode, q, k_cache, v_cache, block_tables, q_start, q_len, ctx_len, work_seq, work_tile,
                    out, part_o=None, part_ml=None, part=0, nparts=1):
    """Causal GQA attention of each sequence's queries over its paged keys (all work items)."""
    hq, hkv = q.shape[1], k_cache.shape[1]
    G = hq // hkv
    seqs = sorted(set(int(b) for b in work_seq.tolist()))
    for b in seqs:
        ql, ctx = int(q_len[b]), int(ctx_len[b])
        if ql <= 0:
            continue
        qs = int(q_start[b])
        K, V = gather_kv(k_cache, v_cache, block_tables[b], ctx)
        K = K.repeat_interleave(G, dim=1)  # [ctx, hq, 128]
        V = V.repeat_interleave(G, dim=1)
        Q = q[qs: qs + ql].float()          # [ql, hq, 128]
        s = torch.einsum("qhd,khd->hqk", Q, K) / math.sqrt(HEAD_DIM)
        qpos = torch.arange(ctx - ql, ctx)[:, None]
        kpos = torch.arange(ctx)[None, :]
        s = s.masked_fill((kpos > qpos)[None].to(s.device), float("-inf"))
        p = torch.softmax(s, dim=-1)
        o = torch.einsum("hqk,khd->qhd", p, V)
        out[qs: qs + ql] = o.to(out.dtype)


# ---------------------------------------------------------------- sampling
_M0, _M1 = 0xD2511F53, 0xCD9E8D57
_W0, _W1 = 0x9E3779B9, 0xBB67AE85
_U32 = 0xFFFFFFFF


def philox4x32(c0, c1, c2, c3, k0, k1):
    """Vectorised Philox4x32-10 on uint64 numpy arrays holding uint32 values (matches common.h)."""
    c0, c1, c2, c3 = (np.asarray(a, dtype=np.uint64) & _U32 for a in (c0, c1, c2, c3))
    k0 = np.uint64(k0 & _U32)
    k1 = np.uint64(k1 & _U32)
    for _ in range(10):
        p0 = np.uint64(_M0) * c0
        p1 = np.uint64(_M1) * c2
        hi0, lo0 = p0 >> np.uint64(32), p0 & np.uint64(_U32)
        hi1, lo1 = p1 >> np.uint64(32), p1 & np.uint64(_U32)
        c0, c1, c2, c3 = (hi1 ^ c1 ^ k0) & np.uint64(_U32), lo1, (hi0 ^ c3 ^ k1) & np.uint64(_U32), lo0
        k0 = np.uint64((int(k0) + _W0) & _U32)
        k1 = np.uint64((int(k1) + _W1) & _U32)
    return c0, c1, c2, c3


def gumbel_noise(seed_lo: int, seed_hi: int, position: int, gidx: np.ndarray) -> np.ndarray:
    x, _, _, _ = philox4x32(gidx, np.full_like(gidx, position), np.full_like(gidx, 0x5353), np.zeros_like(gidx),
                            seed_lo, seed_hi)
    u = ((x >> np.uint64(8)).astype(np.float64) + 1.0) / 16777216.0
    return -np.log(-np.log(u))


def _kept_mask(xb2: torch.Tensor, top_k: int, top_p: float) -> torch.Tensor:
    """Elements kept by top-k then top-p (ties at the boundary kept), on base-2 scaled logits."""
    keep = torch.ones_like(xb2, dtype=torch.bool)
    if 0 < top_k < xb2.numel():
        kth = torch.topk(xb2, top_k).values[-1]
        keep &= xb2 >= kth
    if top_p < 1.0:
        xmax = xb2.max()
        w = torch.where(keep, torch.exp2(xb2 - xmax), torch.zeros_like(xb2))
        z = w.sum()
        vals, order = torch.sort(torch.where(keep, xb2, torch.full_like(xb2, float("-inf"))), descending=True)
        cum = torch.cumsum(torch.exp2(vals - xmax).nan_to_num(0.0), 0)
        n_keep = int(torch.searchsorted(cum, top_p * z).clamp(max=vals.numel() - 1)) + 1
        thr = vals[n_keep - 1]
        keep &= xb2 >= thr
    return keep


def sample_row(logits: torch.Tensor, temperature: float, top_k: int, top_p: float, seed: tuple, position: int,
               vocab_offset: int = 0):
    """Returns (score, global index) exactly as the HIP sampler computes them."""
    x = logits.double()
    if not temperature > 0:
        i = int(torch.argmax(x))
        return float(x[i]), i + vocab_offset
    xb2 = (x / temperature) * (1.0 / math.log(2.0))
    keep = _kept_mask(xb2, top_k, top_p)
    gidx = np.arange(x.numel(), dtype=np.uint64) + np.uint64(vocab_offset)
    g = torch.from_numpy(gumbel_noise(seed[0], seed[1], position, gidx))
    sc = torch.where(keep, xb2 * math.log(2.0) + g, torch.full_like(xb2, float("-inf")))
    i = int(torch.argmax(sc))
    return float(sc[i]), i + vocab_offset


def sample_candidates(logits, temperature, top_k, top_p, seeds, positions, active, cand, vocab_offset=0):
    """cand [B, C, 2]: the whole-row best goes to chunk 0, other chunks get -inf (same final pick)."""
    B = logits.shape[0]
    sd = seeds.reshape(-1).tolist()
    cand[..., 0] = float("-inf")
    cand[..., 1] = 0.0
    for b in range(B):
        if active is not None and not int(active[b]):
            continue
        seed = (sd[2 * b] & _U32, sd[2 * b + 1] & _U32)
        sc, idx = sample_row(logits[b], float(temperature[b]), int(top_k[b]), float(top_p[b]), seed,
                             int(positions[b]), vocab_offset)
        cand[b, 0, 0] = sc
        cand[b, 0, 1] = float(idx)  # CPU encoding: the index as a float value (GPU: its bit pattern)


def sample_pick(cand_all, active, next_ids, ring=None, ring_counter=None, positions_inc=None, vocab: int = 2**31 - 1):
    world, B, C, _ = cand_all.shape
    for b in range(B):
        if active is not None and not int(active[b]):
            continue
        best, bidx = float("-inf"), None
        for w in range(world):
            for c in range(C):
                s, i = float(cand_all[w, b, c, 0]), int(cand_all[w, b, c, 1])
                if s > best or (s == best and (bidx is None or i < bidx)):
                    best, bidx = s, i
        next_ids[b] = bidx
        if ring is not None:
            ring[int(ring_counter[0]) % ring.shape[0], b] = bidx
        if positions_inc is not None:
            positions_inc[b] += 1


def sample(logits, temperature, top_k, top_p, seeds, positions, active, next_ids, ring=None, ring_counter=None,
           positions_inc=None):
    cand = torch.empty(logits.shape[0], 1, 2)
    sample_candidates(logits, temperature, top_k, top_p, seeds, positions, active, cand)
    sample_pick(cand.unsqueeze(0), active, next_ids, ring, ring_counter, positions_inc)


def prefill_sample_gather(x, meta, slot_meta, xl, smeta):
    """CPU twin of sampler.hip prefill_sample_gather_kernel: meta = [rows | slots | last_pos (NS each) | n | ring_row],
    slot_meta = [active | temperature | top_k | top_p | seeds x 2] (Bm each) -> xl rows, smeta = [active | temperature |
    top_k | top_p | seeds x 2 | position] (NS each)."""
    NS, Bm = xl.shape[0], slot_meta.numel() // 6
    n = int(meta[3 * NS])
    xl.zero_()
    smeta.zero_()
    for i in range(NS):
        on = i < n
        slot = int(meta[NS + i]) if on else 0
        if on:
            xl[i] = x[int(meta[i])]
        smeta[i] = 1 if on else 0
        smeta[NS + i] = slot_meta[Bm + slot]
        smeta[2 * NS + i] = slot_meta[2 * Bm + slot]
        smeta[3 * NS + i] = slot_meta[3 * Bm + slot]
        smeta[4 * NS + 2 * i] = slot_meta[4 * Bm + 2 * slot]
        smeta[4 * NS + 2 * i + 1] = slot_meta[4 * Bm + 2 * slot + 1]
        smeta[6 * NS + i] = int(meta[2 * NS + i]) if on else 0


def prefill_sample_commit(meta, new_ids, ids, ring, positions):
    NS = new_ids.numel()
    n, row = int(meta[3 * NS]), int(meta[3 * NS + 1])
    for i in range(min(n, NS)):
        slot = int(meta[NS + i])
        ids[slot] = new_ids[i]
        ring[row, slot] = new_ids[i]
        positions[slot] = int(meta[2 * NS + i]) + 1
