"""Engine ops: gfx950 HIP kernels on GPU tensors, fp32 PyTorch references on CPU tensors.

The HIP library (``_lib/libdsse_kernels.so``, built by ``_build.build_kernels``) registers the
operators under ``torch.ops.dsse``.  Dispatch is by tensor device only:

* GPU tensor  -> the HIP kernel, always.  If the library is missing or failed to load, the call
  raises: there is no eager-PyTorch fallback on the GPU path.
* CPU tensor  -> the reference implementation in ``ops/reference.py`` (plumbing tests in the
  GPU-less build container).
"""
from __future__ import annotations

import os
from pathlib import Path

import torch

from . import reference as ref

_VARIANT = os.environ.get("DSSE_KERNELS_VARIANT", "")  # "checked" (device index checks) or "nt", see _build.py
_LIB = Path(__file__).resolve().parent.parent / "_lib" / (
    f"libdsse_kernels_{_VARIANT}.so" if _VARIANT else "libdsse_kernels.so")
_loaded = False
_load_error: str | None = None


def load_library(required: bool = False) -> bool:
    """Load the HIP kernel library once.  Returns True when torch.ops.dsse is available."""
    global _loaded, _load_error
    if _loaded:
        return True
    if not _LIB.exists() and os.environ.get("DSSE_AUTOBUILD", "1") == "1":
        try:
            from .._build import build_kernels

            build_kernels(variant=_VARIANT or None)
        except Exception as e:  # noqa: BLE001 - reported below
            _load_error = f"build failed: {e}"
    if _LIB.exists():
        try:
            torch.ops.load_library(str(_LIB))
            _loaded = True
        except Exception as e:  # noqa: BLE001
            _load_error = f"load failed: {e}"
    elif _load_error is None:
        _load_error = f"{_LIB} not built"
    if required and not _loaded:
        raise RuntimeError(f"dsse HIP kernels unavailable ({_load_error}); run `python -m "
                           "distributed_sse_for_llm_response_amd._build kernels`")
    return _loaded


def library_path() -> Path:
    return _LIB


def _hip(t: torch.Tensor) -> bool:
    if t.is_cuda:
        load_library(required=True)
        return True
    return False


def gemm_out(x, w, out):
    """out[M, N] = x[M, K] · w[N, K]ᵀ (bf16 or fp32 out)."""
    if _hip(x):
        torch.ops.dsse.gemm_out(x, w, out)
    else:
        ref.gemm_out(x, w, out)


def gemm_resid(x, w, resid):
    """resid[M, N] (fp32) += x · wᵀ."""
    if _hip(x):
        torch.ops.dsse.gemm_resid(x, w, resid)
    else:
        ref.gemm_resid(x, w, resid)


def gemm_silu(x, w, out):
    """out[M, N/2] = silu(gate) * up with the interleaved gate/up weight rows."""
    if _hip(x):
        torch.ops.dsse.gemm_silu(x, w, out)
    else:
        ref.gemm_silu(x, w, out)


def gemm_qkv_rope(x, w, positions, slots, rope, q_out, k_cache, v_cache, nh, nkv):
    """Fused QKV projection + RoPE + paged KV write (decode)."""
    if _hip(x):
        torch.ops.dsse.gemm_qkv_rope(x, w, positions, slots, rope, q_out, k_cache, v_cache, nh, nkv)
    else:
        ref.gemm_qkv_rope(x, w, positions, slots, rope, q_out, k_cache, v_cache, nh, nkv)


def gemm_resid_split(x, w, resid, part) -> int:
    """resid += x · wᵀ, or (when the X-in-LDS kernel splits K) write fp32 slabs [S, M, N] into `part`
    and return S so the following rmsnorm(part=..., nsplit=S) folds the reduction into the norm."""
    if _hip(x):
        return int(torch.ops.dsse.gemm_resid_split(x, w, resid, part))
    ref.gemm_resid(x, w, resid)
    return 0


def gemm_out_split(x, w, out, part) -> int:
    """out = x · wᵀ (bf16), or (when the chosen kernel splits K) fp32 slabs [S, M, N] into `part` and return S for a
    consumer that sums them (the TP decode step's IPC all-reduce, comm.all_reduce_rmsnorm(part=..., nsplit=S))."""
    if _hip(x):
        return int(torch.ops.dsse.gemm_out_split(x, w, out, part))
    ref.gemm_out(x, w, out)
    return 0


def kernel_cfg_env(**overrides) -> str:
    """The DSSE_KERNEL_CFG string (the kernel library's one configuration override: "key=value,..."; keys in
    csrc/kernels/bindings.cpp env_int, e.g. gemm_impl, t_cfg, s_nw) with `overrides` merged into the current value.
    Set it in the environment, then call refresh_env()."""
    cur = {}
    for item in os.environ.get("DSSE_KERNEL_CFG", "").replace(";", ",").replace(" ", ",").split(","):
        if "=" in item:
            k, v = item.split("=", 1)
            cur[k.strip().lower()] = v.strip()
    for k, v in overrides.items():
        if v is None:
            cur.pop(k, None)
        else:
            cur[k] = str(v)
    return ",".join(f"{k}={v}" for k, v in cur.items())


def refresh_env() -> None:
    """Re-read the DSSE_* kernel tuning variables (cached by the library on first use)."""
    if load_library():
        torch.ops.dsse.refresh_env()


def rmsnorm(resid, w, y, eps, delta=None, embed=None, ids=None, part=None, nsplit=0):
    """resid (+= delta | sum of `nsplit` split-K slabs in `part` | = embed[ids]); y = rmsnorm(resid) * w."""
    if _hip(resid):
        torch.ops.dsse.rmsnorm(resid, w, y, eps, delta, embed, ids, part, nsplit)
    else:
        ref.rmsnorm(resid, w, y, eps, delta, embed, ids, part, nsplit)


def rope_kv_write(qkv, positions, slots, rope, q_out, k_cache, v_cache, nh, nkv):
    if _hip(qkv):
        torch.ops.dsse.rope_kv_write(qkv, positions, slots, rope, q_out, k_cache, v_cache, nh, nkv)
    else:
        ref.rope_kv_write(qkv, positions, slots, rope, q_out, k_cache, v_cache, nh, nkv)


def silu_mul(gu, h):
    if _hip(gu):
        torch.ops.dsse.silu_mul(gu, h)
    else:
        ref.silu_mul(gu, h)


def decode_prep(active, positions, block_tables, slots, ctx_len, q_len, num_blocks: int = 2**31 - 1):
    if _hip(active):
        torch.ops.dsse.decode_prep(active, positions, block_tables, slots, ctx_len, q_len, num_blocks)
    else:
        ref.decode_prep(active, positions, block_tables, slots, ctx_len, q_len)


def ring_advance(counter):
    if _hip(counter):
        torch.ops.dsse.ring_advance(counter)
    else:
        ref.ring_advance(counter)


def paged_attention(mode, q, k_cache, v_cache, block_tables, q_start, q_len, ctx_len, work_seq, work_tile, out,
                    part_o, part_ml, part, nparts):
    """mode 0 = decode (flash-decoding partitions), 1 = prefill on 16-query tiles (decode-style kernel),
    2 = flash prefill on 64-query tiles (LDS-staged K/V, attention_prefill.hip)."""
    if _hip(q):
        torch.ops.dsse.paged_attention(mode, q, k_cache, v_cache, block_tables, q_start, q_len, ctx_len, work_seq,
                                       work_tile, out, part_o, part_ml, part, nparts)
    else:
        ref.paged_attention(mode, q, k_cache, v_cache, block_tables, q_start, q_len, ctx_len, work_seq, work_tile,
                            out, part_o, part_ml, part, nparts)


def flash_prefill_split(q, k_cache, v_cache, block_tables, q_start, q_len, ctx_len, work, comb, out, part_o, part_ml,
                        nslots: int) -> None:
    """Flash prefill with long causal tiles split over key ranges (work = [seq | tile | (kb0, kb1) pairs | slot],
    comb = [(seq, tile, first slot, slots)]; ModelRunner._flash_split_plan): the parts leave partial O in slots that
    a combine kernel merges.  Same result as paged_attention mode 2 up to fp32 summation order."""
    if _hip(q):
        torch.ops.dsse.flash_prefill_split(q, k_cache, v_cache, block_tables, q_start, q_len, ctx_len, work, comb, out,
                                           part_o, part_ml, nslots)
    else:  # the split is a schedule: the reference computes each tile whole (a split tile's items repeat it)
        nw = work.numel() // 5
        ref.paged_attention(2, q, k_cache, v_cache, block_tables, q_start, q_len, ctx_len, work[:nw], work[nw:2 * nw],
                            out, part_o, part_ml, 32, 1)


def qkv_attention_decode(x, w, positions, slots, rope, q_out, k_cache, v_cache, nh, nkv, slabs, block_tables, q_start,
                         q_len, ctx_len, work_seq, work_tile, out, part_o, part_ml, part, nparts) -> int:
    """Decode QKV projection + RoPE + KV write + attention.  HIP: the GEMM leaves fp32 split-K slabs in `slabs`
    and the attention kernel folds the reduction, RoPE and the K/V write in (returns the slab count; 0 = it ran
    gemm_qkv_rope + paged_attention instead).  Same result as those two ops."""
    if _hip(x):
        return int(torch.ops.dsse.qkv_attention_decode(x, w, positions, slots, rope, q_out, k_cache, v_cache, nh, nkv,
                                                       slabs, block_tables, q_start, q_len, ctx_len, work_seq,
                                                       work_tile, out, part_o, part_ml, part, nparts))
    B = x.shape[0]
    ref.gemm_qkv_rope(x, w, positions, slots, rope, q_out, k_cache, v_cache, nh, nkv)
    ref.paged_attention(0, q_out.view(B, nh, 128), k_cache, v_cache, block_tables, q_start, q_len, ctx_len, work_seq,
                        work_tile, out.view(B, nh, 128), part_o, part_ml, part, nparts)
    return 0


def sample_candidates(logits, temperature, top_k, top_p, seeds, positions, active, cand, vocab_offset=0):
    """Per-rank pass: cand [B, C, 2] <- best (score, index) of each vocab chunk (Gumbel-max / argmax)."""
    if _hip(logits):
        torch.ops.dsse.sample_candidates(logits, temperature, top_k, top_p, seeds, positions, active, cand,
                                         vocab_offset)
    else:
        ref.sample_candidates(logits, temperature, top_k, top_p, seeds, positions, active, cand, vocab_offset)


def sample_pick(cand_all, active, next_ids, ring=None, ring_counter=None, positions_inc=None,
                vocab: int = 2**31 - 1):
    """Merge cand_all [world, B, C, 2] and commit: next_ids[b], ring[head][b], positions[b] += 1."""
    if _hip(cand_all):
        torch.ops.dsse.sample_pick(cand_all, active, next_ids, ring, ring_counter, positions_inc, vocab)
    else:
        ref.sample_pick(cand_all, active, next_ids, ring, ring_counter, positions_inc)


def prefill_sample_gather(x, meta, slot_meta, xl, smeta):
    """First-token sampling inside the prefill / mixed graphs: xl = the finishing prompts' last rows of x, smeta =
    their slots' sampling parameters (sampler.hip prefill_sample_gather_kernel has the layouts)."""
    if _hip(x):
        torch.ops.dsse.prefill_sample_gather(x, meta, slot_meta, xl, smeta)
    else:
        ref.prefill_sample_gather(x, meta, slot_meta, xl, smeta)


def prefill_sample_commit(meta, new_ids, ids, ring, positions):
    """ids[slot] = ring[ring_row][slot] = new_ids[i], positions[slot] = last_pos[i] + 1 for the n finishing prompts."""
    if _hip(new_ids):
        torch.ops.dsse.prefill_sample_commit(meta, new_ids, ids, ring, positions)
    else:
        ref.prefill_sample_commit(meta, new_ids, ids, ring, positions)


def sample(logits, temperature, top_k, top_p, seeds, positions, active, next_ids, ring=None, ring_counter=None,
           positions_inc=None, nchunks: int = 16):
    """Single-rank convenience: candidates + pick."""
    B = logits.shape[0]
    cand = torch.empty(B, nchunks if logits.is_cuda else 1, 2, device=logits.device, dtype=torch.float32)
    sample_candidates(logits, temperature, top_k, top_p, seeds, positions, active, cand, 0)
    sample_pick(cand.unsqueeze(0), active, next_ids, ring, ring_counter, positions_inc)


class KernelCheckError(RuntimeError):
    """An out-of-range device index caught by the checked kernel build."""


def kernel_checks(clear: bool = True, raise_on_error: bool = True) -> list:
    """Read the checked build's violation words (``_build.py kernels-checked``, DSSE_KERNELS_VARIANT=checked).

    Returns ``[(file, line, value, bound, count)]`` for every kernel file that recorded an out-of-range
    index since the last clear; raises KernelCheckError when ``raise_on_error`` and any were found.  The
    default build records nothing (empty list).  Synchronises the device.
    """
    load_library(required=True)
    if not torch.ops.dsse.kernels_checked():
        return []
    words = torch.ops.dsse.kernel_checks(clear).tolist()
    files = torch.ops.dsse.kernel_check_files().split(",")
    bad = [(f, *w) for f, w in zip(files, words) if w[3] > 0]
    if bad and raise_on_error:
        raise KernelCheckError("; ".join(f"{f}:{ln} index {v} not below {b} ({n} times)" for f, ln, v, b, n in bad))
    return bad

