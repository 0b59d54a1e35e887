"""Engine weight layout and tensor-parallel sharding.

The decode kernels want, per rank (t = TP degree, r = rank):

* ``wqkv``  [(Hq/t + 2·Hkv/t)·128, H]  — q heads, then k heads, then v heads of this rank, each
  128-row head unit permuted by :func:`ops.reference.rotary_perm` so the fused RoPE epilogue finds
  the rotary partner 8 lanes away (column-parallel: Megatron split by heads).
* ``wo``    [H, Hq/t·128]              — row-parallel (input features split by heads).
* ``wgu``   [2·F/t, H]                 — gate/up rows interleaved in 8-row blocks (column-parallel),
  so the SiLU·mul epilogue pairs gate and up in one MFMA tile.
* ``wd``    [H, F/t]                   — row-parallel.
* ``lm_head`` [V/t, H]                 — vocab-parallel; the sampler merges per-rank candidates.
* ``embed`` [V, H] replicated (256 MiB; HBM is plentiful, and it avoids an all-reduce per step).

Every GEMM of the engine -- decode (gemm_skinny / gemm_stream / gemm_wide) and prefill (gemm_tiled) --
consumes the tiled layout of :func:`ops.reference.tile_weight` (``*_t`` fields, made by :func:`attach_tiled`):
every weight load instruction reads 1 KiB of contiguous HBM, and a (16-column, 32-deep) block is one MFMA B
fragment.  The row-major [out, in] matrices above are only the conversion input; :func:`attach_tiled` drops
them, so the model is resident once (round 1 kept both layouts for the library prefill GEMMs: 14.5 GB more for
Mistral-7B at TP=1, now KV cache).
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import torch

from ..models.mistral import MistralConfig
from ..ops.reference import gate_up_perm, rotary_perm, tile_weight


@dataclass
class LayerWeights:
    attn_norm: torch.Tensor
    wqkv: torch.Tensor   # row-major conversion inputs (None once attach_tiled has run)
    wo: torch.Tensor
    ffn_norm: torch.Tensor
    wgu: torch.Tensor
    wd: torch.Tensor
    # the engine's copies, in the tiled layout (attach_tiled)
    wqkv_t: torch.Tensor = None
    wo_t: torch.Tensor = None
    wgu_t: torch.Tensor = None
    wd_t: torch.Tensor = None


@dataclass
class EngineWeights:
    cfg: MistralConfig
    tp_rank: int
    tp_size: int
    embed: torch.Tensor
    layers: list
    final_norm: torch.Tensor
    lm_head: torch.Tensor
    lm_head_t: torch.Tensor = None

    @property
    def nh(self) -> int:
        return self.cfg.num_heads // self.tp_size

    @property
    def nkv(self) -> int:
        return self.cfg.num_kv_heads // self.tp_size

    @property
    def ffn(self) -> int:
        return self.cfg.intermediate_size // self.tp_size

    @property
    def vocab_local(self) -> int:
        return self.cfg.vocab_size // self.tp_size

    @property
    def vocab_offset(self) -> int:
        return self.tp_rank * self.vocab_local

    def nbytes(self) -> int:
        """Bytes of the resident model (what a decode step streams, plus the embedding table)."""
        n = self.embed.numel() + self.final_norm.numel() + self.lm_head_t.numel()
        for L in self.layers:
            n += sum(t.numel() for t in (L.attn_norm, L.wqkv_t, L.wo_t, L.ffn_norm, L.wgu_t, L.wd_t))
        return 2 * n


@torch.no_grad()
def attach_tiled(w: EngineWeights) -> EngineWeights:
    """Convert every GEMM weight to the tiled layout and drop the row-major input (idempotent)."""
    for L in w.layers:
        if L.wqkv_t is None:
            L.wqkv_t, L.wo_t = tile_weight(L.wqkv), tile_weight(L.wo)
            L.wgu_t, L.wd_t = tile_weight(L.wgu), tile_weight(L.wd)
        L.wqkv = L.wo = L.wgu = L.wd = None
    if w.lm_head_t is None:
        w.lm_head_t = tile_weight(w.lm_head)
    w.lm_head = None
    return w


def _permute_units(w: torch.Tensor) -> torch.Tensor:
    """Permute the rows of each 128-row head unit by rotary_perm (works for q, k and v units)."""
    units = w.shape[0] // 128
    perm = rotary_perm().to(w.device)
    return w.view(units, 128, -1)[:, perm, :].reshape(w.shape)


def convert_standard(cfg: MistralConfig, std, tp_rank: int = 0, tp_size: int = 1, device="cpu") -> EngineWeights:
    """Standard (HF-layout) weights -> this rank's engine weights."""
    cfg.validate(tp_size)
    D = cfg.head_dim
    nh, nkv, F = cfg.num_heads // tp_size, cfg.num_kv_heads // tp_size, cfg.intermediate_size // tp_size
    V = cfg.vocab_size // tp_size
    r = tp_rank
    layers = []
    for L in std["layers"]:
        q = L["q"][r * nh * D:(r + 1) * nh * D]
        k = L["k"][r * nkv * D:(r + 1) * nkv * D]
        v = L["v"][r * nkv * D:(r + 1) * nkv * D]
        wqkv = _permute_units(torch.cat([q, k, v]))
        wo = L["o"][:, r * nh * D:(r + 1) * nh * D]
        gate = L["gate"][r * F:(r + 1) * F]
        up = L["up"][r * F:(r + 1) * F]
        wgu = torch.cat([gate, up])[gate_up_perm(F)]
        wd = L["down"][:, r * F:(r + 1) * F]
        layers.append(LayerWeights(
            attn_norm=L["attn_norm"].contiguous().to(device), wqkv=wqkv.contiguous().to(device),
            wo=wo.contiguous().to(device), ffn_norm=L["ffn_norm"].contiguous().to(device),
            wgu=wgu.contiguous().to(device), wd=wd.contiguous().to(device)))
    return attach_tiled(EngineWeights(
        cfg=cfg, tp_rank=tp_rank, tp_size=tp_size, embed=std["embed"].contiguous().to(device), layers=layers,
        final_norm=std["final_norm"].contiguous().to(device), lm_head=std["lm_head"][r * V:(r + 1) * V].contiguous().to(device)))


@torch.no_grad()
def random_engine_weights(cfg: MistralConfig, tp_rank: int = 0, tp_size: int = 1, device="cuda",
                          seed: int = 0, dtype=torch.bfloat16) -> EngineWeights:
    """Random weights generated directly on the device in engine layout (the 7B bench path).

    Generating 14.5 GB through the standard layout on the host would take minutes; the engine layout
    is a fixed row permutation of the standard one, so the distribution is identical.  Each rank
    draws its own shard (seeded by (seed, rank)), i.e. the global model is a valid random model.
    """
    cfg.validate(tp_size)
    D, H = cfg.head_dim, cfg.hidden_size
    nh, nkv, F = cfg.num_heads // tp_size, cfg.num_kv_heads // tp_size, cfg.intermediate_size // tp_size
    V = cfg.vocab_size // tp_size
    gen = torch.Generator(device=device)
    gen.manual_seed(seed * 1000003 + tp_rank)

    def lin(out_f, in_f):
        t = torch.empty(out_f, in_f, device=device, dtype=dtype)
        t.normal_(0.0, 1.0 / math.sqrt(in_f), generator=gen)
        return t

    def norm(n):
        t = torch.empty(n, device=device, dtype=torch.float32).normal_(1.0, 0.1, generator=gen)
        return t.to(dtype)

    embed_gen = torch.Generator(device=device)
    embed_gen.manual_seed(seed * 1000003 + 999)  # replicated: identical on every rank
    embed = torch.empty(cfg.vocab_size, H, device=device, dtype=dtype).normal_(0.0, 1.0, generator=embed_gen)
    layers = []
    for _ in range(cfg.num_layers):
        L = LayerWeights(attn_norm=norm(H), wqkv=lin((nh + 2 * nkv) * D, H), wo=lin(H, nh * D),
                         ffn_norm=norm(H), wgu=lin(2 * F, H), wd=lin(H, F))
        L.wqkv_t, L.wo_t, L.wgu_t, L.wd_t = (tile_weight(t) for t in (L.wqkv, L.wo, L.wgu, L.wd))
        L.wqkv = L.wo = L.wgu = L.wd = None  # one layer's row-major copy at a time
        layers.append(L)
    return attach_tiled(EngineWeights(cfg=cfg, tp_rank=tp_rank, tp_size=tp_size, embed=embed, layers=layers,
                                      final_norm=norm(H), lm_head=lin(V, H)))


def load_safetensors(cfg: MistralConfig, path: str, tp_rank: int = 0, tp_size: int = 1, device="cpu") -> EngineWeights:
    """Load an HF Mistral checkpoint directory (``*.safetensors``) into the engine layout."""
    from pathlib import Path

    from safetensors.torch import load_file

    tensors = {}
    for f in sorted(Path(path).glob("*.safetensors")):
        tensors.update(load_file(str(f)))
    std = {"embed": tensors["model.embed_tokens.weight"], "final_norm": tensors["model.norm.weight"],
           "lm_head": tensors.get("lm_head.weight", tensors["model.embed_tokens.weight"]), "layers": []}
    for i in range(cfg.num_layers):
        p = f"model.layers.{i}."
        std["layers"].append({
            "attn_norm": tensors[p + "input_layernorm.weight"],
            "q": tensors[p + "self_attn.q_proj.weight"], "k": tensors[p + "self_attn.k_proj.weight"],
            "v": tensors[p + "self_attn.v_proj.weight"], "o": tensors[p + "self_attn.o_proj.weight"],
            "ffn_norm": tensors[p + "post_attention_layernorm.weight"],
            "gate": tensors[p + "mlp.gate_proj.weight"], "up": tensors[p + "mlp.up_proj.weight"],
            "down": tensors[p + "mlp.down_proj.weight"],
        })
    return convert_standard(cfg, std, tp_rank, tp_size, device)
