"""Mistral-7B family: configuration, random-init weights and the PyTorch reference forward.

The reference serves ``mistralai/Mistral-7B-Instruct-v0.3`` through vLLM
(reference ``kubernetes/base/llm/deployment.yaml:18,74,85-97``; ``src/llm-stream-proxy/main.go:74``).
No checkpoints are reachable here, so weights are random-initialised from a seed in the standard
(HF-style) layout ``q/k/v/o/gate/up/down``; :mod:`..engine.weights` converts them into the engine's
MFMA-friendly layout.  :func:`reference_forward` is the fp32 oracle the engine's logits are
compared against.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, asdict

import torch


@dataclass(frozen=True)
class MistralConfig:
    name: str = "mistral-7b-v0.3"
    vocab_size: int = 32768
    hidden_size: int = 4096
    intermediate_size: int = 14336
    num_layers: int = 32
    num_heads: int = 32
    num_kv_heads: int = 8
    head_dim: int = 128
    rope_theta: float = 1_000_000.0
    rms_eps: float = 1e-5
    max_position: int = 32768
    bos_token_id: int = 1
    eos_token_id: int = 2

    @property
    def group(self) -> int:
        return self.num_heads // self.num_kv_heads

    def to_dict(self):
        return asdict(self)

    def num_params(self) -> int:
        H, F, V = self.hidden_size, self.intermediate_size, self.vocab_size
        attn = H * (self.num_heads + 2 * self.num_kv_heads) * self.head_dim + self.num_heads * self.head_dim * H
        mlp = 3 * H * F
        return 2 * V * H + self.num_layers * (attn + mlp + 2 * H) + H

    def validate(self, tp: int = 1) -> None:
        assert self.head_dim == 128, "kernels are specialised for head_dim 128"
        assert self.hidden_size % 1024 == 0 and self.hidden_size <= 8192
        assert self.num_heads % tp == 0 and self.num_kv_heads % tp == 0, "TP must divide the head counts"
        assert 16 % self.group == 0, "GQA group must divide 16"
        assert (self.intermediate_size // tp) % 128 == 0, "per-rank FFN width must be a multiple of 128"
        assert (self.vocab_size // tp) % 16 == 0 and self.vocab_size % tp == 0
        assert (self.num_heads // tp) * self.head_dim % 128 == 0


MISTRAL_7B_V03 = MistralConfig()

# Small configurations with the same structure (head_dim 128, GQA 4:1) for tests and smoke runs.
TINY = MistralConfig(name="mistral-tiny", vocab_size=2048, hidden_size=1024, intermediate_size=2816, num_layers=2,
                     num_heads=8, num_kv_heads=2, max_position=4096)
SMALL = MistralConfig(name="mistral-small", vocab_size=8192, hidden_size=2048, intermediate_size=5632, num_layers=4,
                      num_heads=16, num_kv_heads=4, max_position=8192)

# Eight KV heads (one per rank at TP=8, as Mistral-7B) at toy width: the CPU rehearsal model of TP=8 / DP x TP.
TINY_KV8 = MistralConfig(name="mistral-tiny-kv8", vocab_size=2048, hidden_size=2048, intermediate_size=2048,
                         num_layers=2, num_heads=16, num_kv_heads=8, max_position=4096)

CONFIGS = {c.name: c for c in (MISTRAL_7B_V03, TINY, SMALL, TINY_KV8)}
CONFIGS["mistral-7b"] = MISTRAL_7B_V03


def get_config(name: str) -> MistralConfig:
    try:
        return CONFIGS[name]
    except KeyError:
        raise ValueError(f"unknown model config {name!r}; choose one of {sorted(CONFIGS)}") from None


def init_standard_weights(cfg: MistralConfig, seed: int = 0, device="cpu", dtype=torch.bfloat16):
    """Random weights in the standard layout (what a safetensors checkpoint would hold)."""
    g = torch.Generator(device="cpu").manual_seed(seed)
    H, F, V, D = cfg.hidden_size, cfg.intermediate_size, cfg.vocab_size, cfg.head_dim

    def lin(out_f, in_f):
        return (torch.randn(out_f, in_f, generator=g) / math.sqrt(in_f)).to(dtype).to(device)

    def norm(n):
        return (1.0 + 0.1 * torch.randn(n, generator=g)).to(dtype).to(device)

    w = {"embed": (torch.randn(V, H, generator=g)).to(dtype).to(device), "layers": []}
    for _ in range(cfg.num_layers):
        w["layers"].append({
            "attn_norm": norm(H),
            "q": lin(cfg.num_heads * D, H),
            "k": lin(cfg.num_kv_heads * D, H),
            "v": lin(cfg.num_kv_heads * D, H),
            "o": lin(H, cfg.num_heads * D),
            "ffn_norm": norm(H),
            "gate": lin(F, H),
            "up": lin(F, H),
            "down": lin(H, F),
        })
    w["final_norm"] = norm(H)
    w["lm_head"] = lin(V, H)
    return w


def _rms(x, w, eps):
    return x * torch.rsqrt(x.pow(2).mean(-1, keepdim=True) + eps) * w.float()


def _rope(x, pos, theta):
    D = x.shape[-1]
    inv = theta ** (-torch.arange(0, D, 2, dtype=torch.float64, device=x.device) / D)
    ang = pos.to(x.device).double()[:, None] * inv[None, :]
    cos, sin = ang.cos().float()[:, None, :], ang.sin().float()[:, None, :]
    x1, x2 = x[..., : D // 2], x[..., D // 2:]
    return torch.cat([x1 * cos - x2 * sin, x2 * cos + x1 * sin], dim=-1)


@torch.no_grad()
def reference_forward(cfg: MistralConfig, w, ids: torch.Tensor, positions: torch.Tensor | None = None,
                      kv: list | None = None):
    """fp32 forward over one sequence; returns (logits [T, V], kv) with kv = per-layer (K, V) [S, Hkv, D].

    Passing the returned ``kv`` back continues the sequence (incremental decode oracle).
    """
    T = ids.shape[0]
    D, Hq, Hkv = cfg.head_dim, cfg.num_heads, cfg.num_kv_heads
    start = 0 if not kv else kv[0][0].shape[0]
    if positions is None:
        positions = torch.arange(start, start + T, device=ids.device)
    x = w["embed"][ids.long()].float()
    new_kv = []
    for li, L in enumerate(w["layers"]):
        h = _rms(x, L["attn_norm"], cfg.rms_eps)
        q = (h @ L["q"].float().t()).view(T, Hq, D)
        k = (h @ L["k"].float().t()).view(T, Hkv, D)
        v = (h @ L["v"].float().t()).view(T, Hkv, D)
        q, k = _rope(q, positions, cfg.rope_theta), _rope(k, positions, cfg.rope_theta)
        if kv:
            k = torch.cat([kv[li][0], k])
            v = torch.cat([kv[li][1], v])
        new_kv.append((k, v))
        S = k.shape[0]
        kk = k.repeat_interleave(cfg.group, dim=1)
        vv = v.repeat_interleave(cfg.group, dim=1)
        s = torch.einsum("qhd,khd->hqk", q, kk) / math.sqrt(D)
        mask = torch.arange(S, device=x.device)[None, :] > (torch.arange(S - T, S, device=x.device))[:, None]
        s = s.masked_fill(mask[None], float("-inf"))
        o = torch.einsum("hqk,khd->qhd", torch.softmax(s, -1), vv).reshape(T, Hq * D)
        x = x + o @ L["o"].float().t()
        h = _rms(x, L["ffn_norm"], cfg.rms_eps)
        x = x + (torch.nn.functional.silu(h @ L["gate"].float().t()) * (h @ L["up"].float().t())) @ L["down"].float().t()
    logits = _rms(x, w["final_norm"], cfg.rms_eps) @ w["lm_head"].float().t()
    return logits, new_kv
