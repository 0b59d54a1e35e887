"""Numerics of every gfx950 HIP kernel against the plain-PyTorch fp32 reference of the same op."""
import math
import os

import pytest
import torch

from distributed_sse_for_llm_response_amd import ops
from distributed_sse_for_llm_response_amd.ops import reference as R

pytestmark = pytest.mark.gpu


def _rand(*shape, dev, scale=1.0, dtype=torch.bfloat16, gen=None):
    return (torch.randn(*shape, generator=gen) * scale).to(dtype).to(dev)


def _close(a, b, atol, rtol, what=""):
    a, b = a.float().cpu(), b.float().cpu()
    err = (a - b).abs()
    tol = atol + rtol * b.abs()
    bad = (err > tol).sum().item()
    assert bad == 0, f"{what}: {bad} / {a.numel()} elements off; max err {err.max().item():.4g}"


GEMM_CONFIGS = {
    "auto": {},
    "stream-default": {"gemm_impl": "2", "s_ring": "0"},
    "stream-nt2": {"gemm_impl": "2", "s_nt": "2"},
    "stream-nw4-split2": {"gemm_impl": "2", "s_nw": "4", "s_split": "2"},
    "stream-nw4-split4": {"gemm_impl": "2", "s_nw": "4", "s_split": "4"},
    "ring": {"gemm_impl": "2"},
    "ring-nw4-split2": {"gemm_impl": "2", "s_nw": "4", "s_split": "2"},
    "ring-nw8": {"gemm_impl": "2", "s_nw": "8"},
    "ring2-all": {"gemm_impl": "2", "ring2": "1"},
    "ring1-all": {"gemm_impl": "2", "ring2": "0"},
    "wide-default": {"gemm_impl": "3"},
    "wide-split2-rd": {"gemm_impl": "3", "w_split": "2", "w_rd": "3"},
    "tiled-default": {"gemm_impl": "4"},
    "tiled-128-split2": {"gemm_impl": "4", "t_cfg": "1", "t_split": "2"},
    "tiled-128x256": {"gemm_impl": "4", "t_cfg": "5"},
    "pipe-256sq": {"gemm_impl": "4", "t_cfg": "8"},
    "pipe-192": {"gemm_impl": "4", "t_cfg": "9"},
    "pipe-128": {"gemm_impl": "4", "t_cfg": "10"},
    "skinny-default": {"gemm_impl": "0"},
    "skinny-nt2kw4": {"gemm_impl": "0", "gemm_nt": "2", "gemm_kw": "4"},
    "skinny-nt1kw8": {"gemm_impl": "0", "gemm_nt": "1", "gemm_kw": "8"},
}


@pytest.fixture(autouse=True)
def _fresh_kernel_env():
    """The library caches its DSSE_KERNEL_CFG overrides: re-read them around every test."""
    ops.refresh_env()
    yield
    ops.refresh_env()


@pytest.fixture(params=sorted(GEMM_CONFIGS))
def tiles(request, monkeypatch):
    monkeypatch.setenv("DSSE_KERNEL_CFG", ops.kernel_cfg_env(**GEMM_CONFIGS[request.param]))
    ops.refresh_env()
    yield request.param
    monkeypatch.undo()
    ops.refresh_env()


@pytest.mark.parametrize("M", [1, 7, 16, 17, 40, 64, 65, 130, 256])
def test_gemm_out_bf16_f32(gpu, tiles, M):
    g = torch.Generator().manual_seed(M)
    x = _rand(M, 1024, dev=gpu, gen=g)
    w = R.tile_weight(_rand(512, 1024, dev=gpu, scale=1 / 32, gen=g))
    for dt in (torch.bfloat16, torch.float32):
        out = torch.zeros(M, 512, device=gpu, dtype=dt)
        ref = torch.zeros(M, 512, dtype=dt)
        ops.gemm_out(x, w, out)
        R.gemm_out(x.cpu(), w.cpu(), ref)
        _close(out, ref, 2e-2 if dt == torch.bfloat16 else 1e-3, 1e-2, f"gemm_out {dt}")


@pytest.mark.parametrize("M,K", [(3, 4096), (64, 1536), (33, 14336)])
def test_gemm_resid(gpu, tiles, M, K):
    g = torch.Generator().manual_seed(K)
    x = _rand(M, K, dev=gpu, gen=g)
    w = R.tile_weight(_rand(256, K, dev=gpu, scale=1 / math.sqrt(K), gen=g))
    r0 = torch.randn(M, 256, generator=g)
    r = r0.clone().to(gpu)
    ops.gemm_resid(x, w, r)
    R.gemm_resid(x.cpu(), w.cpu(), r0)
    _close(r, r0, 1e-3, 1e-3, "gemm_resid")


@pytest.mark.parametrize("M,K", [(64, 4096), (40, 14336), (4, 4096), (200, 4096), (256, 14336)])
def test_gemm_resid_split_then_fused_norm(gpu, M, K):
    """Split-K slabs reduced inside the RMSNorm equal resid += x·wᵀ followed by the norm."""
    g = torch.Generator().manual_seed(M + K)
    H = 1024
    x = _rand(M, K, dev=gpu, gen=g)
    w = R.tile_weight(_rand(H, K, dev=gpu, scale=1 / math.sqrt(K), gen=g))
    nw = (1 + 0.1 * torch.randn(H, generator=g)).bfloat16()
    r0 = torch.randn(M, H, generator=g)
    r = r0.clone().to(gpu)
    part = torch.zeros(32 * max(64, M) * H, device=gpu)
    y = torch.zeros(M, H, device=gpu, dtype=torch.bfloat16)
    ns = ops.gemm_resid_split(x, w, r, part)
    if M > 16:
        assert ns > 1
    ops.rmsnorm(r, nw.to(gpu), y, 1e-5, part=part, nsplit=ns)
    yr = torch.zeros(M, H, dtype=torch.bfloat16)
    R.gemm_resid(x.cpu(), w.cpu(), r0)
    R.rmsnorm(r0, nw, yr, 1e-5)
    _close(r, r0, 1e-3, 1e-3, "resid")
    _close(y, yr, 2e-2, 1e-2, "y")


@pytest.mark.parametrize("nw,S", [(8, 8), (6, 4), (5, 4), (4, 16), (8, 4)])
@pytest.mark.parametrize("M,K", [(64, 4096), (33, 14336), (64, 14336)])
def test_resid_split_ring_shapes(gpu, monkeypatch, nw, S, M, K):
    """O / down projection on the ring with resid_nw / resid_split (DSSE_KERNEL_CFG; wider workgroups, deeper K split):
    the slabs reduced by the norm equal resid += x·wᵀ followed by the norm."""
    N = {5: 5120, 6: 3072}.get(nw, 4096)  # N / 16 tiles divisible by nw; N a multiple of 1024 for the norm
    monkeypatch.setenv("DSSE_KERNEL_CFG", ops.kernel_cfg_env(resid_nw=str(nw)))
    monkeypatch.setenv("DSSE_KERNEL_CFG", ops.kernel_cfg_env(resid_split=str(S)))
    ops.refresh_env()
    g = torch.Generator().manual_seed(nw * 1000 + S * 10 + M + K)
    x = _rand(M, K, dev=gpu, gen=g)
    w = R.tile_weight(_rand(N, K, dev=gpu, scale=1 / math.sqrt(K), gen=g))
    nwt = (1 + 0.1 * torch.randn(N, generator=g)).bfloat16()
    r0 = torch.randn(M, N, generator=g)
    r = r0.clone().to(gpu)
    part = torch.zeros(32 * 64 * N, device=gpu)
    y = torch.zeros(M, N, device=gpu, dtype=torch.bfloat16)
    ns = ops.gemm_resid_split(x, w, r, part)
    assert ns == S
    ops.rmsnorm(r, nwt.to(gpu), y, 1e-5, part=part, nsplit=ns)
    yr = torch.zeros(M, N, dtype=torch.bfloat16)
    R.gemm_resid(x.cpu(), w.cpu(), r0)
    R.rmsnorm(r0, nwt, yr, 1e-5)
    _close(r, r0, 1e-3, 1e-3, "resid")
    _close(y, yr, 2e-2, 1e-2, "y")


@pytest.mark.parametrize("M", [1, 20, 64, 150])
def test_gemm_silu(gpu, tiles, M):
    g = torch.Generator().manual_seed(M + 100)
    x = _rand(M, 2048, dev=gpu, gen=g)
    w = R.tile_weight(_rand(2 * 704, 2048, dev=gpu, scale=1 / 45, gen=g))
    out = torch.zeros(M, 704, device=gpu, dtype=torch.bfloat16)
    ref = torch.zeros(M, 704, dtype=torch.bfloat16)
    ops.gemm_silu(x, w, out)
    R.gemm_silu(x.cpu(), w.cpu(), ref)
    _close(out, ref, 2e-2, 2e-2, "gemm_silu")


@pytest.mark.parametrize("r2", ["0", "1"])
@pytest.mark.parametrize("ring,nw", [("1", "4"), ("1", "7"), ("1", "8")])
@pytest.mark.parametrize("M,K,S", [(33, 14336, "1"), (64, 14336, "4"), (48, 1536, "3"), (64, 4096, "2"),
                                   (17, 4096, "2"), (32, 14336, "4"), (100, 4096, "2"), (128, 14336, "4")])
def test_gemm_ring_lds_dma(gpu, monkeypatch, ring, nw, M, K, S, r2):
    """LDS-DMA ring GEMMs (gemm_ring_kernel; r2 = 1: gemm_ring2_kernel, the decoupled weight look-ahead): chunk
    counts per workgroup that are not multiples of the ring depth, split-K slabs reduced by the library, every
    epilogue against the fp32 reference."""
    if M > 64 and nw != "4":
        pytest.skip("65-128 rows: the ring runs the 4-wave shapes only (N = 16 * nw * 5 has no kernel there)")
    g = torch.Generator().manual_seed(M * 7 + K + int(nw))
    N = 16 * int(nw) * 5
    x = _rand(M, K, dev=gpu, gen=g)
    w = R.tile_weight(_rand(N, K, dev=gpu, scale=1 / math.sqrt(K), gen=g))
    monkeypatch.setenv("DSSE_KERNEL_CFG", ops.kernel_cfg_env(gemm_impl="2", s_ring=ring, s_nw=nw, s_split=S, ring2=r2))
    ops.refresh_env()
    out = torch.zeros(M, N, device=gpu, dtype=torch.float32)
    ref = torch.zeros(M, N, dtype=torch.float32)
    ops.gemm_out(x, w, out)
    R.gemm_out(x.cpu(), w.cpu(), ref)
    _close(out, ref, 1e-3, 1e-2, f"ring gemm_out d={ring} nw={nw} S={S}")
    r0 = torch.randn(M, N, generator=g)
    rr = r0.clone().to(gpu)
    ops.gemm_resid(x, w, rr)
    R.gemm_resid(x.cpu(), w.cpu(), r0)
    _close(rr, r0, 1e-3, 1e-3, "ring gemm_resid")
    h = torch.zeros(M, N // 2, device=gpu, dtype=torch.bfloat16)
    hr = torch.zeros(M, N // 2, dtype=torch.bfloat16)
    ops.gemm_silu(x, w, h)
    R.gemm_silu(x.cpu(), w.cpu(), hr)
    _close(h, hr, 2e-2, 2e-2, "ring gemm_silu")


@pytest.mark.parametrize("nw", [2, 3, 5, 6, 7])
@pytest.mark.parametrize("M", [33, 64])
def test_gemm_stream_odd_wave_counts(gpu, monkeypatch, nw, M):
    """X-streaming kernel with 2..7 waves per workgroup (N / 16 a multiple of nw), plain and split-K."""
    g = torch.Generator().manual_seed(nw * 100 + M)
    N, K = 16 * nw * 6, 2048
    x = _rand(M, K, dev=gpu, gen=g)
    w = R.tile_weight(_rand(N, K, dev=gpu, scale=1 / 45, gen=g))
    monkeypatch.setenv("DSSE_KERNEL_CFG", ops.kernel_cfg_env(gemm_impl="2"))
    monkeypatch.setenv("DSSE_KERNEL_CFG", ops.kernel_cfg_env(s_ring="0"))  # the gemm_stream kernel itself (the ring form takes 4 / 8 waves)
    monkeypatch.setenv("DSSE_KERNEL_CFG", ops.kernel_cfg_env(s_nw=str(nw)))
    ops.refresh_env()
    for split in ("1", "2"):
        monkeypatch.setenv("DSSE_KERNEL_CFG", ops.kernel_cfg_env(s_split=split))
        ops.refresh_env()
        out = torch.zeros(M, N, device=gpu, dtype=torch.float32)
        ref = torch.zeros(M, N, dtype=torch.float32)
        ops.gemm_out(x, w, out)
        R.gemm_out(x.cpu(), w.cpu(), ref)
        _close(out, ref, 1e-3, 1e-2, f"gemm_out nw={nw} S={split}")
        h = torch.zeros(M, N // 2, device=gpu, dtype=torch.bfloat16)
        hr = torch.zeros(M, N // 2, dtype=torch.bfloat16)
        ops.gemm_silu(x, w, h)
        R.gemm_silu(x.cpu(), w.cpu(), hr)
        _close(h, hr, 2e-2, 2e-2, f"gemm_silu nw={nw} S={split}")


def test_gemm_silu_full_gate_up(gpu):
    """Mistral-7B gate_up at the bench batch (64 rows: the 7-wave, 256-workgroup configuration)."""
    g = torch.Generator().manual_seed(7)
    M, N, K = 64, 28672, 4096
    x = _rand(M, K, dev=gpu, gen=g)
    w = R.tile_weight(_rand(N, K, dev=gpu, scale=1 / 64, gen=g))
    out = torch.zeros(M, N // 2, device=gpu, dtype=torch.bfloat16)
    ref = torch.zeros(M, N // 2, dtype=torch.bfloat16)
    ops.gemm_silu(x, w, out)
    R.gemm_silu(x.cpu(), w.cpu(), ref)
    _close(out, ref, 2e-2, 2e-2, "gate_up")


@pytest.mark.parametrize("M", [1, 9, 64, 100])
def test_gemm_qkv_rope_and_kv_write(gpu, tiles, M):
    nh, nkv, H = 8, 2, 1024
    g = torch.Generator().manual_seed(M + 7)
    x = _rand(M, H, dev=gpu, gen=g)
    w = R.tile_weight(_rand((nh + 2 * nkv) * 128, H, dev=gpu, scale=1 / 32, gen=g))
    rope = R.rope_table(4096, 1e6, gpu)
    positions = torch.randint(0, 4000, (M,), generator=g, dtype=torch.int32)
    slots = torch.randperm(8 * 32, generator=g)[:M].to(torch.int32)
    slots[0] = -1  # a padding row must not write the cache
    q = torch.zeros(M, nh * 128, device=gpu, dtype=torch.bfloat16)
    kc = torch.zeros(8, nkv, 32, 128, device=gpu, dtype=torch.bfloat16)
    vc = torch.zeros(8, nkv, 128, 32, device=gpu, dtype=torch.bfloat16)
    ops.gemm_qkv_rope(x, w, positions.to(gpu), slots.to(gpu), rope, q, kc, vc, nh, nkv)
    qr, kr, vr = torch.zeros(M, nh * 128, dtype=torch.bfloat16), torch.zeros_like(kc.cpu()), torch.zeros_like(vc.cpu())
    R.gemm_qkv_rope(x.cpu(), w.cpu(), positions, slots, rope.cpu(), qr, kr, vr, nh, nkv)
    _close(q, qr, 3e-2, 2e-2, "q")
    _close(kc, kr, 3e-2, 2e-2, "k cache")
    _close(vc, vr, 3e-2, 2e-2, "v cache")


@pytest.mark.parametrize("cfg", ["auto", "tiled-default", "tiled-128-split2", "tiled-128x256", "pipe-256sq",
                                 "pipe-192", "pipe-128"])
@pytest.mark.parametrize("M", [129, 192, 200, 256])
def test_decode_bucket_epilogues(gpu, monkeypatch, cfg, M):
    """Every epilogue of the 129-256-row decode buckets (bf16 / fp32 store, residual add, SiLU*mul, QKV + RoPE +
    K/V write, split-K slabs reduced by the norm) on the tiled kernels, at row counts that are not multiples of
    the tile height, against the fp32 reference."""
    monkeypatch.setenv("DSSE_KERNEL_CFG", ops.kernel_cfg_env(**GEMM_CONFIGS[cfg]))
    ops.refresh_env()
    g = torch.Generator().manual_seed(M * 7 + len(cfg))
    K = 2048
    x = _rand(M, K, dev=gpu, gen=g)
    w = R.tile_weight(_rand(1024, K, dev=gpu, scale=1 / 45, gen=g))
    for dt in (torch.bfloat16, torch.float32):
        out = torch.zeros(M, 1024, device=gpu, dtype=dt)
        ref = torch.zeros(M, 1024, dtype=dt)
        ops.gemm_out(x, w, out)
        R.gemm_out(x.cpu(), w.cpu(), ref)
        _close(out, ref, 2e-2 if dt == torch.bfloat16 else 1e-3, 1e-2, f"gemm_out {dt}")
    r0 = torch.randn(M, 1024, generator=g)
    r = r0.clone().to(gpu)
    ops.gemm_resid(x, w, r)
    R.gemm_resid(x.cpu(), w.cpu(), r0)
    _close(r, r0, 1e-3, 1e-3, "gemm_resid")
    h = torch.zeros(M, 512, device=gpu, dtype=torch.bfloat16)
    hr = torch.zeros(M, 512, dtype=torch.bfloat16)
    ops.gemm_silu(x, w, h)
    R.gemm_silu(x.cpu(), w.cpu(), hr)
    _close(h, hr, 2e-2, 2e-2, "gemm_silu")
    nh, nkv = 4, 2
    wq = R.tile_weight(_rand((nh + 2 * nkv) * 128, K, dev=gpu, scale=1 / 45, gen=g))
    rope = R.rope_table(4096, 1e6, gpu)
    positions = torch.randint(0, 4000, (M,), generator=g, dtype=torch.int32)
    slots = torch.randperm(16 * 32, generator=g)[:M].to(torch.int32)
    slots[-1] = -1
    q = torch.zeros(M, nh * 128, device=gpu, dtype=torch.bfloat16)
    kc = torch.zeros(16, nkv, 32, 128, device=gpu, dtype=torch.bfloat16)
    vc = torch.zeros(16, nkv, 128, 32, device=gpu, dtype=torch.bfloat16)
    ops.gemm_qkv_rope(x, wq, positions.to(gpu), slots.to(gpu), rope, q, kc, vc, nh, nkv)
    qr, kr, vr = torch.zeros(M, nh * 128, dtype=torch.bfloat16), torch.zeros_like(kc.cpu()), torch.zeros_like(vc.cpu())
    R.gemm_qkv_rope(x.cpu(), wq.cpu(), positions, slots, rope.cpu(), qr, kr, vr, nh, nkv)
    _close(q, qr, 3e-2, 2e-2, "q")
    _close(kc, kr, 3e-2, 2e-2, "k cache")
    _close(vc, vr, 3e-2, 2e-2, "v cache")
    # split-K slabs reduced inside the RMSNorm (the o / down projections of the wide buckets)
    nwt = (1 + 0.1 * torch.randn(1024, generator=g)).bfloat16()
    r0 = torch.randn(M, 1024, generator=g)
    r = r0.clone().to(gpu)
    part = torch.zeros(32 * M * 1024, device=gpu)
    y = torch.zeros(M, 1024, device=gpu, dtype=torch.bfloat16)
    ns = ops.gemm_resid_split(x, w, r, part)
    ops.rmsnorm(r, nwt.to(gpu), y, 1e-5, part=part, nsplit=ns)
    yr = torch.zeros(M, 1024, dtype=torch.bfloat16)
    R.gemm_resid(x.cpu(), w.cpu(), r0)
    R.rmsnorm(r0, nwt, yr, 1e-5)
    _close(r, r0, 1e-3, 1e-3, "split resid")
    _close(y, yr, 2e-2, 1e-2, "split norm")


@pytest.mark.parametrize("mode", [0, 1, 2])
@pytest.mark.parametrize("M,H", [(1, 4096), (37, 4096), (5, 1024), (3, 8192)])
def test_rmsnorm(gpu, mode, M, H):
    g = torch.Generator().manual_seed(M * 3 + mode)
    resid0 = torch.randn(M, H, generator=g)
    w = (1 + 0.1 * torch.randn(H, generator=g)).bfloat16()
    delta = torch.randn(M, H, generator=g).bfloat16() if mode == 1 else None
    embed = torch.randn(64, H, generator=g).bfloat16() if mode == 2 else None
    ids = torch.randint(0, 64, (M,), generator=g, dtype=torch.int32) if mode == 2 else None
    r_gpu = resid0.clone().to(gpu)
    y = torch.zeros(M, H, device=gpu, dtype=torch.bfloat16)
    yr = torch.zeros(M, H, dtype=torch.bfloat16)
    to = (lambda t: None if t is None else t.to(gpu))
    ops.rmsnorm(r_gpu, w.to(gpu), y, 1e-5, to(delta), to(embed), to(ids))
    R.rmsnorm(resid0, w, yr, 1e-5, delta, embed, ids)
    _close(r_gpu, resid0, 1e-5, 1e-5, "resid")
    _close(y, yr, 2e-2, 1e-2, "y")


def test_rmsnorm_back_to_back_modes(gpu):
    """60 back-to-back RMSNorm launches with varying row counts, modes 0 / 1 / 3 and slab counts, every call
    against the fp32 reference (the decode step's residual + norm calls in any order)."""
    g = torch.Generator().manual_seed(11)
    H, cap = 4096, 256
    w = (1 + 0.1 * torch.randn(H, generator=g)).bfloat16()
    wg = w.to(gpu)
    part = torch.zeros(4 * cap * H, device=gpu)
    for it in range(60):
        M = [64, 1, 256, 37, 128, 200][it % 6]
        mode = [3, 0, 1][it % 3]
        resid0 = torch.randn(M, H, generator=g) * (1 + it % 5)
        r_gpu = resid0.clone().to(gpu)
        y = torch.zeros(M, H, device=gpu, dtype=torch.bfloat16)
        yr = torch.zeros(M, H, dtype=torch.bfloat16)
        if mode == 3:
            ns = 1 + it % 4
            slabs = torch.randn(ns, M, H, generator=g)
            part[: ns * M * H] = slabs.reshape(-1).to(gpu)
            ops.rmsnorm(r_gpu, wg, y, 1e-5, part=part, nsplit=ns)
            resid0 += slabs.sum(0)
            R.rmsnorm(resid0, w, yr, 1e-5)
        elif mode == 1:
            delta = torch.randn(M, H, generator=g).bfloat16()
            ops.rmsnorm(r_gpu, wg, y, 1e-5, delta=delta.to(gpu))
            R.rmsnorm(resid0, w, yr, 1e-5, delta)
        else:
            ops.rmsnorm(r_gpu, wg, y, 1e-5)
            R.rmsnorm(resid0, w, yr, 1e-5)
        _close(r_gpu, resid0, 1e-4, 1e-5, f"resid it={it} M={M} mode={mode}")
        _close(y, yr, 2e-2, 1e-2, f"y it={it} M={M} mode={mode}")


@pytest.mark.parametrize("layout", ["scattered", "pages"])
def test_rope_kv_write_and_silu_mul(gpu, layout):
    """layout 'pages': rows 0-63 fill pages 1 and 2 in order (the page-row V path), rows 64-76 start page 0 and the
    last row is padding (slot -1); 'scattered': random slots (the per-element V path)."""
    nh, nkv = 8, 2
    T = 45 if layout == "scattered" else 78
    g = torch.Generator().manual_seed(5)
    qkv = torch.randn(T, (nh + 2 * nkv) * 128, generator=g).bfloat16()
    positions = torch.arange(100, 100 + T, dtype=torch.int32)
    if layout == "scattered":
        slots = torch.randperm(4 * 32, generator=g)[:T].to(torch.int32)
    else:
        slots = torch.cat([torch.arange(32, 96), torch.arange(0, 13), torch.tensor([-1])]).to(torch.int32)
    rope = R.rope_table(1024, 1e6)
    q, kc, vc = (torch.zeros(T, nh, 128, dtype=torch.bfloat16), torch.zeros(4, nkv, 32, 128, dtype=torch.bfloat16),
                 torch.zeros(4, nkv, 128, 32, dtype=torch.bfloat16))
    qg, kg, vg = q.to(gpu), kc.to(gpu), vc.to(gpu)
    ops.rope_kv_write(qkv.to(gpu), positions.to(gpu), slots.to(gpu), rope.to(gpu), qg, kg, vg, nh, nkv)
    R.rope_kv_write(qkv, positions, slots, rope, q, kc, vc, nh, nkv)
    _close(qg, q, 2e-2, 1e-2, "q")
    _close(kg, kc, 2e-2, 1e-2, "k")
    _close(vg, vc, 0, 0, "v")
    gu = torch.randn(T, 2 * 1408, generator=g).bfloat16()
    h, hr = torch.zeros(T, 1408, device=gpu, dtype=torch.bfloat16), torch.zeros(T, 1408, dtype=torch.bfloat16)
    ops.silu_mul(gu.to(gpu), h)
    R.silu_mul(gu, hr)
    _close(h, hr, 1e-2, 1e-2, "silu_mul")


def _attn_setup(ctxs, qlens, hq=32, hkv=8, gen=None, blocks=None):
    B = len(ctxs)
    nblk_seq = [math.ceil(c / 32) for c in ctxs]
    total = sum(nblk_seq) + 2
    perm = torch.randperm(total, generator=gen).tolist()
    kc = torch.randn(total, hkv, 32, 128, generator=gen).bfloat16()
    vc = torch.randn(total, hkv, 128, 32, generator=gen).bfloat16()
    maxb = max(nblk_seq) + 1
    bt = torch.zeros(B, maxb, dtype=torch.int32)
    o = 0
    for b in range(B):
        bt[b, : nblk_seq[b]] = torch.tensor(perm[o:o + nblk_seq[b]], dtype=torch.int32)
        o += nblk_seq[b]
    T = sum(qlens)
    q = torch.randn(T, hq, 128, generator=gen).bfloat16()
    q_start = torch.tensor([sum(qlens[:b]) for b in range(B)], dtype=torch.int32)
    return kc, vc, bt, q, q_start


@pytest.mark.parametrize("ctxs", [[1, 31, 32, 33, 300], [2000, 4096, 77], [1, 1, 1]])
@pytest.mark.parametrize("part", [128, 512, 8192])
def test_paged_attention_decode(gpu, ctxs, part):
    g = torch.Generator().manual_seed(sum(ctxs) + part)
    B = len(ctxs)
    kc, vc, bt, q, q_start = _attn_setup(ctxs, [1] * B, gen=g)
    qlen = torch.ones(B, dtype=torch.int32)
    qlen[-1] = 0 if B > 3 else 1  # an inactive slot
    ctx = torch.tensor(ctxs, dtype=torch.int32)
    ws, wt = torch.arange(B, dtype=torch.int32), torch.zeros(B, dtype=torch.int32)
    nparts = math.ceil(max(ctxs) / part)
    out = torch.zeros_like(q)
    out_g = torch.zeros_like(q).to(gpu)
    po = torch.zeros(B * 8 * nparts * 16 * 128, device=gpu)
    pml = torch.zeros(B * 8 * nparts * 16 * 2, device=gpu)
    ops.paged_attention(0, q.to(gpu), kc.to(gpu), vc.to(gpu), bt.to(gpu), q_start.to(gpu), qlen.to(gpu), ctx.to(gpu),
                        ws.to(gpu), wt.to(gpu), out_g, po, pml, part, nparts)
    R.paged_attention(0, q, kc, vc, bt, q_start, qlen, ctx, ws, wt, out)
    live = qlen.bool()
    _close(out_g.cpu()[live], out[live], 1e-2, 2e-2, "decode attention")


@pytest.mark.parametrize("ctxs", [[1, 31, 32, 33, 300], [2000, 4096, 77], [1, 1, 1], [560] * 8])
@pytest.mark.parametrize("nparts", [2, 4, 8])
@pytest.mark.parametrize("comb", ["1", "0"])
def test_paged_attention_decode_even_partitions(gpu, monkeypatch, ctxs, nparts, comb):
    """part = 0 (round 6): every sequence's keys split evenly over the nparts flash-decoding partitions in whole
    pages (attention.hip part_keys) instead of fixed max-context partitions; the partitions merged by
    attn_combine_kernel (the default) or by their last arriver (attn_comb=1); against the fp32 reference, three calls
    in a row (the last arriver leaves its ticket at zero for the next launch)."""
    monkeypatch.setenv("DSSE_KERNEL_CFG", ops.kernel_cfg_env(attn_comb=comb))
    ops.refresh_env()
    g = torch.Generator().manual_seed(sum(ctxs) + nparts)
    B = len(ctxs)
    kc, vc, bt, q, q_start = _attn_setup(ctxs, [1] * B, gen=g)
    qlen = torch.ones(B, dtype=torch.int32)
    qlen[-1] = 0 if B > 3 else 1  # an inactive slot
    ctx = torch.tensor(ctxs, dtype=torch.int32)
    ws, wt = torch.arange(B, dtype=torch.int32), torch.zeros(B, dtype=torch.int32)
    out = torch.zeros_like(q)
    out_g = torch.zeros_like(q).to(gpu)
    po = torch.zeros(B * 8 * nparts * 16 * 128, device=gpu)
    pml = torch.zeros(B * 8 * nparts * 16 * 2, device=gpu)
    args = [t.to(gpu) for t in (q, kc, vc, bt, q_start, qlen, ctx, ws, wt)]
    R.paged_attention(0, q, kc, vc, bt, q_start, qlen, ctx, ws, wt, out)
    live = qlen.bool()
    for _ in range(3):
        out_g.zero_()
        ops.paged_attention(0, *args, out_g, po, pml, 0, nparts)
        _close(out_g.cpu()[live], out[live], 1e-2, 2e-2, f"decode attention, even partitions, attn_comb={comb}")


@pytest.mark.parametrize("kwv", ["1", "2", "4"])
@pytest.mark.parametrize("M,nparts", [(9, 4), (64, 8)])
def test_qkv_attention_decode_folded_even_partitions(gpu, monkeypatch, kwv, M, nparts):
    """The folded QKV path with even per-sequence partitions (part = 0): the partition holding the newest key (and
    its key-split wave) writes that token's K / V, the others attend over their share."""
    _folded_case(gpu, monkeypatch, "auto", M, 0, kwv, nparts=nparts)


@pytest.mark.parametrize("cfg", ["auto", "stream-nw4-split4", "wide-split2-rd", "tiled-default", "tiled-128-split2",
                                 "skinny-default"])
@pytest.mark.parametrize("M,part", [(1, 128), (9, 512), (64, 128), (64, 8192), (200, 256), (256, 8192)])
def test_qkv_attention_decode_folded_epilogue(gpu, monkeypatch, cfg, M, part):
    """Attention mode 3 (QKV split-K reduce + RoPE + K/V write folded into the decode attention kernel) against
    the two-op path (gemm_qkv_rope + decode attention): same K/V cache bytes, same attention output."""
    _folded_case(gpu, monkeypatch, cfg, M, part, None)


@pytest.mark.parametrize("kwv", ["1", "2", "4", "8"])
@pytest.mark.parametrize("M,part", [(9, 512), (64, 128), (256, 8192)])
def test_qkv_attention_decode_folded_key_split_waves(gpu, monkeypatch, kwv, M, part):
    """The folded path with every key-split wave count (attn_kwv): each wave sums the slabs into its own LDS rows, and
    the wave that attends over the newest key's page writes its K / V."""
    _folded_case(gpu, monkeypatch, "auto", M, part, kwv)


def _folded_case(gpu, monkeypatch, cfg, M, part, kwv, nparts=None):
    monkeypatch.setenv("DSSE_KERNEL_CFG", ops.kernel_cfg_env(**GEMM_CONFIGS[cfg]))
    if kwv is not None:
        monkeypatch.setenv("DSSE_KERNEL_CFG", ops.kernel_cfg_env(attn_kwv=kwv))
    nh, nkv, H = 32, 8, 1024
    g = torch.Generator().manual_seed(M * 31 + part)
    ctxs = torch.randint(1, 700, (M,), generator=g).tolist()
    kc, vc, bt, _, _ = _attn_setup(ctxs, [1] * M, hq=nh, hkv=nkv, gen=g)
    ctx = torch.tensor(ctxs, dtype=torch.int32)
    qlen = torch.ones(M, dtype=torch.int32)
    pos = ctx - 1
    slots = torch.tensor([int(bt[b, (c - 1) // 32]) * 32 + (c - 1) % 32 for b, c in enumerate(ctxs)], dtype=torch.int32)
    if M > 1:  # an inactive slot: no query, no key, no K/V write
        qlen[-1], ctx[-1], slots[-1] = 0, 0, -1
    x = _rand(M, H, dev=gpu, gen=g)
    w = R.tile_weight(_rand((nh + 2 * nkv) * 128, H, dev=gpu, scale=1 / 32, gen=g))
    rope = R.rope_table(1024, 1e6, gpu)
    nparts = nparts or math.ceil(int(ctx.max()) / part)
    dev = {k: t.to(gpu) for k, t in dict(bt=bt, ctx=ctx, qlen=qlen, pos=pos, slots=slots,
                                         qs=torch.arange(M, dtype=torch.int32), ws=torch.arange(M, dtype=torch.int32),
                                         wt=torch.zeros(M, dtype=torch.int32)).items()}
    res = {}
    for fused in (1, 0):
        monkeypatch.setenv("DSSE_KERNEL_CFG", ops.kernel_cfg_env(fused_qkv_attn=str(fused)))
        ops.refresh_env()
        k_, v_ = kc.clone().to(gpu), vc.clone().to(gpu)
        q = torch.zeros(M, nh * 128, device=gpu, dtype=torch.bfloat16)
        out = torch.zeros(M, nh * 128, device=gpu, dtype=torch.bfloat16)
        slabs = torch.full((16 * M * (nh + 2 * nkv) * 128,), float("nan"), device=gpu)
        po = torch.zeros(M * nkv * nparts * 16 * 128, device=gpu)
        pml = torch.zeros(M * nkv * nparts * 16 * 2, device=gpu)
        S = ops.qkv_attention_decode(x, w, dev["pos"], dev["slots"], rope, q, k_, v_, nh, nkv, slabs, dev["bt"],
                                     dev["qs"], dev["qlen"], dev["ctx"], dev["ws"], dev["wt"], out, po, pml, part,
                                     nparts)
        res[fused] = (S, out.cpu(), k_.cpu(), v_.cpu())
    assert res[0][0] == 0
    if cfg != "skinny-default" and M > 16:
        assert res[1][0] >= 1, "the folded path did not run"
    live = qlen.bool()
    # the newest key's score is an fp32 dot instead of an MFMA column: bf16 outputs may round one ulp apart
    _close(res[1][1][live], res[0][1][live], 1.6e-2, 1e-2, "attention out")
    _close(res[1][2], res[0][2], 1e-2, 1e-2, "k cache")  # RoPE: fma contraction may differ by an ulp
    _close(res[1][3], res[0][3], 0, 0, "v cache")


@pytest.mark.parametrize("mode,hq", [(1, 32), (2, 32), (2, 16), (2, 8)])
@pytest.mark.parametrize("case", [([45], [45]), ([300, 17], [300, 17]), ([700, 64], [100, 64]), ([4096], [1000]),
                                  ([129, 1], [65, 1]), ([2048], [2048])])
def test_paged_attention_prefill(gpu, case, mode, hq):
    """mode 1: decode-style kernel on 16-query tiles; mode 2: flash prefill on 64-query tiles (G = hq / 8; the
    small cases split a kv head's q heads over workgroups (HG < G), [2048] keeps them in one (256 workgroups))."""
    ctxs, qlens = case
    g = torch.Generator().manual_seed(sum(ctxs) + hq)
    B = len(ctxs)
    kc, vc, bt, q, q_start = _attn_setup(ctxs, qlens, hq=hq, gen=g)
    qlen, ctx = torch.tensor(qlens, dtype=torch.int32), torch.tensor(ctxs, dtype=torch.int32)
    tile = 16 if mode == 1 else 64
    ws, wt = [], []
    for b in range(B):
        for t in reversed(range(math.ceil(qlens[b] / tile))):
            ws.append(b)
            wt.append(t)
    ws, wt = torch.tensor(ws, dtype=torch.int32), torch.tensor(wt, dtype=torch.int32)
    part = math.ceil(max(ctxs) / 32) * 32
    out = torch.zeros_like(q)
    out_g = torch.zeros_like(q).to(gpu)
    dummy = torch.zeros(1, device=gpu)
    ops.paged_attention(mode, q.to(gpu), kc.to(gpu), vc.to(gpu), bt.to(gpu), q_start.to(gpu), qlen.to(gpu),
                        ctx.to(gpu), ws.to(gpu), wt.to(gpu), out_g, dummy, dummy, part, 1)
    R.paged_attention(mode, q, kc, vc, bt, q_start, qlen, ctx, ws, wt, out)
    _close(out_g, out, 1e-2, 2e-2, f"prefill attention mode {mode}")


@pytest.mark.parametrize("hg", ["auto", "1", "2", "4"])
@pytest.mark.parametrize("case", [([4096], [4096]), ([4800, 300], [4096, 300]), ([200], [200])])
def test_flash_prefill_one_kv_head_head_split(gpu, monkeypatch, case, hg):
    """A TP = 8 rank's prompt attention (4 q heads on ONE kv head): the flash kernel with the group's q heads split
    over 1 / 2 / 4 workgroups (flash_hg; auto = the whole group, the measured best)."""
    if hg != "auto":
        monkeypatch.setenv("DSSE_KERNEL_CFG", ops.kernel_cfg_env(flash_hg=hg))
        ops.refresh_env()
    ctxs, qlens = case
    g = torch.Generator().manual_seed(sum(ctxs) + len(hg))
    B = len(ctxs)
    kc, vc, bt, q, q_start = _attn_setup(ctxs, qlens, hq=4, hkv=1, gen=g)
    qlen, ctx = torch.tensor(qlens, dtype=torch.int32), torch.tensor(ctxs, dtype=torch.int32)
    ws, wt = [], []
    for b in range(B):
        for t in reversed(range(math.ceil(qlens[b] / 64))):
            ws.append(b)
            wt.append(t)
    ws, wt = torch.tensor(ws, dtype=torch.int32), torch.tensor(wt, dtype=torch.int32)
    out = torch.zeros_like(q)
    out_g = torch.zeros_like(q).to(gpu)
    dummy = torch.zeros(1, device=gpu)
    ops.paged_attention(2, q.to(gpu), kc.to(gpu), vc.to(gpu), bt.to(gpu), q_start.to(gpu), qlen.to(gpu), ctx.to(gpu),
                        ws.to(gpu), wt.to(gpu), out_g, dummy, dummy, math.ceil(max(ctxs) / 32) * 32, 1)
    R.paged_attention(2, q, kc, vc, bt, q_start, qlen, ctx, ws, wt, out)
    _close(out_g, out, 1e-2, 2e-2, f"flash prefill, one kv head, hg {hg}")


@pytest.mark.parametrize("case", [
    ((1, 4), [2048], [2048]),                   # a TP = 8 rank's prompt: one kv head
    ((1, 4), [1500, 700], [1500, 300]),         # two sequences, the second a later chunk of its prompt
    ((2, 2), [1333], [1333]),                   # G = 2, two kv heads, a ragged last tile
    ((2, 1), [1100, 1030], [1100, 1030]),       # G = 1
])
def test_flash_prefill_key_split(gpu, case):
    """Flash prefill with long causal tiles cut into key ranges (ModelRunner flash_split_plan; partial slots merged
    by flash_combine_kernel) against the fp32 reference -- forced with small ranges so every shape splits."""
    from distributed_sse_for_llm_response_amd.engine.model_runner import flash_split_plan

    (hkv, G), ctxs, qlens = case
    hq = hkv * G
    g = torch.Generator().manual_seed(sum(ctxs) + hq)
    B = len(ctxs)
    kc, vc, bt, q, q_start = _attn_setup(ctxs, qlens, hq=hq, hkv=hkv, gen=g)
    qlen, ctx = torch.tensor(qlens, dtype=torch.int32), torch.tensor(ctxs, dtype=torch.int32)
    tiles = []
    for b in range(B):
        pos0 = ctxs[b] - qlens[b]
        for t in range(math.ceil(qlens[b] / 64)):
            tiles.append((b, t, math.ceil((pos0 + min(qlens[b], 64 * (t + 1))) / 64)))
    tiles.sort(key=lambda x: -x[2])
    plan = flash_split_plan(tiles, hkv, min_blocks=4, fill=1 << 20, min_target=5)
    assert plan is not None
    work, comb, nslots = plan
    assert len(comb) > 0 and nslots > len(comb) // 4
    out = torch.zeros_like(q)
    ws = torch.tensor([b for b, _, _ in tiles], dtype=torch.int32)
    wt = torch.tensor([t for _, t, _ in tiles], dtype=torch.int32)
    R.paged_attention(2, q, kc, vc, bt, q_start, qlen, ctx, ws, wt, out, None, None, 32, 1)
    out_g = torch.full_like(q, float("nan")).to(gpu)
    po = torch.zeros(nslots * hq * 64 * 128, device=gpu)
    pm = torch.zeros(nslots * hq * 64 * 2, device=gpu)
    for _ in range(2):  # repeatable
        ops.flash_prefill_split(q.to(gpu), kc.to(gpu), vc.to(gpu), bt.to(gpu), q_start.to(gpu), qlen.to(gpu),
                                ctx.to(gpu), torch.from_numpy(work).to(gpu), torch.from_numpy(comb).to(gpu), out_g, po,
                                pm, nslots)
    assert not torch.isnan(out_g).any(), "a query row was never written"
    _close(out_g, out, 1e-2, 2e-2, f"flash prefill key split {case}")


def _sampler_inputs(B, V, gen, temps, topk, topp):
    logits = torch.randn(B, V, generator=gen) * 3
    t = torch.tensor(temps, dtype=torch.float32)
    k = torch.tensor(topk, dtype=torch.int32)
    p = torch.tensor(topp, dtype=torch.float32)
    seeds = torch.randint(0, 2**31 - 1, (B, 2), generator=gen, dtype=torch.int32)
    pos = torch.randint(0, 5000, (B,), generator=gen, dtype=torch.int32)
    return logits, t, k, p, seeds, pos


@pytest.mark.parametrize("V", [32768, 4096, 1000])
@pytest.mark.parametrize("nchunks", [1, 16])
def test_sampler_matches_reference(gpu, V, nchunks):
    g = torch.Generator().manual_seed(V + nchunks)
    temps = [0.0, 1.0, 0.7, 1.3, 1.0, 0.5, 1.0, 2.0]
    topk = [0, 0, 0, 50, 1, 0, 20, 0]
    topp = [1.0, 1.0, 1.0, 1.0, 1.0, 0.9, 0.5, 0.95]
    B = len(temps)
    logits, t, k, p, seeds, pos = _sampler_inputs(B, V, g, temps, topk, topp)
    ids_g = torch.zeros(B, dtype=torch.int32, device=gpu)
    ring = torch.zeros(4, B, dtype=torch.int32, device=gpu)
    ctr = torch.tensor([2], dtype=torch.int32, device=gpu)
    pos_g = pos.clone().to(gpu)
    ops.sample(logits.to(gpu), t.to(gpu), k.to(gpu), p.to(gpu), seeds.to(gpu), pos.to(gpu), None, ids_g, ring, ctr,
               pos_g, nchunks=nchunks)
    ids_r = torch.zeros(B, dtype=torch.int32)
    R.sample(logits, t, k, p, seeds, pos, None, ids_r)
    assert torch.equal(ids_g.cpu(), ids_r), (ids_g.cpu(), ids_r)
    assert torch.equal(ring[2].cpu(), ids_r)
    assert torch.equal(pos_g.cpu(), pos + 1)


def test_sampler_distribution(gpu):
    """Gumbel-max draws follow softmax(logits / T) (chi-square style check on a small vocab)."""
    V, N = 16, 4096
    logits = torch.linspace(-2, 2, V)
    lg = logits.repeat(N, 1).to(gpu)
    t = torch.full((N,), 0.8, device=gpu)
    k = torch.zeros(N, dtype=torch.int32, device=gpu)
    p = torch.ones(N, device=gpu)
    seeds = torch.stack([torch.arange(N, dtype=torch.int32), torch.full((N,), 7, dtype=torch.int32)], 1).to(gpu)
    pos = torch.zeros(N, dtype=torch.int32, device=gpu)
    ids = torch.zeros(N, dtype=torch.int32, device=gpu)
    ops.sample(lg, t, k, p, seeds, pos, None, ids, nchunks=2)
    counts = torch.bincount(ids.cpu().long(), minlength=V).float()
    expect = torch.softmax(logits / 0.8, 0) * N
    assert ((counts - expect).abs() <= 5 * expect.sqrt() + 5).all(), (counts, expect)


def test_sampler_tp_candidates(gpu):
    """Per-shard candidates merged by sample_pick equal the unsharded draw (TP invariance)."""
    g = torch.Generator().manual_seed(11)
    B, V, world = 6, 32768, 4
    logits, t, k, p, seeds, pos = _sampler_inputs(B, V, g, [0.0, 1.0, 0.6, 1.0, 1.2, 0.9], [0, 0, 0, 0, 7, 0],
                                                  [1.0, 1.0, 1.0, 0.8, 1.0, 1.0])
    args = [x.to(gpu) for x in (t, k, p, seeds, pos)]
    full = torch.zeros(B, dtype=torch.int32, device=gpu)
    ops.sample(logits.to(gpu), *args, None, full)
    cands = []
    for r in range(world):
        c = torch.zeros(B, 16, 2, device=gpu)
        sh = logits[:, r * V // world:(r + 1) * V // world].contiguous().to(gpu)
        ops.sample_candidates(sh, *args, None, c, r * V // world)
        cands.append(c)
    picked = torch.zeros(B, dtype=torch.int32, device=gpu)
    ops.sample_pick(torch.stack(cands).contiguous(), None, picked)
    # rows without top-k / top-p are exactly TP-invariant (filtered rows filter per shard)
    for b in (0, 1, 2, 5):
        assert int(picked[b]) == int(full[b])


def test_decode_prep_and_ring(gpu):
    B = 5
    active = torch.tensor([1, 0, 1, 1, 0], dtype=torch.int32)
    positions = torch.tensor([0, 5, 31, 32, 9], dtype=torch.int32)
    bt = torch.arange(B * 4, dtype=torch.int32).view(B, 4)
    outs = [torch.zeros(B, dtype=torch.int32) for _ in range(3)]
    outs_g = [o.clone().to(gpu) for o in outs]
    ops.decode_prep(active.to(gpu), positions.to(gpu), bt.to(gpu), *outs_g)
    R.decode_prep(active, positions, bt, *outs)
    for a, b in zip(outs_g, outs):
        assert torch.equal(a.cpu(), b)
    c = torch.zeros(1, dtype=torch.int32, device=gpu)
    ops.ring_advance(c)
    ops.ring_advance(c)
    assert int(c) == 2


def test_gpu_path_has_no_fallback(gpu):
    """GPU tensors must run the HIP library (the op is registered and loaded from the in-tree .so)."""
    assert ops.load_library(required=True)
    assert os.path.exists(ops.library_path())
    assert torch.ops.dsse.kernels_abi_version() == 16
    assert not torch.ops.dsse.kernels_checked() and ops.kernel_checks() == []  # default build: checks compiled out


def test_checked_build_catches_bad_indices(gpu):
    """The checked build (DSSE_KERNELS_VARIANT=checked) runs the model with no false positives and attributes
    corrupted block tables / token ids / KV slots / RoPE positions to the right kernel without faulting."""
    import subprocess
    import sys

    from distributed_sse_for_llm_response_amd import _build

    _build.build_kernels(variant="checked")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(root, "tools", "check_kernels.py")], capture_output=True,
                       text=True, timeout=600, env={**os.environ, "DSSE_KERNELS_VARIANT": "checked"})
    assert r.returncode == 0 and "CHECKS-OK" in r.stdout, r.stdout[-3000:] + r.stderr[-3000:]



def _mistral_shards(tp):
    """(name, N, K) of every Mistral-7B decode projection as one TP rank holds it (Megatron split)."""
    H, F, V, nh, nkv = 4096, 14336, 32768, 32 // tp, 8 // tp
    return [("qkv", (nh + 2 * nkv) * 128, H), ("o", H, nh * 128), ("gate_up", 2 * F // tp, H),
            ("down", H, F // tp), ("lm_head", V // tp, H)]


@pytest.mark.parametrize("tp", [1, 2, 4, 8])
@pytest.mark.parametrize("M", [1, 16, 64, 128, 192])
def test_decode_gemms_at_tp_shard_shapes(gpu, tp, M):
    """Every rank-local projection shape of TP = 1/2/4/8 at the decode bucket sizes, through the kernel the
    engine picks for it (skinny / X-streaming / wide, split-K or not), against an fp32 reference on the GPU.
    The 8-GPU TP path cannot run on a one-GPU box; this pins its kernels' shapes."""
    g = torch.Generator().manual_seed(tp * 1000 + M)
    for name, N, K in _mistral_shards(tp):
        x = _rand(M, K, dev=gpu, gen=g)
        w = R.tile_weight(_rand(N, K, dev=gpu, scale=1 / math.sqrt(K), gen=g))
        if name == "gate_up":
            out = torch.zeros(M, N // 2, device=gpu, dtype=torch.bfloat16)
            ref = torch.zeros(M, N // 2, device=gpu, dtype=torch.bfloat16)
            ops.gemm_silu(x, w, out)
            R.gemm_silu(x, w, ref)
            _close(out, ref, 2e-2, 2e-2, f"{name} tp={tp} M={M}")
        elif name in ("o", "down"):
            r0 = torch.randn(M, N, generator=g).to(gpu)
            r = r0.clone()
            part = torch.zeros(32 * M * N, device=gpu)
            y = torch.zeros(M, N, device=gpu, dtype=torch.bfloat16)
            nw = torch.ones(N, device=gpu, dtype=torch.bfloat16)
            ns = ops.gemm_resid_split(x, w, r, part)
            ops.rmsnorm(r, nw, y, 1e-5, part=part, nsplit=ns)
            R.gemm_resid(x, w, r0)
            _close(r, r0, 1e-3, 1e-3, f"{name} tp={tp} M={M}")
        else:
            out = torch.zeros(M, N, device=gpu, dtype=torch.float32)
            ref = torch.zeros(M, N, device=gpu, dtype=torch.float32)
            ops.gemm_out(x, w, out)
            R.gemm_out(x, w, ref)
            _close(out, ref, 1e-3, 1e-2, f"{name} tp={tp} M={M}")


@pytest.mark.parametrize("M", [17, 33, 64])
@pytest.mark.parametrize("N,K", [(4096, 1792), (4096, 512), (768, 4096), (3584, 4096)])
def test_tp8_shard_shapes_out_and_split_slabs(gpu, M, N, K):
    """A TP = 8 rank's decode projections (qkv N 768, o K 512, gate_up N 3584, down K 1792): gemm_out against the fp32
    reference, and gemm_out_split's fp32 slabs (when it splits; the IPC all-reduce sums them) against the same.  K =
    1792 runs the LDS-DMA ring kernel since round 6 (K % 128, not K % 512)."""
    g = torch.Generator().manual_seed(M * 7 + N + K)
    x = _rand(M, K, dev=gpu, gen=g)
    w = R.tile_weight(_rand(N, K, dev=gpu, scale=1 / math.sqrt(K), gen=g))
    ref = x.float() @ R.untile_weight(w).float().t()
    out = torch.zeros(M, N, device=gpu, dtype=torch.bfloat16)
    ops.gemm_out(x, w, out)
    _close(out, ref, 2e-2, 1e-2, "gemm_out")
    if K == 1792:
        impl = torch.ops.dsse.gemm_plan(M, N, K)[0]
        assert impl == 2, f"K = 1792 at {M} rows should take the ring kernel, got impl {impl}"
    part = torch.full((16 * M * N,), float("nan"), device=gpu)
    out2 = torch.zeros(M, N, device=gpu, dtype=torch.bfloat16)
    ns = ops.gemm_out_split(x, w, out2, part)
    if ns > 0:
        s = part[: ns * M * N].view(ns, M, N).sum(0)
        _close(s, ref, 1e-3, 1e-3, f"{ns} slabs")
    else:
        _close(out2, ref, 2e-2, 1e-2, "gemm_out_split (no split)")


@pytest.mark.parametrize("M", [17, 33, 64])
@pytest.mark.parametrize("fix", ["1", "0"])
def test_ring_silu_split_k_fix_up(gpu, monkeypatch, M, fix):
    """gate_up of a TP = 8 rank (N 3584) at decode rows: the ring kernel splits K and (s_fix=1, opt-in) combines the
    slices inside the launch, else (the default) slabs + splitk_reduce; both against the fp32 reference."""
    monkeypatch.setenv("DSSE_KERNEL_CFG", ops.kernel_cfg_env(s_fix=fix))
    ops.refresh_env()
    g = torch.Generator().manual_seed(M + int(fix))
    N, K = 3584, 4096
    x = _rand(M, K, dev=gpu, gen=g)
    w = R.tile_weight(_rand(N, K, dev=gpu, scale=1 / 64, gen=g))
    out = torch.zeros(M, N // 2, device=gpu, dtype=torch.bfloat16)
    for _ in range(3):
        ops.gemm_silu(x, w, out)
    gu = (x.float() @ R.untile_weight(w).float().t()).view(M, N // 16, 16)
    ref = (torch.nn.functional.silu(gu[..., :8]) * gu[..., 8:]).reshape(M, N // 2)
    _close(out, ref, 2e-2, 2e-2, f"ring silu s_fix={fix}")
    torch.cuda.synchronize()
    assert torch.ops.dsse.gemm_fix_timeouts(gpu.index or 0) == 0
