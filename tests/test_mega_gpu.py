"""Persistent decode MLP block (csrc/kernels/decode_mega.hip) against plain-PyTorch fp32 references.

Each fused stage is checked at its own scale against the reference computed from the kernel's own previous-stage
output (a whole-block tolerance would hide an O(1)-wrong stage), then the block end to end, repeated launches (the
monotonic counters cross launch boundaries), and a captured graph replayed many times."""
import math

import pytest
import torch

from distributed_sse_for_llm_response_amd import ops
from distributed_sse_for_llm_response_amd.ops import reference as R

pytestmark = pytest.mark.gpu

H, F = 4096, 14336


def _close(a, b, atol, rtol, what):
    a, b = a.float().cpu(), b.float().cpu()
    err = (a - b).abs()
    bad = (err > atol + rtol * b.abs()).sum().item()
    assert bad == 0, f"{what}: {bad} / {a.numel()} elements off; max err {err.max().item():.4g}"


@pytest.fixture(scope="module")
def block(gpu):
    if not ops.mega_supported():
        pytest.skip("persistent MLP kernel needs a 256-CU gfx950 device")
    g = torch.Generator().manual_seed(7)

    def w(n, k):
        return R.tile_weight((torch.randn(n, k, generator=g) / math.sqrt(k)).bfloat16()).to(gpu)

    d = dict(wo=w(H, H), wgu=w(2 * F, H), wd=w(H, F),
             w_ffn=(1 + 0.1 * torch.randn(H, generator=g)).bfloat16().to(gpu),
             w_next=(1 + 0.1 * torch.randn(H, generator=g)).bfloat16().to(gpu))
    # untiled fp32 copies for the reference
    d["Wo"] = R.untile_weight(d["wo"]).float()
    d["Wgu"] = R.untile_weight(d["wgu"]).float()
    d["Wd"] = R.untile_weight(d["wd"]).float()
    d["sync"] = ops.mega_sync(gpu)
    d["err"] = torch.zeros(1, dtype=torch.int32, device=gpu)
    d["slabs"] = torch.zeros(8 * 64 * H, device=gpu)
    return d


def _bufs(M, gpu, seed):
    g = torch.Generator().manual_seed(seed)
    return dict(attn=(torch.randn(M, H, generator=g)).bfloat16().to(gpu),
                resid=torch.randn(M, H, generator=g).to(gpu),
                xm=torch.zeros(M, H, dtype=torch.bfloat16, device=gpu),
                h=torch.zeros(M, F, dtype=torch.bfloat16, device=gpu),
                x=torch.zeros(M, H, dtype=torch.bfloat16, device=gpu))


def _run(d, b, eps=1e-5):
    ops.mega_mlp(b["attn"], d["wo"], d["wgu"], d["wd"], b["resid"], d["w_ffn"], d["w_next"], b["xm"], b["h"], b["x"],
                 d["slabs"], d["sync"], d["err"], eps)


def _norm(r, w, eps=1e-5):
    return (r * torch.rsqrt(r.pow(2).mean(-1, keepdim=True) + eps) * w.float()).bfloat16()


@pytest.mark.parametrize("M", [1, 17, 33, 64])
def test_mega_mlp_stages(gpu, block, M):
    d = block
    b = _bufs(M, gpu, 100 + M)
    r0 = b["resid"].clone()
    _run(d, b)
    torch.cuda.synchronize()
    assert int(d["err"].item()) == 0, "a bounded wait timed out"
    # stage 1: resid1 = r0 + attn Woᵀ, xm = norm(resid1) w_ffn
    r1 = r0 + b["attn"].float() @ d["Wo"].t()
    _close(b["xm"], _norm(r1, d["w_ffn"]), 2e-2, 2e-2, "xm")
    # stage 2: h = silu(gate) up from the kernel's own xm
    y = (b["xm"].float() @ d["Wgu"].t()).view(M, -1, 2, 8)
    h_ref = (torch.nn.functional.silu(y[:, :, 0]) * y[:, :, 1]).reshape(M, F)
    _close(b["h"], h_ref, 2e-2, 2e-2, "h")
    # stage 3: resid2 = resid1 + h Wdᵀ from the kernel's own h, x = norm(resid2) w_next
    r2 = r1 + b["h"].float() @ d["Wd"].t()
    _close(b["resid"], r2, 2e-3, 2e-3, "resid")
    _close(b["x"], _norm(r2, d["w_next"]), 2e-2, 2e-2, "x")


def test_mega_mlp_end_to_end_matches_unfused_ops(gpu, block):
    """The fused block equals the engine's unfused op chain (ops reference on CPU, fp32)."""
    d = block
    M = 64
    b = _bufs(M, gpu, 5)
    cpu = {k: v.cpu().clone() for k, v in b.items()}
    _run(d, b)
    torch.cuda.synchronize()
    R.mega_mlp(cpu["attn"], d["wo"].cpu(), d["wgu"].cpu(), d["wd"].cpu(), cpu["resid"], d["w_ffn"].cpu(),
               d["w_next"].cpu(), cpu["xm"], cpu["h"], cpu["x"], 1e-5)
    _close(b["resid"], cpu["resid"], 5e-2, 2e-2, "resid")
    _close(b["x"], cpu["x"], 6e-2, 4e-2, "x")


def test_mega_mlp_repeated_launches_and_graph_replay(gpu, block):
    """The counters are monotonic across launches (bases read at workgroup start): back-to-back launches, eager and
    from a captured graph replayed 200 times, give bit-identical results to a single launch on the same inputs and
    never time out."""
    d = block
    M = 64
    b = _bufs(M, gpu, 9)
    attn, resid0 = b["attn"].clone(), b["resid"].clone()
    _run(d, b)
    torch.cuda.synchronize()
    want = {k: b[k].clone() for k in ("resid", "xm", "h", "x")}
    for _ in range(5):
        b["resid"].copy_(resid0)
        _run(d, b)
    torch.cuda.synchronize()
    for k, v in want.items():
        assert torch.equal(b[k], v), f"eager relaunch changed {k}"
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        with torch.cuda.graph(graph, stream=s):
            b["resid"].copy_(resid0)
            _run(d, b)
    torch.cuda.current_stream().wait_stream(s)
    for _ in range(200):
        graph.replay()
    torch.cuda.synchronize()
    assert int(d["err"].item()) == 0, "a bounded wait timed out"
    for k, v in want.items():
        assert torch.equal(b[k], v), f"graph replay changed {k}"
    assert torch.equal(b["attn"], attn)


def test_mega_mlp_next_layer_qkv_slabs(gpu, block):
    """The optional last phase: the next layer's QKV projection of x as 4 fp32 split-K slabs (their sum = x·Wqkvᵀ),
    and qkv_attention_decode(slabs_ready=4) on them equals the unfused QKV + RoPE + attention."""
    d = block
    M = 64
    g = torch.Generator().manual_seed(21)
    wq = R.tile_weight((torch.randn(6144, H, generator=g) / math.sqrt(H)).bfloat16()).to(gpu)
    slabs = torch.zeros(8 * M * H, device=gpu)
    b = _bufs(M, gpu, 13)
    ops.mega_mlp(b["attn"], d["wo"], d["wgu"], d["wd"], b["resid"], d["w_ffn"], d["w_next"], b["xm"], b["h"], b["x"],
                 slabs, d["sync"], d["err"], 1e-5, wqkv=wq, qkv_slabs=slabs)
    torch.cuda.synchronize()
    assert int(d["err"].item()) == 0
    got = slabs[: 4 * M * 6144].view(4, M, 6144).sum(0)
    ref = b["x"].float() @ R.untile_weight(wq).float().t()
    _close(got, ref, 2e-3, 2e-3, "qkv slabs")
