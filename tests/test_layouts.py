"""CPU checks of the engine's storage layouts (the contracts the HIP kernels index by)."""
import torch

from distributed_sse_for_llm_response_amd.ops import reference as R


def test_tile_weight_roundtrip_and_fragment_order():
    N, K = 48, 384
    w = torch.arange(N * K, dtype=torch.float32).view(N, K)
    wt = R.tile_weight(w)
    assert wt.shape == (N, K) and wt.is_contiguous()
    assert torch.equal(R.untile_weight(wt), w)
    flat = wt.reshape(-1)
    # element (tile T, chunk c, k-step s, lane l = r + 16 g, j) of the tiled storage
    for T, c, s, lane, j in [(0, 0, 0, 0, 0), (1, 2, 3, 17, 5), (2, 1, 2, 63, 7), (0, 2, 1, 40, 3)]:
        r, g = lane % 16, lane // 16
        off = ((T * (K // 128) + c) * 4 + s) * 512 + lane * 8 + j
        assert flat[off] == w[16 * T + r, 128 * c + 32 * g + 8 * s + j]


def test_reference_gemms_consume_tiled_weights():
    g = torch.Generator().manual_seed(0)
    x = torch.randn(5, 256, generator=g)
    w = torch.randn(64, 256, generator=g)
    out = torch.zeros(5, 64)
    R.gemm_out(x, R.tile_weight(w), out)
    torch.testing.assert_close(out, x @ w.t())
