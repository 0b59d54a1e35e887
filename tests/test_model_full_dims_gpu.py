"""Whole-model numerics at the real Mistral-7B dimensions (H 4096, F 14336, 32 / 8 heads, vocab 32768; two
layers to keep the fp32 oracle fast): the full fp32 logits of the graph-captured decode step, at every decode
path the engine picks by batch bucket (register-streaming skinny at 1, LDS-DMA ring at 64 and 128, the wide-bucket
projections at 192 / 256; prompt passes and mixed steps on gemm_tiled / gemm_pipe -- no library GEMM anywhere), after
plain and chunked prefill, against ``models/mistral.py:reference_forward`` of the same weights.

The criterion is on whole logits rows (cosine similarity and max-abs error relative to the row's scale), not on
the sampled token: an O(1)-wrong sub-stage shows up here even when the argmax survives it.
"""
import math

import pytest
import torch

from distributed_sse_for_llm_response_amd.engine.model_runner import ModelRunner, PrefillSeq
from distributed_sse_for_llm_response_amd.engine.weights import convert_standard
from distributed_sse_for_llm_response_amd.models.mistral import MistralConfig, init_standard_weights, reference_forward

pytestmark = pytest.mark.gpu

CFG = MistralConfig(name="mistral-7b-dims-2l", num_layers=2)  # every dimension of v0.3, two layers
BUCKETS = [1, 64, 128, 192, 256]
PAGES_PER_SEQ = 3  # prompts <= 60 tokens + 2 generated < 96


@pytest.fixture(scope="module")
def model():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from distributed_sse_for_llm_response_amd import ops

    ops.load_library(required=True)
    gpu = torch.device("cuda", 0)
    std = init_standard_weights(CFG, seed=3, device=gpu)
    w = convert_standard(CFG, std, device=gpu)
    r = ModelRunner(w, num_blocks=256 * PAGES_PER_SEQ + 8, max_batch=256, max_model_len=512, device=gpu)
    import os
    os.environ["DSSE_MIXED"] = "1"  # capture the mixed prefill + decode graphs too
    try:
        r.capture(BUCKETS)  # before any prefill: the warm-up pass writes no KV (every slot inactive)
    finally:
        del os.environ["DSSE_MIXED"]
    return std, r


def _compare(ref_row, got_row, what):
    ref_row, got_row = ref_row.float(), got_row.float()
    cos = torch.nn.functional.cosine_similarity(ref_row, got_row, dim=0).item()
    rel = ((ref_row - got_row).abs().max() / ref_row.abs().max()).item()
    assert cos > 0.998 and rel < 0.05, f"{what}: cosine {cos:.5f}, max-abs err / max {rel:.4f}"
    return cos, rel


@pytest.mark.parametrize("B", BUCKETS)
def test_full_dims_decode_logits_match_reference(model, gpu, B):
    _decode_logits_check(*model, gpu, B)


def _decode_logits_check(std, r, gpu, B, bucket=None):
    bucket = bucket or B
    g = torch.Generator().manual_seed(B)
    prompts = [torch.randint(3, CFG.vocab_size, (int(torch.randint(3, 61, (1,), generator=g)),), generator=g).tolist()
               for _ in range(B)]
    tables = [list(range(i * PAGES_PER_SEQ, (i + 1) * PAGES_PER_SEQ)) for i in range(B)]
    r.block_tables.zero_()
    for i, bt in enumerate(tables):
        r.block_tables[i, : len(bt)] = torch.tensor(bt, dtype=torch.int32)
    # every other sequence of a multi-sequence bucket is prefilled in two chunks (chunked prefill)
    first, second = [], []
    for i, p in enumerate(prompts):
        if B > 1 and i % 2 == 1 and len(p) > 16:
            first.append(PrefillSeq(i, p[:16], 0, tables[i], False))
            second.append(PrefillSeq(i, p[16:], 16, tables[i], True))
        else:
            first.append(PrefillSeq(i, p, 0, tables[i], True))
    for batch in (first, second):  # at most 64 sequences (<= 3840 tokens) per prefill call
        for k in range(0, len(batch), 64):
            r.prefill(batch[k:k + 64], ring_row=0)
    r.active.zero_()
    r.active[:B] = 1
    r.temperature.zero_()  # greedy
    gen = [[int(t)] for t in r.ids[:B].cpu()]
    logits = []
    for _ in range(2):
        r.decode(bucket)
        torch.cuda.synchronize()
        logits.append(r.logits[:B].clone())
        for i, t in enumerate(r.ids[:B].cpu()):
            gen[i].append(int(t))
    worst_cos, worst_rel = 1.0, 0.0
    for i in range(B):
        ids = torch.tensor(prompts[i] + gen[i][:2], device=gpu)
        ref, _ = reference_forward(CFG, std, ids)
        L = len(prompts[i])
        # the prefill's sampled token is the argmax of the reference's last prompt row (up to near-ties)
        assert float(ref[L - 1].max() - ref[L - 1, gen[i][0]]) < 0.02 * float(ref[L - 1].abs().max()), f"seq {i}"
        for s in range(2):
            c, e = _compare(ref[L + s], logits[s][i], f"bucket {B} seq {i} step {s}")
            worst_cos, worst_rel = min(worst_cos, c), max(worst_rel, e)
    print(f"bucket {B}: worst cosine {worst_cos:.6f}, worst max-abs / max {worst_rel:.4f}")
    assert not math.isnan(worst_cos)


@pytest.mark.parametrize("mode", ["graph", "eager"])
@pytest.mark.parametrize("B", [64, 128])
def test_mixed_prefill_decode_step_logits_match_reference(model, gpu, B, mode):
    """ModelRunner.mixed (the engine's prefill-in-decode step): B decode rows + two new prompts' rows in one
    forward -- the captured graph of bucket B (prompts within its C rows, padded) or the eager step; the decode
    rows' logits and the new prompts' first tokens against the fp32 reference, then the new sequences decode in
    the next bucket."""
    std, r = model
    assert B in r.mx_graphs, "mixed graphs were not captured"
    g = torch.Generator().manual_seed(1000 + B)
    n_new = 2
    prompts = [torch.randint(3, CFG.vocab_size, (int(torch.randint(3, 61, (1,), generator=g)),), generator=g).tolist()
               for _ in range(B)]
    assert [c for c, _ in r.mx_graphs[B]] == r.mixed_chunks(B) and len(r.mx_graphs[B]) >= 3, "one graph per chunk size"
    C = r.mx_graphs[B][0][0]
    prompts += [torch.randint(3, CFG.vocab_size, (n,), generator=g).tolist() for n in (C // 2 - 5, C // 2 - 9)]
    tables = [list(range(i * PAGES_PER_SEQ, (i + 1) * PAGES_PER_SEQ)) for i in range(B + n_new)]
    r.block_tables.zero_()
    for i, bt in enumerate(tables):
        r.block_tables[i, : len(bt)] = torch.tensor(bt, dtype=torch.int32)
    seqs = [PrefillSeq(i, p, 0, tables[i], True) for i, p in enumerate(prompts[:B])]
    for k in range(0, B, 64):
        r.prefill(seqs[k:k + 64], ring_row=0)
    r.active.zero_()
    r.active[:B] = 1
    r.temperature.zero_()
    gen = [[int(t)] for t in r.ids[:B].cpu()]
    new = [PrefillSeq(B + j, prompts[B + j], 0, tables[B + j], True) for j in range(n_new)]
    saved = r.mx_graphs
    if mode == "eager":
        r.mx_graphs = {}
    try:
        r.mixed(B, new, ring_row=int(r.ring_counter.item()))
        torch.cuda.synchronize()
    finally:
        r.mx_graphs = saved
    mixed_logits = r.logits[:B].clone()
    for i, t in enumerate(r.ids[:B].cpu()):
        gen[i].append(int(t))
    for i in range(0, B, 7):
        ref, _ = reference_forward(CFG, std, torch.tensor(prompts[i] + gen[i][:1], device=gpu))
        _compare(ref[len(prompts[i])], mixed_logits[i], f"mixed step, decode row {i}")
    for j in range(n_new):
        p = prompts[B + j]
        ref, _ = reference_forward(CFG, std, torch.tensor(p, device=gpu))
        tok = int(r.ids[B + j])
        assert float(ref[-1].max() - ref[-1, tok]) < 0.02 * float(ref[-1].abs().max()), f"new prompt {j}"
    # the new sequences join the batch (bucket 2B) and decode like everyone else
    r.active[B:B + n_new] = 1
    r.decode(2 * B if 2 * B in BUCKETS else 256)
    torch.cuda.synchronize()
    for j in range(n_new):
        p = prompts[B + j]
        first = int(r.ring[(int(r.ring_counter.item()) - 2) % r.ring.shape[0], B + j])
        ref, _ = reference_forward(CFG, std, torch.tensor(p + [first], device=gpu))
        _compare(ref[-1], r.logits[B + j], f"new sequence {j} first decode step")


def test_prefill_graph_matches_eager(model, gpu):
    """Prefill batches of <= 16 sequences replay a captured graph of their row bucket (padded rows: slot -1, work
    items on the empty sequence): the K/V pages it writes and the first tokens it samples equal the eager pass."""
    std, r = model
    assert r.pf_graphs, "prefill graphs were not captured"
    g = torch.Generator().manual_seed(77)
    lens = [7, 60, 33, 1, 45]
    prompts = [torch.randint(3, CFG.vocab_size, (n,), generator=g).tolist() for n in lens]
    tables = [list(range(i * PAGES_PER_SEQ, (i + 1) * PAGES_PER_SEQ)) for i in range(len(lens))]
    batches = [[PrefillSeq(i, p, 0, tables[i], True) for i, p in enumerate(prompts) if i != 1],
               [PrefillSeq(1, prompts[1][:20], 0, tables[1], False)],
               [PrefillSeq(1, prompts[1][20:], 20, tables[1], True)]]
    # greedy rows and sampled rows (temperature / top-k / top-p): the graph samples the first tokens inside
    # (_graph_sample) and must commit the same ids, ring row and positions as the eager _prefill_sample
    r.temperature.zero_()
    r.temperature[2:4] = 0.8
    r.top_k[3] = 40
    r.top_p[4] = 0.9
    r.temperature[4] = 1.0
    r.seeds[:len(lens), 0] = torch.arange(11, 11 + len(lens), dtype=torch.int32)
    blocks = torch.tensor([b for t in tables for b in t], device=gpu)
    out = {}
    saved = dict(r.pf_graphs)
    for mode in ("graph", "eager"):
        r.pf_graphs = saved if mode == "graph" else {}
        for li in range(CFG.num_layers):
            r.kv.k[li].index_fill_(0, blocks, 0)
            r.kv.v[li].index_fill_(0, blocks, 0)
        r.ids.zero_()
        r.positions.zero_()
        r.ring[3].fill_(-1)
        for b in batches:
            r.prefill(b, ring_row=3)
        torch.cuda.synchronize()
        out[mode] = ([r.kv.k[li].index_select(0, blocks).float() for li in range(CFG.num_layers)],
                     [r.kv.v[li].index_select(0, blocks).float() for li in range(CFG.num_layers)],
                     r.ids[:len(lens)].cpu().tolist(), r.positions[:len(lens)].cpu().tolist(),
                     r.ring[3, :len(lens)].cpu().tolist())
    r.temperature.zero_()
    r.top_k.zero_()
    r.top_p.fill_(1.0)
    r.pf_graphs = saved
    for li in range(CFG.num_layers):
        for kind, a, b in (("k", out["graph"][0][li], out["eager"][0][li]), ("v", out["graph"][1][li], out["eager"][1][li])):
            err = (a - b).abs().max().item()
            assert err <= 0.02 * max(1.0, b.abs().max().item()), f"layer {li} {kind}: max err {err}"
    assert out["graph"][2] == out["eager"][2]
    assert out["graph"][3] == out["eager"][3] == lens  # positions = prompt length (next token's position)
    assert out["graph"][4] == out["eager"][4] == out["eager"][2]
