"""The static (graph-capturable) prefill and mixed-step paths on CPU: the padded buffers of _PrefillStatic (rows
past T with slot -1, work items on the empty sequence, chunk rows after B decode rows) give the same K/V pages and
first tokens as the eager paths.  On the GPU the same bodies are captured into graphs
(test_model_full_dims_gpu.py::test_prefill_graph_matches_eager, ::test_mixed_prefill_decode_step_logits_match_reference)."""
import torch

from distributed_sse_for_llm_response_amd.engine.model_runner import ModelRunner, PrefillSeq, _PrefillStatic
from distributed_sse_for_llm_response_amd.engine.weights import random_engine_weights
from distributed_sse_for_llm_response_amd.models.mistral import SMALL


def _runner():
    w = random_engine_weights(SMALL, device="cpu", seed=0)
    return ModelRunner(w, num_blocks=96, max_batch=8, max_model_len=512, device="cpu", use_graphs=False)


def _prompts():
    g = torch.Generator().manual_seed(3)
    lens = [5, 70, 1, 33]
    return [torch.randint(3, SMALL.vocab_size, (n,), generator=g).tolist() for n in lens]


def _tables(n):
    return [list(range(8 * i, 8 * i + 8)) for i in range(n)]


def _prefill_static(r, seqs, tb):
    q_start, q_len = r.pf.upload(seqs, tb)
    r._prefill_layers(tb, r.pf.views(tb))
    r._prefill_sample(seqs, r.pf.x, q_start, q_len, ring_row=0)


def test_static_prefill_matches_eager():
    prompts, bts = _prompts(), _tables(4)
    batches = [[PrefillSeq(i, p, 0, bts[i], True) for i, p in enumerate(prompts) if i != 1],
               [PrefillSeq(1, prompts[1][:40], 0, bts[1], False)],
               [PrefillSeq(1, prompts[1][40:], 40, bts[1], True)]]
    a, b = _runner(), _runner()
    b.pf = _PrefillStatic(b, 256)
    for r in (a, b):
        r.temperature.zero_()
    for batch in batches:
        a.prefill(batch, ring_row=0)
        _prefill_static(b, batch, 128)
    assert a.ids[:4].tolist() == b.ids[:4].tolist()
    for li in range(len(a.kv.k)):
        torch.testing.assert_close(a.kv.k[li], b.kv.k[li], rtol=2e-2, atol=2e-2)
        torch.testing.assert_close(a.kv.v[li], b.kv.v[li], rtol=2e-2, atol=2e-2)


def test_static_mixed_step_matches_eager():
    prompts, bts = _prompts(), _tables(6)
    a, b = _runner(), _runner()
    b.pf = _PrefillStatic(b, 256)
    for r in (a, b):
        r.temperature.zero_()
        for i, t in enumerate(bts):
            r.block_tables[i, :len(t)] = torch.tensor(t, dtype=torch.int32)
        r.prefill([PrefillSeq(i, p, 0, bts[i], True) for i, p in enumerate(prompts)], ring_row=0)
        r.active[:4] = 1
    new = [PrefillSeq(4, list(range(10, 30)), 0, bts[4], True), PrefillSeq(5, list(range(40, 47)), 0, bts[5], True)]
    B, C = 4, 64
    a.mixed(B, new, ring_row=1)
    q_start, q_len = b.pf.upload(new, C, row0=B)
    b._mixed_layers(B, C)
    b._prefill_sample(new, b.pf.x, q_start, q_len, ring_row=1)
    assert a.ids[:6].tolist() == b.ids[:6].tolist()
    assert a.positions[:6].tolist() == b.positions[:6].tolist()
    torch.testing.assert_close(a.logits[:B], b.logits[:B], rtol=2e-2, atol=2e-2)
