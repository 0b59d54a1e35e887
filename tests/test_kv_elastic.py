"""Elastic KV: pages are allocated as sequences grow, an exhausted pool preempts the newest sequence (paused
ones first) and re-prefills it later from prompt + published tokens, and decoding sequences are compacted
into low slots so the step runs on the smallest captured bucket.

The oracle for every case is the same engine with a pool large enough that nothing is preempted and no
compaction: the client-visible streams (token ids, sequence numbers, finish reasons) must be identical.
Decoding is greedy, so they are -- except where a re-prefilled KV (prefill arithmetic instead of decode
arithmetic, both bf16) flips an arithmetic near-tie of the random-weight model: the first differing token
of a stream must then be a near-tie of the fp32 reference (``_same_up_to_ties``), after which the two
continuations legitimately differ.
"""
import pytest
import torch

from distributed_sse_for_llm_response_amd.engine.engine import LLMEngine, SamplingParams
from distributed_sse_for_llm_response_amd.engine.model_runner import ModelRunner
from distributed_sse_for_llm_response_amd.engine.weights import convert_standard
from distributed_sse_for_llm_response_amd.models.mistral import TINY, init_standard_weights, reference_forward

_W = {}


def _engine(num_blocks, max_batch=4, device="cpu", use_graphs=False, compact=True):
    key = str(device)
    if key not in _W:
        _W[key] = convert_standard(TINY, init_standard_weights(TINY, seed=11), device=device)
    r = ModelRunner(_W[key], num_blocks=num_blocks, max_batch=max_batch, max_model_len=512, device=device,
                    use_graphs=use_graphs)
    if use_graphs:
        r.capture()
    e = LLMEngine(r, eos_id=-1, prefill_budget=256)
    if not compact:
        e._compact = lambda: None
    return e


def _prompt(i, n):
    g = torch.Generator().manual_seed(1000 + i)
    return torch.randint(3, TINY.vocab_size, (n,), generator=g).tolist()


def _streams(e, reqs, hooks=None, max_steps=4000):
    """Drive the engine; reqs = [(conv, prompt, max_tokens, step_to_add)]; returns conv -> [(tok, seq, done, fin)]."""
    out = {c: [] for c, *_ in reqs}
    for step in range(max_steps):
        for c, p, mt, at in reqs:
            if at == step:
                e.add_request(c, p, SamplingParams(temperature=0.0, max_tokens=mt))
        if hooks and step in hooks:
            hooks[step](e)
        for ev in e.step():
            out[ev.conversation_id].append((ev.token_id, ev.sequence, ev.done, ev.finish))
        if step > max(at for *_, at in reqs) and not e.has_work():
            break
    assert not e.has_work(), "engine did not drain"
    return out


def _check_stream(events, max_tokens):
    toks = [x for x in events if not x[2]]
    assert [s for _, s, _, _ in toks] == list(range(1, len(toks) + 1))
    assert events[-1][2] and events[-1][1] == len(toks) + 1
    assert len(toks) == max_tokens and events[-1][3] == "length"


def _same_up_to_ties(got, want, reqs, tol=0.02):
    std = init_standard_weights(TINY, seed=11)
    prompts = {c: p for c, p, *_ in reqs}
    for c in want:
        a, b = got[c], want[c]
        k = next((k for k, (x, y) in enumerate(zip(a, b)) if x != y), None)
        if k is None:
            assert a == b, c
            continue
        ctx = prompts[c] + [t for t, *_ in b[:k]]
        logits, _ = reference_forward(TINY, std, torch.tensor(ctx))
        row = logits[-1]
        gap = float(row[b[k][0]] - row[a[k][0]]).__abs__()
        assert gap < tol * float(row.abs().max()), f"{c}: token {k} differs ({a[k]} vs {b[k]}), logit gap {gap:.4f}"


REQS = [(f"c{i}", _prompt(i, 20 + 7 * i), 60 + 5 * i, i // 2) for i in range(6)]


def test_pages_are_allocated_lazily():
    e = _engine(num_blocks=64)
    e.add_request("a", _prompt(0, 40), SamplingParams(temperature=0.0, max_tokens=200))
    e.step()
    s = e.by_conv["a"]
    assert len(s.blocks) == 2  # 40 prompt tokens, not prompt + max_tokens (8 pages)
    for _ in range(30):
        e.step()
    assert len(s.blocks) == (40 + s.decode_enqueued) // 32 + 1
    e.run_until_idle()
    assert e.alloc.num_free == 64


def test_exhausted_pool_preempts_and_streams_resume_token_exact():
    want = _streams(_engine(num_blocks=256), REQS)
    e = _engine(num_blocks=12)  # 6 x (~3-4 pages each at the end) > 12: preemption is unavoidable
    got = _streams(e, REQS)
    assert e.stats["preemptions"] > 0
    assert e.alloc.num_free == 12
    for c, _, mt, _ in REQS:
        _check_stream(got[c], mt)
    _same_up_to_ties(got, want, REQS)


def test_paused_sequences_are_preempted_first():
    def pause(e):
        e.set_paused("c0", True)

    def resume(e):
        e.set_paused("c0", False)

    seen = []
    e = _engine(num_blocks=10)
    orig = e._preempt

    def spy(v):
        seen.append((v.conversation_id, v.paused))
        orig(v)

    e._preempt = spy
    got = _streams(e, REQS, hooks={8: pause, 200: resume})
    want = _streams(_engine(num_blocks=256), REQS)
    assert seen and seen[0] == ("c0", True)
    _same_up_to_ties(got, want, REQS)


def test_abort_of_a_preempted_request_finishes_it():
    e = _engine(num_blocks=12)
    hit = {}

    def abort_first_preempted(e):
        w = [s for s in e.waiting if s.base > 0]
        if w:
            hit["conv"] = w[0].conversation_id
            e.abort(w[0].conversation_id)

    hooks = {k: abort_first_preempted for k in range(40, 400)}
    got = _streams(e, REQS, hooks=hooks)
    assert "conv" in hit
    ev = got[hit["conv"]]
    assert ev[-1][2] and ev[-1][3] == "abort"
    assert e.alloc.num_free == 12


def test_request_larger_than_the_pool_is_clamped_not_stuck():
    e = _engine(num_blocks=4)  # 128 tokens of KV in total
    got = _streams(e, [("big", _prompt(1, 40), 500, 0)])
    toks = [x for x in got["big"] if not x[2]]
    assert len(toks) == 4 * 32 - 40 and got["big"][-1][3] == "length"


def test_compaction_moves_decoders_into_the_smallest_bucket():
    # 8 slots; the first six finish early, the two long ones sit in slots 6 and 7 -> bucket 8 without compaction
    reqs = [(f"c{i}", _prompt(i, 12), 6 if i < 6 else 60, 0) for i in range(8)]
    buckets = []
    e = _engine(num_blocks=128, max_batch=8)
    orig = e.r.decode
    e.r.decode = lambda B: (buckets.append(B), orig(B))[1]
    got = _streams(e, reqs)
    assert e.stats["compactions"] > 0
    assert buckets[-1] == 2
    assert got == _streams(_engine(num_blocks=128, max_batch=8, compact=False), reqs)


def test_compaction_swaps_with_paused_sequences():
    reqs = [(f"c{i}", _prompt(i, 12), 8 if i < 2 else 60, 0) for i in range(4)]

    def pause(e):
        e.set_paused("c2", True)

    def resume(e):
        e.set_paused("c2", False)

    e = _engine(num_blocks=128, max_batch=4)
    got = _streams(e, reqs, hooks={4: pause, 30: resume})
    assert e.stats["compactions"] > 0
    assert got == _streams(_engine(num_blocks=128, max_batch=4, compact=False), reqs, hooks={4: pause, 30: resume})


@pytest.mark.gpu
def test_preemption_and_compaction_token_exact_on_gpu_graphs(gpu):
    """The captured-graph path: preemption (re-prefill) and compaction (device slot moves) between replays."""
    want = _streams(_engine(num_blocks=256, device=gpu, use_graphs=True), REQS)
    e = _engine(num_blocks=12, device=gpu, use_graphs=True)
    got = _streams(e, REQS)
    assert e.stats["preemptions"] > 0
    _same_up_to_ties(got, want, REQS)
    reqs = [(f"c{i}", _prompt(i, 12), 6 if i < 6 else 60, 0) for i in range(8)]
    e = _engine(num_blocks=128, max_batch=8, device=gpu, use_graphs=True)
    got = _streams(e, reqs)
    assert e.stats["compactions"] > 0
    assert got == _streams(_engine(num_blocks=128, max_batch=8, device=gpu, use_graphs=True, compact=False), reqs)
