"""Mixed prefill + decode steps (ModelRunner.mixed, engine DSSE_MIXED): one forward over the decode rows and the
prompt chunk rows must produce exactly the tokens of a separate prefill pass followed by the decode step."""
import os

import torch

from distributed_sse_for_llm_response_amd.engine.engine import LLMEngine, SamplingParams
from distributed_sse_for_llm_response_amd.engine.model_runner import ModelRunner, PrefillSeq
from distributed_sse_for_llm_response_amd.engine.weights import convert_standard
from distributed_sse_for_llm_response_amd.models.mistral import TINY, init_standard_weights


def _runner():
    std = init_standard_weights(TINY, seed=5)
    w = convert_standard(TINY, std)
    return ModelRunner(w, num_blocks=128, max_batch=8, max_model_len=512, device="cpu", use_graphs=False)


def _state(r):
    return r.ids.clone(), r.positions.clone(), r.ring.clone(), r.ring_counter.clone()


def test_mixed_forward_equals_prefill_then_decode():
    runs = []
    for mixed in (False, True):
        r = _runner()
        # two streams already decoding (slots 0, 1), then a new prompt (slot 2) arrives in two chunks
        bts = {0: [0, 1], 1: [4, 5], 2: [8, 9, 10]}
        for slot, bt in bts.items():
            r.block_tables[slot, : len(bt)] = torch.tensor(bt, dtype=torch.int32)
        r.temperature[:3] = 0.0
        r.prefill([PrefillSeq(0, [5, 6, 7, 8], 0, bts[0], True), PrefillSeq(1, list(range(20, 31)), 0, bts[1], True)],
                  ring_row=0)
        r.active[:2] = 1
        r.decode(2)
        prompt = list(range(40, 77))
        chunks = [PrefillSeq(2, prompt[:20], 0, bts[2], False), PrefillSeq(2, prompt[20:], 20, bts[2], True)]
        for k, c in enumerate(chunks):
            row = int(r.ring_counter[0])
            if mixed:
                r.mixed(2, [c], ring_row=row)
            else:
                r.prefill([c], ring_row=row)
                r.decode(2)
        r.active[2] = 1
        for _ in range(3):
            r.decode(4)
        runs.append(_state(r))
    for a, b in zip(*runs):
        assert torch.equal(a, b)


def _engine_tokens(mixed: bool):
    os.environ["DSSE_MIXED"] = "1" if mixed else "0"
    try:
        e = LLMEngine(_runner(), eos_id=-1, prefill_budget=64)
    finally:
        os.environ.pop("DSSE_MIXED", None)
    out = {}
    for step in range(60):
        if step in (0, 4, 9):
            for k in range(2):
                e.add_request(f"c{step}-{k}", list(range(3 + step, 3 + step + 13 + 7 * k)),
                              SamplingParams(temperature=0.0, max_tokens=9), rid=100 + 10 * step + k)
        for ev in e.step():
            out.setdefault(ev.conversation_id, []).append((ev.token_id, ev.sequence, ev.done))
    while e.has_work():
        for ev in e.step():
            out.setdefault(ev.conversation_id, []).append((ev.token_id, ev.sequence, ev.done))
    return out, e.stats


def test_engine_mixed_steps_emit_the_same_streams():
    sep, st_sep = _engine_tokens(False)
    mix, st_mix = _engine_tokens(True)
    assert st_mix["mixed_steps"] > 0 and st_sep["mixed_steps"] == 0
    assert mix == sep
    assert all(v[-1][2] and len(v) == 10 for v in mix.values())


def test_mixed_budget_queue_boost():
    """LLMEngine._mixed_budget: one pending prompt is split into even chunks at the default cap (506 -> 2 x 256);
    with two or more prompts pending the cap is the largest captured chunk (the queue drains faster: 40 req/s TTFT
    p50 40 -> 32 ms, profiles/r5/serving_r5.md); mixed_queue_boost = False keeps the default cap."""
    from distributed_sse_for_llm_response_amd.engine.engine import Sequence

    os.environ["DSSE_MIXED"] = "1"
    try:
        e = LLMEngine(_runner(), eos_id=-1, prefill_budget=512)
    finally:
        os.environ.pop("DSSE_MIXED", None)
    e.cost = None
    e.r.mx_graphs = {64: [(128, None), (256, None), (384, None)]}
    e.r.mixed_chunks = lambda B: [128, 256, 384]
    e.r.mixed_chunk = lambda B: 256

    def pending(n):
        for i in range(len(e.slots)):
            e.slots[i] = None
        for i in range(n):
            s = Sequence(rid=i, conversation_id=f"p{i}", prompt=list(range(506)), params=SamplingParams())
            s.state = "prefill"
            e.slots[i] = s

    pending(1)
    assert e._mixed_budget(64) == 256  # 506 tokens: two even 253-token shares, rounded up to 64
    pending(2)
    assert e._mixed_budget(64) == 384  # the boost: cap 384, 1012 tokens in three even shares of 338 -> 384
    e.mixed_queue_boost = False
    assert e._mixed_budget(64) == 256
