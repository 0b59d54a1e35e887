"""Adaptive prefill budget (engine.PassCost): the pass-cost line fit and the budget it gives per decode bucket."""
import pytest

from distributed_sse_for_llm_response_amd.engine.engine import PassCost


def _feed(pc, a=1.5, b=0.016, sizes=(128, 256, 512, 384, 256, 512)):
    for t in sizes:
        pc.observe("prefill", t, a + b * t)


def test_line_recovers_a_linear_pass_cost():
    pc = PassCost(2.0)
    assert pc.line() is None
    pc.observe("prefill", 512, 9.7)
    assert pc.line() is None  # one size: no slope yet
    _feed(pc)
    a, b = pc.line()
    assert a == pytest.approx(1.5, abs=0.05) and b == pytest.approx(0.016, rel=0.02)


def test_budget_keeps_a_step_plus_pass_within_the_ratio():
    pc = PassCost(2.0)
    _feed(pc)
    assert pc.budget(64, 512) is None  # no decode step measured for the bucket yet
    for ms in (4.3, 4.3, 4.3):
        pc.observe("decode", 64, ms)
    for ms in (6.1, 6.1):
        pc.observe("decode", 128, ms)
    b64, b128 = pc.budget(64, 512), pc.budget(128, 512)
    assert b64 % 64 == 0 and b128 % 64 == 0 and 64 <= b64 < b128 <= 512
    for B, bud in ((64, b64), (128, b128)):
        step = pc.step_ms[B]
        assert 1.5 + 0.016 * bud <= (2.0 - 1.0) * step + 1e-6  # the pass fits in one step's time
        assert 1.5 + 0.016 * (bud + 64) > step                 # and is the largest multiple of 64 that does
    # a generous ratio is capped by the configured budget; a step too short for any pass still moves 64 tokens
    assert PassCost(10.0).budget(64, 512) is None
    big = PassCost(10.0)
    _feed(big)
    big.observe("decode", 64, 4.3)
    assert big.budget(64, 512) == 512
    tiny = PassCost(1.1)
    _feed(tiny)
    tiny.observe("decode", 64, 4.3)
    assert tiny.budget(64, 512) == 64


def test_decode_step_ema_and_bad_fits():
    pc = PassCost(2.0)
    pc.observe("decode", 64, 4.0)
    pc.observe("decode", 64, 5.0)
    assert pc.step_ms[64] == pytest.approx(4.2)
    # a falling cost line (noise) is not used
    for t, ms in ((128, 5.0), (512, 3.0), (256, 4.5)):
        pc.observe("prefill", t, ms)
    assert pc.line() is None and pc.budget(64, 512) is None


def test_engine_sizes_prefill_chunks_from_the_cost_model(monkeypatch):
    """Separate prefill passes (DSSE_MIXED=0).  With a PassCost attached (as DSSE_PREFILL_ITL_RATIO does on a GPU), a prompt arriving while streams decode is
    prefilled in chunks of the model's budget for the occupied bucket; a prompt starved past boost_steps gets the full
    PREFILL_BUDGET; the token streams equal the fixed-budget engine's (greedy)."""
    import torch

    from distributed_sse_for_llm_response_amd.engine.engine import LLMEngine, SamplingParams
    from distributed_sse_for_llm_response_amd.engine.model_runner import ModelRunner
    from distributed_sse_for_llm_response_amd.engine.weights import convert_standard
    from distributed_sse_for_llm_response_amd.models.mistral import TINY, init_standard_weights

    monkeypatch.setenv("DSSE_MIXED", "0")
    w = convert_standard(TINY, init_standard_weights(TINY, seed=11))

    def run(cost):
        r = ModelRunner(w, num_blocks=64, max_batch=4, max_model_len=512, device="cpu", use_graphs=False)
        e = LLMEngine(r, eos_id=-1, prefill_budget=256)
        e.cost = cost
        e.boost_steps = 3
        chunks = []
        orig = r.prefill

        def spy(seqs, ring_row):
            chunks.append(sum(len(s.tokens) for s in seqs))
            return orig(seqs, ring_row=ring_row)

        r.prefill = spy
        g = torch.Generator().manual_seed(3)
        out = {}
        e.add_request("a", torch.randint(3, TINY.vocab_size, (20,), generator=g).tolist(),
                      SamplingParams(temperature=0.0, max_tokens=12))
        long_prompt = torch.randint(3, TINY.vocab_size, (300,), generator=g).tolist()
        for step in range(400):
            if step == 2:
                e.add_request("b", long_prompt, SamplingParams(temperature=0.0, max_tokens=4))
            for ev in e.step():
                out.setdefault(ev.conversation_id, []).append(ev.token_id)
            if step > 2 and not e.has_work():
                break
        return chunks, out

    fixed_chunks, fixed_out = run(None)
    pc = PassCost(2.0)
    for t in (64, 128, 256, 128):
        pc.observe("prefill", t, 1.0 + 0.02 * t)
    pc.observe("decode", 1, 2.3)  # bucket 1 (one decoding stream): budget = (2.3 - 1.0) / 0.02 -> 64
    assert pc.budget(1, 256) == 64
    ad_chunks, ad_out = run(pc)
    assert fixed_out == ad_out
    assert 256 in fixed_chunks  # the long prompt's first pass at the fixed budget
    # adaptive: 64-token passes while "a" decodes, until the starvation guard hands the rest the full budget
    assert ad_chunks[1] == 64 and max(ad_chunks) <= 256 and len(ad_chunks) > len(fixed_chunks)


def test_mixed_chunk_from_measured_step_costs():
    """Mixed steps: the extra over the bucket's decode step is fitted against the replayed graph's chunk rows; the
    chunk is the largest captured size whose step stays within ratio x the decode step."""
    pc = PassCost(1.85)
    assert pc.mixed_chunk(128, [128, 256, 384, 512]) is None  # nothing measured yet
    pc.observe("mixed", (128, 256), 10.0)  # ignored: the bucket's decode step is unknown
    pc.observe("decode", 128, 6.0)
    assert pc.mixed_chunk(128, [128, 256, 384, 512]) is None
    pc.observe("mixed", (128, 256), 6.0 + 0.5 + 0.016 * 256)  # one size: proportional, 18 us / row
    assert pc.mixed_chunk(128, [128, 256, 384, 512]) == 256  # 5.1 ms of room / 17.95 us -> 284 rows
    for C in (128, 256, 384, 128, 256):
        pc.observe("mixed", (128, C), 6.0 + 0.5 + 0.016 * C)  # extra = 0.5 ms + 16 us per prompt row
    assert abs(pc.mixed_ms(128, 320) - (6.0 + 0.5 + 0.016 * 320)) < 1e-6
    # room: 0.85 x 6 = 5.1 ms -> C <= 287.5: 256 of the captured sizes
    assert pc.mixed_chunk(128, [128, 256, 384, 512]) == 256
    pc.observe("decode", 64, 2.0)  # room 1.7 ms: not even 128 rows fit -> the smallest size
    assert pc.mixed_chunk(64, [128, 256, 384, 512]) == 128
    pc.observe("decode", 256, 10.0)  # room 8.5 ms -> 500 rows: 384
    assert pc.mixed_chunk(256, [128, 256, 384, 512]) == 384


def test_mixed_backlog_split_into_even_chunks(monkeypatch):
    """A prompt backlog longer than the step's chunk goes out in even 64-row-rounded shares (the longest mixed step,
    which sets the ITL tail, stays short); the streams equal the separate-pass engine's (greedy)."""
    import torch

    from distributed_sse_for_llm_response_amd.engine.engine import LLMEngine, SamplingParams
    from distributed_sse_for_llm_response_amd.engine.model_runner import ModelRunner
    from distributed_sse_for_llm_response_amd.engine.weights import convert_standard
    from distributed_sse_for_llm_response_amd.models.mistral import TINY, init_standard_weights

    w = convert_standard(TINY, init_standard_weights(TINY, seed=12))

    def run(mixed):
        monkeypatch.setenv("DSSE_MIXED", mixed)
        monkeypatch.setenv("DSSE_MIXED_CHUNK", "256")
        r = ModelRunner(w, num_blocks=64, max_batch=4, max_model_len=512, device="cpu", use_graphs=False)
        e = LLMEngine(r, eos_id=-1, prefill_budget=512)
        sizes = []
        orig = r.mixed

        def spy(B, seqs, ring_row):
            sizes.append(sum(len(s.tokens) for s in seqs))
            return orig(B, seqs, ring_row=ring_row)

        r.mixed = spy
        g = torch.Generator().manual_seed(5)
        out = {}
        e.add_request("a", torch.randint(3, TINY.vocab_size, (20,), generator=g).tolist(),
                      SamplingParams(temperature=0.0, max_tokens=12))
        long_prompt = torch.randint(3, TINY.vocab_size, (300,), generator=g).tolist()
        for step in range(200):
            if step == 2:
                e.add_request("b", long_prompt, SamplingParams(temperature=0.0, max_tokens=4))
            for ev in e.step():
                out.setdefault(ev.conversation_id, []).append(ev.token_id)
            if step > 2 and not e.has_work():
                break
        return sizes, out

    mixed_sizes, mixed_out = run("1")
    sep_sizes, sep_out = run("0")
    assert mixed_out == sep_out
    assert sep_sizes == []
    assert mixed_sizes == [192, 108]  # 300 rows over two steps: ceil(150 / 64) * 64 = 192, then the rest


def test_tp_ranks_ignore_their_own_pass_costs(monkeypatch):
    """TP groups run the scheduler on every rank (deterministic mode).  Two ranks whose PassCost fits differ (each
    from its own GPU's event timings) must still pick identical chunk sizes, in mixed and in separate-pass mode:
    different row counts would replay different graphs and mismatch the collectives (engine.py)."""
    import torch

    from distributed_sse_for_llm_response_amd.engine.engine import LLMEngine, SamplingParams
    from distributed_sse_for_llm_response_amd.engine.model_runner import ModelRunner
    from distributed_sse_for_llm_response_amd.engine.weights import convert_standard
    from distributed_sse_for_llm_response_amd.models.mistral import TINY, init_standard_weights

    w = convert_standard(TINY, init_standard_weights(TINY, seed=13))

    def fake_cost(slope):
        pc = PassCost(2.0)
        for t in (64, 128, 256, 128):
            pc.observe("prefill", t, 1.0 + slope * t)
        pc.observe("decode", 1, 2.3)
        pc.observe("decode", 64, 2.0)
        for C in (128, 256, 384):
            pc.observe("mixed", (64, C), 2.0 + slope * C)
        return pc

    # mixed steps: _mixed_budget with captured sizes; the two "ranks" see different fits
    monkeypatch.setenv("DSSE_MIXED", "1")
    budgets = {}
    for det in (True, False):
        for slope in (0.001, 0.02):
            r = ModelRunner(w, num_blocks=64, max_batch=4, max_model_len=512, device="cpu", use_graphs=False)
            e = LLMEngine(r, eos_id=-1, prefill_budget=512, deterministic=det)
            e.cost = fake_cost(slope)
            r.mx_graphs = {1: object()}
            r.mixed_chunks = lambda B: [128, 256, 384]
            r.mixed_chunk = lambda B: 128
            budgets[(det, slope)] = e._mixed_budget(64)
    assert budgets[(False, 0.001)] != budgets[(False, 0.02)]  # the fits do move the chunk when not in TP mode
    assert budgets[(True, 0.001)] == budgets[(True, 0.02)] == 128

    # separate prefill passes: the chunk list of a whole run is identical across the two ranks
    monkeypatch.setenv("DSSE_MIXED", "0")

    def run(slope):
        r = ModelRunner(w, num_blocks=64, max_batch=4, max_model_len=512, device="cpu", use_graphs=False)
        e = LLMEngine(r, eos_id=-1, prefill_budget=256, deterministic=True)
        e.cost = fake_cost(slope)
        chunks = []
        orig = r.prefill

        def spy(seqs, ring_row):
            chunks.append(sum(len(s.tokens) for s in seqs))
            return orig(seqs, ring_row=ring_row)

        r.prefill = spy
        g = torch.Generator().manual_seed(3)
        e.add_request("a", torch.randint(3, TINY.vocab_size, (20,), generator=g).tolist(),
                      SamplingParams(temperature=0.0, max_tokens=8))
        long_prompt = torch.randint(3, TINY.vocab_size, (300,), generator=g).tolist()
        for step in range(300):
            if step == 2:
                e.add_request("b", long_prompt, SamplingParams(temperature=0.0, max_tokens=4))
            e.step()
            if step > 2 and not e.has_work():
                break
        return chunks

    assert run(0.001) == run(0.02)


def test_flash_split_plan_covers_every_key_block_once():
    """flash_split_plan (ModelRunner, the flash prefill key split): only an under-filled grid with long tiles is
    split; every tile's key blocks are covered once, by one direct item or by its consecutive slots."""
    from distributed_sse_for_llm_response_amd.engine.model_runner import flash_split_plan

    tiles = [(0, t, t + 1) for t in reversed(range(128))]  # an 8k prompt, fresh: tile t walks t + 1 blocks
    assert flash_split_plan(tiles, 8) is None               # 1024 workgroups: already fills the chip
    assert flash_split_plan(tiles[-20:], 1) is None         # short tiles only
    work, comb, nslots = flash_split_plan(tiles, 1)
    nw = len(work) // 5
    seq, tile, kb, slot = work[:nw], work[nw:2 * nw], work[2 * nw:4 * nw].reshape(nw, 2), work[4 * nw:]
    assert nw <= 256 and max(e - a for a, e in kb) <= 43  # one round of 256 workgroups
    ranges = {}
    for i in range(nw):
        ranges.setdefault(int(tile[i]), []).append((int(kb[i, 0]), int(kb[i, 1]), int(slot[i])))
    cmap = {int(comb[4 * c + 1]): (int(comb[4 * c + 2]), int(comb[4 * c + 3])) for c in range(len(comb) // 4)}
    for t, rs in ranges.items():
        rs.sort()
        assert rs[0][0] == 0 and rs[-1][1] == t + 1
        assert all(a[1] == b[0] for a, b in zip(rs, rs[1:]))
        if len(rs) == 1:
            assert rs[0][2] == -1 and t not in cmap
        else:
            s0, n = cmap[t]
            assert sorted(r[2] for r in rs) == list(range(s0, s0 + n))
    assert nslots == sum(n for _, n in cmap.values())
    assert (seq == 0).all()
