"""The production TP decode step, captured: 2 and 4 TP ranks sharing the one MI355X, the Mistral-7B dimensions (two
layers), decode graphs of buckets 1 and 64 captured and replayed 200 times.  The step's collectives are the
hand-written IPC kernels only (allreduce.hip: the fused all-reduce + RMSNorm twice per layer and the candidate
all-gather), so nothing in it needs RCCL -- the ranks' host group is gloo here, which cannot be captured at all.

Checks: every rank samples the same token at every replay; the first replays' full logits (the ranks' vocab shards
concatenated) match the fp32 ``reference_forward`` of the same weights and the TP = 1 engine within bf16 tolerance;
the health word (a timed-out peer wait) stays clear.  Reference: SURVEY.md §2.4 C1-C3, VERDICT round 4 item 4."""
import math
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from distributed_sse_for_llm_response_amd.models.mistral import MistralConfig, init_standard_weights, reference_forward

pytestmark = pytest.mark.gpu

CFG = MistralConfig(name="mistral-7b-dims-2l", num_layers=2)  # every dimension of v0.3, two layers
PAGES = 10          # 32-token pages per sequence: prompts <= 60 tokens + 200 generated < 320
REPLAYS = 200
B64 = 64


def _prompts():
    g = torch.Generator().manual_seed(77)
    return [torch.randint(3, CFG.vocab_size, (int(torch.randint(3, 61, (1,), generator=g)),), generator=g).tolist()
            for _ in range(B64)]


def _run_rank(rank, world, gpu):
    """Prefill, then phase 1 (bucket 1, one sequence, 20 replays) and phase 2 (bucket 64, 64 sequences, 200
    replays).  Returns the tokens of every replay and the first two replays' logits (this rank's vocab shard)."""
    from distributed_sse_for_llm_response_amd import ops
    from distributed_sse_for_llm_response_amd.engine.model_runner import ModelRunner, PrefillSeq
    from distributed_sse_for_llm_response_amd.engine.weights import convert_standard
    from distributed_sse_for_llm_response_amd.parallel.comm import TPComm

    ops.load_library(required=True)
    std = init_standard_weights(CFG, seed=3, device=gpu)
    comm = TPComm(rank=rank, size=world) if world > 1 else TPComm()
    w = convert_standard(CFG, std, tp_rank=rank, tp_size=world, device=gpu)
    del std
    r = ModelRunner(w, num_blocks=B64 * PAGES + 8, max_batch=B64, max_model_len=512, device=gpu, comm=comm)
    if world > 1:
        assert r.ipc_decode(), f"IPC collectives not up: {r.fast_ar_reason}"
    r.capture([1, B64])
    assert r.use_graphs and set(r.graphs) == {1, B64}, "decode graphs were not captured"
    out = {}
    prompts = _prompts()
    for phase, (B, steps) in enumerate(((1, 20), (B64, REPLAYS))):
        tables = [list(range(i * PAGES, (i + 1) * PAGES)) for i in range(B)]
        r.block_tables.zero_()
        for i, bt in enumerate(tables):
            r.block_tables[i, : len(bt)] = torch.tensor(bt, dtype=torch.int32)
        r.prefill([PrefillSeq(i, prompts[i], 0, tables[i], True) for i in range(B)], ring_row=0)
        r.active.zero_()
        r.active[:B] = 1
        r.temperature.zero_()
        toks = [r.ids[:B].cpu().tolist()]
        logits = []
        for s in range(steps):
            r.decode(B)  # the captured graph of bucket B
            if s < 2:
                torch.cuda.synchronize(gpu)
                logits.append(r.logits[:B].cpu())
            toks.append(r.ids[:B].cpu().tolist())
        torch.cuda.synchronize(gpu)
        out[phase] = (toks, logits)
    health = r.health.cpu().tolist()
    r.close()
    return out, health


def _worker(rank, world, port, res):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        res[rank] = _run_rank(rank, world, torch.device("cuda", 0))
    finally:
        dist.destroy_process_group()


def _compare(ref_row, got_row, what):
    ref_row, got_row = ref_row.float(), got_row.float()
    cos = torch.nn.functional.cosine_similarity(ref_row, got_row, dim=0).item()
    rel = ((ref_row - got_row).abs().max() / ref_row.abs().max()).item()
    assert cos > 0.998 and rel < 0.05, f"{what}: cosine {cos:.5f}, max-abs err / max {rel:.4f}"
    return cos, rel


@pytest.fixture(scope="module")
def tp1():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return _run_rank(0, 1, torch.device("cuda", 0))


@pytest.mark.timeout(600)
@pytest.mark.parametrize("world", [2, 4])
def test_tp_decode_graph_ipc_collectives(tp1, world):
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    with mp.get_context("spawn").Manager() as m:
        res = m.dict()
        mp.spawn(_worker, args=(world, port, res), nprocs=world, join=True)
        res = [res[q] for q in range(world)]
    for q in range(world):
        assert not any(res[q][1]), f"rank {q} health words set: {res[q][1]} (a peer wait timed out)"
    gpu = torch.device("cuda", 0)
    std = init_standard_weights(CFG, seed=3, device=gpu)
    prompts = _prompts()
    one, _ = tp1
    worst = (1.0, 0.0)
    for phase in (0, 1):
        toks = res[0][0][phase][0]
        for q in range(1, world):
            assert res[q][0][phase][0] == toks, f"phase {phase}: TP ranks disagree on the sampled tokens"
        B = len(toks[0])
        assert len(toks) == (21 if phase == 0 else REPLAYS + 1)
        # full-vocab logits of the first two replays: the ranks' shards in rank order
        full = [torch.cat([res[q][0][phase][1][s] for q in range(world)], dim=1) for s in range(2)]
        tp1_logits = one[phase][1]
        rows = range(B) if B == 1 else range(0, B, 4)
        for i in rows:
            gen = [toks[s][i] for s in range(3)]
            ids = torch.tensor(prompts[i] + gen[:2], device=gpu)
            ref, _ = reference_forward(CFG, std, ids)
            L = len(prompts[i])
            for s in range(2):
                c, e = _compare(ref[L + s].cpu(), full[s][i], f"TP={world} phase {phase} seq {i} replay {s} vs fp32")
                worst = (min(worst[0], c), max(worst[1], e))
                if one[phase][0][s][i] == gen[s]:  # same history as the TP = 1 run: logits within bf16 tolerance
                    _compare(tp1_logits[s][i], full[s][i], f"TP={world} phase {phase} seq {i} replay {s} vs TP=1")
    print(f"TP={world}: worst cosine vs fp32 {worst[0]:.6f}, worst max-abs / max {worst[1]:.4f}")
    assert not math.isnan(worst[0])
