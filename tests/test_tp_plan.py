"""TP plan wire format and channels (serving/tp.py): exact round trip of every admitted parameter (seeds above
2^31 included), the shared-memory rings and the gloo fallback delivering identical plans to every follower."""
import os
import socket

import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from distributed_sse_for_llm_response_amd.engine.engine import SamplingParams
from distributed_sse_for_llm_response_amd.serving.tp import (GlooPlanChannel, Plan, ShmPlanChannel, _messages,
                                                             _Reassembly)


def _plan(n_prompt=5):
    p = Plan(step=True)
    p.adds.append((7, list(range(n_prompt)), SamplingParams(temperature=0.7, top_p=0.9, top_k=40, max_tokens=33,
                                                            seed=(1 << 40) + 12345, ignore_eos=True), (1 << 52) + 99))
    p.adds.append((8, [1, 2, 3], SamplingParams(temperature=0.0, max_tokens=4), 5))
    p.aborts += [3, 4]
    p.flow += [(7, True), (9, False)]
    return p


def _key(plan):
    return (plan.step, plan.stop, plan.sync,
            [(rid, list(pr), sp.temperature, sp.top_p, sp.top_k, sp.max_tokens, sp.seed, sp.ignore_eos, arr)
             for rid, pr, sp, arr in plan.adds], list(plan.aborts), list(plan.flow))


def test_plan_roundtrip_keeps_large_seeds_and_float32_params():
    p = _plan()
    q = p.roundtrip()
    assert q.adds[0][2].seed == (1 << 40) + 12345  # was cut to 31 bits before round 3
    assert q.adds[0][3] == (1 << 52) + 99
    assert q.adds[1][2].seed is None
    assert abs(q.adds[0][2].temperature - 0.7) < 1e-7 and q.adds[0][2].top_k == 40 and q.adds[0][2].ignore_eos
    assert q.aborts == [3, 4] and q.flow == [(7, True), (9, False)]
    assert _key(q.roundtrip()) == _key(q)  # decoding is a fixed point: leader and followers apply the same plan


def test_plan_rejects_out_of_range_seed():
    p = Plan(step=True)
    p.adds.append((1, [1], SamplingParams(seed=1 << 62), 0))
    with pytest.raises(ValueError):
        p.encode()


def test_large_plan_is_split_and_reassembled():
    p = _plan(n_prompt=3000)
    msgs = _messages(p, room=1000)
    assert len(msgs) > 3
    re = _Reassembly()
    got = [re.feed(m) for m in msgs]
    assert all(g is None for g in got[:-1])
    assert _key(got[-1]) == _key(p.roundtrip())


def test_empty_step_plan_is_one_header():
    msgs = _messages(Plan(step=True), room=1000)
    assert len(msgs) == 1 and len(msgs[0]) == 6  # 24 bytes per follower per idle step


def _worker(rank, world, port, kind, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        ranks = list(range(world))
        ch = (ShmPlanChannel(None, 0, rank, ranks, tag=f"test-{port}") if kind == "shm"
              else GlooPlanChannel(None, 0))
        plans = [Plan(step=True), _plan(), _plan(n_prompt=300_000), Plan(sync=True), Plan(stop=True)]
        if rank == 0:
            for p in plans:
                ch.send(p)
            out[rank] = [_key(p.roundtrip()) for p in plans]
        else:
            got = []
            while True:
                p = ch.recv()
                got.append(_key(p))
                if p.stop:
                    break
            out[rank] = got
        dist.barrier()
    finally:
        dist.destroy_process_group()


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.timeout(300)
@pytest.mark.parametrize("kind", ["shm", "gloo"])
def test_plan_channel_delivers_identical_plans(kind):
    world = 3
    with mp.Manager() as m:
        out = m.dict()
        mp.spawn(_worker, args=(world, _port(), kind, out), nprocs=world, join=True)
        res = [out[r] for r in range(world)]
    assert res[1] == res[0] and res[2] == res[0]
