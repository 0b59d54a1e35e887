"""Checked-kernel run (SURVEY.md §5.2 "HIP-side bounds-check debug build").

Run with the checked library: ``DSSE_KERNELS_VARIANT=checked python tools/check_kernels.py``
(``python -m distributed_sse_for_llm_response_amd._build kernels-checked`` builds it).

1. A clean pass: the tiny Mistral through prefill + graph-captured decode must record no violation.
2. Corrupted inputs (a block-table page past the cache, a token id past the vocabulary, a KV slot past
   the cache, a RoPE position past the table) must each be caught and attributed to the right kernel
   file — without a GPU fault, because the checked build substitutes a safe index after recording.

Prints ``CHECKS-OK`` on success; exits non-zero otherwise.
"""
from __future__ import annotations

import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from distributed_sse_for_llm_response_amd import ops  # noqa: E402
from distributed_sse_for_llm_response_amd.engine.model_runner import ModelRunner, PrefillSeq  # noqa: E402
from distributed_sse_for_llm_response_amd.engine.weights import convert_standard  # noqa: E402
from distributed_sse_for_llm_response_amd.models.mistral import TINY, init_standard_weights  # noqa: E402


def expect(fn, file: str, what: str):
    ops.kernel_checks()  # clear
    fn()
    bad = ops.kernel_checks(raise_on_error=False)
    files = [b[0] for b in bad]
    if file not in files:
        raise SystemExit(f"{what}: expected a violation in {file}, got {bad}")
    print(f"caught {what}: {[b for b in bad if b[0] == file][0]}")


def main():
    dev = torch.device("cuda", 0)
    ops.load_library(required=True)
    if not torch.ops.dsse.kernels_checked():
        raise SystemExit("not the checked build: set DSSE_KERNELS_VARIANT=checked")

    # ---- 1. clean model run
    cfg = TINY
    w = convert_standard(cfg, init_standard_weights(cfg, seed=1), device=dev)
    r = ModelRunner(w, num_blocks=64, max_batch=4, max_model_len=512, device=dev, use_graphs=True)
    prompts = [[5, 17, 99, 3, 8, 1000, 42], list(range(100, 170)), [7] * 33]
    bts = [[0, 1, 2], [10, 4, 5, 6], [20, 21, 22]]
    for i, bt in enumerate(bts):
        r.block_tables[i, : len(bt)] = torch.tensor(bt, dtype=torch.int32)
    r.prefill([PrefillSeq(i, p, 0, bts[i], True) for i, p in enumerate(prompts)], ring_row=0)
    r.active[:3] = 1
    r.capture([4])
    for _ in range(6):
        r.decode(4)
    clean = ops.kernel_checks(raise_on_error=False)
    if clean:
        raise SystemExit(f"false positive on a valid model run: {clean}")
    print("clean model run: no violations")

    # ---- 2. corrupted inputs
    g = torch.Generator().manual_seed(0)
    nblk, hkv, hq = 8, 8, 32
    kc = torch.randn(nblk, hkv, 32, 128, generator=g).bfloat16().to(dev)
    vc = torch.randn(nblk, hkv, 128, 32, generator=g).bfloat16().to(dev)
    q = torch.randn(1, hq, 128, generator=g).bfloat16().to(dev)
    bt = torch.tensor([[0, 1, nblk + 1000]], dtype=torch.int32, device=dev)  # third page is past the cache
    i32 = dict(dtype=torch.int32, device=dev)
    out = torch.zeros_like(q)
    po = torch.zeros(8 * 16 * 128 * 4, device=dev)
    pml = torch.zeros(8 * 16 * 2 * 4, device=dev)

    expect(lambda: ops.paged_attention(0, q, kc, vc, bt, torch.zeros(1, **i32), torch.ones(1, **i32),
                                       torch.tensor([90], **i32), torch.zeros(1, **i32), torch.zeros(1, **i32),
                                       out, po, pml, 128, 1), "attention.hip", "decode attention: bad page id")

    qp = torch.randn(90, hq, 128, generator=g).bfloat16().to(dev)
    outp = torch.zeros_like(qp)
    expect(lambda: ops.paged_attention(2, qp, kc, vc, bt, torch.zeros(1, **i32), torch.tensor([90], **i32),
                                       torch.tensor([90], **i32), torch.zeros(math.ceil(90 / 64), **i32),
                                       torch.arange(math.ceil(90 / 64), **i32), outp, po, pml, 96, 1),
           "attention_prefill.hip", "flash prefill: bad page id")

    H = 1024
    emb = torch.randn(100, H, generator=g).bfloat16().to(dev)
    resid = torch.zeros(2, H, device=dev)
    y = torch.zeros(2, H, dtype=torch.bfloat16, device=dev)
    nw = torch.ones(H, dtype=torch.bfloat16, device=dev)
    expect(lambda: ops.rmsnorm(resid, nw, y, 1e-5, embed=emb, ids=torch.tensor([3, 100 + 7], **i32)),
           "elementwise.hip", "embedding gather: token id past the vocabulary")

    nkv, nh = 8, 32
    qkv = torch.randn(1, (nh + 2 * nkv) * 128, generator=g).bfloat16().to(dev)
    rope = torch.zeros(64, 64, 2, device=dev)
    qo = torch.zeros(1, nh, 128, dtype=torch.bfloat16, device=dev)
    expect(lambda: ops.rope_kv_write(qkv, torch.tensor([3], **i32), torch.tensor([nblk * 32 + 5], **i32), rope, qo,
                                     kc, vc, nh, nkv), "elementwise.hip", "KV write: slot past the cache")
    expect(lambda: ops.rope_kv_write(qkv, torch.tensor([64 + 9], **i32), torch.tensor([4], **i32), rope, qo,
                                     kc, vc, nh, nkv), "elementwise.hip", "RoPE: position past the table")

    act = torch.ones(1, **i32)
    expect(lambda: ops.decode_prep(act, torch.tensor([70], **i32), bt, torch.zeros(1, **i32), torch.zeros(1, **i32),
                                   torch.zeros(1, **i32), nblk), "elementwise.hip", "decode_prep: bad page id")
    torch.cuda.synchronize()
    print("CHECKS-OK")


if __name__ == "__main__":
    main()
