"""Anatomy of the captured decode step from in-kernel stamps (where the 64-stream step's time
above its byte floor goes, split per kernel into first-load latency, steady stream and tail).

    DSSE_KERNELS_VARIANT=stamps python tools/step_stamps.py [--streams 64] [--steps 4] [--out stamps.json]
    python tools/step_stamps.py --analyse stamps.json
    rocprofv3 --pmc ... -- python3 tools/step_stamps.py --pmc-pass    (eager steps for a counter pass)

Needs the diagnostic `stamps` build (`python -c "from distributed_sse_for_llm_response_amd import _build;
_build.build_kernels(variant='stamps')"`; `.gpurunignore` keeps it off GPU pushes, so drop that line for a run on the
box; common.h `stamps::record`): every wave of the
ring GEMMs (`gemm_ring_kernel`: qkv, o, down, gate_up, LM head at 17-64 rows) and of `rmsnorm_kernel` appends
[tag, grid, block, t0, t1, t2, t3, wave] with s_memrealtime (100 MHz, one clock for the whole chip) into one of 256
sub-buffers (by workgroup; a single shared record counter serialised the waves' exits and stretched every kernel):

  * ring GEMM: t0 entry, t1 first K chunk (X + weights) landed in LDS for the whole workgroup, t2 K loop done
    (every DMA drained), t3 epilogue stores drained;
  * RMSNorm: t0 entry, t1 the row (and its split-K slabs) loaded, t2 block reduction done, t3 stores drained.

The TP = 1 Mistral-7B runner (random-init bf16 weights, synthetic prompts of --prompt-len tokens, the bench.py
shape) captures its decode graph; the stamped steps are graph replays after --warmup replays.  Launches are
recovered by sorting records by t0 (kernels of one stream never overlap: a record whose t0 is past the current
launch's last t3 opens the next launch).  Per launch class (tag, mode, grid): span (first t0 -> last t3), start
spread (last t0 - first t0: dispatch ramp), median first-load, stream and tail per wave, end spread (last t3 -
median t3: stragglers), and the idle gap to the previous stamped launch's end.
"""
from __future__ import annotations

import argparse
import collections
import gzip
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

TAGS = {1: "ring", 2: "rmsnorm", 3: "attn", 4: "pipe"}
US = 0.01  # s_memrealtime tick, us


def collect(args):
    import torch

    from distributed_sse_for_llm_response_amd import ops
    from distributed_sse_for_llm_response_amd.engine.kv_cache import PAGE, blocks_needed
    from distributed_sse_for_llm_response_amd.engine.model_runner import ModelRunner, PrefillSeq
    from distributed_sse_for_llm_response_amd.engine.weights import random_engine_weights
    from distributed_sse_for_llm_response_amd.models.mistral import MISTRAL_7B_V03

    ops.load_library(required=True)
    device = torch.device("cuda", 0)
    torch.cuda.set_device(device)
    cfg = MISTRAL_7B_V03
    w = random_engine_weights(cfg, device=device, seed=7)
    B = args.streams
    max_len = args.max_model_len
    per_stream = blocks_needed(args.prompt_len + args.steps + args.warmup + 2 * PAGE)
    r = ModelRunner(w, num_blocks=B * per_stream + 8, max_batch=B, max_model_len=max_len, device=device,
                    use_graphs=not args.pmc_pass)
    if not args.pmc_pass:
        r.capture([B])
    gen = torch.Generator().manual_seed(5)
    tables = [list(range(i * per_stream, (i + 1) * per_stream)) for i in range(B)]
    for i, bt in enumerate(tables):
        r.block_tables[i, : len(bt)] = torch.tensor(bt, dtype=torch.int32)
    prompts = [torch.randint(3, cfg.vocab_size, (args.prompt_len,), generator=gen).tolist() for _ in range(B)]
    per_pass = max(1, 8192 // args.prompt_len)
    for a in range(0, B, per_pass):
        r.prefill([PrefillSeq(i, prompts[i], 0, tables[i], True) for i in range(a, min(B, a + per_pass))], ring_row=0)
    r.active[:B] = 1
    r.temperature[:B] = 0.0
    for _ in range(args.warmup):
        r.decode(B)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(args.steps):
        r.decode(B)
    e1.record()
    torch.cuda.synchronize()
    step_ms = e0.elapsed_time(e1) / args.steps
    if args.pmc_pass:  # eager decode steps for rocprofv3 --pmc (tools/gpu_run.sh pmc64); no stamps
        print(json.dumps({"streams": B, "eager_step_ms": step_ms, "health": r.health.cpu().tolist()}))
        r.close()
        return None
    armed = torch.ops.dsse.step_stamps_arm(0, args.cap)
    if not armed:
        raise SystemExit("the default kernel build records no stamps: run with DSSE_KERNELS_VARIANT=stamps")
    e0.record()
    for _ in range(args.steps):
        r.decode(B)
    e1.record()
    torch.cuda.synchronize()
    stamped_ms = e0.elapsed_time(e1) / args.steps
    rec = torch.ops.dsse.step_stamps_read(0)
    torch.ops.dsse.step_stamps_arm(0, 0)
    out = {"streams": B, "prompt_len": args.prompt_len, "steps": args.steps, "step_ms_unstamped_replays": step_ms,
           "step_ms_stamped": stamped_ms,
           "records": rec.tolist(), "health": r.health.cpu().tolist()}
    r.close()
    return out


def launches(records):
    """Group records into launches (see the module docstring)."""
    rows = sorted(records, key=lambda x: x[3])
    out, cur = [], None
    for x in rows:
        key = (x[0], x[1])
        if cur is None or key != cur["key"] or x[3] > cur["t3max"]:
            cur = {"key": key, "recs": [], "t3max": x[6]}
            out.append(cur)
        cur["recs"].append(x)
        cur["t3max"] = max(cur["t3max"], x[6])
    return out


def analyse(data, md=False):
    L = launches(data["records"])
    by = collections.defaultdict(list)
    prev_end = None
    for la in L:
        rs = la["recs"]
        t0 = [x[3] for x in rs]
        t1 = [x[4] for x in rs]
        t2 = [x[5] for x in rs]
        t3 = [x[6] for x in rs]
        tag, grid = la["key"]
        m = {
            "span": (max(t3) - min(t0)) * US,
            "start_spread": (max(t0) - min(t0)) * US,
            "first": statistics.median(b - a for a, b in zip(t0, t1)) * US,
            "stream": statistics.median(b - a for a, b in zip(t1, t2)) * US,
            "tail": statistics.median(b - a for a, b in zip(t2, t3)) * US,
            "end_spread": (max(t3) - statistics.median(t3)) * US,
            "gap": None if prev_end is None else (min(t0) - prev_end) * US,
            "waves": len(rs),
        }
        prev_end = max(t3)
        name = f"{TAGS.get(tag & 0xFF, tag & 0xFF)} mode {(tag >> 8) & 0xF}{' fix' if tag >> 12 & 1 else ''}"
        by[(name, f"{grid & 0xFFFFFFFF}x{grid >> 32}")].append(m)
    steps = max(1, data.get("steps", 1))
    lines = []
    lines.append(f"streams {data['streams']}, {steps} stamped steps, {len(L)} stamped launches, "
                 f"replays {data.get('step_ms_unstamped_replays', 0):.4f} ms/step unstamped, "
                 f"{data.get('step_ms_stamped', 0):.4f} stamped")
    hdr = ["kernel", "grid", "launches/step", "waves", "span", "start spread", "first load", "stream", "tail",
           "end spread", "gap before", "us/step"]
    lines.append("| " + " | ".join(hdr) + " |")
    lines.append("|" + "---|" * len(hdr))
    for (name, grid), ms in sorted(by.items(), key=lambda kv: -sum(m["span"] for m in kv[1])):
        def med(k):
            v = [m[k] for m in ms if m[k] is not None]
            return statistics.median(v) if v else float("nan")
        lines.append(
            f"| {name} | {grid} | {len(ms) / steps:.0f} | {ms[0]['waves']} | {med('span'):.2f} | "
            f"{med('start_spread'):.2f} | {med('first'):.2f} | {med('stream'):.2f} | {med('tail'):.2f} | "
            f"{med('end_spread'):.2f} | {med('gap'):.2f} | {sum(m['span'] for m in ms) / steps:.1f} |")
    text = "\n".join(lines)
    print(text)
    return text


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--streams", type=int, default=64)
    ap.add_argument("--prompt-len", type=int, default=512)
    ap.add_argument("--max-model-len", type=int, default=4096)
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--warmup", type=int, default=8)
    ap.add_argument("--cap", type=int, default=1 << 12, help="records per sub-buffer (256 sub-buffers)")
    ap.add_argument("--out", default=None)
    ap.add_argument("--analyse", default=None)
    ap.add_argument("--md", action="store_true")
    ap.add_argument("--pmc-pass", action="store_true", help="eager decode steps, no stamps (a counter pass)")
    args = ap.parse_args()
    if args.analyse:
        with (gzip.open if args.analyse.endswith(".gz") else open)(args.analyse, "rt") as f:
            analyse(json.load(f), args.md)
        return
    data = collect(args)
    if data is None:
        return
    if args.out:  # records as [n, 8] int lists; .gz: gzip (a 4-step record set is tens of MB as text)
        with (gzip.open if args.out.endswith(".gz") else open)(args.out, "wt") as f:
            json.dump(data, f)
    analyse(data)


if __name__ == "__main__":
    main()
