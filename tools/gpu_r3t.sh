#!/bin/bash
# Round-3 step T: engine step trace (DSSE_TRACE) under Poisson arrivals at 13 req/s, budgets 512 and 128, to
# attribute the in-flight ITL tail (p99 26-37 ms, max 130-205 ms in every serving run so far).
set -o pipefail
out=gpurun_out/${1:-r3t}
mkdir -p $out
export TMPDIR=/tmp
for b in 512 128; do
  DSSE_TRACE=$out/trace_b$b.jsonl timeout -k 10 400 python -u tools/bench_serving.py --rates 13 --requests 300 \
    --max-tokens 1000 --prefill-budget $b > $out/serving_b$b.jsonl 2> $out/serving_b$b.err || exit 1
done
