#!/bin/bash
# Round-3 step Y: serving under arrivals with early-drained first tokens published before the engine blocks
# (LLMEngine.on_flush), 13 req/s x 1000 and 40 req/s x 200 tokens; one 64-stream bench as a regression check.
set -o pipefail
out=gpurun_out/${1:-r3y}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $out/bench64.log 2>&1 || exit 1
timeout -k 10 400 python -u tools/bench_serving.py --rates 13 --requests 300 --max-tokens 1000 \
  --prefill-budget 512 > $out/serving13.jsonl 2> $out/serving13.err || exit 1
timeout -k 10 400 python -u tools/bench_serving.py --rates 40 --requests 600 --max-tokens 200 \
  --prefill-budget 512 > $out/serving40.jsonl 2> $out/serving40.err
