#!/bin/bash
# Round-3 soak: 2000 requests at 30 req/s (300 tokens, some 4k-token prompts) through POST /chat on the default
# tree, then the same with mixed steps: every request must complete with no client error.
set -o pipefail
out=gpurun_out/${1:-r3soak}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 500 python -u tools/bench_serving.py --rates 30 --requests 2000 --max-tokens 300 --long-every 100 \
  --long-words 4000 --prefill-budget 512 > $out/soak_default.jsonl 2> $out/soak_default.err || exit 1
DSSE_MIXED=1 DSSE_MIXED_CHUNK=256 timeout -k 10 500 python -u tools/bench_serving.py --rates 30 --requests 1000 \
  --max-tokens 300 --prefill-budget 512 > $out/soak_mixed.jsonl 2> $out/soak_mixed.err
