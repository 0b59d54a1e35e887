#!/bin/bash
# Round-3 step AL: separate passes vs 256-row mixed chunks at 20 / 30 req/s x 300 tokens (no long prompts).
set -o pipefail
out=gpurun_out/${1:-r3al}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 500 python -u tools/bench_serving.py --rates 20,30 --requests 600 --max-tokens 300 \
  --prefill-budget 512 > $out/separate.jsonl 2> $out/separate.err || exit 1
DSSE_MIXED=1 DSSE_MIXED_CHUNK=256 timeout -k 10 500 python -u tools/bench_serving.py --rates 20,30 --requests 600 \
  --max-tokens 300 --prefill-budget 512 > $out/mixed.jsonl 2> $out/mixed.err
