#!/bin/bash
# Round-3 step W: mixed prefill+decode steps with a fixed prompt chunk (DSSE_MIXED_CHUNK 512 / 256: a whole short
# prompt rides in one decode step) vs separate passes (budget 512), 13 req/s x 1000 and 40 req/s x 200 tokens.
set -o pipefail
out=gpurun_out/${1:-r3w}
mkdir -p $out
export TMPDIR=/tmp
for c in 512 256; do
  DSSE_MIXED=1 DSSE_MIXED_CHUNK=$c timeout -k 10 400 python -u tools/bench_serving.py --rates 13,40 --requests 300 \
    --max-tokens 1000 --prefill-budget 512 > $out/mixed_c$c.jsonl 2> $out/mixed_c$c.err || exit 1
done
timeout -k 10 400 python -u tools/bench_serving.py --rates 13,40 --requests 300 --max-tokens 1000 \
  --prefill-budget 512 > $out/separate.jsonl 2> $out/separate.err
