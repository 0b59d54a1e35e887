#!/bin/bash
# Round-3 step V: mixed prefill+decode steps (DSSE_MIXED=1) vs separate passes after the non-blocking first-token
# sampling fix, at 13 req/s x 1000 tokens and 40 req/s x 200 tokens.
set -o pipefail
out=gpurun_out/${1:-r3v}
mkdir -p $out
export TMPDIR=/tmp
DSSE_MIXED=1 DSSE_TRACE=$out/trace_mixed13.jsonl timeout -k 10 400 python -u tools/bench_serving.py --rates 13 --requests 300 \
  --max-tokens 1000 --prefill-budget 2048 > $out/mixed13.jsonl 2> $out/mixed13.err || exit 1
DSSE_MIXED=1 timeout -k 10 400 python -u tools/bench_serving.py --rates 40 --requests 600 \
  --max-tokens 200 --prefill-budget 2048 > $out/mixed40.jsonl 2> $out/mixed40.err || exit 1
timeout -k 10 400 python -u tools/bench_serving.py --rates 40 --requests 600 \
  --max-tokens 200 --prefill-budget 512,2048 > $out/separate40.jsonl 2> $out/separate40.err
