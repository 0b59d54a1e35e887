#!/bin/bash
# Round-3 step AJ: mixed steps with a 256-row chunk on the final tree (pipeline depth 1, early first tokens).
set -o pipefail
out=gpurun_out/${1:-r3aj}
mkdir -p $out
export TMPDIR=/tmp
DSSE_MIXED=1 DSSE_MIXED_CHUNK=256 timeout -k 10 400 python -u tools/bench_serving.py --rates 13 --requests 300 \
  --max-tokens 1000 --prefill-budget 512 > $out/mixed13.jsonl 2> $out/mixed13.err || exit 1
DSSE_MIXED=1 DSSE_MIXED_CHUNK=256 timeout -k 10 400 python -u tools/bench_serving.py --rates 40 --requests 600 \
  --max-tokens 200 --prefill-budget 512 > $out/mixed40.jsonl 2> $out/mixed40.err
