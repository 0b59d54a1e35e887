#!/bin/bash
# Round-3 step AM: DSSE_MIXED=auto (mixed 256-row chunks only from the 192-row decode bucket up) vs separate
# passes: the 30 req/s soak with 4k prompts, and 13 req/s (where auto must equal separate).
set -o pipefail
out=gpurun_out/${1:-r3am}
mkdir -p $out
export TMPDIR=/tmp
DSSE_MIXED=auto timeout -k 10 500 python -u tools/bench_serving.py --rates 30 --requests 2000 --max-tokens 300 \
  --long-every 100 --long-words 4000 --prefill-budget 512 > $out/soak_auto.jsonl 2> $out/soak_auto.err || exit 1
DSSE_MIXED=auto timeout -k 10 400 python -u tools/bench_serving.py --rates 13 --requests 300 --max-tokens 1000 \
  --prefill-budget 512 > $out/auto13.jsonl 2> $out/auto13.err || exit 1
timeout -k 10 500 python -u tools/bench_serving.py --rates 30 --requests 2000 --max-tokens 300 \
  --long-every 100 --long-words 4000 --prefill-budget 512 > $out/soak_separate.jsonl 2> $out/soak_separate.err
