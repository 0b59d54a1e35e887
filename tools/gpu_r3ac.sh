#!/bin/bash
# Round-3 step AC: adaptive pipeline depth (1 while requests arrive, 2 otherwise; the new default): 64-stream
# benches and serving at 13 / 40 req/s.
set -o pipefail
out=gpurun_out/${1:-r3ac}
mkdir -p $out
export TMPDIR=/tmp
for i in 1 2; do timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $out/bench64_$i.log 2>&1 || exit 1; done
timeout -k 10 400 python -u tools/bench_serving.py --rates 13 --requests 300 --max-tokens 1000 \
  --prefill-budget 512 > $out/serving13.jsonl 2> $out/serving13.err || exit 1
timeout -k 10 400 python -u tools/bench_serving.py --rates 40 --requests 600 --max-tokens 200 \
  --prefill-budget 512 > $out/serving40.jsonl 2> $out/serving40.err
