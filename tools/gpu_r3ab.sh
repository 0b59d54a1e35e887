#!/bin/bash
# Round-3 step AB: pipeline depth 1 vs 2, alternating: 64 / 256-stream benches, serving at 40 req/s.
set -o pipefail
out=gpurun_out/${1:-r3ab}
mkdir -p $out
export TMPDIR=/tmp
for i in 1 2; do for d in 1 2; do
  DSSE_PIPELINE_DEPTH=$d timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $out/bench64_d${d}_$i.log 2>&1 || exit 1
  DSSE_PIPELINE_DEPTH=$d timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --streams 256 > $out/bench256_d${d}_$i.log 2>&1 || exit 1
done; done
for d in 1 2; do
  DSSE_PIPELINE_DEPTH=$d timeout -k 10 400 python -u tools/bench_serving.py --rates 40 --requests 600 --max-tokens 200 \
    --prefill-budget 512 > $out/serving40_d$d.jsonl 2> $out/serving40_d$d.err || exit 1
done
