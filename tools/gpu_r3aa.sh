#!/bin/bash
# Round-3 step AA: engine pipeline depth (DSSE_PIPELINE_DEPTH 1 / 2 / 3) under arrivals (TTFT, ITL) and in the
# steady 64-stream bench.
set -o pipefail
out=gpurun_out/${1:-r3aa}
mkdir -p $out
export TMPDIR=/tmp
for d in 1 3 2; do
  DSSE_PIPELINE_DEPTH=$d timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $out/bench64_d$d.log 2>&1 || exit 1
  DSSE_PIPELINE_DEPTH=$d timeout -k 10 400 python -u tools/bench_serving.py --rates 13 --requests 300 --max-tokens 1000 \
    --prefill-budget 512 > $out/serving13_d$d.jsonl 2> $out/serving13_d$d.err || exit 1
done
