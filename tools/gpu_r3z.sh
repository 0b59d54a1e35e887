#!/bin/bash
# Round-3 step Z: GPU suite + smoke after removing the row-split norm kernel; 64-stream bench; serving at 40 req/s
# twice (TTFT p99 spread of the early-publish change).
set -o pipefail
out=gpurun_out/${1:-r3z}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $out/smoke.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $out/bench64.log 2>&1 || exit 1
for i in 1 2; do
  timeout -k 10 400 python -u tools/bench_serving.py --rates 40 --requests 600 --max-tokens 200 \
    --prefill-budget 512 > $out/serving40_$i.jsonl 2> $out/serving40_$i.err || exit 1
done
