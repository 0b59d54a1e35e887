#!/bin/bash
# Round-3 step AD: default tree (pipeline depth 1): GPU suite, smoke, 64 / 256-stream benches, serving 13 / 40 req/s.
set -o pipefail
out=gpurun_out/${1:-r3ad}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $out/smoke.log 2>&1 || exit 1
for i in 1 2 3; do timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $out/bench64_$i.log 2>&1 || exit 1; done
for i in 1 2; do timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --streams 256 > $out/bench256_$i.log 2>&1 || exit 1; done
timeout -k 10 400 python -u tools/bench_serving.py --rates 13 --requests 300 --max-tokens 1000 \
  --prefill-budget 512 > $out/serving13.jsonl 2> $out/serving13.err || exit 1
timeout -k 10 400 python -u tools/bench_serving.py --rates 40 --requests 600 --max-tokens 200 \
  --prefill-budget 512 > $out/serving40.jsonl 2> $out/serving40.err
