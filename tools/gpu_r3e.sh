#!/bin/bash
# Round-3 step E: mixed-step numerics, fill-rate microbenchmark, serving under arrivals mixed vs separate.
set -o pipefail
out=gpurun_out/${1:-r3e}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_model_full_dims_gpu.py -x -v --timeout 200 --timeout-method thread \
  > $out/pytest.log 2>&1 || exit 1
timeout -k 10 120 ./tools/fillbench > $out/fillbench.log 2>&1 || exit 1
for mixed in 1 0; do
  DSSE_MIXED=$mixed timeout -k 10 300 python -u tools/bench_serving.py --rates 13 --requests 300 --max-tokens 1000 \
    > $out/serving_moderate_mixed$mixed.jsonl 2> $out/serving_moderate_mixed$mixed.err || exit 1
  DSSE_MIXED=$mixed timeout -k 10 300 python -u tools/bench_serving.py --rates 40 --requests 500 --max-tokens 200 \
    > $out/serving_heavy_mixed$mixed.jsonl 2> $out/serving_heavy_mixed$mixed.err || exit 1
done
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > $out/bench64.log 2>&1
