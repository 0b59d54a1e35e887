#!/bin/bash
# Round-3 step K: captured mixed prefill + decode steps -- numerics, then serving under Poisson arrivals, mixed
# (captured) vs separate prefill passes.
set -o pipefail
out=gpurun_out/${1:-r3k}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_model_full_dims_gpu.py -x -v --timeout 300 --timeout-method thread \
  > $out/pytest.log 2>&1 || exit 1
for mixed in 1 0; do
  DSSE_MIXED=$mixed timeout -k 10 300 python -u tools/bench_serving.py --rates 13 --requests 300 --max-tokens 1000 \
    > $out/serving_moderate_mixed$mixed.jsonl 2> $out/serving_moderate_mixed$mixed.err || exit 1
  DSSE_MIXED=$mixed timeout -k 10 300 python -u tools/bench_serving.py --rates 40 --requests 500 --max-tokens 200 \
    > $out/serving_heavy_mixed$mixed.jsonl 2> $out/serving_heavy_mixed$mixed.err || exit 1
done
