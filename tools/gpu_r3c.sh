#!/bin/bash
# Round-3 step C: TP rehearsal tests (IPC all-reduce engaged), whole-model numerics, QKV ring A/B, serving under
# Poisson arrivals, config 5 on the box CPU.
set -o pipefail
out=gpurun_out/${1:-r3c}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_tp_gpu.py tests/test_model_full_dims_gpu.py -x -v --timeout 240 \
  --timeout-method thread > $out/pytest_tp.log 2>&1
echo "rc=$?" >> $out/pytest_tp.log
bash tools/ab_multi.sh r3c_qkv.log 64 1 "DSSE_QKV_NW=6 DSSE_QKV_SPLIT=4" "-" "DSSE_QKV_SPLIT=4" && mv gpurun_out/r3c_qkv.log $out/ &&
timeout -k 10 400 python -u tools/bench_serving.py --rates 40,70 --requests 500 --max-tokens 200 --prefill-budget 512,2048 \
  > $out/serving.jsonl 2> $out/serving.err &&
timeout -k 10 300 python -u tools/bench_serving.py --rates 60 --requests 400 --max-tokens 200 --prefill-budget 1024 \
  --long-every 40 --long-words 8000 > $out/serving_long.jsonl 2> $out/serving_long.err
bash tools/config5_box.sh r3c/config5
