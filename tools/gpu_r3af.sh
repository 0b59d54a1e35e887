#!/bin/bash
# Round-3 step AF: prefill-chunk tile rule (257-1024 rows): GEMM tests, TTFT at 512 / 1024 / 8192 tokens, serving.
set -o pipefail
out=gpurun_out/${1:-r3af}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gemm_tiled_gpu.py tests/test_model_full_dims_gpu.py -x -q --timeout 300 --timeout-method thread > $out/pytest.log 2>&1 || exit 1
for n in 512 1024; do
  timeout -k 10 300 python3 tools/bench_ttft.py --prompt-len $n --iters 5 --decode-steps 4 > $out/ttft$n.log 2>&1 || exit 1
  DSSE_T_NARROW_CFG=1 timeout -k 10 300 python3 tools/bench_ttft.py --prompt-len $n --iters 5 --decode-steps 4 > $out/ttft${n}_old.log 2>&1 || exit 1
done
timeout -k 10 300 python3 tools/bench_ttft.py --prompt-len 8192 --iters 3 > $out/ttft8192.log 2>&1 || exit 1
timeout -k 10 400 python -u tools/bench_serving.py --rates 13 --requests 300 --max-tokens 1000 \
  --prefill-budget 512 > $out/serving13.jsonl 2> $out/serving13.err
