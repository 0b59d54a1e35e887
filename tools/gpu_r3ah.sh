#!/bin/bash
# Round-3 step AH: 256 / 192-stream step with the per-shape narrow rule (qkv, down on 256x128; o on 128x128) vs
# the round-2 rule (all narrow on 128x128: DSSE_T_NARROW_CFG=1), alternating; decode-bucket GEMM tests.
set -o pipefail
out=gpurun_out/${1:-r3ah}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -k "decode_bucket or qkv_attention or resid" -x -q --timeout 300 --timeout-method thread > $out/pytest.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_model_full_dims_gpu.py -x -q --timeout 300 --timeout-method thread > $out/pytest_model.log 2>&1 || exit 1
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --streams 256 > $out/bench256_new_$i.log 2>&1 || exit 1
  DSSE_T_NARROW_CFG=1 timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --streams 256 > $out/bench256_old_$i.log 2>&1 || exit 1
done
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --streams 192 > $out/bench192_new.log 2>&1 || exit 1
DSSE_T_NARROW_CFG=1 timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --streams 192 > $out/bench192_old.log 2>&1
