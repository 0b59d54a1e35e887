#!/bin/bash
# Round-3 step G: ring2 (decoupled weight look-ahead) and tiled2 (separate X / W rings) numerics; A/B at
# 64 / 128 / 256 streams.
set -o pipefail
out=gpurun_out/${1:-r3g}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py \
  -k "ring or resid_split or gemm_out or gemm_silu or qkv or tiled or decode_bucket" \
  -x -q --timeout 120 --timeout-method thread > $out/pytest.log 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest tests/test_model_full_dims_gpu.py -x -q --timeout 200 --timeout-method thread \
  > $out/pytest_model.log 2>&1 || exit 1
bash tools/ab_multi.sh r3g_ring64.log 64 3 "DSSE_RING2=0" "-" || exit 1
mv gpurun_out/r3g_ring64.log $out/
bash tools/ab_multi.sh r3g_ab256.log 256 1 "-" "DSSE_T_NARROW_CFG=7" "DSSE_T_NARROW_CFG=9" "DSSE_T_WIDE_CFG=8" \
  "DSSE_T_NARROW_CFG=7 DSSE_T_WIDE_CFG=8" || exit 1
mv gpurun_out/r3g_ab256.log $out/
bash tools/ab_multi.sh r3g_ring128.log 128 2 "DSSE_RING2=0" "-" || exit 1
mv gpurun_out/r3g_ring128.log $out/
