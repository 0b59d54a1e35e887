#!/bin/bash
# Round-3 step F: 256-row decode GEMM decompositions (gemm_tiled cfg knobs), A/B at 256 streams; new-config numerics.
set -o pipefail
out=gpurun_out/${1:-r3f}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -k "tiled or resid_split" -x -q --timeout 120 \
  --timeout-method thread > $out/pytest.log 2>&1 || exit 1
bash tools/ab_multi.sh r3f_ab256.log 256 2 "-" "DSSE_T_WIDE_CFG=4" "DSSE_T_NARROW_CFG=4" "DSSE_T_NARROW_CFG=5" \
  "DSSE_T_NARROW_CFG=6" "DSSE_T_WIDE_CFG=4 DSSE_T_NARROW_CFG=4"
mv gpurun_out/r3f_ab256.log $out/
