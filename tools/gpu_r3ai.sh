#!/bin/bash
# Round-3 step AI: 65-128-row bucket GEMMs: the default dispatch (ring2 / gemm_wide) vs every gemm_tiled config.
set -o pipefail
out=gpurun_out/${1:-r3ai}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python3 tools/bench_gemm_tiled.py --M 96,128 --cfg auto,0,1,3,4 --no-library --rounds 3 \
  --iters 20 > $out/gemm_m128.log 2>&1
