#!/bin/bash
# Round-3 step AG: 192 / 256-row decode-bucket GEMMs over every gemm_tiled config and split target (isolated).
set -o pipefail
out=gpurun_out/${1:-r3ag}
mkdir -p $out
export TMPDIR=/tmp
for mw in 160 256; do
  DSSE_T_MIN_WGS=$mw timeout -k 10 300 python3 tools/bench_gemm_tiled.py --M 192,256 --cfg 0,1,2,3,4 \
    --no-library --rounds 3 --iters 20 > $out/gemm_minwgs$mw.log 2>&1 || exit 1
done
