#!/bin/bash
# Round-3 step AE: prefill-chunk GEMMs (512 / 1024 / 2048 rows) over every gemm_tiled config and split-K target,
# to re-tune the 129-512-row rule (chosen for the 256-stream decode bucket) for prompt chunks.
set -o pipefail
out=gpurun_out/${1:-r3ae}
mkdir -p $out
export TMPDIR=/tmp
for mw in 160 256 64 1; do
  DSSE_T_MIN_WGS=$mw timeout -k 10 300 python3 tools/bench_gemm_tiled.py --M 512,1024,2048 --cfg 0,1,2,3,4 \
    --no-library --rounds 3 --iters 10 > $out/gemm_minwgs$mw.log 2>&1 || exit 1
done
