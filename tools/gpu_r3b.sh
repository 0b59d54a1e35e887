#!/bin/bash
# Round-3 step B: IPC all-reduce multi-process test, ring GEMM numerics, split/nw A/B at 64 streams.
set -o pipefail
out=gpurun_out/${1:-r3b}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_custom_ar_gpu.py -x -v --timeout 200 --timeout-method thread > $out/pytest_ar.log 2>&1
echo "ar rc=$?" >> $out/pytest_ar.log
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -k "ring or resid_split or rmsnorm" -x -q --timeout 120 --timeout-method thread > $out/pytest_k.log 2>&1 &&
bash tools/ab_multi.sh r3b_ab64.log 64 2 "-" "DSSE_RESID_NW=8 DSSE_RESID_SPLIT=8" "DSSE_QKV_NW=6 DSSE_QKV_SPLIT=4" \
  "DSSE_RESID_NW=8 DSSE_RESID_SPLIT=8 DSSE_QKV_NW=6 DSSE_QKV_SPLIT=4" \
  "DSSE_RESID_NW=8 DSSE_RESID_SPLIT=8 DSSE_QKV_NW=6 DSSE_QKV_SPLIT=4 DSSE_NORM_SPLIT=0" "DSSE_NORM_SPLIT=0" &&
mv gpurun_out/r3b_ab64.log $out/
