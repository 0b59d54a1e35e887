#!/bin/bash
# A/B of decode-GEMM variants (run on the GPU box): X-streaming kernel across M (is the M = 64 cost
# X traffic or the MT = 4 body?) with default vs non-temporal weight loads.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
CFGS="${CFGS:-s;s:DSSE_S_NW=4}"
MS="${MS:-33,40,48,56,64}"
timeout -k 10 300 python tools/tune_gemm.py --M "$MS" --iters 30 --configs "$CFGS" > gpurun_out/ab_default.log 2>&1 || exit $?
DSSE_KERNELS_VARIANT=nt timeout -k 10 300 python tools/tune_gemm.py --M "$MS" --iters 30 --configs "$CFGS" > gpurun_out/ab_nt.log 2>&1 || exit $?
echo "--- default"; grep -A30 "best per" gpurun_out/ab_default.log; echo "--- nt"; grep -A30 "best per" gpurun_out/ab_nt.log
