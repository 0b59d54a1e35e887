#!/bin/bash
# Round-3 step N: decode-attention shape at 256 / 128 streams with non-temporal K/V loads; non-temporal tiled
# weight staging (variant "tnt") at 256 streams; kernel summary of a 512-token prefill.
set -o pipefail
out=gpurun_out/${1:-r3n}
mkdir -p $out
export TMPDIR=/tmp
bash tools/ab_multi.sh r3n_ab256.log 256 2 "DSSE_ATTN_KWV=1 DSSE_ATTN_PD=1" "DSSE_ATTN_KWV=1 DSSE_ATTN_PD=2" \
  "DSSE_ATTN_KWV=2 DSSE_ATTN_PD=1" "-" "DSSE_ATTN_KWV=1 DSSE_ATTN_PD=1 DSSE_KERNELS_VARIANT=tnt" || exit 1
bash tools/ab_multi.sh r3n_ab128.log 128 2 "-" "DSSE_ATTN_KWV=4" "DSSE_ATTN_KWV=1 DSSE_ATTN_PD=2" || exit 1
mv gpurun_out/r3n_ab256.log gpurun_out/r3n_ab128.log $out/
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/pttft512 -o run -- \
  python3 tools/bench_ttft.py --prompt-len 512 --iters 4 --decode-steps 2 > $out/pttft512.log 2>&1 &&
python3 tools/prof_sum.py $out/pttft512/run_results.db --div 5 > $out/pttft512.md 2>&1
rc=$?
rm -f $out/pttft512/run_results.db
exit $rc
