#!/bin/bash
# Round-3 step N: decode-attention shape at 256 streams with non-temporal K/V loads (2 rounds).
set -o pipefail
out=gpurun_out/${1:-r3n}
mkdir -p $out
export TMPDIR=/tmp
bash tools/ab_multi.sh r3n_ab256.log 256 2 "DSSE_ATTN_KWV=1 DSSE_ATTN_PD=1" "DSSE_ATTN_KWV=1 DSSE_ATTN_PD=2" \
  "DSSE_ATTN_KWV=2 DSSE_ATTN_PD=1" "-" || exit 1
bash tools/ab_multi.sh r3n_ab128.log 128 2 "-" "DSSE_ATTN_KWV=4" "DSSE_ATTN_KWV=1 DSSE_ATTN_PD=2" || exit 1
mv gpurun_out/r3n_ab256.log gpurun_out/r3n_ab128.log $out/
