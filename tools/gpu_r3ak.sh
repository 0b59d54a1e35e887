#!/bin/bash
# Round-3 step AK: 64-stream knob re-check on the final tree (non-temporal attention changed the balance since
# round 2's tuning): O / down split, QKV wave count, attention key-split waves.
set -o pipefail
mkdir -p gpurun_out/r3ak
bash tools/ab_multi.sh r3ak/ab64.log 64 2 "-" "DSSE_RESID_NW=4 DSSE_RESID_SPLIT=2" "DSSE_RESID_NW=8 DSSE_RESID_SPLIT=4" \
  "DSSE_RESID_NW=2 DSSE_RESID_SPLIT=8" "DSSE_QKV_RING3=0" "DSSE_ATTN_KWV=4" "DSSE_ATTN_KWV=1"
