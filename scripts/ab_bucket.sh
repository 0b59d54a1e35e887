#!/usr/bin/env bash
# A/B of the decode-GEMM path for one stream count: STREAMS:MAX_M pairs, each a bench.py run with
# DSSE_DECODE_GEMM_MAX_M=MAX_M (buckets above it take the hipBLASLt + gemm_wide path).
# Usage: scripts/ab_bucket.sh 192:192 192:128 ...   (logs under gpurun_out/)
set -o pipefail
mkdir -p gpurun_out
for cfg in "$@"; do
  s=${cfg%%:*}
  m=${cfg##*:}
  log=gpurun_out/ab_s${s}_m${m}.log
  DSSE_DECODE_GEMM_MAX_M=$m timeout -k 10 200 python bench.py --streams "$s" --steps 48 --warmup 8 > "$log" 2>&1 || exit $?
  echo "streams=$s max_m=$m $(tail -1 "$log")"
done
