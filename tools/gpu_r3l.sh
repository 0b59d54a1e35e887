#!/bin/bash
# Round-3 step L: small prefill budgets (captured prefill passes) under arrivals; fused vs unfused QKV attention at
# 256 streams; 8k TTFT (default vs flash MFMA-priority variant) and its kernel summary.
set -o pipefail
out=gpurun_out/${1:-r3l}
mkdir -p $out
export TMPDIR=/tmp
DSSE_MIXED=0 timeout -k 10 400 python -u tools/bench_serving.py --rates 13 --requests 300 --max-tokens 1000 \
  --prefill-budget 128,256,512 > $out/serving_budget.jsonl 2> $out/serving_budget.err || exit 1
bash tools/ab_multi.sh r3l_qkv256.log 256 1 "-" "DSSE_FUSED_QKV_ATTN=0 DSSE_ATTN_KWV=1 DSSE_ATTN_PD=2" \
  "DSSE_ATTN_KWV=1 DSSE_ATTN_PD=2" "DSSE_FUSED_QKV_ATTN=0" || exit 1
mv gpurun_out/r3l_qkv256.log $out/
timeout -k 10 300 python3 tools/bench_ttft.py --prompt-len 8192 --iters 3 > $out/ttft8k.log 2>&1 &&
DSSE_KERNELS_VARIANT=pfprio timeout -k 10 300 python3 tools/bench_ttft.py --prompt-len 8192 --iters 3 > $out/ttft8k_pfprio.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/pttft8k -o run -- \
  python3 tools/bench_ttft.py --prompt-len 8192 --iters 1 --decode-steps 2 > $out/pttft8k.log 2>&1 &&
python3 tools/prof_sum.py $out/pttft8k/run_results.db --div 2 > $out/pttft8k.md 2>&1
rc=$?
rm -f $out/pttft8k/run_results.db
exit $rc
