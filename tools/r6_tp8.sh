#!/bin/bash
# Round 6: one TP = 8 rank's work on one GPU -- kernel traces of its decode step and 8k prefill, and its shard GEMMs.
#   bash tools/r6_tp8.sh OUTDIR
set -e
out=${1:-gpurun_out/r6_tp8}; mkdir -p "$out"; export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 300 rocprofv3 --kernel-trace -d "$out/prof_dec" -o run --output-format csv -- python3 tools/bench_tp_rank.py --tp 8 --phase decode --steps 20 --profile-marker > "$out/tp8_dec.log" 2>&1
python3 tools/trace_sum.py "$(ls "$out"/prof_dec/*/run_kernel_trace.csv "$out"/prof_dec/run_kernel_trace.csv 2>/dev/null | head -1)" --div 20 --after-kernel bitwise_not --title "TP=8 rank 0, 64-stream decode step (20 replays)" > "$out/tp8_dec.md" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace -d "$out/prof_pf" -o run --output-format csv -- python3 tools/bench_tp_rank.py --tp 8 --phase prefill --iters 3 --profile-marker > "$out/tp8_pf.log" 2>&1
python3 tools/trace_sum.py "$(ls "$out"/prof_pf/*/run_kernel_trace.csv "$out"/prof_pf/run_kernel_trace.csv 2>/dev/null | head -1)" --div 3 --after-kernel bitwise_not --title "TP=8 rank 0, 8192-token prefill (3 prompts)" > "$out/tp8_pf.md" 2>&1
B="timeout -k 10 300 python tools/bench_decode_gemm.py"
$B --shape qkv_tp8,gate_up_tp8,lm_tp8 --M 64,8192 --variants out > "$out/gemm_col.log" 2>&1
$B --shape o_tp8,down_tp8 --M 64,8192 --variants out,split_norm > "$out/gemm_row.log" 2>&1
