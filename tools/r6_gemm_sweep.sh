#!/bin/bash
# Round-6 mid-row GEMM sweep: the cost-model dispatch (default) against the round-5 table (t_model=0) and forced
# gemm_pipe candidates with in-launch split-K (t_fix=1), at 192-1024 rows, every projection of Mistral-7B.
#   bash tools/r6_gemm_sweep.sh OUTDIR [M list]
set -e
out=${1:-gpurun_out/r6_sweep}
M=${2:-192,256,320,384,448,512,576,640,768,896,1024}
mkdir -p "$out"
export PYTHONUNBUFFERED=1
B="timeout -k 10 300 python tools/bench_decode_gemm.py"
$B --shape gate_up --M $M --variants "silu,silu:t_model=0,silu:t_cfg=8;t_split=2;t_fix=1,silu:t_cfg=9;t_split=2;t_fix=1,silu:t_cfg=10;t_split=2;t_fix=1" > "$out/gu.log" 2>&1
$B --shape qkv --M $M --variants "out,out:t_model=0,out:t_cfg=8;t_split=2;t_fix=1,out:t_cfg=8;t_split=4;t_fix=1,out:t_cfg=10;t_split=2;t_fix=1,out:t_cfg=9;t_split=4;t_fix=1" > "$out/qkv.log" 2>&1
$B --shape o,down --M $M --variants "split_norm,split_norm:t_model=0,resid:t_cfg=8;t_split=4;t_fix=1,resid:t_cfg=9;t_split=4;t_fix=1,resid:t_cfg=10;t_split=2;t_fix=1,split_norm:t_cfg=9;t_split=8" > "$out/od.log" 2>&1
