set -e
out=$1; mkdir -p $out; export PYTHONUNBUFFERED=1
B="timeout -k 10 300 python tools/bench_decode_gemm.py"
$B --shape gate_up --M 256,576 --variants "silu:t_model=0,silu:t_cfg=8;t_split=2;t_fix=1,silu:t_cfg=9;t_split=2;t_fix=1,silu:t_model=0" > $out/gu.log 2>&1
$B --shape qkv --M 320,512 --variants "out:t_model=0,out:t_cfg=8;t_split=4;t_fix=1,out:t_cfg=9;t_split=4;t_fix=1,out:t_cfg=10;t_split=2;t_fix=1,out:t_model=0" > $out/qkv.log 2>&1
