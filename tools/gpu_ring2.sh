set -o pipefail
mkdir -p gpurun_out/ring2
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "ring or stream or silu" > gpurun_out/ring2/pytest.log 2>&1 &&
timeout -k 10 300 python -u tools/tune_gemm.py --M 64 --graph --iters 40 --ops qkv,o,down,gate_up --configs "s;s:DSSE_S_RING7=0;s:DSSE_S_NW=8,DSSE_S_SPLIT=8;s:DSSE_S_NW=8,DSSE_S_SPLIT=4;s:DSSE_S_NW=4,DSSE_S_SPLIT=8" > gpurun_out/ring2/tune.log 2>&1 &&
tools/ab_bench.sh gpurun_out/ring2/ab 2 "X=0" "DSSE_S_RING7=0"
