set -o pipefail
mkdir -p gpurun_out/ring3
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "ring or stream or silu or gemm_out" > gpurun_out/ring3/pytest.log 2>&1 &&
BENCH_ARGS="--steps 40 --warmup 5 --streams 32" tools/ab_bench.sh gpurun_out/ring3/ab32 2 "X=0" "DSSE_S_RING_SMALL=1" &&
BENCH_ARGS="--steps 40 --warmup 5 --streams 16" tools/ab_bench.sh gpurun_out/ring3/ab16 2 "X=0" "DSSE_S_RING_SMALL=1"
