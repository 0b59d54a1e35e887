#!/bin/bash
# Round-3 step J: ring / ring2 numerics; attention sweeps at 64 and 256 streams (page order, waves, page ring);
# three driver-style 256-stream runs (p99 / p50) and two 64-stream runs on the current defaults.
set -o pipefail
out=gpurun_out/${1:-r3j}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -k "ring or gemm_out or decode_bucket" -x -q \
  --timeout 120 --timeout-method thread > $out/pytest.log 2>&1 &&
timeout -k 10 200 python3 tools/bench_attn.py --B 256 --ctx 560 --configs "KWV=1;KWV=2;KWV=1,PD=2;KWV=2,PD=2;KWV=4" \
  > $out/attn256.log 2>&1 &&
timeout -k 10 200 python3 tools/bench_attn.py --B 256 --ctx 560 --seq-pages --configs "KWV=1;KWV=2,PD=2" \
  > $out/attn256_seq.log 2>&1 &&
timeout -k 10 200 python3 tools/bench_attn.py --B 64 --ctx 560 --configs "KWV=2;KWV=2,PD=2;KWV=1,PD=2;KWV=4" \
  > $out/attn64.log 2>&1 &&
timeout -k 10 200 python3 tools/bench_attn.py --B 64 --ctx 560 --seq-pages --configs "KWV=2;KWV=4" \
  > $out/attn64_seq.log 2>&1 &&
for i in 1 2 3; do timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --streams 256 > $out/bench256_$i.log 2>&1 || exit 1; done &&
for i in 1 2; do timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $out/bench64_$i.log 2>&1 || exit 1; done
