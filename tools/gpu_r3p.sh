#!/bin/bash
# Round-3 step P: GPU suite + smoke on the rebuilt tree, driver-style benches, and the phased 256x256 tile
# (split-K) for the 256-stream bucket's wide / narrow projections (DSSE_T_WIDE_CFG / DSSE_T_NARROW_CFG = 4).
set -o pipefail
out=gpurun_out/${1:-r3p}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $out/bench64_1.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --streams 256 > $out/bench256_def.log 2>&1 || exit 1
DSSE_T_WIDE_CFG=4 timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --streams 256 > $out/bench256_w4.log 2>&1 || exit 1
DSSE_T_WIDE_CFG=4 DSSE_T_NARROW_CFG=4 timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --streams 256 > $out/bench256_w4n4.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --streams 256 > $out/bench256_def2.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $out/bench64_2.log 2>&1
