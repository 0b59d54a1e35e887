#!/bin/bash
# Round-3 step O: GPU test suite + smoke + driver-style benches at 64 / 128 / 256 streams on the current defaults.
set -o pipefail
out=gpurun_out/${1:-r3o}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || exit 1
for i in 1 2; do timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $out/bench64_$i.log 2>&1 || exit 1; done
for i in 1 2; do timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --streams 256 > $out/bench256_$i.log 2>&1 || exit 1; done
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --streams 128 > $out/bench128.log 2>&1
