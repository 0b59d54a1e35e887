#!/bin/bash
# Round-3 step Q: norm-folded decode GEMMs (tests, then 64-stream A/B: fold off / on with 1- and 2-wave O
# projection workgroups), the phased 256x256 tile for the 256-stream bucket, full GPU suite + smoke.
set -o pipefail
out=gpurun_out/${1:-r3q}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_norm_fold_gpu.py -x -v --timeout 120 --timeout-method thread > $out/pytest_fold.log 2>&1 || exit 1
for i in 1 2; do
  DSSE_NORM_FOLD=0 timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $out/bench64_nofold_$i.log 2>&1 || exit 1
  DSSE_OPROJ_NW=1 timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $out/bench64_fold1_$i.log 2>&1 || exit 1
  DSSE_OPROJ_NW=2 timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $out/bench64_fold2_$i.log 2>&1 || exit 1
done
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --streams 256 > $out/bench256_def.log 2>&1 || exit 1
DSSE_T_WIDE_CFG=4 timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --streams 256 > $out/bench256_w4.log 2>&1 || exit 1
DSSE_T_WIDE_CFG=4 DSSE_T_NARROW_CFG=4 timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --streams 256 > $out/bench256_w4n4.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1
