#!/bin/bash
# Round-3 step S: norm-folded O projection on the register-streaming kernel (K split over 4 / 8 waves per
# 16-column workgroup) vs the separate-norm step; per-grid breakdown of the K-split-8 form.
set -o pipefail
out=gpurun_out/${1:-r3s}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_norm_fold_gpu.py -x -q --timeout 120 --timeout-method thread > $out/pytest_fold.log 2>&1 || exit 1
for i in 1 2; do
  DSSE_NORM_FOLD=0 timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $out/bench64_nofold_$i.log 2>&1 || exit 1
  DSSE_OPROJ_NW=-8 timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $out/bench64_k8_$i.log 2>&1 || exit 1
  DSSE_OPROJ_NW=-4 timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $out/bench64_k4_$i.log 2>&1 || exit 1
done
DSSE_OPROJ_NW=-8 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/p64_k8 -o run -- \
  python3 bench.py --steps 12 --warmup 3 > $out/p64_k8.log 2>&1 &&
python3 tools/prof_step.py $out/p64_k8/run_results.db --last 6 --by-grid > $out/p64_k8.md 2>&1
rc=$?
rm -f $out/p64_k8/run_results.db
exit $rc
