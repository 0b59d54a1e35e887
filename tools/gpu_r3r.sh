#!/bin/bash
# Round-3 step R: per-grid kernel breakdown of the 64-stream step with the norm-folded path (1- and 2-wave O
# projection) and without it; then the rest of the GPU suite and smoke.
set -o pipefail
out=gpurun_out/${1:-r3r}
mkdir -p $out
export TMPDIR=/tmp
prof() {  # name streams env...
  local name=$1 streams=$2; shift 2
  env "$@" timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/$name -o run -- \
    python3 bench.py --steps 12 --warmup 3 --streams $streams > $out/$name.log 2>&1 &&
  python3 tools/prof_step.py $out/$name/run_results.db --last 6 --by-grid > $out/$name.md 2>&1
  local rc=$?
  rm -f $out/$name/run_results.db
  return $rc
}
prof p64_fold1 64 DSSE_OPROJ_NW=1 || exit 1
prof p64_fold2 64 DSSE_OPROJ_NW=2 || exit 1
prof p64_nofold 64 DSSE_NORM_FOLD=0 || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1
