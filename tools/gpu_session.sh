#!/bin/bash
# One GPU-box session: tests -> smoke -> bench -> rocprof.  Each GPU step has its own time limit;
# a crash / fault / timeout (exit status other than 0 or 1) ends the session immediately.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
STEPS="${STEPS:-tests smoke bench prof}"
run() {  # name, timeout, cmd...
  local name=$1 t=$2; shift 2
  echo "=== $name: $*" | tee -a gpurun_out/session.log
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a gpurun_out/session.log
  tail -5 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "fatal rc=$rc in $name; stopping"; exit $rc; fi
  return 0
}
for s in $STEPS; do
  case $s in
    tests) run pytest_gpu 900 python -m pytest tests -m gpu -q -x ${PYTEST_ARGS:-} ;;
    tune) run tune 600 python tools/tune_gemm.py ${TUNE_ARGS:---M 16,32,64 --iters 30} ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run bench 900 python bench.py ${BENCH_ARGS:---steps 32 --warmup 4} ;;
    prof) run prof 900 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 8 --warmup 2 ${PROF_ARGS:-} ;;
  esac
done
echo "session done"
