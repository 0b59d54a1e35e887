#!/bin/bash
# Round-3 step X: verification of the session-L tree: GPU suite, smoke, driver-style benches at 64 / 128 / 256
# streams, per-grid step profiles at 64 and 256 streams, 8k TTFT.
set -o pipefail
out=gpurun_out/${1:-r3x}
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
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $out/smoke.log 2>&1 || exit 1
for i in 1 2 3; do timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $out/bench64_$i.log 2>&1 || exit 1; done
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --streams 128 > $out/bench128.log 2>&1 || exit 1
for i in 1 2; do timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --streams 256 > $out/bench256_$i.log 2>&1 || exit 1; done
timeout -k 10 300 python3 tools/bench_ttft.py --prompt-len 8192 --iters 3 > $out/ttft8k.log 2>&1 || exit 1
prof step_p64 64 || exit 1
prof step_p256 256 || exit 1
timeout -k 10 400 python -u tools/bench_serving.py --rates 13 --requests 300 --max-tokens 1000 \
  --prefill-budget 512 > $out/serving13.jsonl 2> $out/serving13.err || exit 1
timeout -k 10 400 python -u tools/bench_serving.py --rates 40 --requests 600 --max-tokens 200 \
  --prefill-budget 512 > $out/serving40.jsonl 2> $out/serving40.err
