#!/bin/bash
# Round-3 session-L final verification: GPU suite, smoke, driver-style benches at 64 / 128 / 192 / 256 streams,
# TTFT at 1024 / 8192 tokens, serving under arrivals, 64-stream step profile.
set -o pipefail
out=gpurun_out/${1:-r3final}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $out/smoke.log 2>&1 || exit 1
for i in 1 2 3; do timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $out/bench64_$i.log 2>&1 || exit 1; done
for s in 128 192 256; do timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --streams $s > $out/bench$s.log 2>&1 || exit 1; done
timeout -k 10 300 python3 tools/bench_ttft.py --prompt-len 1024 --iters 5 --decode-steps 4 > $out/ttft1024.log 2>&1 || exit 1
timeout -k 10 300 python3 tools/bench_ttft.py --prompt-len 8192 --iters 3 > $out/ttft8192.log 2>&1 || exit 1
timeout -k 10 400 python -u tools/bench_serving.py --rates 13 --requests 300 --max-tokens 1000 \
  --prefill-budget 512 > $out/serving13.jsonl 2> $out/serving13.err || exit 1
timeout -k 10 400 python -u tools/bench_serving.py --rates 40 --requests 600 --max-tokens 200 \
  --prefill-budget 512 > $out/serving40.jsonl 2> $out/serving40.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/step_p64 -o run -- \
  python3 bench.py --steps 12 --warmup 3 > $out/step_p64.log 2>&1 &&
python3 tools/prof_step.py $out/step_p64/run_results.db --last 6 --by-grid > $out/step_p64.md 2>&1
rc=$?
rm -f $out/step_p64/run_results.db
exit $rc
