#!/bin/bash
# Round-3 step H: kernel traces of the 64 / 128 / 256-stream steps (ring2 / tiled2 on and off), summarised on the
# box (tools/prof_step.py; the 20+ MB trace databases are deleted); short-prompt TTFT with and without the
# captured prefill graphs.
set -o pipefail
out=gpurun_out/${1:-r3h}
mkdir -p $out
export TMPDIR=/tmp
prof() {  # name streams env...
  local name=$1 streams=$2; shift 2
  env "$@" timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/$name -o run -- \
    python3 bench.py --steps 12 --warmup 3 --streams $streams > $out/$name.log 2>&1 &&
  python3 tools/prof_step.py $out/$name/run_results.db --last 6 > $out/$name.md 2>&1
  local rc=$?
  rm -f $out/$name/run_results.db
  return $rc
}
timeout -k 10 300 python -u -m pytest tests/test_model_full_dims_gpu.py -x -q --timeout 200 --timeout-method thread \
  > $out/pytest_model.log 2>&1 &&
timeout -k 10 200 python3 tools/bench_ttft.py --prompt-len 512 --iters 5 --decode-steps 4 > $out/ttft512.log 2>&1 &&
DSSE_PREFILL_GRAPHS=0 timeout -k 10 200 python3 tools/bench_ttft.py --prompt-len 512 --iters 5 --decode-steps 4 > $out/ttft512_eager.log 2>&1 &&
timeout -k 10 200 python3 tools/bench_ttft.py --prompt-len 512 --prompts 4 --iters 5 --decode-steps 4 > $out/ttft512x4.log 2>&1 &&
DSSE_PREFILL_GRAPHS=0 timeout -k 10 200 python3 tools/bench_ttft.py --prompt-len 512 --prompts 4 --iters 5 --decode-steps 4 > $out/ttft512x4_eager.log 2>&1 &&
prof p64_r2 64 DSSE_RING2=1 &&
prof p64_r0 64 DSSE_RING2=0 &&
prof p256_def 256 DSSE_RING2=1 &&
prof p256_t2 256 DSSE_T_NARROW_CFG=7 DSSE_T_WIDE_CFG=8 &&
prof p128_r2 128 DSSE_RING2=1 &&
prof p128_r0 128 DSSE_RING2=0
du -sh $out
