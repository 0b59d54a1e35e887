#!/bin/bash
# Round-3 step H: kernel traces of the 64- and 256-stream steps, ring2 / tiled2 on and off.
set -o pipefail
out=gpurun_out/${1:-r3h}
mkdir -p $out
export TMPDIR=/tmp
prof() {  # name streams env...
  local name=$1 streams=$2; shift 2
  env "$@" timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/$name -o run -- \
    python3 bench.py --steps 12 --warmup 3 --streams $streams > $out/$name.log 2>&1
}
prof p64_r2 64 DSSE_RING2=1 &&
prof p64_r0 64 DSSE_RING2=0 &&
prof p256_def 256 DSSE_RING2=1 &&
prof p256_t2 256 DSSE_T_NARROW_CFG=7 DSSE_T_WIDE_CFG=8 &&
prof p128_r2 128 DSSE_RING2=1 &&
prof p128_r0 128 DSSE_RING2=0
