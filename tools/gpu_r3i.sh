#!/bin/bash
# Round-3 step I: Infinity-Cache prefetch experiment; attention knob sweep at 64 streams.
set -o pipefail
out=gpurun_out/${1:-r3i}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 240 python3 tools/bench_prefetch.py --rows 64 > $out/prefetch64.log 2>&1 &&
timeout -k 10 240 python3 tools/bench_prefetch.py --rows 256 --wgs 256 > $out/prefetch256.log 2>&1 &&
timeout -k 10 240 python3 tools/bench_attn.py --B 64 --ctx 560 --configs "KWV=2;KWV=4;KWV=8;KWV=1" --target-wgs 512,1024 \
  > $out/attn64.log 2>&1
