#!/bin/bash
# A/B of kernel environment settings on the bench (alternating runs on one box): ab_env.sh OUT STREAMS "ENV_A" "ENV_B" [rounds]
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
out=gpurun_out/$1; streams=$2; a=$3; b=$4; rounds=${5:-2}
for i in $(seq 1 "$rounds"); do
  for e in "$a" "$b"; do
    r=$(env $e timeout -k 10 400 python bench.py --steps 20 --warmup 5 --streams "$streams" 2>&1 | tail -1 |
        python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['value'], d.get('p50_itl_ms'))")
    echo "$e $r" | tee -a "$out"
  done
done
