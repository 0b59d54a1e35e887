#!/bin/bash
# A/B of engine/kernel environment knobs on the 64-stream bench: each config runs REPS times, interleaved.
# usage: tools/ab_bench.sh OUTDIR REPS "ENV1" "ENV2" ...   (an ENV is "" or "A=1 B=2"; extra bench args in BENCH_ARGS)
out=$1; reps=$2; shift 2
mkdir -p "$out"
for rep in $(seq 1 "$reps"); do
  i=0
  for cfg in "$@"; do
    i=$((i + 1))
    log="$out/cfg${i}_rep${rep}.log"
    env $cfg timeout -k 10 240 python -u bench.py ${BENCH_ARGS:---steps 100 --warmup 10} > "$log" 2>&1 || { echo "cfg $i failed rc=$?"; exit 1; }
    ms=$(grep -o '"ms_per_step": [0-9.]*' "$log" | tail -1)
    cad=$(grep -o '"step_cadence_ms": {"p50": [0-9.]*' "$log" | tail -1)
    echo "rep $rep cfg $i [$cfg] $ms $cad" | tee -a "$out/summary.txt"
  done
done
