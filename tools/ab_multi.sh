#!/bin/bash
# Interleaved A/B/C/... of kernel environment settings on the bench (one box):
#   ab_multi.sh OUT STREAMS ROUNDS "ENV_A" "ENV_B" ...   ("-" = no extra environment)
# One line per run ("env | ms_per_step tok/s p50_itl p99_itl"); a failed run logs its tail and the series goes on.
export TMPDIR=/tmp
mkdir -p gpurun_out
out=gpurun_out/$1; streams=$2; rounds=$3; shift 3
for i in $(seq 1 "$rounds"); do
  for e in "$@"; do
    envs=$([ "$e" = "-" ] && echo "" || echo "$e")
    log=$(mktemp)
    env $envs timeout -k 10 400 python bench.py --steps 20 --warmup 5 --streams "$streams" > "$log" 2>&1
    rc=$?
    r=$(tail -1 "$log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['value'], d.get('p50_itl_ms'), d.get('p99_itl_ms'))" 2>/dev/null)
    if [ -z "$r" ]; then r="FAILED rc=$rc: $(tail -5 "$log" | tr '\n' ' ' | cut -c1-600)"; fi
    echo "$e | $r" | tee -a "$out"
    rm -f "$log"
    [ $rc -eq 124 ] || [ $rc -eq 137 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ] && exit $rc
  done
done
exit 0
