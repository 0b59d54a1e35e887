#!/bin/bash
# BASELINE config 5 on the GPU box's CPU (no GPU use): dsse-server with the RESP ingest + the native load generator
# at 10,000 conversations x 50 tokens (the reference's demo/load-generator workload), two runs.
out=gpurun_out/${1:-config5}
mkdir -p $out
L=distributed_sse_for_llm_response_amd/_lib
nproc > $out/nproc.txt
for run in 1 2; do
  SSE_PORT=18080 METRICS_PORT=19090 ORIGIN_PORT=18081 RESP_PORT=16379 STUB_TOKENS=20 IO_THREADS=8 $L/dsse-server > $out/server_$run.log 2>&1 &
  sp=$!
  sleep 1
  timeout -k 5 120 $L/dsse-loadgen -mode both -redis 127.0.0.1:16379 -sse http://127.0.0.1:18080 -conversations 10000 \
    -tokens 50 -token-delay 50 -duration 30s -json -threads 8 -pool 64 > $out/loadgen_$run.json 2>&1
  curl -s http://127.0.0.1:19090/metrics > $out/metrics_$run.txt 2>/dev/null || true
  kill $sp; wait $sp 2>/dev/null
done
cat $out/loadgen_*.json
