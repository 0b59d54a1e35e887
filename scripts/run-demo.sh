#!/usr/bin/env bash
# Demo menu against a running deployment (or a local `serve`), like the reference's scripts/run-demo.sh:
#   1) stream one conversation with curl (POST /chat)      2) time-to-first-byte of /healthz per endpoint
#   3) fake LLM stream: publish tokens over RESP (no engine) and watch them on GET /stream/<id>
#   4) open N idle /stream connections and read sse_active_connections
# Usage: scripts/run-demo.sh <1-4> [sse_url=http://127.0.0.1:8080] [resp=127.0.0.1:6379] [metrics=http://127.0.0.1:9090]
set -euo pipefail
cd "$(dirname "$0")/.."
SSE=${2:-http://127.0.0.1:8080}
RESP=${3:-127.0.0.1:6379}
MET=${4:-http://127.0.0.1:9090}
LG=distributed_sse_for_llm_response_amd/_lib/dsse-loadgen
case "${1:-1}" in
  1) curl -sN -X POST "$SSE/chat" -H 'Content-Type: application/json' \
       -d '{"message":"Explain server-sent events in two sentences.","max_tokens":64}' ;;
  2) for u in $SSE ${EXTRA_ENDPOINTS:-}; do
       printf '%-40s ' "$u"; curl -s -o /dev/null -w 'ttfb %{time_starttransfer}s total %{time_total}s\n' "$u/healthz"
     done ;;
  3) ID=demo-$(date +%s%N)
     (curl -sN "$SSE/stream/$ID" & echo $! > /tmp/dsse-demo-curl.pid; wait) &
     sleep 0.5
     # nanosecond timestamps (the reference demo sent milliseconds; consumers tolerate both)
     for i in $(seq 1 10); do
       python3 - "$RESP" "$ID" "$i" <<'PY'
import socket, sys, time, json
host, port = sys.argv[1].rsplit(":", 1)
cid, i = sys.argv[2], int(sys.argv[3])
msg = json.dumps({"conversation_id": cid, "token": f"tok{i} ", "sequence": i, "done": i == 10,
                  "timestamp": time.time_ns()}, separators=(",", ":"))
ch = f"llm:tokens:{cid}"
s = socket.create_connection((host, int(port)))
s.sendall(f"*3\r\n$7\r\nPUBLISH\r\n${len(ch)}\r\n{ch}\r\n${len(msg)}\r\n{msg}\r\n".encode())
s.recv(64)
PY
       sleep 0.2
     done
     sleep 0.5; kill "$(cat /tmp/dsse-demo-curl.pid)" 2>/dev/null || true ;;
  4) N=${N:-1000}
     for i in $(seq 1 "$N"); do curl -sN "$SSE/stream/idle-$i" >/dev/null & done
     sleep 2; curl -s "$MET/metrics" | grep '^sse_active_connections'
     kill $(jobs -p) 2>/dev/null || true ;;
  5) # the reference load-test workload through the native load generator
     "$LG" -mode both -redis "$RESP" -sse "$SSE" -conversations "${CONV:-100}" -tokens 50 -token-delay 50 -duration 30s ;;
  *) echo "choose 1-5" >&2; exit 2 ;;
esac
