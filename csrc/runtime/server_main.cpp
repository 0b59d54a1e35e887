// dsse-server: standalone delivery server (no GPU).  BASELINE config 1 (CPU plumbing): the edge SSE
// server, origin admission API, RESP ingest shim and metrics, with either the built-in stub token
// generator (STUB_TOKENS > 0) or LLM_PROXY_URL forwarding.  Environment variables follow the reference
// services (src/sse-adapter/main.go:29-40, src/llm-stream-proxy/main.go:70-96):
//   SSE_PORT (8080) METRICS_PORT (9090) ORIGIN_PORT (8081, or PORT) RESP_PORT (-1 = off; 6379)
//   LLM_PROXY_URL UPSTREAM_URL (edge: relay tokens from the origin's SSE port) INSPECTION_MODE
//   INSPECTION_BUFFER_MS LOG_LEVEL IO_THREADS FLOW_HIGH_WATER
//   UI_PATH (chat page served at GET /) STUB_TOKENS (50; 0 = no stub) STUB_TOKEN_DELAY_MS (50) STUB_WORKERS (2)
#include <csignal>
#include <cstdio>
#include <fstream>
#include <sstream>
#include <thread>

#include "server.h"
#include "util.h"

using namespace dsse;

static volatile std::sig_atomic_t g_stop = 0;
static void on_signal(int) { g_stop = 1; }

int main() {
  ServerConfig c;
  c.sse_port = (int)env_long("SSE_PORT", 8080);
  c.metrics_port = (int)env_long("METRICS_PORT", 9090);
  c.origin_port = (int)env_long("ORIGIN_PORT", env_long("PORT", 8081));
  c.resp_port = (int)env_long("RESP_PORT", -1);
  c.io_threads = (int)env_long("IO_THREADS", 4);
  c.llm_proxy_url = env_str("LLM_PROXY_URL", "");
  c.upstream_url = env_str("UPSTREAM_URL", "");
  if (const std::string ui = env_str("UI_PATH", ""); !ui.empty()) {  // chat page at GET /
    std::ifstream f(ui);
    std::stringstream ss;
    ss << f.rdbuf();
    c.ui_html = ss.str();
  }
  c.inspection = parse_inspection_mode(env_str("INSPECTION_MODE", "disabled"));
  c.inspection_buffer_ms = (int)env_long("INSPECTION_BUFFER_MS", 150);
  c.inspection_endpoint = env_str("INSPECTION_ENDPOINT", "");
  c.inspection_timeout_ms = (int)env_long("INSPECTION_TIMEOUT_MS", c.inspection_timeout_ms);
  c.inspection_fail_open = env_long("INSPECTION_FAIL_OPEN", 0) != 0;
  c.dedupe_window_s = (int)env_long("DEDUPE_WINDOW_SEC", c.dedupe_window_s);
  c.flow_high_water = (size_t)env_long("FLOW_HIGH_WATER", (long)c.flow_high_water);
  const int stub_tokens = (int)env_long("STUB_TOKENS", 50);
  const int stub_delay = (int)env_long("STUB_TOKEN_DELAY_MS", 50);
  c.local_engine = stub_tokens > 0;
  BusConfig bc;
  bc.dedupe_window_s = c.dedupe_window_s;
  auto bus = std::make_shared<Bus>(bc);
  Server server(c, bus);
  std::string err;
  if (!server.start(&err)) {
    fprintf(stderr, "dsse-server: %s\n", err.c_str());
    return 1;
  }
  std::unique_ptr<StubEngine> stub;
  if (stub_tokens > 0) stub = std::make_unique<StubEngine>(server, stub_tokens, stub_delay, (int)env_long("STUB_WORKERS", 2));
  log_json(LogLevel::kInfo, "dsse-server listening",
           "\"sse_port\":" + std::to_string(server.bound_port("edge")) + ",\"origin_port\":" +
               std::to_string(server.bound_port("origin")) + ",\"metrics_port\":" +
               std::to_string(server.bound_port("metrics")) + ",\"resp_port\":" + std::to_string(server.bound_port("resp")));
  std::signal(SIGINT, on_signal);
  std::signal(SIGTERM, on_signal);
  while (!g_stop) std::this_thread::sleep_for(std::chrono::milliseconds(100));
  log_json(LogLevel::kInfo, "shutting down");
  if (stub) stub->stop();
  server.stop();
  return 0;
}
