#include "metrics.h"

#include <cmath>
#include <cstdio>

namespace dsse {

Histogram::Histogram(std::vector<double> buckets)
    : bounds_(std::move(buckets)), counts_(new std::atomic<uint64_t>[bounds_.size() + 1]) {
  for (size_t i = 0; i <= bounds_.size(); ++i) counts_[i].store(0);
}

void Histogram::observe(double v) {
  size_t i = 0;
  while (i < bounds_.size() && v > bounds_[i]) ++i;
  counts_[i].fetch_add(1, std::memory_order_relaxed);
  sum_.add(v);
  n_.fetch_add(1, std::memory_order_relaxed);
}

static void fmt_num(std::string& out, double v) {
  char b[64];
  if (std::isinf(v)) {
    out += v > 0 ? "+Inf" : "-Inf";
    return;
  }
  if (v == std::floor(v) && std::fabs(v) < 1e15) snprintf(b, sizeof b, "%.0f", v);
  else snprintf(b, sizeof b, "%.9g", v);
  out += b;
}

void Histogram::render(std::string& out, const std::string& name) const {
  uint64_t cum = 0;
  for (size_t i = 0; i <= bounds_.size(); ++i) {
    cum += counts_[i].load(std::memory_order_relaxed);
    out += name + "_bucket{le=\"";
    if (i < bounds_.size()) fmt_num(out, bounds_[i]);
    else out += "+Inf";
    out += "\"} ";
    fmt_num(out, (double)cum);
    out += '\n';
  }
  out += name + "_sum ";
  fmt_num(out, sum_.get());
  out += '\n' + name + "_count ";
  fmt_num(out, (double)n_.load());
  out += '\n';
}

Metrics::Metrics()
    : sse_connection_duration_seconds({1, 5, 10, 30, 60, 120, 300, 600}),
      sse_delivery_latency_seconds({0.0001, 0.00025, 0.0005, 0.001, 0.0025, 0.005, 0.01, 0.025, 0.05, 0.1, 0.5}),
      engine_decode_step_seconds({0.001, 0.002, 0.003, 0.005, 0.0075, 0.01, 0.015, 0.02, 0.03, 0.05, 0.1}),
      engine_ttft_seconds({0.01, 0.025, 0.05, 0.1, 0.25, 0.5, 1, 2.5, 5, 10}),
      engine_itl_seconds({0.001, 0.002, 0.003, 0.005, 0.0075, 0.01, 0.015, 0.02, 0.03, 0.05, 0.1}),
      engine_host_step_seconds({0.0001, 0.0002, 0.0005, 0.001, 0.002, 0.003, 0.005, 0.01, 0.02, 0.05, 0.1}) {}

namespace {
void line(std::string& out, const char* name, const char* help, const char* type, double v) {
  out += "# HELP ";
  out += name;
  out += ' ';
  out += help;
  out += "\n# TYPE ";
  out += name;
  out += ' ';
  out += type;
  out += '\n';
  out += name;
  out += ' ';
  fmt_num(out, v);
  out += '\n';
}
void hist(std::string& out, const char* name, const char* help, const Histogram& h) {
  out += "# HELP ";
  out += name;
  out += ' ';
  out += help;
  out += "\n# TYPE ";
  out += name;
  out += " histogram\n";
  h.render(out, name);
}
}  // namespace

std::string Metrics::render() const {
  std::string o;
  o.reserve(4096);
  line(o, "sse_active_connections", "Number of active SSE connections", "gauge", sse_active_connections.get());
  line(o, "sse_total_connections", "Total number of SSE connections", "counter", sse_total_connections.get());
  line(o, "sse_messages_delivered_total", "Total number of messages delivered via SSE", "counter",
       sse_messages_delivered_total.get());
  hist(o, "sse_connection_duration_seconds", "Duration of SSE connections", sse_connection_duration_seconds);
  hist(o, "sse_delivery_latency_seconds", "Token timestamp to socket write (server-side delivery latency)",
       sse_delivery_latency_seconds);
  line(o, "active_chats", "Chats currently generating on the local engine", "gauge", active_chats.get());
  line(o, "bus_published_total", "Token messages published on the in-node bus", "counter", bus_published_total.get());
  line(o, "bus_dropped_tokens_total", "Token frames dropped for slow subscribers", "counter",
       bus_dropped_tokens_total.get());
  line(o, "bus_backpressure_events_total", "Subscriber queues that crossed the high-water mark", "counter",
       bus_backpressure_events_total.get());
  line(o, "bus_backpressure_pauses_total", "Conversations whose decode was paused for slow subscribers", "counter",
       bus_backpressure_pauses_total.get());
  line(o, "bus_paused_conversations", "Conversations currently paused by flow control", "gauge",
       bus_paused_conversations.get());
  line(o, "bus_replayed_total", "Token frames replayed from the conversation ring (Last-Event-ID)", "counter",
       bus_replayed_total.get());
  line(o, "bus_conversations", "Conversations tracked by the bus (live + retained)", "gauge", bus_conversations.get());
  line(o, "resp_publish_total", "PUBLISH commands accepted by the RESP ingest shim", "counter",
       resp_publish_total.get());
  line(o, "bus_duplicates_dropped_total", "Frames dropped as duplicates (dedupe window) or after a conversation ended",
       "counter", bus_duplicates_dropped_total.get());
  line(o, "control_kills_total", "Conversations killed through chat.<id>.control / chat.control.kill", "counter",
       control_kills_total.get());
  line(o, "inspection_remote_errors_total", "INSPECTION_ENDPOINT calls that failed", "counter",
       inspection_remote_errors_total.get());
  line(o, "inspection_fail_open_total", "Frames delivered uninspected (INSPECTION_FAIL_OPEN=1)", "counter",
       inspection_fail_open_total.get());
  line(o, "inspection_fail_closed_total", "Conversations ended because inspection was unavailable", "counter",
       inspection_fail_closed_total.get());
  line(o, "inspection_redacted_total", "Tokens redacted by the security inspector", "counter",
       inspection_redacted_total.get());
  line(o, "inspection_dropped_total", "Tokens dropped by the security inspector", "counter",
       inspection_dropped_total.get());
  line(o, "inspection_killed_total", "Conversations stopped by the asynchronous inspector", "counter",
       inspection_killed_total.get());
  line(o, "engine_batch_size", "Sequences in the current decode batch", "gauge", engine_batch_size.get());
  line(o, "engine_kv_blocks_free", "Free KV-cache pages", "gauge", engine_kv_blocks_free.get());
  line(o, "engine_tokens_total", "Tokens generated by the engine", "counter", engine_tokens_total.get());
  hist(o, "engine_decode_step_seconds", "Engine decode step latency", engine_decode_step_seconds);
  hist(o, "engine_ttft_seconds", "Time to first token", engine_ttft_seconds);
  hist(o, "engine_itl_seconds", "Inter-token latency", engine_itl_seconds);
  hist(o, "engine_host_step_seconds", "Host time of an engine step (scheduling, launches, token processing; drain waits excluded)",
       engine_host_step_seconds);
  line(o, "dp_workers_alive", "Data-parallel engine workers with a live heartbeat", "gauge", dp_workers_alive.get());
  line(o, "dp_requests_routed_total", "Chat requests routed to data-parallel engine workers", "counter",
       dp_requests_routed_total.get());
  line(o, "dp_requeued_total", "Requests moved to another worker after a worker failure", "counter",
       dp_requeued_total.get());
  line(o, "dp_worker_failures_total", "Data-parallel workers declared dead (heartbeat timeout)", "counter",
       dp_worker_failures_total.get());
  line(o, "relay_upstream_connections", "Upstream SSE connections relaying conversations from the origin", "gauge",
       relay_upstream_connections.get());
  line(o, "relay_frames_total", "Token frames received from the origin and republished on this edge", "counter",
       relay_frames_total.get());
  std::lock_guard<std::mutex> g(extra_mu_);
  for (auto& kv : extra_) o += kv.second();
  return o;
}

void Metrics::set_extra(const std::string& key, std::function<std::string()> fn) {
  std::lock_guard<std::mutex> g(extra_mu_);
  extra_[key] = std::move(fn);
}

void Metrics::clear_extra(const std::string& key) {
  std::lock_guard<std::mutex> g(extra_mu_);
  extra_.erase(key);
}

std::string Metrics::render_origin() const {
  char b[64];
  snprintf(b, sizeof b, "active_chats %lld\n", (long long)active_chats.get());
  return b;
}

Metrics& metrics() {
  static Metrics m;
  return m;
}

}  // namespace dsse
