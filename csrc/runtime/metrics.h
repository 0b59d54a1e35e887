// Prometheus text-exposition metrics registry (lock-free counters/gauges, bucketed histograms).
//
// Names the reference dashboard and HPA depend on are kept exactly
// (src/sse-adapter/sse_handler.go:22-43; demo/dashboards/sse-metrics.json):
//   sse_active_connections, sse_total_connections, sse_messages_delivered_total,
//   sse_connection_duration_seconds{1,5,10,30,60,120,300,600}
// plus the origin's `active_chats` (src/llm-stream-proxy/main.go:110-112) and the engine / bus
// metrics this framework adds.
#pragma once
#include <atomic>
#include <cstdint>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

namespace dsse {

class Counter {
 public:
  void inc(double v = 1.0) { add(v); }
  void add(double v) {
    double cur = val_.load(std::memory_order_relaxed);
    while (!val_.compare_exchange_weak(cur, cur + v, std::memory_order_relaxed)) {}
  }
  void set(double v) { val_.store(v, std::memory_order_relaxed); }
  double get() const { return val_.load(std::memory_order_relaxed); }

 private:
  std::atomic<double> val_{0.0};
};

using Gauge = Counter;  // same storage; exposition type differs

class Histogram {
 public:
  explicit Histogram(std::vector<double> buckets);
  void observe(double v);
  void render(std::string& out, const std::string& name) const;

 private:
  std::vector<double> bounds_;
  std::unique_ptr<std::atomic<uint64_t>[]> counts_;  // bounds_.size() + 1 (the +Inf bucket)
  Counter sum_;
  std::atomic<uint64_t> n_{0};
};

class Metrics {
 public:
  Metrics();
  // sse-adapter (exact reference names)
  Gauge sse_active_connections;
  Counter sse_total_connections;
  Counter sse_messages_delivered_total;
  Histogram sse_connection_duration_seconds;
  // token timestamp (engine drain / producer publish) -> written to the subscriber's socket
  Histogram sse_delivery_latency_seconds;
  // origin proxy
  Gauge active_chats;
  // bus / delivery
  Counter bus_published_total;
  Counter bus_dropped_tokens_total;
  Counter bus_backpressure_events_total;
  Counter bus_replayed_total;
  Counter bus_backpressure_pauses_total;  // conversations paused by flow control (server.h flow_high_water)
  Gauge bus_paused_conversations;
  Gauge bus_conversations;
  Counter resp_publish_total;
  Counter bus_duplicates_dropped_total;  // dedupe window / frames after a conversation's terminal frame
  Counter control_kills_total;           // chat.<id>.control / chat.control.kill
  Counter inspection_remote_errors_total;  // INSPECTION_ENDPOINT calls that failed
  Counter inspection_fail_open_total;      // frames delivered uninspected (INSPECTION_FAIL_OPEN=1 only)
  Counter inspection_fail_closed_total;    // conversations ended because inspection was unavailable / overloaded
  Counter inspection_redacted_total;
  Counter inspection_dropped_total;
  Counter inspection_killed_total;
  // engine (set from the Python engine loop)
  Gauge engine_batch_size;
  Gauge engine_kv_blocks_free;
  Counter engine_tokens_total;
  Histogram engine_decode_step_seconds;
  Histogram engine_ttft_seconds;
  Histogram engine_itl_seconds;
  Histogram engine_host_step_seconds;  // host (Python + launch) time of an engine step, drain waits excluded
  // data-parallel router (dp.h)
  Gauge dp_workers_alive;
  Counter dp_requests_routed_total;
  Counter dp_requeued_total;
  Counter dp_worker_failures_total;
  // edge relay (relay.h)
  Gauge relay_upstream_connections;
  Counter relay_frames_total;

  // Labelled series rendered by their owners (e.g. per-GPU DP worker gauges); appended to render().
  void set_extra(const std::string& key, std::function<std::string()> fn);
  void clear_extra(const std::string& key);

  std::string render() const;        // full exposition for :9090/metrics
  std::string render_origin() const;  // "active_chats N\n" (origin /metrics)

 private:
  mutable std::mutex extra_mu_;
  std::map<std::string, std::function<std::string()>> extra_;
};

Metrics& metrics();

}  // namespace dsse
