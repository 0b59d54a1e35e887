// Upstream relay: the edge side of a two-tier (origin -> edge regions) deployment.
//
// The reference carries tokens from the origin to each region over NATS: core cluster -> leaf node
// per edge -> sse-adapter subscriptions, with interest propagation so that only subjects somebody
// subscribed to cross the WAN (docs/architecture.md:26-93, kubernetes/base/nats-leaf/leaf-node.yaml,
// README.md:296-309).  Here an edge server configured with UPSTREAM_URL does the same with one HTTP
// connection per conversation: the first local subscriber of `chat.<id>.tokens` opens
// `GET <upstream>/stream/<id>?replay=1` on the origin's SSE port and every token frame received is
// republished on the edge's bus (same sequence numbers and timestamps), which fans it out to all
// local subscribers.  Interest-based: when the last local subscriber leaves, the upstream connection
// closes.  Reconnects resume with `Last-Event-ID` from the origin's replay ring (the JetStream-style
// replay the reference designed but never wired up, docs/architecture.md:142-145), so the relay loses
// nothing across a dropped WAN connection; `?replay=1` also closes the subscribe-vs-first-token race
// of the reference.
#pragma once
#include <atomic>
#include <cstdint>
#include <deque>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>

#include "bus.h"

namespace dsse {

class UpstreamRelay {
 public:
  UpstreamRelay(Bus& bus, std::string upstream_url, int max_retries = 5);
  ~UpstreamRelay();
  bool start(std::string* err);
  void stop();
  // Make sure `conv_id` is being relayed (thread-safe, idempotent).
  void ensure(const std::string& conv_id);
  size_t active();

 private:
  struct Link;
  void run();
  bool open_link(Link& l);
  void close_link(Link& l);
  void on_readable(Link& l);
  bool parse(Link& l);

  Bus& bus_;
  std::string url_, host_, port_, base_;
  int max_retries_;
  int ep_ = -1, evfd_ = -1;
  std::atomic<bool> running_{false};
  std::thread thread_;
  std::mutex mu_;
  std::deque<std::string> wanted_;
  std::unordered_map<std::string, std::unique_ptr<Link>> links_;  // owned by the relay thread
  std::atomic<size_t> n_active_{0};
};

}  // namespace dsse
