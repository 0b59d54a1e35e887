// In-node token bus: replaces Redis pub/sub -> redis-nats-bridge -> NATS core/leaf (reference
// README.md:59-68, docs/architecture.md:18-93, src/redis-nats-bridge/main.go:115-179).
//
// * Subjects are conversations: `chat.<conversation_id>.tokens`.  Subscribers register per
//   conversation (exact subject) or as wildcard taps (`chat.*.tokens`), which is NATS's
//   interest-based routing collapsed into one process: a token of a conversation nobody listens to
//   costs one ring append and nothing else.
// * Each conversation keeps a bounded replay ring of formatted SSE frames (JetStream-like
//   retention: `replay_max` frames, `retention_s` after completion), so a reconnecting client with
//   `Last-Event-ID: n` gets every frame with sequence > n (the reference only filters and loses seq
//   n+1).
// * Frames are formatted ONCE per token (shared_ptr) and fanned out to any number of subscribers.
// * Subscribers are sinks owned by server I/O threads; publishing only enqueues (no socket I/O under
//   the bus locks).  The bus is sharded by conversation id to keep publisher/subscriber contention low.
#pragma once
#include <atomic>
#include <cstdint>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "json.h"

namespace dsse {

struct Frame {
  std::string bytes;   // full SSE event: "event: token\nid: N\ndata: {...}\n\n"
  std::string json;    // the TokenMessage JSON (for RESP / tap consumers)
  std::string conversation_id;
  int64_t seq = 0;
  bool done = false;
  int64_t timestamp = 0;
  uint8_t finish = kFinishNone;  // TokenMessage::finish
  int32_t prompt_tokens = -1;
};
using FramePtr = std::shared_ptr<const Frame>;

class Sink {
 public:
  virtual ~Sink() = default;
  // Enqueue a frame for delivery.  Must be thread-safe and non-blocking.  Returns false when the
  // subscriber is over its high-water mark (the frame was still queued; the bus counts it).
  virtual bool push(const FramePtr& f) = 0;
  // Called once after a publish batch so sinks can coalesce wakeups.
  virtual void flush() {}
};
using SinkPtr = std::shared_ptr<Sink>;

struct BusConfig {
  size_t replay_max = 4096;     // frames kept per conversation
  int64_t retention_s = 300;    // JetStream CHAT_TOKENS max-age (kubernetes/base/nats-core/core-cluster.yaml:233-244)
  int shards = 64;
};

class Bus {
 public:
  explicit Bus(BusConfig cfg = {});

  static std::string subject_for(const std::string& conversation_id) { return "chat." + conversation_id + ".tokens"; }
  static FramePtr make_frame(const TokenMessage& m);

  // Register a subscriber for one conversation.  Frames with seq > after_seq already in the ring are
  // returned in `replay` (in order) atomically with the registration, so no frame is missed or
  // duplicated.  after_seq < 0 = live only.
  void subscribe(const std::string& conversation_id, const SinkPtr& s, int64_t after_seq, std::vector<FramePtr>* replay);
  void unsubscribe(const std::string& conversation_id, const SinkPtr& s);
  void add_tap(const SinkPtr& s);
  void remove_tap(const SinkPtr& s);

  // Publish one token message; returns the number of subscribers that received it.
  int publish(const TokenMessage& m);
  int publish(const FramePtr& f);
  // Publish many (one flush per distinct sink at the end).
  void publish_batch(const std::vector<FramePtr>& frames);

  size_t subscriber_count(const std::string& conversation_id);
  bool conversation_done(const std::string& conversation_id);
  int64_t last_sequence(const std::string& conversation_id);
  size_t conversations() const { return n_convs_.load(); }
  // Drop finished conversations older than the retention window without subscribers.
  size_t gc(int64_t now_ns);

 private:
  struct Conv {
    std::vector<SinkPtr> subs;
    std::deque<FramePtr> ring;
    int64_t last_seq = 0;
    bool done = false;
    int64_t done_ns = 0;
  };
  struct Shard {
    std::mutex mu;
    std::unordered_map<std::string, Conv> convs;
  };
  Shard& shard(const std::string& id);
  int deliver(const FramePtr& f, std::vector<SinkPtr>* flush_list);

  BusConfig cfg_;
  std::vector<std::unique_ptr<Shard>> shards_;
  std::mutex taps_mu_;
  std::vector<SinkPtr> taps_;
  std::atomic<bool> have_taps_{false};
  std::atomic<size_t> n_convs_{0};
};

}  // namespace dsse
