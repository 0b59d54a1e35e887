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
// * Frames are formatted ONCE per token (shared_ptr; the JSON is a view into the SSE bytes) and fanned
//   out to any number of subscribers.
// * Subscribers are sinks owned by server I/O threads; publishing only enqueues (no socket I/O under
//   the bus locks).  The bus is sharded by conversation id to keep publisher/subscriber contention low;
//   a conversation's subscriber list is copy-on-write (subscribe / unsubscribe build a new one), so a
//   publish takes a reference to it instead of copying it per token.
// * Duplicate suppression (the CHAT_TOKENS stream's 30 s dupe window, kubernetes/base/nats-core/
//   core-cluster.yaml:240, and the bridge's DEDUPE_WINDOW_SEC, src/redis-nats-bridge/main.go:36): a frame
//   whose (conversation, sequence) was delivered within `dedupe_window_s` is dropped, and so is a frame at
//   or past a conversation's terminal sequence (late out-of-order tokens below it still pass; a new
//   stream that restarts at sequence 1 reopens the conversation).
// * An optional gate (remote inline / hybrid inspection) takes frames before fan-out and hands them back
//   through deliver_gated() in per-conversation order.
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
  uint32_t json_off = 0, json_len = 0;  // the TokenMessage JSON inside `bytes` (RESP / tap consumers)
  std::string_view json() const { return std::string_view(bytes).substr(json_off, json_len); }
  std::string conversation_id;
  int64_t seq = 0;
  bool done = false;
  int64_t timestamp = 0;
  uint8_t finish = kFinishNone;  // TokenMessage::finish
  int32_t prompt_tokens = -1;
  int64_t created_mono = 0;      // formatting time (dedupe window clock)
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
  int64_t dedupe_window_s = 30;  // 0 disables duplicate suppression
};

// Holds frames back before fan-out (e.g. remote inspection); returns true when it took `f` and will hand it
// (or a replacement) back through Bus::deliver_gated, in per-conversation order.
class FrameGate {
 public:
  virtual ~FrameGate() = default;
  virtual bool admit(const FramePtr& f) = 0;
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
  // Fan out frames a gate took, bypassing the gate.
  void deliver_gated(const std::vector<FramePtr>& frames);
  // End a conversation now: a terminal frame (done, `token`, sequence = last + 1, assigned under the
  // conversation's lock so it cannot collide with a racing token) bypassing the gate.  False if the
  // conversation already ended.
  bool terminate(const std::string& conversation_id, const std::string& token, uint8_t finish);
  void set_gate(std::shared_ptr<FrameGate> g);

  size_t subscriber_count(const std::string& conversation_id);
  bool conversation_done(const std::string& conversation_id);
  int64_t last_sequence(const std::string& conversation_id);
  size_t conversations() const { return n_convs_.load(); }
  // Drop finished conversations older than the retention window without subscribers.
  size_t gc(int64_t now_ns);

 private:
  using SubList = std::vector<SinkPtr>;
  struct Conv {
    std::shared_ptr<const SubList> subs;  // copy-on-write
    std::deque<FramePtr> ring;
    int64_t last_seq = 0;
    bool done = false;
    int64_t done_seq = 0;
    int64_t done_ns = 0;
    int64_t done_ts = 0;    // producer timestamp of the terminal frame
    int64_t done_mono = 0;  // its created_mono
  };
  struct Shard {
    std::mutex mu;
    std::unordered_map<std::string, Conv> convs;
  };
  Shard& shard(const std::string& id);
  int deliver(const FramePtr& f, std::vector<SinkPtr>* flush_list);
  bool duplicate_locked(Conv& c, const Frame& f, int64_t now);
  static void flush_all(std::vector<SinkPtr>& flush);

  BusConfig cfg_;
  std::vector<std::unique_ptr<Shard>> shards_;
  std::mutex taps_mu_;
  std::vector<SinkPtr> taps_;
  std::atomic<bool> have_taps_{false};
  std::atomic<size_t> n_convs_{0};
  std::mutex gate_mu_;
  std::shared_ptr<FrameGate> gate_;
  std::atomic<bool> have_gate_{false};
};

}  // namespace dsse
