// Data-parallel serving across GPUs: one router process owns the sockets and the bus, one engine
// worker process per GPU (BASELINE config 3: DP=8 on one node).
//
//   clients ──HTTP/SSE──► Server (edge/origin) ──RequestQueue──► DpRouter.dispatch ──shm ring──► worker g
//   worker g ──shm ring (token batches)──► DpRouter.drain[g] ──► Bus ──► epoll writers ──► clients
//
// * Routing: least outstanding conversations among live workers; a conversation stays on the worker
//   that owns its KV cache (cancellations follow it).
// * Liveness: workers send a heartbeat at least every 500 ms; a worker silent for `worker_timeout_ms`
//   is declared dead: conversations it had not started streaming are requeued on another worker
//   (restart from the prompt), streaming ones get a terminal `[ERROR]` token (the reference's
//   upstream-error convention, src/llm-stream-proxy/main.go:166-186).  /readyz is ready while at least
//   one worker is live.
// * Token text is resolved here from the vocabulary (set_vocab), so workers ship 4-byte ids.
#pragma once
#include <atomic>
#include <cstdint>
#include <cstring>
#include <deque>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "server.h"
#include "shm_ring.h"

namespace dsse {

namespace dpwire {
enum : uint8_t { kRequest = 1, kCancel = 2, kShutdown = 3, kFlow = 4, kHello = 10, kTokens = 11, kStats = 12, kHeartbeat = 13, kBye = 14 };

class Writer {
 public:
  void u8(uint8_t v) { b_.push_back((char)v); }
  void i32(int32_t v) { raw(&v, 4); }
  void i64(int64_t v) { raw(&v, 8); }
  void f64(double v) { raw(&v, 8); }
  void str(const std::string& s) {
    i32((int32_t)s.size());
    b_ += s;
  }
  const std::string& data() const { return b_; }

 private:
  void raw(const void* p, size_t n) { b_.append(static_cast<const char*>(p), n); }
  std::string b_;
};

class Reader {
 public:
  explicit Reader(const std::string& b) : b_(b) {}
  uint8_t u8() { return ok(1) ? (uint8_t)b_[p_++] : 0; }
  int32_t i32() { int32_t v = 0; get(&v, 4); return v; }
  int64_t i64() { int64_t v = 0; get(&v, 8); return v; }
  double f64() { double v = 0; get(&v, 8); return v; }
  std::string str() {
    const int32_t n = i32();
    if (n < 0 || !ok((size_t)n)) { bad_ = true; return {}; }
    std::string s = b_.substr(p_, (size_t)n);
    p_ += (size_t)n;
    return s;
  }
  bool good() const { return !bad_; }

 private:
  bool ok(size_t n) {
    if (p_ + n > b_.size()) bad_ = true;
    return !bad_;
  }
  void get(void* v, size_t n) {
    if (ok(n)) {
      std::memcpy(v, b_.data() + p_, n);
      p_ += n;
    }
  }
  const std::string& b_;
  size_t p_ = 0;
  bool bad_ = false;
};

std::string encode_request(const ChatRequest& r);
bool decode_request(Reader& rd, ChatRequest* r);
}  // namespace dpwire

std::string dp_ring_name(const std::string& prefix, int worker, bool to_worker);

struct DpWorkerInfo {
  bool ready = false, alive = true;
  int64_t last_seen_ms = 0;
  int64_t outstanding = 0;
  double batch = 0, kv_free = 0, active = 0;
};

class DpRouter {
 public:
  DpRouter(Server& server, std::string prefix, int workers, size_t ring_bytes = 8 << 20, int worker_timeout_ms = 10000);
  ~DpRouter();
  bool start(std::string* err);
  void stop();
  void set_vocab(std::vector<std::string> pieces);
  std::vector<DpWorkerInfo> workers();
  int num_workers() const { return n_; }

 private:
  struct Conv {
    int worker = -1;
    int64_t last_seq = 0;
    ChatRequest req;
  };
  void dispatch_loop();
  void drain_loop(int w);
  int pick_worker_locked(const std::string& conv_id);
  bool send_request_locked(ChatRequest r);
  void check_liveness_locked(int64_t now_ms);
  void handle_tokens(int w, dpwire::Reader& rd);
  void update_readiness_locked();

  Server& server_;
  std::string prefix_;
  int n_;
  int rr_ = 0;  // first worker examined by the next pick: ties on outstanding rotate over the replicas
  size_t ring_bytes_;
  int timeout_ms_;
  std::vector<std::unique_ptr<ShmRing>> to_w_, from_w_;
  std::mutex mu_;
  std::vector<DpWorkerInfo> info_;
  std::unordered_map<std::string, Conv> convs_;
  std::deque<ChatRequest> pending_;  // arrived before any worker was ready
  std::mutex vocab_mu_;
  std::shared_ptr<const std::vector<std::string>> vocab_;
  std::atomic<bool> running_{false};
  std::thread dispatch_;
  std::vector<std::thread> drains_;
};

// Worker side of the channel (one per engine process).  Mirrors the Runtime calls the engine loop makes.
class DpWorker {
 public:
  DpWorker(const std::string& prefix, int worker, int open_timeout_ms);
  ~DpWorker();
  bool ok() const { return to_router_ && from_router_; }
  const std::string& error() const { return err_; }
  // Requests routed to this worker; cancellations and shutdown are returned through the out-params.
  std::vector<ChatRequest> poll(size_t max, int timeout_ms, std::vector<std::string>* cancels, bool* shutdown,
                                std::vector<std::pair<std::string, bool>>* flow = nullptr);
  bool publish_tokens(const std::vector<std::string>& conv_ids, const std::vector<int>& token_ids,
                      const std::vector<int64_t>& seqs, const std::vector<bool>& dones, int64_t ts,
                      const std::vector<std::string>& texts, const std::vector<int>& finish = {},
                      const std::vector<int>& prompt_tokens = {});
  void hello();
  void bye();
  void stats(double step_s, double batch, double kv_free, double active, const std::vector<double>& ttft,
             const std::vector<double>& itl, const std::vector<double>& host = {});

 private:
  void heartbeat_if_due();
  bool send(const std::string& msg);
  int worker_;
  std::unique_ptr<ShmRing> from_router_, to_router_;
  std::string err_;
  int64_t last_sent_ms_ = 0;
  std::mutex send_mu_;
};

}  // namespace dsse
