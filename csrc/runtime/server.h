// Native epoll HTTP/1.1 + SSE server, origin admission API, RESP ingest shim and metrics endpoint.
//
// One process serves every role the reference splits over Go services and Redis/NATS:
//   edge  (SSE_PORT, default 8080)   POST /chat -> SSE, GET /stream/{id}, /healthz, /readyz
//                                    (src/sse-adapter/sse_handler.go:80-450, main.go:96-139)
//   origin (ORIGIN_PORT, default 8081) POST /chat -> {"conversation_id","status":"streaming"},
//                                    GET /health, GET /metrics (src/llm-stream-proxy/main.go:89-146)
//   metrics (METRICS_PORT, 9090)     Prometheus text (src/sse-adapter/main.go:134-139)
//   resp  (RESP_PORT, 6379 or 0)     PUBLISH/SUBSCRIBE/PSUBSCRIBE ingest compatible with go-redis, so
//                                    demo/load-generator's producer works unchanged
//                                    (demo/load-generator/main.go:204-240)
//   extra: POST /publish/<subject>   (src/spin-functions/nats-publisher), POST /inspect
//                                    (src/spin-functions/nats-subscriber), GET / (chat page)
//
// Threading: `io_threads` event loops, each with its own SO_REUSEPORT listeners, epoll set and
// eventfd-woken outbox.  The bus pushes frames into the owning thread's outbox; sockets are only
// touched by their own thread.  Chat requests from either /chat endpoint are queued for the engine
// (RequestQueue), or, when LLM_PROXY_URL is set and no local engine is attached, forwarded to the
// remote origin over HTTP exactly like the reference adapter.
#pragma once
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "bus.h"
#include "inspector.h"
#include "relay.h"

namespace dsse {

struct ServerConfig {
  std::string host = "0.0.0.0";
  int sse_port = 8080;      // < 0 = disabled, 0 = ephemeral
  int origin_port = 8081;   // < 0 = disabled
  int metrics_port = 9090;  // < 0 = disabled
  int resp_port = -1;       // < 0 = disabled (6379 for the load-generator producer)
  int io_threads = 4;
  std::string llm_proxy_url;  // edge mode: forward POST /chat here when no local engine is attached
  std::string upstream_url;   // edge mode: relay conversations from this origin SSE endpoint (relay.h)
  bool local_engine = false;  // POST /chat goes straight into the in-process request queue
  std::string model_name = "mistralai/Mistral-7B-Instruct-v0.3";
  InspectionMode inspection = InspectionMode::kDisabled;
  int inspection_buffer_ms = 150;
  // INSPECTION_ENDPOINT: remote inspector URL (inline / hybrid / async verdicts come from it instead of the
  // built-in keyword rules)
  std::string inspection_endpoint;
  int inspection_timeout_ms = 250;
  // INSPECTION_FAIL_OPEN: what inline / hybrid inspection does when the endpoint fails or the gate is overloaded.
  // false (default, the reference's inline contract "inspector down = streaming stops",
  // docs/security-inspection-patterns.md:38): the affected conversation ends with [ERROR] and nothing uninspected
  // is delivered; true: frames pass uninspected, counted in inspection_fail_open_total.
  bool inspection_fail_open = false;
  int dedupe_window_s = 30;  // DEDUPE_WINDOW_SEC (the bus's duplicate window; 0 = off)
  int keepalive_ms = 15000;          // sse_handler.go:182
  int first_token_timeout_ms = 30000;  // sse_handler.go:395
  size_t max_pending_bytes = 4 << 20;  // per-connection output cap before token frames are dropped
  // Per-conversation flow control: when every subscriber of a conversation has more than this many
  // bytes queued, the engine pauses that sequence's decode (others keep going) until the queues drain
  // below a quarter of it.  0 disables (slow consumers then only lose frames past max_pending_bytes).
  size_t flow_high_water = 256 << 10;
  int socket_sndbuf = 0;  // SO_SNDBUF for accepted sockets (0 = kernel autotuning); smaller = earlier backpressure
  size_t replay_max = 4096;
  int retention_s = 300;
  std::string ui_html;  // served at GET / when non-empty
};

// Chat request handed to the engine (or the stub generator).
struct ChatRequest {
  uint64_t id = 0;
  std::string conversation_id;
  std::string message;
  int64_t arrival_ns = 0;
  int max_tokens = -1;       // optional body fields beyond the reference's {message, conversation_id}
  double temperature = -1;
  double top_p = -1;
  int top_k = -1;
  int64_t seed = -1;
  bool ignore_eos = false;
  bool from_edge = false;    // submitted by the edge /chat (a subscriber exists)
  // OpenAI chat (POST /v1/chat/completions): the conversation as normalised JSON
  // [{"role":..,"content":..},..]; empty = `message` is a single user turn
  std::string messages_json;
};

class RequestQueue {
 public:
  void push(ChatRequest r);
  // Pop up to `max` requests, waiting at most timeout_ms for the first.
  std::vector<ChatRequest> pop(size_t max, int timeout_ms);
  size_t size();
  void close();

 private:
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<ChatRequest> q_;
  bool closed_ = false;
};

class IoThread;
class AsyncInspector;
class InspectionGate;

class Server {
 public:
  Server(ServerConfig cfg, std::shared_ptr<Bus> bus);
  ~Server();
  bool start(std::string* err = nullptr);
  void stop();
  bool running() const { return running_.load(); }

  RequestQueue& requests() { return requests_; }
  Bus& bus() { return *bus_; }
  const ServerConfig& config() const { return cfg_; }
  void set_local_engine(bool on) { local_engine_.store(on); }
  void set_ready(bool on) { ready_.store(on); }
  // Conversations whose last subscriber left before completion (engine may abort them).
  std::vector<std::string> pop_cancellations();
  // Flow-control transitions since the last call: (conversation, paused).
  std::vector<std::pair<std::string, bool>> pop_flow_events();
  // Actual bound ports (useful with port 0 requests in tests): role -> port.
  int bound_port(const std::string& role) const;

  // internal (used by IoThread)
  void submit_chat(ChatRequest r);
  void note_cancel(const std::string& conv_id);
  // Kill a conversation (chat.<id>.control, chat.control.kill, or an inspection verdict): subscribers get a
  // terminal `token` frame (done) and the engine a cancellation.  False if it had already ended.
  bool kill_conversation(const std::string& conv_id, const std::string& token, const std::string& why);
  // A remote inline / hybrid inspection gate holds frames before fan-out (per-connection inspection off).
  bool remote_inspection() const { return gate_ != nullptr; }
  // A subscriber of `conv_id` crossed the high-water mark (+1), drained (-1), or the subscriber set
  // changed (0): re-evaluate whether the conversation is paused.
  void flow_update(const std::string& conv_id, int delta);
  bool flow_paused(const std::string& conv_id);
  bool local_engine() const { return local_engine_.load(); }
  bool ready() const { return ready_.load(); }
  // Edge without a local engine: start relaying `conv_id` from the upstream origin (no-op otherwise).
  void relay_ensure(const std::string& conv_id) {
    if (relay_ && !local_engine_.load()) relay_->ensure(conv_id);
  }
  void forward_to_proxy(uint64_t conn_id, IoThread* io, const std::string& conv_id, const std::string& message);

 private:
  ServerConfig cfg_;
  std::shared_ptr<Bus> bus_;
  RequestQueue requests_;
  std::vector<std::unique_ptr<IoThread>> io_;
  std::vector<std::thread> threads_;
  std::thread housekeeping_;
  std::unique_ptr<UpstreamRelay> relay_;
  std::shared_ptr<AsyncInspector> inspector_;
  std::shared_ptr<InspectionGate> gate_;
  std::atomic<bool> running_{false};
  std::atomic<bool> local_engine_{false};
  std::atomic<bool> ready_{true};
  std::atomic<uint64_t> next_req_{1};
  std::mutex cancel_mu_;
  std::vector<std::string> cancels_;
  std::mutex flow_mu_;
  std::unordered_map<std::string, std::pair<int, bool>> flow_;  // congested subscribers, paused
  std::vector<std::pair<std::string, bool>> flow_events_;  // bounded: consumers also time pauses out
  std::atomic<int> n_paused_{0};
  std::vector<std::pair<std::string, int>> ports_;
  friend class IoThread;
};

// INSPECTION_MODE=async: tokens reach clients immediately; this wildcard tap (`chat.*.tokens`) inspects
// them on its own thread and kills a conversation whose token gets a `drop` verdict: subscribers get a
// terminal "[BLOCKED]" token (done=true) and the engine a cancellation — the reference's
// security-inspection "async" pattern with its kill signal on chat.<id>.control
// (docs/security-inspection-patterns.md:70-126), which the reference never implemented.
class AsyncInspector : public Sink, public std::enable_shared_from_this<AsyncInspector> {
 public:
  explicit AsyncInspector(Server& s);
  ~AsyncInspector() override;
  void start();
  void stop();
  bool push(const FramePtr& f) override;

 private:
  void run();
  Server& srv_;
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<FramePtr> q_;
  std::vector<std::string> killed_;
  bool stop_ = false;
  std::thread thread_;
  std::unique_ptr<RemoteInspector> remote_;  // INSPECTION_ENDPOINT
};

// INSPECTION_MODE=inline|hybrid with INSPECTION_ENDPOINT: a bus gate that holds every token frame until the
// remote inspector's verdict, so one call per token serves every subscriber (the reference's inline hook
// ran per token per connection).  Workers are sharded by conversation, so each conversation's frames keep
// their order.  inline: allow -> deliver, redact -> deliver redacted_content, drop -> withhold the token.
// hybrid: the first INSPECTION_BUFFER_MS of a conversation's tokens are held and inspected as one text;
// allow -> release them and pass the rest through, redact -> one frame with redacted_content, drop -> kill.
class InspectionGate : public FrameGate, public std::enable_shared_from_this<InspectionGate> {
 public:
  InspectionGate(Server& s, int workers);
  ~InspectionGate() override;
  void start();
  void stop();
  bool admit(const FramePtr& f) override;

 private:
  struct Worker {
    std::mutex mu;
    std::condition_variable cv;
    std::deque<FramePtr> q;
    std::thread thread;
    // conversations this worker ended fail-closed (their later frames drop) -> when (mono ns); an entry leaves with
    // the conversation's done frame, or after kDeadAgeNs if that frame never comes
    std::unordered_map<std::string, int64_t> dead;
  };
  struct Held {  // hybrid: per conversation
    int64_t first_mono = 0;
    std::vector<FramePtr> frames;
    bool cleared = false;
    int64_t last_mono = 0;
  };
  void run(Worker& w);
  // returns true when the frame's conversation was ended fail-closed
  bool inline_frame(RemoteInspector& ri, const FramePtr& f, std::vector<FramePtr>& out);
  void hybrid_frame(RemoteInspector& ri, std::unordered_map<std::string, Held>& held, const FramePtr& f,
                    std::vector<FramePtr>& out);
  void hybrid_flush(RemoteInspector& ri, const std::string& conv, Held& h, std::vector<FramePtr>& out);
  static constexpr size_t kBypassDepth = 4096;     // fail-open mode: deliver a backlog past this uninspected
  static constexpr size_t kOverloadDepth = 65536;  // fail-closed mode: end the conversations of a backlog past this
  void fail_closed(const std::string& conv, const std::string& why);
  Server& srv_;
  std::vector<std::unique_ptr<Worker>> workers_;
  std::atomic<bool> stop_{false};
};

// Stub token generator (BASELINE config 1, CPU plumbing): consumes the request queue and streams
// `tokens` words per conversation with `delay_ms` (+ uniform jitter up to delay/2, like the Go
// load generator's producer) between tokens, then "[DONE]".
class StubEngine {
 public:
  StubEngine(Server& server, int tokens, int delay_ms, int workers = 2);
  ~StubEngine();
  void stop();

 private:
  void run();
  Server& server_;
  int tokens_, delay_ms_;
  std::atomic<bool> stop_{false};
  std::vector<std::thread> threads_;
};

}  // namespace dsse
