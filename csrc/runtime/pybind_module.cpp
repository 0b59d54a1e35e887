// Python bindings of the host runtime (module `_dsse_runtime`).
//
// The engine loop (Python, one per GPU) drives the runtime through a handful of calls per decode
// step: poll_requests() for new chats, publish_tokens() with the step's sampled token ids (detokenised
// and JSON-encoded here, in C++), pop_cancellations(), and engine metric updates.  Blocking calls
// release the GIL.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <memory>
#include <string>
#include <vector>

#include "bus.h"
#include "dp.h"
#include "inspector.h"
#include "json.h"
#include "metrics.h"
#include "server.h"
#include "shm_ring.h"
#include "util.h"

namespace py = pybind11;
using namespace dsse;

namespace {

py::dict request_dict(const ChatRequest& r) {
  py::dict d;
  d["id"] = r.id;
  d["conversation_id"] = r.conversation_id;
  d["message"] = r.message;
  d["arrival_ns"] = r.arrival_ns;
  d["max_tokens"] = r.max_tokens;
  d["temperature"] = r.temperature;
  d["top_p"] = r.top_p;
  d["top_k"] = r.top_k;
  d["seed"] = r.seed;
  d["ignore_eos"] = r.ignore_eos;
  d["from_edge"] = r.from_edge;
  d["messages"] = r.messages_json;
  return d;
}

class Runtime {
 public:
  explicit Runtime(py::dict cfg) {
    auto geti = [&](const char* k, int d) { return cfg.contains(k) ? cfg[k].cast<int>() : d; };
    auto gets = [&](const char* k, const std::string& d) { return cfg.contains(k) ? cfg[k].cast<std::string>() : d; };
    ServerConfig c;
    c.host = gets("host", c.host);
    c.sse_port = geti("sse_port", c.sse_port);
    c.origin_port = geti("origin_port", c.origin_port);
    c.metrics_port = geti("metrics_port", c.metrics_port);
    c.resp_port = geti("resp_port", c.resp_port);
    c.io_threads = geti("io_threads", c.io_threads);
    c.llm_proxy_url = gets("llm_proxy_url", "");
    c.upstream_url = gets("upstream_url", "");
    c.local_engine = cfg.contains("local_engine") && cfg["local_engine"].cast<bool>();
    c.model_name = gets("model_name", c.model_name);
    c.inspection = parse_inspection_mode(gets("inspection_mode", "disabled"));
    c.inspection_buffer_ms = geti("inspection_buffer_ms", c.inspection_buffer_ms);
    c.inspection_endpoint = gets("inspection_endpoint", "");
    c.inspection_timeout_ms = geti("inspection_timeout_ms", c.inspection_timeout_ms);
    c.inspection_fail_open = geti("inspection_fail_open", 0) != 0;
    c.dedupe_window_s = geti("dedupe_window_s", c.dedupe_window_s);
    c.keepalive_ms = geti("keepalive_ms", c.keepalive_ms);
    c.first_token_timeout_ms = geti("first_token_timeout_ms", c.first_token_timeout_ms);
    c.max_pending_bytes = (size_t)geti("max_pending_bytes", (int)c.max_pending_bytes);
    c.flow_high_water = (size_t)geti("flow_high_water", (int)c.flow_high_water);
    c.socket_sndbuf = geti("socket_sndbuf", c.socket_sndbuf);
    c.replay_max = (size_t)geti("replay_max", (int)c.replay_max);
    c.retention_s = geti("retention_s", c.retention_s);
    c.ui_html = gets("ui_html", "");
    BusConfig bc;
    bc.replay_max = c.replay_max;
    bc.retention_s = c.retention_s;
    bc.dedupe_window_s = c.dedupe_window_s;
    bus_ = std::make_shared<Bus>(bc);
    server_ = std::make_unique<Server>(c, bus_);
  }
  ~Runtime() { stop(); }

  void start() {
    std::string err;
    bool ok;
    {
      py::gil_scoped_release nogil;
      ok = server_->start(&err);
    }
    if (!ok) throw std::runtime_error("runtime start failed: " + err);
  }
  void stop() {
    py::gil_scoped_release nogil;
    if (dp_) dp_->stop();
    dp_.reset();
    if (stub_) stub_->stop();
    stub_.reset();
    if (server_) server_->stop();
  }
  int bound_port(const std::string& role) { return server_->bound_port(role); }

  py::list poll_requests(size_t max, int timeout_ms) {
    std::vector<ChatRequest> rs;
    {
      py::gil_scoped_release nogil;
      rs = server_->requests().pop(max, timeout_ms);
    }
    py::list out;
    for (auto& r : rs) out.append(request_dict(r));
    return out;
  }
  void submit(const std::string& conv_id, const std::string& message, int max_tokens) {
    ChatRequest r;
    r.conversation_id = conv_id;
    r.message = message;
    r.max_tokens = max_tokens;
    server_->submit_chat(std::move(r));
  }

  void set_vocab(std::vector<std::string> pieces) {
    if (dp_) dp_->set_vocab(pieces);
    vocab_ = std::move(pieces);
  }

  // Data-parallel mode: this runtime becomes the router for `workers` engine processes (dp.h).
  void start_dp_router(const std::string& prefix, int workers, int ring_mb, int worker_timeout_ms) {
    dp_ = std::make_unique<DpRouter>(*server_, prefix, workers, (size_t)ring_mb << 20, worker_timeout_ms);
    dp_->set_vocab(vocab_);
    std::string err;
    if (!dp_->start(&err)) {
      dp_.reset();
      throw std::runtime_error("dp router start failed: " + err);
    }
  }
  py::list dp_workers() {
    py::list out;
    if (!dp_) return out;
    for (auto& i : dp_->workers()) {
      py::dict d;
      d["ready"] = i.ready;
      d["alive"] = i.alive;
      d["outstanding"] = i.outstanding;
      d["batch"] = i.batch;
      d["kv_free"] = i.kv_free;
      d["active"] = i.active;
      out.append(d);
    }
    return out;
  }

  // Publish one engine step: conversation ids, token ids, sequence numbers, done flags.  Token text
  // comes from the vocabulary; `texts` (optional) overrides per entry (e.g. "[DONE]", "[ERROR]").
  int publish_tokens(const std::vector<std::string>& conv_ids, const std::vector<int>& token_ids,
                     const std::vector<int64_t>& seqs, const std::vector<bool>& dones, int64_t ts,
                     const std::vector<std::string>& texts, const std::vector<int>& finish,
                     const std::vector<int>& prompt_tokens) {
    const size_t n = conv_ids.size();
    if (token_ids.size() != n || seqs.size() != n || dones.size() != n)
      throw std::invalid_argument("publish_tokens: length mismatch");
    std::vector<FramePtr> frames;
    frames.reserve(n);
    {
      py::gil_scoped_release nogil;
      const int64_t t = ts > 0 ? ts : now_ns();
      TokenMessage m;
      for (size_t i = 0; i < n; ++i) {
        m.conversation_id = conv_ids[i];
        if (i < texts.size() && !texts[i].empty()) m.token = texts[i];
        else if (token_ids[i] >= 0 && (size_t)token_ids[i] < vocab_.size()) m.token = vocab_[token_ids[i]];
        else m.token = "<" + std::to_string(token_ids[i]) + ">";
        m.sequence = seqs[i];
        m.done = dones[i];
        m.timestamp = t;
        m.finish = i < finish.size() ? (uint8_t)finish[i] : kFinishNone;
        m.prompt_tokens = i < prompt_tokens.size() ? prompt_tokens[i] : -1;
        frames.push_back(Bus::make_frame(m));
      }
      bus_->publish_batch(frames);
    }
    metrics().engine_tokens_total.add((double)n);
    return (int)n;
  }
  int publish(const std::string& conv_id, const std::string& token, int64_t seq, bool done, int64_t ts) {
    TokenMessage m{conv_id, token, seq, done, ts > 0 ? ts : now_ns()};
    py::gil_scoped_release nogil;
    return bus_->publish(m);
  }
  std::vector<std::string> pop_cancellations() { return server_->pop_cancellations(); }
  std::vector<std::pair<std::string, bool>> pop_flow_events() { return server_->pop_flow_events(); }
  size_t subscriber_count(const std::string& id) { return bus_->subscriber_count(id); }
  int64_t last_sequence(const std::string& id) { return bus_->last_sequence(id); }
  size_t queued_requests() { return server_->requests().size(); }
  void set_ready(bool r) { server_->set_ready(r); }
  void set_local_engine(bool on) { server_->set_local_engine(on); }
  void start_stub(int tokens, int delay_ms, int workers) {
    stub_ = std::make_unique<StubEngine>(*server_, tokens, delay_ms, workers);
  }
  std::string metrics_text() { return metrics().render(); }

 private:
  std::shared_ptr<Bus> bus_;
  std::unique_ptr<Server> server_;
  std::unique_ptr<StubEngine> stub_;
  std::unique_ptr<DpRouter> dp_;
  std::vector<std::string> vocab_;
};

// Engine-worker end of a DP channel: the same calls the engine loop makes on a Runtime.
class DpWorkerPy {
 public:
  DpWorkerPy(const std::string& prefix, int worker, int open_timeout_ms) {
    {
      py::gil_scoped_release nogil;
      w_ = std::make_unique<DpWorker>(prefix, worker, open_timeout_ms);
    }
    if (!w_->ok()) throw std::runtime_error("dp worker attach failed: " + w_->error());
  }
  py::list poll_requests(size_t max, int timeout_ms) {
    std::vector<ChatRequest> rs;
    {
      py::gil_scoped_release nogil;
      std::vector<std::string> cancels;
      bool sd = false;
      std::vector<std::pair<std::string, bool>> flow;
      rs = w_->poll(max, timeout_ms, &cancels, &sd, &flow);
      cancels_.insert(cancels_.end(), cancels.begin(), cancels.end());
      flow_.insert(flow_.end(), flow.begin(), flow.end());
      if (sd) shutdown_ = true;
    }
    py::list out;
    for (auto& r : rs) out.append(request_dict(r));
    return out;
  }
  std::vector<std::string> pop_cancellations() {
    std::vector<std::string> out;
    out.swap(cancels_);
    return out;
  }
  std::vector<std::pair<std::string, bool>> pop_flow_events() {
    std::vector<std::pair<std::string, bool>> out;
    out.swap(flow_);
    return out;
  }
  bool shutdown_requested() const { return shutdown_; }
  int publish_tokens(const std::vector<std::string>& conv_ids, const std::vector<int>& token_ids,
                     const std::vector<int64_t>& seqs, const std::vector<bool>& dones, int64_t ts,
                     const std::vector<std::string>& texts, const std::vector<int>& finish,
                     const std::vector<int>& prompt_tokens) {
    const size_t n = conv_ids.size();
    if (token_ids.size() != n || seqs.size() != n || dones.size() != n)
      throw std::invalid_argument("publish_tokens: length mismatch");
    py::gil_scoped_release nogil;
    if (!w_->publish_tokens(conv_ids, token_ids, seqs, dones, ts, texts, finish, prompt_tokens))
      throw std::runtime_error("dp worker: token ring closed or full");
    return (int)n;
  }
  void set_ready(bool r) {
    py::gil_scoped_release nogil;
    if (r) w_->hello();
    else w_->bye();
  }
  void observe(double step_s, double batch, double kv_free, double active, const std::vector<double>& ttft,
               const std::vector<double>& itl, const std::vector<double>& host) {
    py::gil_scoped_release nogil;
    w_->stats(step_s, batch, kv_free, active, ttft, itl, host);
  }
  void set_vocab(const std::vector<std::string>&) {}  // text is resolved by the router

 private:
  std::unique_ptr<DpWorker> w_;
  std::vector<std::string> cancels_;
  std::vector<std::pair<std::string, bool>> flow_;
  bool shutdown_ = false;
};

// One direction of a same-node control channel (bytes messages) over a POSIX shm SPSC ring: the TP leader's
// per-step plan to each follower (serving/tp.py ShmPlanChannel).  The creator owns (and unlinks) the ring.
class ShmChannelPy {
 public:
  ShmChannelPy(const std::string& name, bool create, size_t capacity, int open_timeout_ms) {
    std::string err;
    {
      py::gil_scoped_release nogil;
      r_ = create ? ShmRing::create(name, capacity, true, &err) : ShmRing::open(name, open_timeout_ms, &err);
    }
    if (!r_) throw std::runtime_error("shm channel: " + err);
  }
  bool push(const py::bytes& b, int timeout_ms) {
    std::string s = b;
    py::gil_scoped_release nogil;
    return timeout_ms > 0 ? r_->push_wait(s.data(), (uint32_t)s.size(), timeout_ms) : r_->push(s.data(), (uint32_t)s.size());
  }
  py::object pop(int timeout_ms, int spin_us) {
    std::string out;
    bool got;
    {
      py::gil_scoped_release nogil;
      got = timeout_ms > 0 || spin_us > 0 ? r_->pop_wait(&out, timeout_ms, spin_us) : r_->pop(&out);
    }
    if (!got) return py::none();
    return py::bytes(out);
  }
  void close() { r_->close(); }
  bool closed() const { return r_->closed(); }
  const std::string& name() const { return r_->name(); }

 private:
  std::unique_ptr<ShmRing> r_;
};

// The TP leader's side of the plan channel: one ring per follower, every message pushed to all of them in one
// call without the GIL.
class ShmFanoutPy {
 public:
  ShmFanoutPy(const std::vector<std::string>& names, size_t capacity) {
    std::string err;
    py::gil_scoped_release nogil;
    for (const auto& n : names) {
      auto r = ShmRing::create(n, capacity, true, &err);
      if (!r) throw std::runtime_error("shm fanout: " + err);
      rings_.push_back(std::move(r));
    }
  }
  bool push(const py::bytes& b, int timeout_ms) {
    char* data = nullptr;
    Py_ssize_t len = 0;
    PyBytes_AsStringAndSize(b.ptr(), &data, &len);
    py::gil_scoped_release nogil;
    for (auto& r : rings_)
      if (!(r->push(data, (uint32_t)len) || (timeout_ms > 0 && r->push_wait(data, (uint32_t)len, timeout_ms))))
        return false;
    return true;
  }
  void close() {
    for (auto& r : rings_) r->close();
  }

 private:
  std::vector<std::unique_ptr<ShmRing>> rings_;
};

}  // namespace

PYBIND11_MODULE(_dsse_runtime, m) {
  m.doc() = "MI355X streaming-token delivery runtime (bus, SSE server, RESP ingest, inspector, metrics)";
  py::class_<Runtime>(m, "Runtime")
      .def(py::init<py::dict>(), py::arg("config") = py::dict())
      .def("start", &Runtime::start)
      .def("stop", &Runtime::stop)
      .def("bound_port", &Runtime::bound_port)
      .def("poll_requests", &Runtime::poll_requests, py::arg("max") = 256, py::arg("timeout_ms") = 0)
      .def("submit", &Runtime::submit, py::arg("conversation_id"), py::arg("message"), py::arg("max_tokens") = -1)
      .def("set_vocab", &Runtime::set_vocab)
      .def("publish_tokens", &Runtime::publish_tokens, py::arg("conversation_ids"), py::arg("token_ids"),
           py::arg("sequences"), py::arg("dones"), py::arg("timestamp_ns") = 0,
           py::arg("texts") = std::vector<std::string>{}, py::arg("finish") = std::vector<int>{},
           py::arg("prompt_tokens") = std::vector<int>{})
      .def("publish", &Runtime::publish, py::arg("conversation_id"), py::arg("token"), py::arg("sequence"),
           py::arg("done") = false, py::arg("timestamp_ns") = 0)
      .def("pop_cancellations", &Runtime::pop_cancellations)
      .def("pop_flow_events", &Runtime::pop_flow_events)
      .def("subscriber_count", &Runtime::subscriber_count)
      .def("last_sequence", &Runtime::last_sequence)
      .def("queued_requests", &Runtime::queued_requests)
      .def("set_ready", &Runtime::set_ready)
      .def("set_local_engine", &Runtime::set_local_engine)
      .def("start_stub", &Runtime::start_stub, py::arg("tokens") = 50, py::arg("delay_ms") = 50, py::arg("workers") = 2)
      .def("metrics_text", &Runtime::metrics_text)
      .def("start_dp_router", &Runtime::start_dp_router, py::arg("prefix"), py::arg("workers"), py::arg("ring_mb") = 8,
           py::arg("worker_timeout_ms") = 10000)
      .def("dp_workers", &Runtime::dp_workers);

  py::class_<DpWorkerPy>(m, "DpWorker")
      .def(py::init<const std::string&, int, int>(), py::arg("prefix"), py::arg("worker"),
           py::arg("open_timeout_ms") = 60000)
      .def("poll_requests", &DpWorkerPy::poll_requests, py::arg("max") = 256, py::arg("timeout_ms") = 0)
      .def("pop_cancellations", &DpWorkerPy::pop_cancellations)
      .def("pop_flow_events", &DpWorkerPy::pop_flow_events)
      .def("shutdown_requested", &DpWorkerPy::shutdown_requested)
      .def("publish_tokens", &DpWorkerPy::publish_tokens, py::arg("conversation_ids"), py::arg("token_ids"),
           py::arg("sequences"), py::arg("dones"), py::arg("timestamp_ns") = 0,
           py::arg("texts") = std::vector<std::string>{}, py::arg("finish") = std::vector<int>{},
           py::arg("prompt_tokens") = std::vector<int>{})
      .def("set_ready", &DpWorkerPy::set_ready)
      .def("observe", &DpWorkerPy::observe, py::arg("step_s"), py::arg("batch"), py::arg("kv_free"), py::arg("active"),
           py::arg("ttft"), py::arg("itl"), py::arg("host") = std::vector<double>{})
      .def("set_vocab", &DpWorkerPy::set_vocab);
  m.def("dp_ring_name", &dp_ring_name);

  py::class_<ShmChannelPy>(m, "ShmChannel")
      .def(py::init<const std::string&, bool, size_t, int>(), py::arg("name"), py::arg("create"),
           py::arg("capacity") = 1 << 20, py::arg("open_timeout_ms") = 60000)
      .def("push", &ShmChannelPy::push, py::arg("data"), py::arg("timeout_ms") = 5000)
      .def("pop", &ShmChannelPy::pop, py::arg("timeout_ms") = 0, py::arg("spin_us") = 0)
      .def("close", &ShmChannelPy::close)
      .def("closed", &ShmChannelPy::closed)
      .def_property_readonly("name", &ShmChannelPy::name);
  py::class_<ShmFanoutPy>(m, "ShmFanout")
      .def(py::init<const std::vector<std::string>&, size_t>(), py::arg("names"), py::arg("capacity") = 1 << 20)
      .def("push", &ShmFanoutPy::push, py::arg("data"), py::arg("timeout_ms") = 5000)
      .def("close", &ShmFanoutPy::close);

  m.def("encode_token_message", [](const std::string& cid, const std::string& tok, int64_t seq, bool done, int64_t ts) {
    return encode_token_message(TokenMessage{cid, tok, seq, done, ts});
  });
  m.def("parse_token_message", [](const std::string& s) -> py::object {
    TokenMessage t;
    if (!parse_token_message(s, t)) return py::none();
    py::dict d;
    d["conversation_id"] = t.conversation_id;
    d["token"] = t.token;
    d["sequence"] = t.sequence;
    d["done"] = t.done;
    d["timestamp"] = t.timestamp;
    return d;
  });
  m.def("sse_frame", [](const std::string& cid, const std::string& tok, int64_t seq, bool done, int64_t ts) {
    return py::bytes(Bus::make_frame(TokenMessage{cid, tok, seq, done, ts})->bytes);
  });
  m.def("inspect", [](const std::string& content) {
    InspectionResult r = inspect_message(content);
    py::dict d;
    d["action"] = action_name(r.action);
    d["reason"] = r.reason.empty() ? py::object(py::none()) : py::object(py::str(r.reason));
    d["redacted_content"] = r.action == InspectAction::kRedact ? py::object(py::str(r.redacted_content)) : py::object(py::none());
    return d;
  });
  m.def("inspection_json", [](const std::string& content) { return inspection_result_json(inspect_message(content)); });
  m.def("engine_observe", [](double step_s, double batch, double kv_free, double host_s) {
    if (step_s > 0) metrics().engine_decode_step_seconds.observe(step_s);
    if (host_s >= 0) metrics().engine_host_step_seconds.observe(host_s);
    metrics().engine_batch_size.set(batch);
    metrics().engine_kv_blocks_free.set(kv_free);
  }, py::arg("step_s"), py::arg("batch"), py::arg("kv_free"), py::arg("host_s") = -1.0);
  m.def("observe_ttft", [](double s) { metrics().engine_ttft_seconds.observe(s); });
  m.def("observe_itl", [](double s) { metrics().engine_itl_seconds.observe(s); });
  m.def("set_active_chats", [](double n) { metrics().active_chats.set(n); });
  m.def("uuid4", &uuid4);
}
