#include "dp.h"

#include <algorithm>
#include <chrono>

#include "metrics.h"
#include "util.h"

namespace dsse {

namespace {
int64_t mono_ms() {
  return std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}
}  // namespace

namespace dpwire {
std::string encode_request(const ChatRequest& r) {
  Writer w;
  w.u8(kRequest);
  w.i64((int64_t)r.id);
  w.str(r.conversation_id);
  w.str(r.message);
  w.i64(r.arrival_ns);
  w.i32(r.max_tokens);
  w.f64(r.temperature);
  w.f64(r.top_p);
  w.i32(r.top_k);
  w.i64(r.seed);
  w.u8(r.ignore_eos ? 1 : 0);
  w.u8(r.from_edge ? 1 : 0);
  w.str(r.messages_json);
  return w.data();
}

bool decode_request(Reader& rd, ChatRequest* r) {
  r->id = (uint64_t)rd.i64();
  r->conversation_id = rd.str();
  r->message = rd.str();
  r->arrival_ns = rd.i64();
  r->max_tokens = rd.i32();
  r->temperature = rd.f64();
  r->top_p = rd.f64();
  r->top_k = rd.i32();
  r->seed = rd.i64();
  r->ignore_eos = rd.u8() != 0;
  r->from_edge = rd.u8() != 0;
  r->messages_json = rd.str();
  return rd.good();
}
}  // namespace dpwire

std::string dp_ring_name(const std::string& prefix, int worker, bool to_worker) {
  std::string p = prefix;
  if (p.empty() || p[0] != '/') p = "/" + p;
  std::replace(p.begin() + 1, p.end(), '/', '_');
  return p + "-w" + std::to_string(worker) + (to_worker ? "-req" : "-tok");
}

// ------------------------------------------------------------------------------------------ router
DpRouter::DpRouter(Server& server, std::string prefix, int workers, size_t ring_bytes, int worker_timeout_ms)
    : server_(server), prefix_(std::move(prefix)), n_(workers), ring_bytes_(ring_bytes), timeout_ms_(worker_timeout_ms),
      info_((size_t)workers), vocab_(std::make_shared<std::vector<std::string>>()) {}

DpRouter::~DpRouter() { stop(); }

bool DpRouter::start(std::string* err) {
  for (int w = 0; w < n_; ++w) {
    auto a = ShmRing::create(dp_ring_name(prefix_, w, true), ring_bytes_, true, err);
    auto b = ShmRing::create(dp_ring_name(prefix_, w, false), ring_bytes_, true, err);
    if (!a || !b) return false;
    to_w_.push_back(std::move(a));
    from_w_.push_back(std::move(b));
  }
  server_.set_local_engine(true);  // /chat admits into the request queue this router drains
  server_.set_ready(false);
  // per-GPU series: dp_worker_{up,outstanding,batch_size,kv_blocks_free,active_chats}{worker="g"}
  metrics().set_extra("dp", [this] {
    std::string o;
    const auto ws = workers();
    const char* names[] = {"dp_worker_up", "dp_worker_outstanding", "dp_worker_batch_size", "dp_worker_kv_blocks_free",
                           "dp_worker_active_chats"};
    for (int k = 0; k < 5; ++k) {
      o += std::string("# TYPE ") + names[k] + " gauge\n";
      for (size_t w = 0; w < ws.size(); ++w) {
        const auto& i = ws[w];
        const double v = k == 0 ? (i.ready && i.alive ? 1.0 : 0.0)
                         : k == 1 ? (double)i.outstanding
                         : k == 2 ? i.batch
                         : k == 3 ? i.kv_free
                                  : i.active;
        char b[128];
        snprintf(b, sizeof b, "%s{worker=\"%zu\"} %.17g\n", names[k], w, v);
        o += b;
      }
    }
    return o;
  });
  running_ = true;
  dispatch_ = std::thread([this] { dispatch_loop(); });
  for (int w = 0; w < n_; ++w) drains_.emplace_back([this, w] { drain_loop(w); });
  return true;
}

void DpRouter::stop() {
  if (!running_.exchange(false)) return;
  metrics().clear_extra("dp");
  {
    dpwire::Writer m;
    m.u8(dpwire::kShutdown);
    for (auto& r : to_w_) r->push(m.data().data(), (uint32_t)m.data().size());
  }
  if (dispatch_.joinable()) dispatch_.join();
  for (auto& t : drains_)
    if (t.joinable()) t.join();
  drains_.clear();
  for (auto& r : to_w_) r->close();
  for (auto& r : from_w_) r->close();
  to_w_.clear();
  from_w_.clear();
}

void DpRouter::set_vocab(std::vector<std::string> pieces) {
  auto v = std::make_shared<const std::vector<std::string>>(std::move(pieces));
  std::lock_guard<std::mutex> g(vocab_mu_);
  vocab_ = std::move(v);
}

std::vector<DpWorkerInfo> DpRouter::workers() {
  std::lock_guard<std::mutex> g(mu_);
  return info_;
}

int DpRouter::pick_worker_locked(const std::string& conv_id) {
  auto it = convs_.find(conv_id);
  if (it != convs_.end() && it->second.worker >= 0 && info_[(size_t)it->second.worker].alive) return it->second.worker;
  // least outstanding; ties rotate (a low request rate would otherwise always land on the lowest index)
  int best = -1;
  for (int k = 0; k < n_; ++k) {
    const int w = (rr_ + k) % n_;
    const auto& i = info_[(size_t)w];
    if (!i.ready || !i.alive) continue;
    if (best < 0 || i.outstanding < info_[(size_t)best].outstanding) best = w;
  }
  if (best >= 0) rr_ = (best + 1) % n_;
  return best;
}

bool DpRouter::send_request_locked(ChatRequest r) {
  const int w = pick_worker_locked(r.conversation_id);
  if (w < 0) return false;
  const std::string msg = dpwire::encode_request(r);
  if (!to_w_[(size_t)w]->push_wait(msg.data(), (uint32_t)msg.size(), 1000)) return false;
  auto& c = convs_[r.conversation_id];
  if (c.worker != w) info_[(size_t)w].outstanding++;
  c.worker = w;
  c.last_seq = 0;
  c.req = std::move(r);
  metrics().dp_requests_routed_total.inc();
  return true;
}

void DpRouter::update_readiness_locked() {
  int alive = 0;
  for (auto& i : info_) alive += (i.ready && i.alive) ? 1 : 0;
  metrics().dp_workers_alive.set(alive);
  server_.set_ready(alive > 0);
}

void DpRouter::check_liveness_locked(int64_t now_ms) {
  for (int w = 0; w < n_; ++w) {
    auto& i = info_[(size_t)w];
    if (!i.ready || !i.alive || now_ms - i.last_seen_ms <= timeout_ms_) continue;
    i.alive = false;
    metrics().dp_worker_failures_total.inc();
    log_json(LogLevel::kWarn, "dp worker lost", "\"worker\":" + std::to_string(w));
    std::vector<ChatRequest> requeue;
    std::vector<FramePtr> errors;
    for (auto it = convs_.begin(); it != convs_.end();) {
      if (it->second.worker != w) {
        ++it;
        continue;
      }
      if (it->second.last_seq == 0) {
        requeue.push_back(std::move(it->second.req));
      } else {
        TokenMessage m{it->first, "[ERROR]", it->second.last_seq + 1, true, now_ns()};
        errors.push_back(Bus::make_frame(m));
      }
      it = convs_.erase(it);
    }
    i.outstanding = 0;
    if (!errors.empty()) server_.bus().publish_batch(errors);
    for (auto& r : requeue) {
      metrics().dp_requeued_total.inc();
      if (!send_request_locked(r)) pending_.push_back(std::move(r));
    }
  }
  update_readiness_locked();
}

void DpRouter::dispatch_loop() {
  while (running_) {
    auto reqs = server_.requests().pop(256, 20);
    auto cancels = server_.pop_cancellations();
    auto flow = server_.pop_flow_events();
    std::lock_guard<std::mutex> g(mu_);
    check_liveness_locked(mono_ms());
    while (!pending_.empty()) {
      if (!send_request_locked(pending_.front())) break;
      pending_.pop_front();
    }
    for (auto& r : reqs) {
      if (!pending_.empty() || !send_request_locked(r)) pending_.push_back(std::move(r));
    }
    for (auto& c : cancels) {
      auto it = convs_.find(c);
      if (it == convs_.end() || it->second.worker < 0) continue;
      dpwire::Writer m;
      m.u8(dpwire::kCancel);
      m.str(c);
      to_w_[(size_t)it->second.worker]->push_wait(m.data().data(), (uint32_t)m.data().size(), 100);
    }
    for (auto& [c, paused] : flow) {  // flow control follows the conversation to its worker
      auto it = convs_.find(c);
      if (it == convs_.end() || it->second.worker < 0) continue;
      dpwire::Writer m;
      m.u8(dpwire::kFlow);
      m.str(c);
      m.u8(paused ? 1 : 0);
      to_w_[(size_t)it->second.worker]->push_wait(m.data().data(), (uint32_t)m.data().size(), 100);
    }
  }
}

void DpRouter::handle_tokens(int w, dpwire::Reader& rd) {
  const int32_t n = rd.i32();
  if (n <= 0) return;
  std::shared_ptr<const std::vector<std::string>> vocab;
  {
    std::lock_guard<std::mutex> g(vocab_mu_);
    vocab = vocab_;
  }
  const int64_t ts_all = rd.i64();
  std::vector<FramePtr> frames;
  frames.reserve((size_t)n);
  std::vector<std::pair<std::string, std::pair<int64_t, bool>>> progress;
  progress.reserve((size_t)n);
  TokenMessage m;
  m.timestamp = ts_all > 0 ? ts_all : now_ns();
  for (int32_t i = 0; i < n && rd.good(); ++i) {
    m.conversation_id = rd.str();
    const int32_t tok = rd.i32();
    m.sequence = rd.i64();
    m.done = rd.u8() != 0;
    std::string text = rd.str();
    m.finish = rd.u8();
    m.prompt_tokens = rd.i32();
    if (!text.empty()) m.token = std::move(text);
    else if (tok >= 0 && (size_t)tok < vocab->size()) m.token = (*vocab)[(size_t)tok];
    else m.token = "<" + std::to_string(tok) + ">";
    frames.push_back(Bus::make_frame(m));
    progress.push_back({m.conversation_id, {m.sequence, m.done}});
  }
  server_.bus().publish_batch(frames);
  metrics().engine_tokens_total.add((double)frames.size());
  std::lock_guard<std::mutex> g(mu_);
  for (auto& p : progress) {
    auto it = convs_.find(p.first);
    if (it == convs_.end() || it->second.worker != w) continue;
    it->second.last_seq = std::max(it->second.last_seq, p.second.first);
    if (p.second.second) {
      info_[(size_t)w].outstanding = std::max<int64_t>(0, info_[(size_t)w].outstanding - 1);
      convs_.erase(it);
    }
  }
}

void DpRouter::drain_loop(int w) {
  std::string msg;
  while (running_) {
    if (!from_w_[(size_t)w]->pop_wait(&msg, 50)) continue;
    dpwire::Reader rd(msg);
    const uint8_t type = rd.u8();
    if (type == dpwire::kTokens) handle_tokens(w, rd);
    std::lock_guard<std::mutex> g(mu_);
    auto& i = info_[(size_t)w];
    i.last_seen_ms = mono_ms();
    if (type == dpwire::kHello) {
      i.ready = true;
      i.alive = true;
      log_json(LogLevel::kInfo, "dp worker ready", "\"worker\":" + std::to_string(w));
      update_readiness_locked();
    } else if (type == dpwire::kBye) {
      i.ready = false;
      update_readiness_locked();
    } else if (type == dpwire::kStats) {
      const double step_s = rd.f64();
      i.batch = rd.f64();
      i.kv_free = rd.f64();
      i.active = rd.f64();
      const int32_t nt = rd.i32();
      for (int32_t k = 0; k < nt && rd.good(); ++k) metrics().engine_ttft_seconds.observe(rd.f64());
      const int32_t ni = rd.i32();
      for (int32_t k = 0; k < ni && rd.good(); ++k) metrics().engine_itl_seconds.observe(rd.f64());
      const int32_t nh = rd.good() ? rd.i32() : 0;
      for (int32_t k = 0; k < nh && rd.good(); ++k) metrics().engine_host_step_seconds.observe(rd.f64());
      if (step_s > 0) metrics().engine_decode_step_seconds.observe(step_s);
      double batch = 0, kv = 0, active = 0;
      for (auto& x : info_) {
        batch += x.batch;
        kv += x.kv_free;
        active += x.active;
      }
      metrics().engine_batch_size.set(batch);
      metrics().engine_kv_blocks_free.set(kv);
      metrics().active_chats.set(active);
    }
  }
}

// ------------------------------------------------------------------------------------------ worker
DpWorker::DpWorker(const std::string& prefix, int worker, int open_timeout_ms) : worker_(worker) {
  from_router_ = ShmRing::open(dp_ring_name(prefix, worker, true), open_timeout_ms, &err_);
  if (from_router_) to_router_ = ShmRing::open(dp_ring_name(prefix, worker, false), open_timeout_ms, &err_);
}

DpWorker::~DpWorker() = default;

bool DpWorker::send(const std::string& msg) {
  std::lock_guard<std::mutex> g(send_mu_);
  last_sent_ms_ = mono_ms();
  return to_router_->push_wait(msg.data(), (uint32_t)msg.size(), 5000);
}

void DpWorker::heartbeat_if_due() {
  if (mono_ms() - last_sent_ms_ < 500) return;
  dpwire::Writer m;
  m.u8(dpwire::kHeartbeat);
  send(m.data());
}

std::vector<ChatRequest> DpWorker::poll(size_t max, int timeout_ms, std::vector<std::string>* cancels, bool* shutdown,
                                        std::vector<std::pair<std::string, bool>>* flow) {
  std::vector<ChatRequest> out;
  heartbeat_if_due();
  std::string msg;
  bool got = timeout_ms > 0 ? from_router_->pop_wait(&msg, std::min(timeout_ms, 400)) : from_router_->pop(&msg);
  while (got) {
    dpwire::Reader rd(msg);
    const uint8_t type = rd.u8();
    if (type == dpwire::kRequest) {
      ChatRequest r;
      if (dpwire::decode_request(rd, &r)) out.push_back(std::move(r));
    } else if (type == dpwire::kCancel) {
      cancels->push_back(rd.str());
    } else if (type == dpwire::kFlow) {
      std::string c = rd.str();
      const bool paused = rd.u8() != 0;
      if (flow) flow->emplace_back(std::move(c), paused);
    } else if (type == dpwire::kShutdown) {
      *shutdown = true;
    }
    if (out.size() >= max) break;
    got = from_router_->pop(&msg);
  }
  if (from_router_->closed()) *shutdown = true;
  return out;
}

bool DpWorker::publish_tokens(const std::vector<std::string>& conv_ids, const std::vector<int>& token_ids,
                              const std::vector<int64_t>& seqs, const std::vector<bool>& dones, int64_t ts,
                              const std::vector<std::string>& texts, const std::vector<int>& finish,
                              const std::vector<int>& prompt_tokens) {
  const size_t n = conv_ids.size();
  dpwire::Writer m;
  m.u8(dpwire::kTokens);
  m.i32((int32_t)n);
  m.i64(ts > 0 ? ts : now_ns());
  static const std::string empty;
  for (size_t i = 0; i < n; ++i) {
    m.str(conv_ids[i]);
    m.i32(token_ids[i]);
    m.i64(seqs[i]);
    m.u8(dones[i] ? 1 : 0);
    m.str(i < texts.size() ? texts[i] : empty);
    m.u8(i < finish.size() ? (uint8_t)finish[i] : 0);
    m.i32(i < prompt_tokens.size() ? prompt_tokens[i] : -1);
  }
  return send(m.data());
}

void DpWorker::hello() {
  dpwire::Writer m;
  m.u8(dpwire::kHello);
  m.i32(worker_);
  send(m.data());
}

void DpWorker::bye() {
  dpwire::Writer m;
  m.u8(dpwire::kBye);
  send(m.data());
}

void DpWorker::stats(double step_s, double batch, double kv_free, double active, const std::vector<double>& ttft,
                     const std::vector<double>& itl, const std::vector<double>& host) {
  dpwire::Writer m;
  m.u8(dpwire::kStats);
  m.f64(step_s);
  m.f64(batch);
  m.f64(kv_free);
  m.f64(active);
  m.i32((int32_t)ttft.size());
  for (double v : ttft) m.f64(v);
  m.i32((int32_t)itl.size());
  for (double v : itl) m.f64(v);
  m.i32((int32_t)host.size());
  for (double v : host) m.f64(v);
  send(m.data());
}

}  // namespace dsse
