#include "server.h"

#include <arpa/inet.h>
#include <fcntl.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/epoll.h>
#include <sys/eventfd.h>
#include <sys/socket.h>
#include <sys/uio.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <cmath>
#include <cstring>
#include <ctime>
#include <map>
#include <random>
#include <unordered_map>

#include "json.h"
#include "metrics.h"
#include "util.h"

namespace dsse {

// ------------------------------------------------------------------ logging
LogLevel& log_level() {
  static LogLevel lvl = [] {
    std::string s = env_str("LOG_LEVEL", "info");
    if (s == "debug") return LogLevel::kDebug;
    if (s == "warn") return LogLevel::kWarn;
    if (s == "error") return LogLevel::kError;
    return LogLevel::kInfo;
  }();
  return lvl;
}

void log_json(LogLevel lvl, const std::string& msg, const std::string& kv) {
  if ((int)lvl < (int)log_level()) return;
  static const char* names[] = {"DEBUG", "INFO", "WARN", "ERROR"};
  char ts[64];
  const int64_t ns = now_ns();
  time_t secs = (time_t)(ns / 1000000000);
  struct tm tmv;
  gmtime_r(&secs, &tmv);
  strftime(ts, sizeof ts, "%Y-%m-%dT%H:%M:%S", &tmv);
  std::string line = "{\"time\":\"";
  line += ts;
  char frac[16];
  snprintf(frac, sizeof frac, ".%03dZ\"", (int)((ns / 1000000) % 1000));
  line += frac;
  line += ",\"level\":\"";
  line += names[(int)lvl];
  line += "\",\"msg\":";
  json_append_string(line, msg);
  if (!kv.empty()) {
    line += ',';
    line += kv;
  }
  line += "}\n";
  fwrite(line.data(), 1, line.size(), stderr);
}

// ------------------------------------------------------------------ request queue
void RequestQueue::push(ChatRequest r) {
  {
    std::lock_guard<std::mutex> g(mu_);
    q_.push_back(std::move(r));
  }
  cv_.notify_one();
}

std::vector<ChatRequest> RequestQueue::pop(size_t max, int timeout_ms) {
  std::vector<ChatRequest> out;
  std::unique_lock<std::mutex> lk(mu_);
  // system_clock deadline: libstdc++ maps steady-clock waits to pthread_cond_clockwait, which the
  // ThreadSanitizer runtime of this toolchain does not intercept (it then reports false double locks
  // and races on everything the mutex protects); pthread_cond_timedwait is understood.
  if (q_.empty() && timeout_ms > 0 && !closed_)
    cv_.wait_until(lk, std::chrono::system_clock::now() + std::chrono::milliseconds(timeout_ms),
                   [&] { return !q_.empty() || closed_; });
  while (!q_.empty() && out.size() < max) {
    out.push_back(std::move(q_.front()));
    q_.pop_front();
  }
  return out;
}

size_t RequestQueue::size() {
  std::lock_guard<std::mutex> g(mu_);
  return q_.size();
}

void RequestQueue::close() {
  {
    std::lock_guard<std::mutex> g(mu_);
    closed_ = true;
  }
  cv_.notify_all();
}

// ------------------------------------------------------------------ HTTP helpers
namespace {

enum class Role { kEdge, kOrigin, kMetrics, kResp };

std::string http_date() {
  char b[64];
  time_t t = time(nullptr);
  struct tm tmv;
  gmtime_r(&t, &tmv);
  strftime(b, sizeof b, "%a, %d %b %Y %H:%M:%S GMT", &tmv);
  return b;
}

const char* status_text(int code) {
  switch (code) {
    case 200: return "OK";
    case 202: return "Accepted";
    case 400: return "Bad Request";
    case 404: return "Not Found";
    case 405: return "Method Not Allowed";
    case 411: return "Length Required";
    case 413: return "Request Entity Too Large";
    case 500: return "Internal Server Error";
    case 503: return "Service Unavailable";
  }
  return "Unknown";
}

struct HttpRequest {
  std::string method, target, path, query, version;
  std::vector<std::pair<std::string, std::string>> headers;  // lower-cased names
  std::string body;
  bool keep_alive = true;
  std::string header(const std::string& name) const {
    for (const auto& h : headers)
      if (h.first == name) return h.second;
    return "";
  }
};

std::string lower(std::string s) {
  for (auto& c : s) c = (char)tolower((unsigned char)c);
  return s;
}
std::string trim(const std::string& s) {
  size_t a = s.find_first_not_of(" \t"), b = s.find_last_not_of(" \t");
  return a == std::string::npos ? "" : s.substr(a, b - a + 1);
}

// Parse one request from `buf`.  Returns >0 bytes consumed, 0 = need more data, -1 = malformed,
// -2 = unsupported body encoding, -3 = too large.
long parse_http(const std::string& buf, HttpRequest& req) {
  const size_t hdr_end = buf.find("\r\n\r\n");
  if (hdr_end == std::string::npos) return buf.size() > 65536 ? -3 : 0;
  size_t pos = buf.find("\r\n");
  const std::string line = buf.substr(0, pos);
  size_t s1 = line.find(' '), s2 = line.rfind(' ');
  if (s1 == std::string::npos || s2 == s1) return -1;
  req.method = line.substr(0, s1);
  req.target = line.substr(s1 + 1, s2 - s1 - 1);
  req.version = line.substr(s2 + 1);
  const size_t qm = req.target.find('?');
  req.path = qm == std::string::npos ? req.target : req.target.substr(0, qm);
  req.query = qm == std::string::npos ? "" : req.target.substr(qm + 1);
  size_t p = pos + 2;
  long content_length = 0;
  bool chunked = false;
  req.keep_alive = req.version == "HTTP/1.1";
  while (p < hdr_end) {
    size_t e = buf.find("\r\n", p);
    const std::string h = buf.substr(p, e - p);
    p = e + 2;
    const size_t c = h.find(':');
    if (c == std::string::npos) continue;
    std::string name = lower(trim(h.substr(0, c))), val = trim(h.substr(c + 1));
    if (name == "content-length") content_length = strtol(val.c_str(), nullptr, 10);
    if (name == "transfer-encoding" && lower(val).find("chunked") != std::string::npos) chunked = true;
    if (name == "connection") {
      const std::string lv = lower(val);
      if (lv.find("close") != std::string::npos) req.keep_alive = false;
      if (lv.find("keep-alive") != std::string::npos) req.keep_alive = true;
    }
    req.headers.emplace_back(std::move(name), std::move(val));
  }
  const size_t body_start = hdr_end + 4;
  if (chunked) {
    // decode a chunked request body
    size_t q = body_start;
    std::string body;
    while (true) {
      size_t e = buf.find("\r\n", q);
      if (e == std::string::npos) return 0;
      long n = strtol(buf.substr(q, e - q).c_str(), nullptr, 16);
      if (n < 0) return -1;
      if (n == 0) {
        size_t fin = buf.find("\r\n", e + 2);
        if (fin == std::string::npos) return 0;
        req.body = std::move(body);
        return (long)(fin + 2);
      }
      if (buf.size() < e + 2 + n + 2) return 0;
      body.append(buf, e + 2, n);
      q = e + 2 + n + 2;
      if (body.size() > (1 << 20)) return -3;
    }
  }
  if (content_length < 0) return -1;
  if (content_length > (1 << 20)) return -3;
  if (buf.size() < body_start + (size_t)content_length) return 0;
  req.body = buf.substr(body_start, content_length);
  return (long)(body_start + content_length);
}

// Go http.Error(): text/plain body with a trailing newline.
std::string simple_response(int code, const std::string& body, const std::string& ctype, bool keep_alive,
                            const std::vector<std::string>& extra = {}) {
  std::string r = "HTTP/1.1 " + std::to_string(code) + " " + status_text(code) + "\r\n";
  for (const auto& h : extra) r += h + "\r\n";
  if (!ctype.empty()) r += "Content-Type: " + ctype + "\r\n";
  r += "Date: " + http_date() + "\r\n";
  r += "Content-Length: " + std::to_string(body.size()) + "\r\n";
  if (!keep_alive) r += "Connection: close\r\n";
  r += "\r\n";
  r += body;
  return r;
}
// Optional sampling fields of a /chat body ({message, conversation_id} plus max_tokens, temperature, top_p,
// top_k, seed, ignore_eos).  Integers must be integral and in range BEFORE any conversion (a double outside the
// target type's range is undefined behaviour to cast): false with *err otherwise -> 400.
bool parse_sampling(const std::map<std::string, JsonValue>& o, ChatRequest& r, std::string* err) {
  auto num = [&](const char* k, double dflt) {
    auto it = o.find(k);
    return (it != o.end() && it->second.kind == JsonValue::kNumber) ? it->second.num : dflt;
  };
  auto int_param = [&](const char* k, double lo, double hi, int64_t* out) {
    const double v = num(k, -1);
    if (v == -1) return true;  // absent (or the legacy "unset" marker)
    if (!(v >= lo && v <= hi) || v != std::floor(v)) {
      *err = std::string(k) + " must be an integer in [" + std::to_string((long long)lo) + ", " +
             std::to_string((long long)hi) + "]";
      return false;
    }
    *out = (int64_t)v;
    return true;
  };
  int64_t max_tokens = -1, top_k = -1, seed = -1;
  if (!int_param("max_tokens", 1, 1 << 20, &max_tokens) || !int_param("top_k", -1, 1 << 20, &top_k) ||
      !int_param("seed", 0, 9007199254740991.0, &seed))  // 2^53 - 1: every such double is exact
    return false;
  const double temperature = num("temperature", -1), top_p = num("top_p", -1);
  if (!std::isfinite(temperature) || !std::isfinite(top_p)) {
    *err = "temperature and top_p must be finite";
    return false;
  }
  r.max_tokens = (int)max_tokens;
  r.top_k = (int)top_k;
  r.seed = seed;
  r.temperature = temperature;
  r.top_p = top_p;
  auto ie = o.find("ignore_eos");
  r.ignore_eos = ie != o.end() && ie->second.kind == JsonValue::kBool && ie->second.b;
  return true;
}

std::string http_error(int code, const std::string& msg, bool ka) {
  return simple_response(code, msg + "\n", "text/plain; charset=utf-8", ka, {"X-Content-Type-Options: nosniff"});
}

const char* kSseHeaders =
    "HTTP/1.1 200 OK\r\n"
    "Access-Control-Allow-Origin: *\r\n"
    "Cache-Control: no-cache\r\n"
    "Connection: keep-alive\r\n"
    "Content-Type: text/event-stream\r\n"
    "X-Accel-Buffering: no\r\n"
    "Transfer-Encoding: chunked\r\n";

void append_chunk(std::string& out, const char* data, size_t n) {
  if (n == 0) return;
  char h[24];
  int k = snprintf(h, sizeof h, "%zx\r\n", n);
  out.append(h, k);
  out.append(data, n);
  out += "\r\n";
}

bool glob_match(const char* p, const char* s) {
  for (; *p; ++p, ++s) {
    if (*p == '*') {
      while (*p == '*') ++p;
      if (!*p) return true;
      for (; *s; ++s)
        if (glob_match(p, s)) return true;
      return false;
    }
    if (!*s) return false;
    if (*p != '?' && *p != *s) return false;
  }
  return !*s;
}

std::string resp_bulk(std::string_view s) {
  std::string o = "$" + std::to_string(s.size()) + "\r\n";
  o.append(s.data(), s.size());
  o += "\r\n";
  return o;
}

// The conversation a control-subject message targets, or "" when `subject` is not a control subject:
//   chat.<id>.control   (the CHAT_CONTROL stream, kubernetes/base/nats-core/core-cluster.yaml:246-255)
//   chat.control.kill   payload = the conversation id, raw or {"conversation_id": ...}
//                       (docs/security-inspection-patterns.md:118-123)
std::string control_target(const std::string& subject, const std::string& payload) {
  if (subject == "chat.control.kill") {
    std::map<std::string, JsonValue> o;
    if (parse_json_object(payload, o)) {
      auto it = o.find("conversation_id");
      return (it != o.end() && it->second.kind == JsonValue::kString) ? it->second.str : std::string();
    }
    size_t b = payload.find_first_not_of(" \t\r\n\""), e = payload.find_last_not_of(" \t\r\n\"");
    return b == std::string::npos ? std::string() : payload.substr(b, e - b + 1);
  }
  const std::string pre = "chat.", suf = ".control";
  if (subject.size() > pre.size() + suf.size() && subject.rfind(pre, 0) == 0 &&
      subject.compare(subject.size() - suf.size(), suf.size(), suf) == 0)
    return subject.substr(pre.size(), subject.size() - pre.size() - suf.size());
  return std::string();
}
bool is_control_subject(const std::string& subject) {
  return subject == "chat.control.kill" ||
         (subject.rfind("chat.", 0) == 0 && subject.size() > 13 && subject.compare(subject.size() - 8, 8, ".control") == 0);
}

}  // namespace

// ------------------------------------------------------------------ connections / I/O thread
struct Conn {
  int fd = -1;
  uint64_t id = 0;
  Role role = Role::kEdge;
  std::string in;
  std::string out;
  size_t out_off = 0;
  bool want_write = false;
  bool close_after_write = false;
  bool keep_alive = true;
  // SSE session
  bool sse = false;
  bool chat_mode = false;
  bool got_first = false;
  bool congested = false;  // output queue above flow_high_water (counted in Server::flow_)
  std::string conv_id;
  int64_t sse_start_mono = 0, last_write_mono = 0, first_deadline_mono = 0;
  int64_t after_seq = -1;
  SinkPtr sink;
  std::deque<std::pair<int64_t, FramePtr>> held;  // hybrid inspection delay queue (release time, frame)
  // OpenAI chat completions (vLLM-compatible): frames are re-encoded as chat.completion chunks
  bool openai = false;
  bool oa_stream = true;
  std::string oa_model, oa_text;
  int64_t oa_created = 0;
  int oa_count = 0, oa_max_tokens = -1;
  // RESP
  bool resp_pubsub = false;
  std::vector<std::string> resp_channels, resp_patterns;
};

enum class OutKind { kToken, kError, kResp };
struct OutItem {
  uint64_t conn;
  OutKind kind;
  FramePtr frame;
  std::string text;
};

class IoThread {
 public:
  IoThread(Server& s, int index) : srv_(s), index_(index) {}
  ~IoThread() {
    for (auto& kv : conns_) ::close(kv.first);
    for (auto& l : listeners_) ::close(l.first);
    if (epfd_ >= 0) ::close(epfd_);
    if (evfd_ >= 0) ::close(evfd_);
  }

  bool init(std::string* err);
  bool listen_on(Role role, const std::string& host, int port, int* bound, std::string* err);
  void run();
  void stop() {
    stop_.store(true);
    wake();
  }
  // thread-safe (any thread)
  void enqueue(OutItem item) {
    std::lock_guard<std::mutex> g(out_mu_);
    outbox_.push_back(std::move(item));
  }
  void wake() {
    if (!wake_pending_.exchange(true)) {
      uint64_t one = 1;
      ssize_t r = ::write(evfd_, &one, sizeof one);
      (void)r;
    }
  }
  int index() const { return index_; }

 private:
  struct ConnSink : Sink {
    IoThread* io;
    uint64_t conn;
    std::atomic<size_t>* pending;
    size_t cap;
    bool push(const FramePtr& f) override {
      io->enqueue(OutItem{conn, OutKind::kToken, f, {}});
      return pending->load(std::memory_order_relaxed) < cap;
    }
    void flush() override { io->wake(); }
  };
  struct RespTapSink : Sink {
    IoThread* io;
    uint64_t conn;
    bool push(const FramePtr& f) override {
      io->enqueue(OutItem{conn, OutKind::kResp, f, {}});
      return true;
    }
    void flush() override { io->wake(); }
  };

  void accept_all(int lfd, Role role);
  void on_readable(Conn& c);
  void on_writable(Conn& c);
  void handle_request(Conn& c, HttpRequest& req);
  void handle_resp(Conn& c);
  void start_sse(Conn& c, const std::string& conv_id, bool chat, int64_t after_seq, const std::string& first_bytes,
                 std::vector<FramePtr>* replay);
  void end_sse(Conn& c, bool write_terminator);
  void write_raw(Conn& c, const std::string& data);
  void write_sse_bytes(Conn& c, const std::string& data);
  void deliver_token(Conn& c, const FramePtr& f);
  void handle_openai(Conn& c, HttpRequest& req);
  void deliver_openai(Conn& c, const FramePtr& f);
  void finish_openai(Conn& c, const char* finish_reason, int prompt_tokens = -1);
  void flush_out(Conn& c);
  void close_conn(Conn& c);
  void drain_outbox();
  void timers();
  void update_epoll(Conn& c);

  Server& srv_;
  int index_;
  int epfd_ = -1, evfd_ = -1;
  std::atomic<bool> stop_{false};
  std::atomic<bool> wake_pending_{false};
  std::vector<std::pair<int, Role>> listeners_;
  std::unordered_map<int, Conn> conns_;
  std::unordered_map<uint64_t, int> by_id_;
  std::unordered_map<uint64_t, std::unique_ptr<std::atomic<size_t>>> pending_;
  std::mutex out_mu_;
  std::vector<OutItem> outbox_;
  uint64_t next_id_ = 1;
  int64_t last_timer_ = 0;
};

bool IoThread::init(std::string* err) {
  epfd_ = epoll_create1(EPOLL_CLOEXEC);
  evfd_ = eventfd(0, EFD_NONBLOCK | EFD_CLOEXEC);
  if (epfd_ < 0 || evfd_ < 0) {
    if (err) *err = strerror(errno);
    return false;
  }
  epoll_event ev{};
  ev.events = EPOLLIN;
  ev.data.fd = evfd_;
  epoll_ctl(epfd_, EPOLL_CTL_ADD, evfd_, &ev);
  return true;
}

bool IoThread::listen_on(Role role, const std::string& host, int port, int* bound, std::string* err) {
  int fd = socket(AF_INET, SOCK_STREAM | SOCK_NONBLOCK | SOCK_CLOEXEC, 0);
  if (fd < 0) {
    if (err) *err = strerror(errno);
    return false;
  }
  int one = 1;
  setsockopt(fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
  setsockopt(fd, SOL_SOCKET, SO_REUSEPORT, &one, sizeof one);
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_port = htons((uint16_t)port);
  a.sin_addr.s_addr = host == "0.0.0.0" ? INADDR_ANY : inet_addr(host.c_str());
  if (bind(fd, (sockaddr*)&a, sizeof a) < 0 || listen(fd, 4096) < 0) {
    if (err) *err = std::string("bind/listen port ") + std::to_string(port) + ": " + strerror(errno);
    ::close(fd);
    return false;
  }
  socklen_t len = sizeof a;
  getsockname(fd, (sockaddr*)&a, &len);
  if (bound) *bound = ntohs(a.sin_port);
  epoll_event ev{};
  ev.events = EPOLLIN;
  ev.data.fd = fd;
  epoll_ctl(epfd_, EPOLL_CTL_ADD, fd, &ev);
  listeners_.emplace_back(fd, role);
  return true;
}

void IoThread::update_epoll(Conn& c) {
  epoll_event ev{};
  ev.events = EPOLLIN | EPOLLRDHUP | (c.want_write ? EPOLLOUT : 0);
  ev.data.fd = c.fd;
  epoll_ctl(epfd_, EPOLL_CTL_MOD, c.fd, &ev);
}

void IoThread::accept_all(int lfd, Role role) {
  while (true) {
    int fd = accept4(lfd, nullptr, nullptr, SOCK_NONBLOCK | SOCK_CLOEXEC);
    if (fd < 0) return;
    int one = 1;
    setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
    if (srv_.config().socket_sndbuf > 0)
      setsockopt(fd, SOL_SOCKET, SO_SNDBUF, &srv_.config().socket_sndbuf, sizeof(int));
    Conn c;
    c.fd = fd;
    c.id = ((uint64_t)index_ << 48) | next_id_++;
    c.role = role;
    by_id_[c.id] = fd;
    pending_[c.id] = std::make_unique<std::atomic<size_t>>(0);
    conns_.emplace(fd, std::move(c));
    epoll_event ev{};
    ev.events = EPOLLIN | EPOLLRDHUP;
    ev.data.fd = fd;
    epoll_ctl(epfd_, EPOLL_CTL_ADD, fd, &ev);
  }
}

void IoThread::close_conn(Conn& c) {
  if (c.sse) end_sse(c, false);
  if (c.role == Role::kResp && c.sink) srv_.bus().remove_tap(c.sink);
  epoll_ctl(epfd_, EPOLL_CTL_DEL, c.fd, nullptr);
  ::close(c.fd);
  by_id_.erase(c.id);
  pending_.erase(c.id);
  const int fd = c.fd;
  conns_.erase(fd);
}

void IoThread::flush_out(Conn& c) {
  while (c.out_off < c.out.size()) {
    ssize_t n = ::send(c.fd, c.out.data() + c.out_off, c.out.size() - c.out_off, MSG_NOSIGNAL);
    if (n > 0) {
      c.out_off += (size_t)n;
      continue;
    }
    if (n < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) break;
    c.out.clear();
    c.out_off = 0;
    c.close_after_write = true;  // peer gone
    break;
  }
  if (c.out_off == c.out.size()) {
    c.out.clear();
    c.out_off = 0;
  } else if (c.out_off > (1 << 16)) {
    c.out.erase(0, c.out_off);
    c.out_off = 0;
  }
  const size_t pend = c.out.size() - c.out_off;
  auto pit = pending_.find(c.id);
  if (pit != pending_.end()) pit->second->store(pend, std::memory_order_relaxed);
  const size_t hw = srv_.config().flow_high_water;
  if (hw && c.sse && c.sink) {
    if (!c.congested && pend > hw) {
      c.congested = true;
      srv_.flow_update(c.conv_id, +1);
    } else if (c.congested && pend < hw / 4) {
      c.congested = false;
      srv_.flow_update(c.conv_id, -1);
    }
  }
  const bool ww = c.out_off < c.out.size();
  if (ww != c.want_write) {
    c.want_write = ww;
    update_epoll(c);
  }
}

void IoThread::write_raw(Conn& c, const std::string& data) {
  c.out += data;
  flush_out(c);
}

void IoThread::write_sse_bytes(Conn& c, const std::string& data) {
  append_chunk(c.out, data.data(), data.size());
  c.last_write_mono = mono_ns();
  flush_out(c);
}

void IoThread::start_sse(Conn& c, const std::string& conv_id, bool chat, int64_t after_seq,
                         const std::string& first_bytes, std::vector<FramePtr>* replay) {
  c.sse = true;
  c.chat_mode = chat;
  c.got_first = false;
  c.conv_id = conv_id;
  c.after_seq = after_seq;
  c.sse_start_mono = c.last_write_mono = mono_ns();
  c.first_deadline_mono = c.sse_start_mono + (int64_t)srv_.config().first_token_timeout_ms * 1000000LL;
  metrics().sse_active_connections.add(1);
  metrics().sse_total_connections.inc();
  std::string hdr = kSseHeaders;
  hdr += "Date: " + http_date() + "\r\n\r\n";
  c.out += hdr;
  append_chunk(c.out, first_bytes.data(), first_bytes.size());
  c.last_write_mono = mono_ns();
  flush_out(c);
  if (replay) {
    for (const auto& f : *replay) {
      if (!c.sse) break;
      deliver_token(c, f);
    }
  }
}

void IoThread::end_sse(Conn& c, bool write_terminator) {
  if (!c.sse) return;
  c.sse = false;
  if (c.sink) {
    srv_.bus().unsubscribe(c.conv_id, c.sink);
    srv_.flow_update(c.conv_id, c.congested ? -1 : 0);
    c.congested = false;
    if (c.chat_mode && !srv_.bus().conversation_done(c.conv_id) && srv_.bus().subscriber_count(c.conv_id) == 0)
      srv_.note_cancel(c.conv_id);
    c.sink.reset();
  }
  c.held.clear();
  c.openai = false;
  metrics().sse_active_connections.add(-1);
  metrics().sse_connection_duration_seconds.observe((mono_ns() - c.sse_start_mono) / 1e9);
  if (write_terminator) {
    c.out += "0\r\n\r\n";
    if (!c.keep_alive) c.close_after_write = true;
    flush_out(c);
  }
}

void IoThread::deliver_token(Conn& c, const FramePtr& f) {
  if (!c.sse) return;
  // Last-Event-ID filter (strictly greater: fixes the reference's off-by-one)
  if (c.after_seq >= 0 && f->seq <= c.after_seq && !f->done) return;
  if (c.openai) {
    deliver_openai(c, f);
    return;
  }
  // with a remote inspection gate the bus has already applied the verdict to this frame
  const InspectionMode mode = srv_.remote_inspection() ? InspectionMode::kDisabled : srv_.config().inspection;
  if (mode == InspectionMode::kHybrid) {
    c.held.emplace_back(mono_ns() + (int64_t)srv_.config().inspection_buffer_ms * 1000000LL, f);
    return;
  }
  FramePtr out = f;
  if (mode == InspectionMode::kInline && !f->done) {
    TokenMessage m;
    if (parse_token_message(f->json(), m)) {
      InspectionResult r = inspect_message(m.token);
      if (r.action == InspectAction::kDrop) {
        metrics().inspection_dropped_total.inc();
        return;
      }
      if (r.action == InspectAction::kRedact) {
        metrics().inspection_redacted_total.inc();
        m.token = r.redacted_content;
        out = Bus::make_frame(m);
      }
    }
  }
  const size_t pend = c.out.size() - c.out_off;
  if (pend > srv_.config().max_pending_bytes && !out->done) {
    metrics().bus_dropped_tokens_total.inc();
    return;
  }
  c.got_first = true;
  append_chunk(c.out, out->bytes.data(), out->bytes.size());
  c.last_write_mono = mono_ns();
  metrics().sse_messages_delivered_total.inc();
  if (out->timestamp > 0) {  // producers may send ms timestamps (run-demo.sh): keep plausible values only
    const double d = (now_ns() - out->timestamp) * 1e-9;
    if (d >= 0 && d < 60) metrics().sse_delivery_latency_seconds.observe(d);
  }
  if (out->done) {
    end_sse(c, true);
    return;
  }
  flush_out(c);
}

// ---- OpenAI-compatible chat completions (the vLLM surface the reference proxy consumes) ----------------
// POST /v1/chat/completions {"model","messages":[{"role","content"}..],"stream",...} -> either an SSE stream of
// chat.completion.chunk objects ending with `data: [DONE]` (stream: true; the exact lines the reference's
// llm-stream-proxy parses, src/llm-stream-proxy/main.go:34-52,192-227) or one chat.completion object.  The
// request goes to the same engine queue as POST /chat; the engine's TokenMessages for the conversation are
// re-encoded per connection.  GET /v1/models lists the served model.
namespace {
std::string openai_error(int code, const std::string& msg, const char* type) {
  return "{\"object\":\"error\",\"message\":" + json_quote(msg) + ",\"type\":\"" + type + "\",\"param\":null,\"code\":" +
         std::to_string(code) + "}";
}
}  // namespace

void IoThread::handle_openai(Conn& c, HttpRequest& req) {
  const bool ka = req.keep_alive;
  const std::string& model = srv_.config().model_name;
  if (req.path == "/v1/models") {
    const std::string body = "{\"object\":\"list\",\"data\":[{\"id\":" + json_quote(model) +
                             ",\"object\":\"model\",\"created\":" + std::to_string((long long)time(nullptr)) +
                             ",\"owned_by\":\"dsse\",\"root\":" + json_quote(model) + ",\"parent\":null}]}";
    write_raw(c, simple_response(200, body, "application/json", ka));
    return;
  }
  auto bad = [&](int code, const std::string& m) {
    write_raw(c, simple_response(code, openai_error(code, m, code == 404 ? "NotFoundError" : "BadRequestError"),
                                 "application/json", ka));
  };
  if (req.method != "POST") {
    write_raw(c, http_error(405, "Method not allowed", ka));
    return;
  }
  if (!srv_.local_engine()) {
    write_raw(c, simple_response(503, openai_error(503, "no engine attached", "ServiceUnavailableError"),
                                 "application/json", ka));
    return;
  }
  std::map<std::string, JsonValue> o;
  if (!parse_json_object(req.body, o)) return bad(400, "Invalid JSON body");
  auto mi = o.find("messages");
  std::vector<std::map<std::string, JsonValue>> msgs;
  if (mi == o.end() || mi->second.kind != JsonValue::kArray || !parse_json_array_of_objects(mi->second.raw, msgs) ||
      msgs.empty())
    return bad(400, "messages must be a non-empty array of {role, content} objects");
  std::string norm = "[", last_user;
  // The Mistral instruct template accepts system messages first, then user/assistant turns that alternate
  // starting and ending with user (vLLM returns 400 on anything else): validate here, so a malformed
  // conversation never reaches the engine's tokenizer.
  std::string expect = "user";
  bool seen_turn = false;
  for (size_t i = 0; i < msgs.size(); ++i) {
    auto& m = msgs[i];
    auto r = m.find("role");
    auto ct = m.find("content");
    if (r == m.end() || r->second.kind != JsonValue::kString) return bad(400, "every message needs a string role");
    const std::string& role = r->second.str;
    if (role != "system" && role != "user" && role != "assistant")
      return bad(400, "unsupported message role '" + role + "' (system, user, assistant)");
    if (role == "system") {
      if (seen_turn) return bad(400, "system messages must come before the conversation turns");
    } else {
      if (role != expect) return bad(400, "conversation roles must alternate user/assistant/user/...");
      expect = role == "user" ? "assistant" : "user";
      seen_turn = true;
    }
    std::string text;
    if (ct != m.end() && ct->second.kind == JsonValue::kString) {
      text = ct->second.str;
    } else if (ct != m.end() && ct->second.kind == JsonValue::kArray) {  // [{"type":"text","text":..}]
      std::vector<std::map<std::string, JsonValue>> parts;
      if (!parse_json_array_of_objects(ct->second.raw, parts)) return bad(400, "invalid content parts");
      for (auto& pt : parts) {
        auto tx = pt.find("text");
        if (tx != pt.end() && tx->second.kind == JsonValue::kString) text += tx->second.str;
      }
    } else if (!(ct != m.end() && ct->second.kind == JsonValue::kNull)) {
      return bad(400, "every message needs string content");
    }
    if (r->second.str == "user") last_user = text;
    norm += (i ? ",{\"role\":" : "{\"role\":") + json_quote(r->second.str) + ",\"content\":" + json_quote(text) + "}";
  }
  norm += "]";
  if (expect != "assistant") return bad(400, "the last conversation turn must be a user message");
  auto num = [&](const char* k, double dflt) {
    auto it2 = o.find(k);
    return (it2 != o.end() && it2->second.kind == JsonValue::kNumber) ? it2->second.num : dflt;
  };
  // integer parameters: reject fractional / out-of-range values before any conversion (a double outside
  // the target range is undefined behaviour to cast)
  std::string int_err;
  auto int_param = [&](const char* k, double lo, double hi) -> int64_t {
    const double v = num(k, -1);
    if (v == -1) return -1;
    if (!(v >= lo && v <= hi) || v != std::floor(v)) {
      if (int_err.empty()) int_err = std::string(k) + " must be an integer in [" + std::to_string((long long)lo) + ", " +
                                     std::to_string((long long)hi) + "]";
      return -1;
    }
    return (int64_t)v;
  };
  if (num("n", 1) != 1) return bad(400, "only n = 1 is supported");
  int64_t max_tokens = int_param("max_tokens", 1, 1 << 20);
  if (max_tokens < 0) max_tokens = int_param("max_completion_tokens", 1, 1 << 20);
  const int64_t top_k = int_param("top_k", -1, 1 << 20);
  const int64_t seed = int_param("seed", 0, 9007199254740991.0);  // 2^53 - 1: every such double is exact
  if (!int_err.empty()) return bad(400, int_err);
  const double temperature = num("temperature", -1), top_p = num("top_p", -1);
  if (!std::isfinite(temperature) || !std::isfinite(top_p)) return bad(400, "temperature and top_p must be finite");
  auto st = o.find("stream");
  const bool stream = st != o.end() && st->second.kind == JsonValue::kBool && st->second.b;
  std::string id = uuid4();
  id.erase(std::remove(id.begin(), id.end(), '-'), id.end());
  const std::string conv = "chatcmpl-" + id;
  ChatRequest r;
  r.conversation_id = conv;
  r.message = last_user;
  r.messages_json = norm;
  r.max_tokens = (int)max_tokens;
  r.temperature = temperature;
  r.top_p = top_p;
  r.top_k = (int)top_k;
  r.seed = seed;
  {
    auto ie = o.find("ignore_eos");
    r.ignore_eos = ie != o.end() && ie->second.kind == JsonValue::kBool && ie->second.b;
  }
  r.from_edge = true;
  auto mo = o.find("model");
  c.openai = true;
  c.oa_stream = stream;
  c.oa_model = (mo != o.end() && mo->second.kind == JsonValue::kString && !mo->second.str.empty()) ? mo->second.str : model;
  c.oa_created = (int64_t)time(nullptr);
  c.oa_count = 0;
  c.oa_max_tokens = r.max_tokens;
  c.oa_text.clear();
  // subscribe before submitting, as POST /chat does
  auto sink = std::make_shared<ConnSink>();
  sink->io = this;
  sink->conn = c.id;
  sink->pending = pending_[c.id].get();
  sink->cap = srv_.config().max_pending_bytes;
  c.sink = sink;
  srv_.bus().subscribe(conv, sink, -1, nullptr);
  srv_.flow_update(conv, 0);
  if (stream) {
    const std::string first = "data: {\"id\":" + json_quote(conv) + ",\"object\":\"chat.completion.chunk\",\"created\":" +
                              std::to_string(c.oa_created) + ",\"model\":" + json_quote(c.oa_model) +
                              ",\"choices\":[{\"index\":0,\"delta\":{\"role\":\"assistant\",\"content\":\"\"},"
                              "\"logprobs\":null,\"finish_reason\":null}]}\n\n";
    start_sse(c, conv, true, -1, first, nullptr);
  } else {  // buffered: no HTTP response until the completion is done
    c.sse = true;
    c.chat_mode = true;
    c.got_first = false;
    c.conv_id = conv;
    c.after_seq = -1;
    c.sse_start_mono = c.last_write_mono = mono_ns();
    c.first_deadline_mono = c.sse_start_mono + (int64_t)srv_.config().first_token_timeout_ms * 1000000LL;
    metrics().sse_active_connections.add(1);
    metrics().sse_total_connections.inc();
  }
  srv_.submit_chat(std::move(r));
}

void IoThread::deliver_openai(Conn& c, const FramePtr& f) {
  TokenMessage m;
  if (!parse_token_message(f->json(), m)) return;
  if (f->done) {
    // vLLM's finish_reason: the engine's own reason when it sent one (EOS = stop; max_tokens or the context
    // limit = length; cancelled = abort), else from the terminal token and the count
    const char* reason;
    if (f->finish == kFinishStop) reason = "stop";
    else if (f->finish == kFinishLength) reason = "length";
    else if (f->finish == kFinishAbort || m.token == "[ERROR]" || m.token == "[BLOCKED]" || m.token == "[KILLED]") reason = "abort";
    else reason = c.oa_max_tokens > 0 && c.oa_count >= c.oa_max_tokens ? "length" : "stop";
    return finish_openai(c, reason, f->prompt_tokens);
  }
  c.got_first = true;
  ++c.oa_count;
  metrics().sse_messages_delivered_total.inc();
  if (!c.oa_stream) {
    c.oa_text += m.token;
    return;
  }
  const size_t pend = c.out.size() - c.out_off;
  if (pend > srv_.config().max_pending_bytes) {
    metrics().bus_dropped_tokens_total.inc();
    return;
  }
  std::string ev = "data: {\"id\":";
  json_append_string(ev, c.conv_id);
  ev += ",\"object\":\"chat.completion.chunk\",\"created\":" + std::to_string(c.oa_created) + ",\"model\":";
  json_append_string(ev, c.oa_model);
  ev += ",\"choices\":[{\"index\":0,\"delta\":{\"content\":";
  json_append_string(ev, m.token);
  ev += "},\"logprobs\":null,\"finish_reason\":null}]}\n\n";
  write_sse_bytes(c, ev);
}

void IoThread::finish_openai(Conn& c, const char* finish_reason, int prompt_tokens) {
  if (!c.sse) return;
  const int pt = std::max(0, prompt_tokens);
  const std::string head = "{\"id\":" + json_quote(c.conv_id) + ",\"object\":\"chat.completion" +
                           std::string(c.oa_stream ? ".chunk" : "") + "\",\"created\":" + std::to_string(c.oa_created) +
                           ",\"model\":" + json_quote(c.oa_model) + ",\"choices\":[{\"index\":0,";
  const std::string usage = "\"usage\":{\"prompt_tokens\":" + std::to_string(pt) + ",\"total_tokens\":" +
                            std::to_string(pt + c.oa_count) + ",\"completion_tokens\":" + std::to_string(c.oa_count) + "}";
  if (c.oa_stream) {
    std::string ev = "data: " + head + "\"delta\":{},\"logprobs\":null,\"finish_reason\":\"" + finish_reason +
                     "\",\"stop_reason\":null}]}\n\ndata: [DONE]\n\n";
    append_chunk(c.out, ev.data(), ev.size());
    end_sse(c, true);
    return;
  }
  const bool ka = c.keep_alive;
  std::string body = head + "\"message\":{\"role\":\"assistant\",\"content\":" + json_quote(c.oa_text) +
                     ",\"tool_calls\":[]},\"logprobs\":null,\"finish_reason\":\"" + finish_reason +
                     "\",\"stop_reason\":null}]," + usage + "}";
  // buffered mode never wrote headers: close the pseudo-SSE session, then send one JSON response (and close
  // the connection after it when the client asked for Connection: close)
  end_sse(c, false);
  c.oa_text.clear();
  write_raw(c, simple_response(200, body, "application/json", ka));
  if (!ka) {
    c.close_after_write = true;
    flush_out(c);
  }
}

void IoThread::drain_outbox() {
  std::vector<OutItem> items;
  {
    std::lock_guard<std::mutex> g(out_mu_);
    items.swap(outbox_);
  }
  wake_pending_.store(false);
  for (auto& it : items) {
    auto b = by_id_.find(it.conn);
    if (b == by_id_.end()) continue;
    auto cit = conns_.find(b->second);
    if (cit == conns_.end()) continue;
    Conn& c = cit->second;
    switch (it.kind) {
      case OutKind::kToken: deliver_token(c, it.frame); break;
      case OutKind::kError:
        if (c.sse) {
          c.out.reserve(c.out.size() + it.text.size() + 16);
          append_chunk(c.out, it.text.data(), it.text.size());
          end_sse(c, true);
        }
        break;
      case OutKind::kResp: {
        if (!c.resp_pubsub) break;
        const std::string subj = Bus::subject_for(it.frame->conversation_id);
        std::string msg;
        for (const auto& ch : c.resp_channels)
          if (ch == subj) msg += "*3\r\n$7\r\nmessage\r\n" + resp_bulk(ch) + resp_bulk(it.frame->json());
        for (const auto& p : c.resp_patterns)
          if (glob_match(p.c_str(), subj.c_str()))
            msg += "*4\r\n$8\r\npmessage\r\n" + resp_bulk(p) + resp_bulk(subj) + resp_bulk(it.frame->json());
        if (!msg.empty()) write_raw(c, msg);
        break;
      }
    }
    if (c.close_after_write && c.out_off >= c.out.size()) close_conn(c);
  }
}

void IoThread::timers() {
  const int64_t now = mono_ns();
  if (now - last_timer_ < 50 * 1000000LL) return;
  last_timer_ = now;
  const int64_t ka = (int64_t)srv_.config().keepalive_ms * 1000000LL;
  std::vector<int> to_close;
  for (auto& kv : conns_) {
    Conn& c = kv.second;
    if (!c.sse) continue;
    // hybrid inspection: release frames whose buffer window has passed
    while (!c.held.empty() && c.held.front().first <= now && c.sse) {
      FramePtr f = c.held.front().second;
      c.held.pop_front();
      TokenMessage m;
      if (!f->done && parse_token_message(f->json(), m)) {
        InspectionResult r = inspect_message(m.token);
        if (r.action == InspectAction::kDrop) {
          metrics().inspection_dropped_total.inc();
          continue;
        }
        if (r.action == InspectAction::kRedact) {
          metrics().inspection_redacted_total.inc();
          m.token = r.redacted_content;
          f = Bus::make_frame(m);
        }
      }
      c.got_first = true;
      append_chunk(c.out, f->bytes.data(), f->bytes.size());
      c.last_write_mono = now;
      metrics().sse_messages_delivered_total.inc();
      if (f->done) end_sse(c, true);
      else flush_out(c);
    }
    if (!c.sse) continue;
    if (c.openai) {
      if (!c.got_first && now >= c.first_deadline_mono) finish_openai(c, "abort");
      else if (c.oa_stream && now - c.last_write_mono >= ka) write_sse_bytes(c, ": keep-alive\n\n");
      if (c.close_after_write && c.out_off >= c.out.size()) to_close.push_back(c.fd);
      continue;
    }
    if (c.chat_mode && !c.got_first && now >= c.first_deadline_mono) {
      const std::string e = "event: error\ndata: {\"error\":\"timeout waiting for response\"}\n\n";
      append_chunk(c.out, e.data(), e.size());
      end_sse(c, true);
      continue;
    }
    if (now - c.last_write_mono >= ka) write_sse_bytes(c, ": keep-alive\n\n");
    if (c.close_after_write && c.out_off >= c.out.size()) to_close.push_back(c.fd);
  }
  for (int fd : to_close) {
    auto it = conns_.find(fd);
    if (it != conns_.end()) close_conn(it->second);
  }
}

void IoThread::on_writable(Conn& c) {
  flush_out(c);
  if (c.close_after_write && c.out_off >= c.out.size()) close_conn(c);
}

void IoThread::on_readable(Conn& c) {
  char buf[16384];
  bool peer_closed = false;
  while (true) {
    ssize_t n = ::recv(c.fd, buf, sizeof buf, 0);
    if (n > 0) {
      if (!c.sse) c.in.append(buf, (size_t)n);
      continue;
    }
    if (n == 0) peer_closed = true;
    else if (errno != EAGAIN && errno != EWOULDBLOCK) peer_closed = true;
    break;
  }
  if (c.role == Role::kResp) {
    handle_resp(c);
  } else {
    while (!c.sse && !c.in.empty() && !c.close_after_write) {
      HttpRequest req;
      long used = parse_http(c.in, req);
      if (used == 0) break;
      if (used < 0) {
        write_raw(c, http_error(used == -3 ? 413 : (used == -2 ? 411 : 400),
                                used == -3 ? "request too large" : "malformed request", false));
        c.close_after_write = true;
        c.in.clear();
        break;
      }
      c.in.erase(0, (size_t)used);
      c.keep_alive = req.keep_alive;
      handle_request(c, req);
      if (!c.keep_alive && !c.sse) c.close_after_write = true;
    }
  }
  auto it = conns_.find(c.fd);
  if (it == conns_.end()) return;
  if (peer_closed || (c.close_after_write && c.out_off >= c.out.size())) close_conn(c);
}

void IoThread::handle_request(Conn& c, HttpRequest& req) {
  const bool ka = req.keep_alive;
  const std::string& path = req.path;
  if (c.role == Role::kMetrics) {
    if (path == "/metrics") write_raw(c, simple_response(200, metrics().render(), "text/plain; version=0.0.4", ka));
    else write_raw(c, http_error(404, "404 page not found", ka));
    return;
  }
  if (path == "/v1/chat/completions" || path == "/v1/models") {  // vLLM's OpenAI surface, both HTTP roles
    handle_openai(c, req);
    return;
  }
  if (c.role == Role::kOrigin) {
    if (path == "/health") {
      write_raw(c, simple_response(200, "ok", "text/plain; charset=utf-8", ka));
    } else if (path == "/metrics") {
      write_raw(c, simple_response(200, metrics().render_origin(), "text/plain; charset=utf-8", ka));
    } else if (path == "/chat") {
      if (req.method != "POST") {
        write_raw(c, http_error(405, "Method not allowed", ka));
        return;
      }
      std::map<std::string, JsonValue> o;
      if (!parse_json_object(req.body, o)) {
        write_raw(c, http_error(400, "Invalid request body", ka));
        return;
      }
      auto mi = o.find("message");
      auto ci = o.find("conversation_id");
      if ((mi != o.end() && mi->second.kind != JsonValue::kString && mi->second.kind != JsonValue::kNull) ||
          (ci != o.end() && ci->second.kind != JsonValue::kString && ci->second.kind != JsonValue::kNull)) {
        write_raw(c, http_error(400, "Invalid request body", ka));
        return;
      }
      const std::string msg = mi == o.end() ? "" : mi->second.str;
      if (msg.empty()) {
        write_raw(c, http_error(400, "Message is required", ka));
        return;
      }
      std::string conv = ci == o.end() ? "" : ci->second.str;
      if (conv.empty()) conv = uuid4();
      ChatRequest r;
      r.conversation_id = conv;
      r.message = msg;
      std::string perr;
      if (!parse_sampling(o, r, &perr)) {
        write_raw(c, http_error(400, perr, ka));
        return;
      }
      srv_.submit_chat(std::move(r));
      write_raw(c, simple_response(200, "{\"conversation_id\":" + json_quote(conv) + ",\"status\":\"streaming\"}\n",
                                   "application/json", ka));
    } else {
      write_raw(c, http_error(404, "404 page not found", ka));
    }
    return;
  }
  // ---- edge role ----
  if (path == "/healthz" || path == "/readyz") {
    if (!srv_.ready()) write_raw(c, http_error(503, "engine not ready", ka));
    else write_raw(c, simple_response(200, path == "/healthz" ? "ok" : "ready", "text/plain; charset=utf-8", ka));
    return;
  }
  if (path == "/chat") {
    if (req.method != "POST") {
      if (req.method == "OPTIONS") {
        write_raw(c, simple_response(200, "", "", ka,
                                     {"Access-Control-Allow-Headers: Content-Type",
                                      "Access-Control-Allow-Methods: POST, OPTIONS", "Access-Control-Allow-Origin: *"}));
        return;
      }
      write_raw(c, http_error(405, "Method not allowed", ka));
      return;
    }
    const bool local = srv_.local_engine();
    if (!local && srv_.config().llm_proxy_url.empty()) {
      write_raw(c, http_error(503, "LLM proxy not configured", ka));
      return;
    }
    std::map<std::string, JsonValue> o;
    if (!parse_json_object(req.body, o)) {
      write_raw(c, http_error(400, "Invalid JSON body", ka));
      return;
    }
    auto mi = o.find("message");
    auto ci = o.find("conversation_id");
    if ((mi != o.end() && mi->second.kind != JsonValue::kString && mi->second.kind != JsonValue::kNull) ||
        (ci != o.end() && ci->second.kind != JsonValue::kString && ci->second.kind != JsonValue::kNull)) {
      write_raw(c, http_error(400, "Invalid JSON body", ka));
      return;
    }
    const std::string msg = mi == o.end() ? "" : mi->second.str;
    if (msg.empty()) {
      write_raw(c, http_error(400, "message is required", ka));
      return;
    }
    ChatRequest sampling;
    std::string perr;
    if (!parse_sampling(o, sampling, &perr)) {  // before any SSE byte: a bad parameter is a plain 400
      write_raw(c, http_error(400, perr, ka));
      return;
    }
    std::string conv = ci == o.end() ? "" : ci->second.str;
    if (conv.empty()) conv = uuid4();
    // subscribe BEFORE the request leaves (sse_handler.go:313), so no token can be missed
    auto sink = std::make_shared<ConnSink>();
    sink->io = this;
    sink->conn = c.id;
    sink->pending = pending_[c.id].get();
    sink->cap = srv_.config().max_pending_bytes;
    c.sink = sink;
    srv_.bus().subscribe(conv, sink, -1, nullptr);
    srv_.flow_update(conv, 0);  // an uncongested subscriber resumes a paused conversation
    start_sse(c, conv, true, -1, "event: connected\ndata: {\"conversation_id\":" + json_quote(conv) + "}\n\n", nullptr);
    srv_.relay_ensure(conv);
    if (local) {
      ChatRequest r = std::move(sampling);
      r.conversation_id = conv;
      r.message = msg;
      r.from_edge = true;
      srv_.submit_chat(std::move(r));
    } else {
      srv_.forward_to_proxy(c.id, this, conv, msg);
    }
    return;
  }
  if (path.rfind("/stream/", 0) == 0) {
    std::string conv = path.substr(8);
    while (!conv.empty() && conv.back() == '/') conv.pop_back();
    if (conv.empty()) {
      write_raw(c, http_error(400, "conversation_id required", ka));
      return;
    }
    int64_t after = -1;
    const std::string lei = req.header("last-event-id");
    if (!lei.empty()) after = strtoll(lei.c_str(), nullptr, 10);
    if (req.query.find("replay=1") != std::string::npos && after < 0) after = 0;
    auto sink = std::make_shared<ConnSink>();
    sink->io = this;
    sink->conn = c.id;
    sink->pending = pending_[c.id].get();
    sink->cap = srv_.config().max_pending_bytes;
    c.sink = sink;
    std::vector<FramePtr> replay;
    srv_.bus().subscribe(conv, sink, after, after >= 0 ? &replay : nullptr);
    srv_.flow_update(conv, 0);
    start_sse(c, conv, false, after, ": connected to " + conv + "\n\n", &replay);
    srv_.relay_ensure(conv);
    return;
  }
  if (path.rfind("/publish/", 0) == 0) {
    if (req.method != "POST") {
      write_raw(c, http_error(405, "Method not allowed", ka));
      return;
    }
    // subject chat.<id>.tokens (or a bare conversation id); body: a TokenMessage JSON.  Control subjects
    // (chat.<id>.control, chat.control.kill) end the conversation instead.
    std::string subject = path.substr(9);
    if (is_control_subject(subject)) {
      const std::string conv = control_target(subject, req.body);
      if (conv.empty()) {
        write_raw(c, http_error(400, "control message names no conversation", ka));
        return;
      }
      const bool killed = srv_.kill_conversation(conv, "[KILLED]", "control subject " + subject);
      if (killed) metrics().control_kills_total.inc();
      write_raw(c, simple_response(200, std::string("{\"status\": \"") + (killed ? "killed" : "published") +
                                            "\", \"conversation_id\": " + json_quote(conv) + "}",
                                   "application/json", ka));
      return;
    }
    TokenMessage m;
    if (!parse_token_message(req.body, m)) {
      write_raw(c, http_error(400, "Invalid JSON body", ka));
      return;
    }
    if (m.conversation_id.empty()) {
      std::string id = subject;
      if (id.rfind("chat.", 0) == 0) id = id.substr(5);
      const size_t dot = id.rfind(".tokens");
      if (dot != std::string::npos && dot + 7 == id.size()) id = id.substr(0, dot);
      m.conversation_id = id;
    }
    if (m.timestamp == 0) m.timestamp = now_ns();
    srv_.bus().publish(m);
    write_raw(c, simple_response(200, "{\"status\": \"published\"}", "application/json", ka));
    return;
  }
  if (path == "/inspect") {
    std::map<std::string, JsonValue> o;
    if (!parse_json_object(req.body, o) || o.find("data") == o.end() || o["data"].kind != JsonValue::kString) {
      write_raw(c, http_error(400, "Invalid JSON body", ka));
      return;
    }
    write_raw(c, simple_response(200, inspection_result_json(inspect_message(o["data"].str)), "application/json", ka));
    return;
  }
  if (path == "/" && !srv_.config().ui_html.empty()) {
    write_raw(c, simple_response(200, srv_.config().ui_html, "text/html; charset=utf-8", ka));
    return;
  }
  write_raw(c, http_error(404, "404 page not found", ka));
}

void IoThread::handle_resp(Conn& c) {
  std::string& b = c.in;
  size_t p = 0;
  while (p < b.size()) {
    std::vector<std::string> args;
    size_t q = p;
    if (b[q] == '*') {
      size_t e = b.find("\r\n", q);
      if (e == std::string::npos) break;
      long n = strtol(b.c_str() + q + 1, nullptr, 10);
      q = e + 2;
      bool ok = true;
      for (long i = 0; i < n; ++i) {
        if (q >= b.size()) { ok = false; break; }
        if (b[q] != '$') {
          write_raw(c, "-ERR Protocol error: expected '$'\r\n");
          c.close_after_write = true;
          b.clear();
          return;
        }
        size_t e2 = b.find("\r\n", q);
        if (e2 == std::string::npos) { ok = false; break; }
        long len = strtol(b.c_str() + q + 1, nullptr, 10);
        if (len < 0 || len > (512 << 20)) {
          write_raw(c, "-ERR Protocol error: invalid bulk length\r\n");
          c.close_after_write = true;
          b.clear();
          return;
        }
        if (b.size() < e2 + 2 + (size_t)len + 2) { ok = false; break; }
        args.emplace_back(b, e2 + 2, (size_t)len);
        q = e2 + 2 + (size_t)len + 2;
      }
      if (!ok) break;
    } else {  // inline command
      size_t e = b.find('\n', q);
      if (e == std::string::npos) break;
      std::string line = b.substr(q, e - q);
      if (!line.empty() && line.back() == '\r') line.pop_back();
      q = e + 1;
      size_t s = 0;
      while (s < line.size()) {
        size_t t = line.find(' ', s);
        if (t == std::string::npos) t = line.size();
        if (t > s) args.push_back(line.substr(s, t - s));
        s = t + 1;
      }
    }
    p = q;
    if (args.empty()) continue;
    std::string cmd = lower(args[0]);
    if (cmd == "ping") {
      if (c.resp_pubsub) write_raw(c, "*2\r\n$4\r\npong\r\n" + resp_bulk(args.size() > 1 ? args[1] : ""));
      else write_raw(c, args.size() > 1 ? resp_bulk(args[1]) : "+PONG\r\n");
    } else if (cmd == "publish" && args.size() == 3 && is_control_subject(args[1])) {
      // kill signal: PUBLISH chat.<id>.control <any> / PUBLISH chat.control.kill <conversation id>
      const std::string conv = control_target(args[1], args[2]);
      const bool killed = srv_.kill_conversation(conv, "[KILLED]", "control subject " + args[1]);
      if (killed) metrics().control_kills_total.inc();
      write_raw(c, killed ? ":1\r\n" : ":0\r\n");
    } else if (cmd == "publish" && args.size() == 3) {
      TokenMessage m;
      int n = 0;
      if (parse_token_message(args[2], m) && !m.conversation_id.empty()) {
        // subject from the payload's conversation_id, like the bridge (redis-nats-bridge/main.go:160)
        n = srv_.bus().publish(m);
        metrics().resp_publish_total.inc();
      } else {
        log_json(LogLevel::kWarn, "RESP PUBLISH payload is not a TokenMessage", "\"channel\":" + json_quote(args[1]));
      }
      write_raw(c, ":" + std::to_string(n) + "\r\n");
    } else if ((cmd == "subscribe" || cmd == "psubscribe") && args.size() >= 2) {
      if (!c.resp_pubsub) {
        auto tap = std::make_shared<RespTapSink>();
        tap->io = this;
        tap->conn = c.id;
        c.sink = tap;
        srv_.bus().add_tap(tap);
        c.resp_pubsub = true;
      }
      for (size_t i = 1; i < args.size(); ++i) {
        auto& lst = cmd == "subscribe" ? c.resp_channels : c.resp_patterns;
        lst.push_back(args[i]);
        write_raw(c, "*3\r\n" + resp_bulk(cmd) + resp_bulk(args[i]) + ":" +
                         std::to_string(c.resp_channels.size() + c.resp_patterns.size()) + "\r\n");
      }
    } else if (cmd == "hello") {
      write_raw(c, "-ERR unknown command 'HELLO', with args beginning with: \r\n");
    } else if (cmd == "client" || cmd == "select" || cmd == "auth" || cmd == "readonly") {
      write_raw(c, "+OK\r\n");
    } else if (cmd == "quit") {
      write_raw(c, "+OK\r\n");
      c.close_after_write = true;
      b.clear();
      return;
    } else if (cmd == "echo" && args.size() == 2) {
      write_raw(c, resp_bulk(args[1]));
    } else if (cmd == "info") {
      write_raw(c, resp_bulk("# Server\r\nredis_version:7.0.0\r\nredis_mode:standalone\r\n"));
    } else if (cmd == "command") {
      write_raw(c, "*0\r\n");
    } else {
      write_raw(c, "-ERR unknown command '" + args[0] + "'\r\n");
    }
  }
  b.erase(0, p);
}

void IoThread::run() {
  epoll_event evs[256];
  while (!stop_.load()) {
    int n = epoll_wait(epfd_, evs, 256, 50);
    for (int i = 0; i < n; ++i) {
      const int fd = evs[i].data.fd;
      if (fd == evfd_) {
        uint64_t v;
        ssize_t r = ::read(evfd_, &v, sizeof v);
        (void)r;
        drain_outbox();
        continue;
      }
      bool is_listener = false;
      for (auto& l : listeners_)
        if (l.first == fd) {
          accept_all(fd, l.second);
          is_listener = true;
        }
      if (is_listener) continue;
      auto it = conns_.find(fd);
      if (it == conns_.end()) continue;
      Conn& c = it->second;
      if (evs[i].events & (EPOLLERR)) {
        close_conn(c);
        continue;
      }
      if (evs[i].events & EPOLLOUT) {
        on_writable(c);
        if (conns_.find(fd) == conns_.end()) continue;
      }
      if (evs[i].events & (EPOLLIN | EPOLLRDHUP | EPOLLHUP)) on_readable(it->second);
    }
    drain_outbox();
    timers();
  }
}

// ------------------------------------------------------------------ Server
Server::Server(ServerConfig cfg, std::shared_ptr<Bus> bus) : cfg_(std::move(cfg)), bus_(std::move(bus)) {
  local_engine_.store(cfg_.local_engine);
}

Server::~Server() { stop(); }

bool Server::start(std::string* err) {
  if (running_.load()) return true;
  const int n = std::max(1, cfg_.io_threads);
  std::vector<std::pair<Role, int>> roles;
  // port < 0 = role disabled, 0 = ephemeral (thread 0 binds, the other threads reuse its port)
  if (cfg_.sse_port >= 0) roles.emplace_back(Role::kEdge, cfg_.sse_port);
  if (cfg_.origin_port >= 0) roles.emplace_back(Role::kOrigin, cfg_.origin_port);
  if (cfg_.metrics_port >= 0) roles.emplace_back(Role::kMetrics, cfg_.metrics_port);
  if (cfg_.resp_port >= 0) roles.emplace_back(Role::kResp, cfg_.resp_port);
  auto want = [](int p) { return p; };
  static const char* names[] = {"edge", "origin", "metrics", "resp"};
  for (int i = 0; i < n; ++i) {
    auto io = std::make_unique<IoThread>(*this, i);
    if (!io->init(err)) return false;
    for (auto& rp : roles) {
      int port = want(rp.second);
      if (i > 0) {
        for (auto& kv : ports_)
          if (kv.first == names[(int)rp.first]) port = kv.second;
      }
      int bound = 0;
      if (!io->listen_on(rp.first, cfg_.host, port, &bound, err)) return false;
      if (i == 0) ports_.emplace_back(names[(int)rp.first], bound);
    }
    io_.push_back(std::move(io));
  }
  if (cfg_.inspection == InspectionMode::kAsync) {
    inspector_ = std::make_shared<AsyncInspector>(*this);
    inspector_->start();
    bus_->add_tap(inspector_);
  }
  if (!cfg_.inspection_endpoint.empty() &&
      (cfg_.inspection == InspectionMode::kInline || cfg_.inspection == InspectionMode::kHybrid)) {
    gate_ = std::make_shared<InspectionGate>(*this, 4);
    gate_->start();
    bus_->set_gate(gate_);
  }
  if (!cfg_.upstream_url.empty()) {
    relay_ = std::make_unique<UpstreamRelay>(*bus_, cfg_.upstream_url);
    if (!relay_->start(err)) return false;
  }
  running_.store(true);
  for (auto& io : io_) threads_.emplace_back([p = io.get()] { p->run(); });
  housekeeping_ = std::thread([this] {
    int64_t last_gc = mono_ns();
    while (running_.load()) {
      std::this_thread::sleep_for(std::chrono::milliseconds(200));
      if (mono_ns() - last_gc > 5000000000LL) {
        bus_->gc(now_ns());
        last_gc = mono_ns();
      }
    }
  });
  log_json(LogLevel::kInfo, "server started",
           "\"io_threads\":" + std::to_string(n) + ",\"inspection_mode\":" + json_quote(inspection_mode_name(cfg_.inspection)));
  return true;
}

void Server::stop() {
  if (!running_.exchange(false)) return;
  requests_.close();
  for (auto& io : io_) io->stop();
  for (auto& t : threads_) t.join();
  threads_.clear();
  if (housekeeping_.joinable()) housekeeping_.join();
  if (relay_) relay_->stop();
  relay_.reset();
  if (inspector_) {
    bus_->remove_tap(inspector_);
    inspector_->stop();
    inspector_.reset();
  }
  if (gate_) {
    bus_->set_gate(nullptr);
    gate_->stop();
    gate_.reset();
  }
  io_.clear();
}

int Server::bound_port(const std::string& role) const {
  for (auto& kv : ports_)
    if (kv.first == role) return kv.second;
  return -1;
}

void Server::submit_chat(ChatRequest r) {
  r.id = next_req_.fetch_add(1);
  r.arrival_ns = now_ns();
  requests_.push(std::move(r));
}

void Server::note_cancel(const std::string& conv_id) {
  std::lock_guard<std::mutex> g(cancel_mu_);
  cancels_.push_back(conv_id);
}

bool Server::kill_conversation(const std::string& conv_id, const std::string& token, const std::string& why) {
  if (conv_id.empty() || !bus_->terminate(conv_id, token, kFinishAbort)) return false;
  note_cancel(conv_id);
  log_json(LogLevel::kWarn, "conversation killed",
           "\"conversation_id\":" + json_quote(conv_id) + ",\"token\":" + json_quote(token) + ",\"reason\":" + json_quote(why));
  return true;
}



void Server::flow_update(const std::string& conv_id, int delta) {
  std::lock_guard<std::mutex> g(flow_mu_);  // lock order: flow_mu_ -> bus shard (the bus never calls back)
  auto it = flow_.find(conv_id);
  if (it == flow_.end()) {
    if (delta <= 0) return;
    it = flow_.emplace(conv_id, std::make_pair(0, false)).first;
  }
  int& n = it->second.first;
  n = std::max(0, n + delta);
  const bool paused = n > 0 && (size_t)n >= bus_->subscriber_count(conv_id);
  if (paused != it->second.second) {
    it->second.second = paused;
    if (flow_events_.size() < (1u << 16)) flow_events_.emplace_back(conv_id, paused);
    n_paused_.fetch_add(paused ? 1 : -1);
    if (paused) metrics().bus_backpressure_pauses_total.inc();
    metrics().bus_paused_conversations.add(paused ? 1 : -1);
  }
  if (n == 0) flow_.erase(it);
}

bool Server::flow_paused(const std::string& conv_id) {
  if (n_paused_.load(std::memory_order_relaxed) == 0) return false;
  std::lock_guard<std::mutex> g(flow_mu_);
  auto it = flow_.find(conv_id);
  return it != flow_.end() && it->second.second;
}

std::vector<std::pair<std::string, bool>> Server::pop_flow_events() {
  std::lock_guard<std::mutex> g(flow_mu_);
  std::vector<std::pair<std::string, bool>> out;
  out.swap(flow_events_);
  return out;
}

std::vector<std::string> Server::pop_cancellations() {
  std::lock_guard<std::mutex> g(cancel_mu_);
  std::vector<std::string> out;
  out.swap(cancels_);
  return out;
}

// Blocking HTTP POST to <LLM_PROXY_URL>/chat in a detached thread (sse_handler.go:359-388).
void Server::forward_to_proxy(uint64_t conn_id, IoThread* io, const std::string& conv_id, const std::string& message) {
  std::string url = cfg_.llm_proxy_url;
  std::thread([conn_id, io, conv_id, message, url] {
    auto fail = [&](const std::string& why) {
      io->enqueue(OutItem{conn_id, OutKind::kError, nullptr,
                          "event: error\ndata: {\"error\":" + json_quote(why) + "}\n\n"});
      io->wake();
    };
    std::string u = url;
    if (u.rfind("http://", 0) == 0) u = u.substr(7);
    while (!u.empty() && u.back() == '/') u.pop_back();
    std::string hostport = u.substr(0, u.find('/'));
    std::string base = u.find('/') == std::string::npos ? "" : u.substr(u.find('/'));
    std::string host = hostport, port = "80";
    if (hostport.find(':') != std::string::npos) {
      host = hostport.substr(0, hostport.find(':'));
      port = hostport.substr(hostport.find(':') + 1);
    }
    addrinfo hints{}, *res = nullptr;
    hints.ai_socktype = SOCK_STREAM;
    if (getaddrinfo(host.c_str(), port.c_str(), &hints, &res) != 0 || !res) {
      fail("Post \"" + url + "/chat\": dial tcp: lookup " + host + ": no such host");
      return;
    }
    int fd = socket(res->ai_family, SOCK_STREAM, 0);
    if (fd < 0 || connect(fd, res->ai_addr, res->ai_addrlen) < 0) {
      freeaddrinfo(res);
      if (fd >= 0) close(fd);
      fail("Post \"" + url + "/chat\": dial tcp " + hostport + ": connect: connection refused");
      return;
    }
    freeaddrinfo(res);
    const std::string body = "{\"conversation_id\":" + json_quote(conv_id) + ",\"message\":" + json_quote(message) + "}";
    const std::string req = "POST " + base + "/chat HTTP/1.1\r\nHost: " + hostport +
                            "\r\nUser-Agent: dsse-edge\r\nContent-Type: application/json\r\nContent-Length: " +
                            std::to_string(body.size()) + "\r\nConnection: close\r\n\r\n" + body;
    if (send(fd, req.data(), req.size(), MSG_NOSIGNAL) != (ssize_t)req.size()) {
      close(fd);
      fail("forward failed");
      return;
    }
    char buf[512];
    ssize_t n = recv(fd, buf, sizeof buf - 1, 0);
    close(fd);
    if (n <= 0) {
      fail("forward failed: empty response");
      return;
    }
    buf[n] = 0;
    int code = 0;
    sscanf(buf, "HTTP/%*s %d", &code);
    if (code != 200 && code != 202) fail("LLM proxy error: " + std::to_string(code));
  }).detach();
}

// ------------------------------------------------------------------ stub engine
namespace {
const char* kStubWords[] = {"Streaming", "tokens", "leave", "the", "decode", "engine", "as", "soon", "as",
                            "they", "are", "sampled,", "travel", "through", "the", "in-node", "bus", "and",
                            "reach", "every", "subscribed", "browser", "as", "server-sent", "events.", "Each",
                            "frame", "carries", "its", "sequence", "number", "and", "a", "nanosecond",
                            "timestamp", "for", "latency", "accounting."};
constexpr int kNumStubWords = sizeof(kStubWords) / sizeof(kStubWords[0]);
}  // namespace

// ------------------------------------------------------------------ async inspection
AsyncInspector::AsyncInspector(Server& s) : srv_(s) {
  if (!s.config().inspection_endpoint.empty())
    remote_ = std::make_unique<RemoteInspector>(s.config().inspection_endpoint, s.config().inspection_timeout_ms);
}
AsyncInspector::~AsyncInspector() { stop(); }

void AsyncInspector::start() { thread_ = std::thread([this] { run(); }); }

void AsyncInspector::stop() {
  {
    std::lock_guard<std::mutex> g(mu_);
    stop_ = true;
  }
  cv_.notify_all();
  if (thread_.joinable()) thread_.join();
}

bool AsyncInspector::push(const FramePtr& f) {
  {
    std::lock_guard<std::mutex> g(mu_);
    q_.push_back(f);
  }
  cv_.notify_one();
  return true;
}

void AsyncInspector::run() {
  while (true) {
    std::deque<FramePtr> batch;
    {
      std::unique_lock<std::mutex> lk(mu_);
      cv_.wait_until(lk, std::chrono::system_clock::now() + std::chrono::milliseconds(100),
                     [&] { return stop_ || !q_.empty(); });
      if (stop_) return;
      batch.swap(q_);
    }
    for (auto& f : batch) {
      if (f->done) continue;
      if (std::find(killed_.begin(), killed_.end(), f->conversation_id) != killed_.end()) continue;
      TokenMessage m;
      if (!parse_token_message(f->json(), m)) continue;
      InspectionResult r;
      if (remote_) {
        if (!remote_->inspect(Bus::subject_for(f->conversation_id), m.token, m.sequence, m.timestamp, &r)) {
          metrics().inspection_remote_errors_total.inc();
          continue;  // fail open
        }
      } else {
        r = inspect_message(m.token);
      }
      if (r.action == InspectAction::kRedact) metrics().inspection_redacted_total.inc();
      if (r.action != InspectAction::kDrop) continue;
      // kill: terminal token for every subscriber, cancellation for the engine
      killed_.push_back(f->conversation_id);
      if (killed_.size() > 4096) killed_.erase(killed_.begin(), killed_.begin() + 2048);
      metrics().inspection_killed_total.inc();
      srv_.kill_conversation(f->conversation_id, "[BLOCKED]", "inspection: " + r.reason);
    }
  }
}

// ------------------------------------------------------------------ remote inline / hybrid inspection
InspectionGate::InspectionGate(Server& s, int workers) : srv_(s) {
  for (int i = 0; i < std::max(1, workers); ++i) workers_.emplace_back(new Worker);
}

InspectionGate::~InspectionGate() { stop(); }

void InspectionGate::start() {
  for (auto& w : workers_) {
    Worker* wp = w.get();
    wp->thread = std::thread([this, wp] { run(*wp); });
  }
}

void InspectionGate::stop() {
  if (stop_.exchange(true)) return;
  for (auto& w : workers_) {
    w->cv.notify_all();
    if (w->thread.joinable()) w->thread.join();
  }
}

bool InspectionGate::admit(const FramePtr& f) {
  if (stop_.load(std::memory_order_relaxed)) return false;
  Worker& w = *workers_[std::hash<std::string>{}(f->conversation_id) % workers_.size()];
  {
    std::lock_guard<std::mutex> g(w.mu);
    w.q.push_back(f);
  }
  w.cv.notify_one();
  return true;
}

namespace {
FramePtr with_token(const FramePtr& f, const std::string& token) {
  TokenMessage m;
  parse_token_message(f->json(), m);
  m.token = token;
  m.finish = f->finish;
  m.prompt_tokens = f->prompt_tokens;
  return Bus::make_frame(m);
}
}  // namespace

void InspectionGate::fail_closed(const std::string& conv, const std::string& why) {
  metrics().inspection_fail_closed_total.inc();
  srv_.kill_conversation(conv, "[ERROR]", why);
}

bool InspectionGate::inline_frame(RemoteInspector& ri, const FramePtr& f, std::vector<FramePtr>& out) {
  TokenMessage m;
  if (f->done || !parse_token_message(f->json(), m)) {
    out.push_back(f);
    return false;
  }
  InspectionResult r;
  if (!ri.inspect(Bus::subject_for(f->conversation_id), m.token, m.sequence, m.timestamp, &r)) {
    metrics().inspection_remote_errors_total.inc();
    if (srv_.config().inspection_fail_open) {
      metrics().inspection_fail_open_total.inc();
      out.push_back(f);
      return false;
    }
    fail_closed(f->conversation_id, "inspection unavailable");
    return true;
  }
  if (r.action == InspectAction::kDrop) {
    metrics().inspection_dropped_total.inc();
    return false;
  }
  if (r.action == InspectAction::kRedact) {
    metrics().inspection_redacted_total.inc();
    out.push_back(with_token(f, r.redacted_content));
    return false;
  }
  out.push_back(f);
  return false;
}

void InspectionGate::hybrid_flush(RemoteInspector& ri, const std::string& conv, Held& h, std::vector<FramePtr>& out) {
  h.cleared = true;
  if (h.frames.empty()) return;
  std::string text;
  int64_t seq = 0, ts = 0;
  for (const auto& f : h.frames) {
    TokenMessage m;
    if (f->done || !parse_token_message(f->json(), m)) continue;
    text += m.token;
    seq = m.sequence;
    ts = m.timestamp;
  }
  InspectionResult r;
  if (text.empty()) {
    r.action = InspectAction::kAllow;
  } else if (!ri.inspect(Bus::subject_for(conv), text, seq, ts, &r)) {
    metrics().inspection_remote_errors_total.inc();
    if (!srv_.config().inspection_fail_open) {
      h.frames.clear();
      fail_closed(conv, "inspection unavailable");
      return;
    }
    metrics().inspection_fail_open_total.inc((double)h.frames.size());
    r.action = InspectAction::kAllow;
  }
  if (r.action == InspectAction::kDrop) {
    metrics().inspection_killed_total.inc();
    h.frames.clear();
    srv_.kill_conversation(conv, "[BLOCKED]", "inspection: " + r.reason);
    return;
  }
  if (r.action == InspectAction::kRedact) {  // the held text becomes one frame (sequence of the last token)
    metrics().inspection_redacted_total.inc();
    FramePtr last_tok;
    for (const auto& f : h.frames)
      if (!f->done) last_tok = f;
    if (last_tok) out.push_back(with_token(last_tok, r.redacted_content));
    for (const auto& f : h.frames)
      if (f->done) out.push_back(f);
  } else {
    out.insert(out.end(), h.frames.begin(), h.frames.end());
  }
  h.frames.clear();
}

void InspectionGate::hybrid_frame(RemoteInspector& ri, std::unordered_map<std::string, Held>& held, const FramePtr& f,
                                  std::vector<FramePtr>& out) {
  auto [it, inserted] = held.try_emplace(f->conversation_id);
  Held& h = it->second;
  h.last_mono = mono_ns();
  if (inserted) h.first_mono = h.last_mono;
  if (h.cleared) {
    out.push_back(f);
  } else {
    h.frames.push_back(f);
    if (f->done) hybrid_flush(ri, f->conversation_id, h, out);
  }
  if (f->done) held.erase(it);
}

constexpr int64_t kDeadAgeNs = 600LL * 1000000000LL;  // 10 minutes

void InspectionGate::run(Worker& w) {
  const ServerConfig& cfg = srv_.config();
  RemoteInspector ri(cfg.inspection_endpoint, cfg.inspection_timeout_ms);
  const bool hybrid = cfg.inspection == InspectionMode::kHybrid;
  const int64_t window = (int64_t)cfg.inspection_buffer_ms * 1000000LL;
  std::unordered_map<std::string, Held> held;
  int64_t next_age_scan = 0;  // the dead map's age-out scan runs at most once a second (a full-map walk)
  while (!stop_.load()) {
    std::deque<FramePtr> batch;
    {
      std::unique_lock<std::mutex> lk(w.mu);
      w.cv.wait_for(lk, std::chrono::milliseconds(hybrid ? 5 : 50), [&] { return stop_.load() || !w.q.empty(); });
      batch.swap(w.q);
    }
    std::vector<FramePtr> out;
    // overload (a slow endpoint, a token burst): the backlog stays bounded either way.  Fail-open: past kBypassDepth
    // queued frames the batch is forwarded uninspected, in order.  Fail-closed: every frame is inspected; only past
    // kOverloadDepth are the backlog's conversations ended with [ERROR] (nothing uninspected reaches a client).
    if (!hybrid && cfg.inspection_fail_open && batch.size() > kBypassDepth) {
      metrics().inspection_fail_open_total.inc((double)batch.size());
      out.assign(batch.begin(), batch.end());
      batch.clear();
    } else if (!hybrid && batch.size() > kOverloadDepth) {
      const int64_t now = mono_ns();
      for (const auto& f : batch) {
        if (w.dead.emplace(f->conversation_id, now).second) fail_closed(f->conversation_id, "inspection overloaded");
        if (f->done) w.dead.erase(f->conversation_id);  // its done frame was in this batch: no later frame comes
      }
      batch.clear();
    }
    for (const auto& f : batch) {
      if (w.dead.count(f->conversation_id)) {  // ended fail-closed: later frames (its [DONE] too) are dropped
        if (f->done) w.dead.erase(f->conversation_id);
        continue;
      }
      if (hybrid) {
        hybrid_frame(ri, held, f, out);
      } else {
        if (inline_frame(ri, f, out) && !f->done) w.dead.emplace(f->conversation_id, mono_ns());
      }
    }
    if (w.dead.size() > 4096 && mono_ns() >= next_age_scan) {  // age out entries whose done frame never arrived
      const int64_t now = mono_ns();                            // (never a wholesale clear)
      next_age_scan = now + 1000000000LL;
      for (auto it = w.dead.begin(); it != w.dead.end();) it = now - it->second > kDeadAgeNs ? w.dead.erase(it) : std::next(it);
    }
    if (hybrid) {  // buffer windows that ran out; forget conversations idle for 10 minutes
      const int64_t now = mono_ns();
      for (auto it = held.begin(); it != held.end();) {
        Held& h = it->second;
        if (!h.cleared && now - h.first_mono >= window) hybrid_flush(ri, it->first, h, out);
        if (h.cleared && h.frames.empty() && now - h.last_mono > 600LL * 1000000000LL) it = held.erase(it);
        else ++it;
      }
    }
    if (!out.empty()) srv_.bus().deliver_gated(out);
  }
}

StubEngine::StubEngine(Server& server, int tokens, int delay_ms, int workers)
    : server_(server), tokens_(tokens), delay_ms_(delay_ms) {
  server_.set_local_engine(true);
  for (int i = 0; i < std::max(1, workers); ++i) threads_.emplace_back([this] { run(); });
}

StubEngine::~StubEngine() { stop(); }

void StubEngine::stop() {
  if (stop_.exchange(true)) return;
  for (auto& t : threads_) t.join();
  threads_.clear();
}

void StubEngine::run() {
  struct Item {
    ChatRequest req;
    int n = 0;       // tokens to emit before [DONE]
    int next = 0;    // index of the next token
    bool finished = false;
    int64_t due_ns = 0;
  };
  std::vector<Item> live;
  std::mt19937 rng{std::random_device{}()};
  while (!stop_.load()) {
    for (auto& r : server_.requests().pop(256, live.empty() ? 50 : 0)) {
      Item it;
      it.n = r.max_tokens > 0 ? r.max_tokens : tokens_;
      it.req = std::move(r);
      it.due_ns = mono_ns();
      live.push_back(std::move(it));
      metrics().active_chats.add(1);
    }
    int64_t now = mono_ns(), next_due = now + 5000000;
    std::vector<FramePtr> batch;
    for (auto& it : live) {
      if (!it.finished && it.due_ns <= now && server_.flow_paused(it.req.conversation_id)) {
        it.due_ns = now + std::max(delay_ms_, 1) * 1000000LL;  // flow control: hold this stream only
        next_due = std::min(next_due, it.due_ns);
        continue;
      }
      while (!it.finished && it.due_ns <= now) {
        TokenMessage m;
        m.conversation_id = it.req.conversation_id;
        m.timestamp = now_ns();
        if (it.next < it.n) {
          m.token = std::string(it.next ? " " : "") + kStubWords[it.next % kNumStubWords];
          m.sequence = it.next + 1;
          ++it.next;
        } else {  // terminal message: sequence last+1, done (llm-stream-proxy/main.go:207-210)
          m.token = "[DONE]";
          m.sequence = it.n + 1;
          m.done = true;
          it.finished = true;
        }
        batch.push_back(Bus::make_frame(m));
        const int jitter = delay_ms_ > 1 ? (int)(rng() % (unsigned)(delay_ms_ / 2)) : 0;
        it.due_ns += (int64_t)(delay_ms_ + jitter) * 1000000LL;
        if (delay_ms_ > 0) break;
      }
      if (!it.finished) next_due = std::min(next_due, it.due_ns);
    }
    if (!batch.empty()) server_.bus().publish_batch(batch);
    const size_t before = live.size();
    live.erase(std::remove_if(live.begin(), live.end(), [](const Item& it) { return it.finished; }), live.end());
    metrics().active_chats.add(-(double)(before - live.size()));
    now = mono_ns();
    if (!live.empty() && next_due > now)
      std::this_thread::sleep_for(std::chrono::nanoseconds(std::min<int64_t>(next_due - now, 2000000)));
  }
}

}  // namespace dsse
