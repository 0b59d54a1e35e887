// dsse-loadgen: native load generator and SSE bench client.
//
// Same workload and flags as the reference harness (demo/load-generator/main.go:100-319) and its Python
// twin (distributed_sse_for_llm_response_amd/tools_loadgen.py):
//   -mode producer|consumer|both   consumers GET /stream/<id>; producers PUBLISH llm:tokens:<id> over
//                                  RESP with delay + U[0, delay/2) ms between tokens (main.go:204-240);
//   -chat                          consumers POST /chat instead (engine-generated tokens);
//   -conversations N -tokens T -token-delay MS -duration 30s -redis host:port -sse http://host:port
// plus what a 10k-connection / 100k-token/s run needs and Python cannot deliver: T epoll threads, a
// RESP connection pool, per-token arrival records (-arrivals FILE: int32 stream, int32 sequence,
// int64 recv_ns, int64 msg_timestamp_ns), and a JSON summary (-json) with latency and inter-token
// percentiles.  Chat extras: -message, -max-tokens, -ignore-eos, -id-prefix.
// Serving under continuous arrivals (tools/bench_serving.py): -rate R starts the chat streams as a Poisson
// process of R requests/s (seeded by -seed) instead of all at once, and records each request's send time as an
// arrival with sequence 0 (TTFT = first token - that); -long-every K -long-words W makes every K-th request a
// W-word prompt (one synthetic token per word: an 8k-token prompt is -long-words 8000).
#include <arpa/inet.h>
#include <fcntl.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <signal.h>
#include <sys/epoll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cerrno>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <queue>
#include <random>
#include <string>
#include <thread>
#include <vector>

namespace {

int64_t now_ns() {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::system_clock::now().time_since_epoch())
      .count();
}

struct Args {
  std::string mode = "both";
  std::string redis = "localhost:6379";
  std::string sse = "http://localhost:8080";
  int conversations = 5;
  int tokens = 50;
  int token_delay_ms = 50;
  double duration_s = 30;
  bool chat = false;
  std::string message = "Tell me about streaming token delivery.";
  int max_tokens = -1;
  bool ignore_eos = false;
  std::string id_prefix;
  int threads = 4;
  int pool = 16;
  std::string arrivals;
  bool json = false;
  double rate = 0;         // chat: Poisson request arrivals per second (0 = all at once)
  int long_every = 0;      // chat: every K-th request gets the long prompt
  int long_words = 0;
  uint64_t seed = 42;
  int connect_batch = 512;  // connections started per thread per loop iteration
};

double parse_duration(const std::string& s) {
  char* end = nullptr;
  double v = std::strtod(s.c_str(), &end);
  std::string suf = end ? end : "";
  if (suf == "ms") return v / 1000;
  if (suf == "m") return v * 60;
  if (suf == "h") return v * 3600;
  return v;  // "s" or bare seconds
}

bool split_hostport(const std::string& hp, std::string* host, int* port) {
  auto c = hp.rfind(':');
  if (c == std::string::npos) return false;
  *host = hp.substr(0, c);
  if (host->empty()) *host = "127.0.0.1";
  *port = std::atoi(hp.c_str() + c + 1);
  return *port > 0;
}

bool resolve(const std::string& host, int port, sockaddr_in* out) {
  std::memset(out, 0, sizeof *out);
  out->sin_family = AF_INET;
  out->sin_port = htons((uint16_t)port);
  std::string h = host == "localhost" ? "127.0.0.1" : host;
  if (inet_pton(AF_INET, h.c_str(), &out->sin_addr) == 1) return true;
  addrinfo hints{}, *res = nullptr;
  hints.ai_family = AF_INET;
  if (getaddrinfo(h.c_str(), nullptr, &hints, &res) != 0 || !res) return false;
  out->sin_addr = reinterpret_cast<sockaddr_in*>(res->ai_addr)->sin_addr;
  freeaddrinfo(res);
  return true;
}

int connect_nb(const sockaddr_in& a) {
  int fd = socket(AF_INET, SOCK_STREAM | SOCK_NONBLOCK | SOCK_CLOEXEC, 0);
  if (fd < 0) return -1;
  int one = 1;
  setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
  if (connect(fd, reinterpret_cast<const sockaddr*>(&a), sizeof a) < 0 && errno != EINPROGRESS) {
    close(fd);
    return -1;
  }
  return fd;
}

// JSON string escaping for the request body (message may contain anything).
std::string jesc(const std::string& s) {
  std::string o;
  for (unsigned char c : s) {
    if (c == '"' || c == '\\') { o += '\\'; o += (char)c; }
    else if (c < 0x20) { char b[8]; snprintf(b, sizeof b, "\\u%04x", c); o += b; }
    else o += (char)c;
  }
  return o;
}

// Minimal field extraction from a TokenMessage JSON (keys are unique and values simple).
bool find_int(const std::string& j, const char* key, int64_t* v) {
  std::string k = std::string("\"") + key + "\":";
  auto p = j.find(k);
  if (p == std::string::npos) return false;
  *v = std::strtoll(j.c_str() + p + k.size(), nullptr, 10);
  return true;
}
bool find_bool(const std::string& j, const char* key) {
  std::string k = std::string("\"") + key + "\":";
  auto p = j.find(k);
  return p != std::string::npos && j.compare(p + k.size(), 4, "true") == 0;
}

struct Arrival {
  int32_t stream, seq;
  int64_t recv_ns, ts_ns;
};

struct Stats {
  std::atomic<int64_t> published{0}, received{0}, opened{0}, closed{0}, errors{0};
  std::mutex mu;
  std::vector<Arrival> arrivals;
};

// ------------------------------------------------------------------------------ SSE consumer
struct Consumer {
  int idx = 0;
  int fd = -1;
  std::string out;
  size_t out_off = 0;
  std::string in;        // raw bytes not yet consumed
  bool headers_done = false, chunked = false, finished = false;
  int status = 0;
  int64_t chunk_left = -1;  // -1: expecting a size line
  std::string sse;       // decoded body bytes not yet parsed into events
  std::vector<Arrival> local;
};

class ConsumerThread {
 public:
  ConsumerThread(const Args& a, const sockaddr_in& addr, const std::string& host, std::vector<std::string> ids,
                 std::vector<int> idx, Stats* st, int64_t deadline_ns, std::vector<int64_t> start_at = {},
                 const std::string* long_msg = nullptr)
      : a_(a), addr_(addr), host_(host), ids_(std::move(ids)), idx_(std::move(idx)), st_(st), deadline_(deadline_ns),
        start_at_(std::move(start_at)), long_msg_(long_msg) {}

  void run() {
    ep_ = epoll_create1(EPOLL_CLOEXEC);
    conns_.resize(ids_.size());
    size_t next = 0, live = 0;
    epoll_event evs[256];
    while (true) {
      // open connections in batches so a 10k-connection run does not flood the listen backlog; with -rate, each at
      // its Poisson arrival time
      const int64_t t_now = now_ns();
      for (int k = 0; k < a_.connect_batch && next < ids_.size(); ++k, ++next) {
        if (!start_at_.empty() && start_at_[next] > t_now) break;
        if (start(next)) ++live;
      }
      if (live == 0 && next >= ids_.size()) break;
      if (t_now > deadline_ + 5'000'000'000LL) break;
      int n = epoll_wait(ep_, evs, 256, next < ids_.size() ? 1 : 100);
      for (int i = 0; i < n; ++i) {
        Consumer& c = conns_[evs[i].data.u32];
        if (c.finished) continue;
        bool ok = true;
        if (evs[i].events & EPOLLOUT) ok = flush(c);
        if (ok && (evs[i].events & (EPOLLIN | EPOLLHUP | EPOLLERR))) ok = readable(c);
        if (!ok || c.finished) {
          finish(c, ok);
          --live;
        }
      }
    }
    for (auto& c : conns_)
      if (c.fd >= 0 && !c.finished) finish(c, now_ns() > deadline_);
    close(ep_);
    std::lock_guard<std::mutex> g(st_->mu);
    for (auto& c : conns_) st_->arrivals.insert(st_->arrivals.end(), c.local.begin(), c.local.end());
  }

 private:
  bool start(size_t i) {
    Consumer& c = conns_[i];
    c.idx = idx_[i];
    c.fd = connect_nb(addr_);
    if (c.fd < 0) {
      st_->errors++;
      c.finished = true;
      return false;
    }
    const std::string& id = ids_[i];
    if (a_.chat) {
      const bool is_long = long_msg_ && a_.long_every > 0 && c.idx % a_.long_every == a_.long_every - 1;
      std::string body = "{\"message\":\"" + jesc(is_long ? *long_msg_ : a_.message) + "\",\"conversation_id\":\"" +
                         jesc(id) + "\"";
      if (a_.max_tokens > 0) body += ",\"max_tokens\":" + std::to_string(a_.max_tokens);
      if (a_.ignore_eos) body += ",\"ignore_eos\":true";
      body += "}";
      c.out = "POST /chat HTTP/1.1\r\nHost: " + host_ + "\r\nContent-Type: application/json\r\nAccept: text/event-stream\r\n"
              "Content-Length: " + std::to_string(body.size()) + "\r\n\r\n" + body;
    } else {
      c.out = "GET /stream/" + id + " HTTP/1.1\r\nHost: " + host_ +
              "\r\nAccept: text/event-stream\r\nCache-Control: no-cache\r\n\r\n";
    }
    epoll_event ev{};
    ev.events = EPOLLIN | EPOLLOUT | EPOLLRDHUP;
    ev.data.u32 = (uint32_t)i;
    epoll_ctl(ep_, EPOLL_CTL_ADD, c.fd, &ev);
    if (!start_at_.empty()) c.local.push_back({c.idx, 0, now_ns(), 0});  // request sent (TTFT origin)
    return true;
  }

  bool flush(Consumer& c) {
    while (c.out_off < c.out.size()) {
      ssize_t n = send(c.fd, c.out.data() + c.out_off, c.out.size() - c.out_off, MSG_NOSIGNAL);
      if (n < 0) return errno == EAGAIN || errno == EWOULDBLOCK;
      c.out_off += (size_t)n;
    }
    epoll_event ev{};
    ev.events = EPOLLIN | EPOLLRDHUP;
    ev.data.u32 = (uint32_t)(&c - conns_.data());
    epoll_ctl(ep_, EPOLL_CTL_MOD, c.fd, &ev);
    return true;
  }

  bool readable(Consumer& c) {
    char buf[65536];
    while (true) {
      ssize_t n = recv(c.fd, buf, sizeof buf, 0);
      if (n > 0) {
        c.in.append(buf, (size_t)n);
        if (!parse(c)) return false;
        if (c.finished) return true;
        continue;
      }
      if (n == 0) {  // server closed: a complete stream ends with done (already finished)
        c.finished = true;
        return c.headers_done && c.status == 200;
      }
      return errno == EAGAIN || errno == EWOULDBLOCK;
    }
  }

  bool parse(Consumer& c) {
    if (!c.headers_done) {
      auto e = c.in.find("\r\n\r\n");
      if (e == std::string::npos) return true;
      std::string head = c.in.substr(0, e);
      c.in.erase(0, e + 4);
      c.status = std::atoi(head.c_str() + head.find(' ') + 1);
      std::string lower = head;
      std::transform(lower.begin(), lower.end(), lower.begin(), ::tolower);
      c.chunked = lower.find("transfer-encoding: chunked") != std::string::npos;
      c.headers_done = true;
      if (c.status != 200) return false;
      st_->opened++;
    }
    if (c.chunked) {
      size_t p = 0;
      while (p < c.in.size()) {
        if (c.chunk_left < 0) {
          auto e = c.in.find("\r\n", p);
          if (e == std::string::npos) break;
          c.chunk_left = std::strtoll(c.in.c_str() + p, nullptr, 16);
          p = e + 2;
          if (c.chunk_left == 0) {
            c.finished = true;
            break;
          }
        } else {
          size_t take = std::min<size_t>((size_t)c.chunk_left, c.in.size() - p);
          c.sse.append(c.in, p, take);
          p += take;
          c.chunk_left -= (int64_t)take;
          if (c.chunk_left == 0) {
            if (c.in.size() - p < 2) {
              c.chunk_left = 0;  // wait for the CRLF
              break;
            }
            p += 2;
            c.chunk_left = -1;
          }
        }
      }
      c.in.erase(0, p);
      if (c.chunk_left == 0 && c.in.size() >= 2) {
        c.in.erase(0, 2);
        c.chunk_left = -1;
      }
    } else {
      c.sse += c.in;
      c.in.clear();
    }
    return events(c);
  }

  bool events(Consumer& c) {
    size_t p = 0;
    while (true) {
      auto e = c.sse.find("\n\n", p);
      if (e == std::string::npos) break;
      std::string ev = "message", data;
      size_t q = p;
      while (q < e) {
        auto nl = c.sse.find('\n', q);
        if (nl == std::string::npos || nl > e) nl = e;
        if (c.sse.compare(q, 6, "event:") == 0) {
          ev = c.sse.substr(q + 6, nl - q - 6);
          if (!ev.empty() && ev[0] == ' ') ev.erase(0, 1);
        } else if (c.sse.compare(q, 5, "data:") == 0) {
          data = c.sse.substr(q + 5, nl - q - 5);
          if (!data.empty() && data[0] == ' ') data.erase(0, 1);
        }
        q = nl + 1;
      }
      p = e + 2;
      if (data.empty() || ev == "connected") continue;
      if (ev == "error") {
        st_->errors++;
        c.finished = true;
        break;
      }
      if (data.find("\"token\"") == std::string::npos) continue;
      int64_t seq = 0, ts = 0;
      find_int(data, "sequence", &seq);
      find_int(data, "timestamp", &ts);
      c.local.push_back({c.idx, (int32_t)seq, now_ns(), ts});
      st_->received++;
      if (find_bool(data, "done")) {
        c.finished = true;
        break;
      }
    }
    c.sse.erase(0, p);
    if (!c.finished && now_ns() > deadline_) c.finished = true;
    return true;
  }

  void finish(Consumer& c, bool ok) {
    if (c.fd >= 0) {
      epoll_ctl(ep_, EPOLL_CTL_DEL, c.fd, nullptr);
      close(c.fd);
      c.fd = -1;
    }
    c.finished = true;
    if (ok) st_->closed++;
    else st_->errors++;
  }

  const Args& a_;
  sockaddr_in addr_;
  std::string host_;
  std::vector<std::string> ids_;
  std::vector<int> idx_;
  Stats* st_;
  int64_t deadline_;
  std::vector<int64_t> start_at_;
  const std::string* long_msg_;
  int ep_ = -1;
  std::vector<Consumer> conns_;
};

// ------------------------------------------------------------------------------ RESP producer
const char* kSample[] = {"Streaming", "tokens", "travel", "from", "the", "sampler", "through", "the", "in-node", "bus",
                         "to", "every", "subscribed", "browser", "as", "server-sent", "events"};

class ProducerThread {
 public:
  ProducerThread(const Args& a, const sockaddr_in& addr, std::vector<std::string> ids, Stats* st, int64_t deadline,
                 int pool, uint64_t seed)
      : a_(a), addr_(addr), ids_(std::move(ids)), st_(st), deadline_(deadline), pool_(pool), rng_(seed) {}

  bool run() {
    ep_ = epoll_create1(EPOLL_CLOEXEC);
    for (int i = 0; i < pool_; ++i) {
      int fd = connect_nb(addr_);
      if (fd < 0) return false;
      conns_.push_back({fd, {}, 0, {}, 0});
      epoll_event ev{};
      ev.events = EPOLLIN | EPOLLOUT;
      ev.data.u32 = (uint32_t)i;
      epoll_ctl(ep_, EPOLL_CTL_ADD, fd, &ev);
    }
    using Item = std::pair<int64_t, size_t>;  // (due ns, conversation)
    std::priority_queue<Item, std::vector<Item>, std::greater<Item>> due;
    std::vector<int> sent(ids_.size(), 0);
    const int64_t t0 = now_ns();
    for (size_t i = 0; i < ids_.size(); ++i) due.push({t0, i});
    epoll_event evs[64];
    while (!due.empty() || pending()) {
      const int64_t now = now_ns();
      if (now > deadline_ + 2'000'000'000LL) break;
      while (!due.empty() && due.top().first <= now) {
        size_t i = due.top().second;
        due.pop();
        if (now > deadline_) continue;
        const int k = sent[i]++;
        const bool done = k == a_.tokens - 1;
        char js[512];
        int n = snprintf(js, sizeof js, "{\"conversation_id\":\"%s\",\"token\":\"%s\",\"sequence\":%d,\"done\":%s,\"timestamp\":%lld}",
                         ids_[i].c_str(), kSample[k % (sizeof kSample / sizeof *kSample)], k + 1, done ? "true" : "false",
                         (long long)now_ns());
        std::string ch = "llm:tokens:" + ids_[i];
        Conn& c = conns_[i % conns_.size()];
        c.out += "*3\r\n$7\r\nPUBLISH\r\n$" + std::to_string(ch.size()) + "\r\n" + ch + "\r\n$" + std::to_string(n) + "\r\n";
        c.out.append(js, (size_t)n);
        c.out += "\r\n";
        c.expect++;
        st_->published++;
        if (!done) {
          int jitter = a_.token_delay_ms >= 2 ? (int)(rng_() % (uint64_t)(a_.token_delay_ms / 2)) : 0;
          due.push({now + (int64_t)(a_.token_delay_ms + jitter) * 1'000'000LL, i});
        }
      }
      for (auto& c : conns_) write_some(c);
      int timeout = 50;
      if (!due.empty()) timeout = (int)std::max<int64_t>(0, (due.top().first - now_ns()) / 1'000'000LL);
      int n = epoll_wait(ep_, evs, 64, std::min(timeout, 50));
      for (int i = 0; i < n; ++i) {
        Conn& c = conns_[evs[i].data.u32];
        if (evs[i].events & EPOLLIN) read_replies(c);
        if (evs[i].events & EPOLLOUT) write_some(c);
      }
    }
    for (auto& c : conns_) close(c.fd);
    close(ep_);
    return true;
  }

 private:
  struct Conn {
    int fd;
    std::string out;
    size_t off;
    std::string in;
    int64_t expect;
  };
  bool pending() const {
    for (auto& c : conns_)
      if (c.expect > 0 || c.off < c.out.size()) return true;
    return false;
  }
  void write_some(Conn& c) {
    while (c.off < c.out.size()) {
      ssize_t n = send(c.fd, c.out.data() + c.off, c.out.size() - c.off, MSG_NOSIGNAL);
      if (n <= 0) break;
      c.off += (size_t)n;
    }
    if (c.off == c.out.size()) {
      c.out.clear();
      c.off = 0;
    }
  }
  void read_replies(Conn& c) {
    char buf[16384];
    ssize_t n;
    while ((n = recv(c.fd, buf, sizeof buf, 0)) > 0) c.in.append(buf, (size_t)n);
    size_t p = 0;
    while (true) {
      auto e = c.in.find("\r\n", p);
      if (e == std::string::npos) break;
      if (c.in[p] != ':') st_->errors++;
      c.expect--;
      p = e + 2;
    }
    c.in.erase(0, p);
  }

  const Args& a_;
  sockaddr_in addr_;
  std::vector<std::string> ids_;
  Stats* st_;
  int64_t deadline_;
  int pool_;
  std::mt19937_64 rng_;
  int ep_ = -1;
  std::vector<Conn> conns_;
};

double pct(std::vector<double>& v, double p) {
  if (v.empty()) return 0;
  size_t k = std::min(v.size() - 1, (size_t)(p / 100.0 * (double)v.size()));
  std::nth_element(v.begin(), v.begin() + (long)k, v.end());
  return v[k];
}

void usage() {
  fprintf(stderr,
          "usage: dsse-loadgen [-mode producer|consumer|both] [-chat] [-redis host:port] [-sse http://host:port]\n"
          "  [-conversations N] [-tokens T] [-token-delay MS] [-duration 30s] [-threads T] [-pool P]\n"
          "  [-message TEXT] [-max-tokens N] [-ignore-eos] [-id-prefix P] [-arrivals FILE] [-json]\n"
          "  [-rate REQ_PER_S] [-long-every K -long-words W] [-seed S]\n");
}

}  // namespace

int main(int argc, char** argv) {
  signal(SIGPIPE, SIG_IGN);
  Args a;
  for (int i = 1; i < argc; ++i) {
    std::string k = argv[i];
    while (k.size() > 1 && k[0] == '-' && k[1] == '-') k.erase(0, 1);
    auto val = [&]() -> std::string {
      if (i + 1 >= argc) {
        usage();
        std::exit(2);
      }
      return argv[++i];
    };
    if (k == "-mode") a.mode = val();
    else if (k == "-redis") a.redis = val();
    else if (k == "-sse") a.sse = val();
    else if (k == "-conversations") a.conversations = std::atoi(val().c_str());
    else if (k == "-tokens") a.tokens = std::atoi(val().c_str());
    else if (k == "-token-delay") a.token_delay_ms = std::atoi(val().c_str());
    else if (k == "-duration") a.duration_s = parse_duration(val());
    else if (k == "-chat") a.chat = true;
    else if (k == "-message") a.message = val();
    else if (k == "-max-tokens") a.max_tokens = std::atoi(val().c_str());
    else if (k == "-ignore-eos") a.ignore_eos = true;
    else if (k == "-id-prefix") a.id_prefix = val();
    else if (k == "-threads") a.threads = std::max(1, std::atoi(val().c_str()));
    else if (k == "-pool") a.pool = std::max(1, std::atoi(val().c_str()));
    else if (k == "-arrivals") a.arrivals = val();
    else if (k == "-json") a.json = true;
    else if (k == "-rate") a.rate = std::atof(val().c_str());
    else if (k == "-long-every") a.long_every = std::atoi(val().c_str());
    else if (k == "-long-words") a.long_words = std::atoi(val().c_str());
    else if (k == "-seed") a.seed = (uint64_t)std::strtoull(val().c_str(), nullptr, 10);
    else if (k == "-h" || k == "-help") { usage(); return 0; }
    else { fprintf(stderr, "unknown flag %s\n", argv[i]); usage(); return 2; }
  }
  std::string hp = a.sse;
  if (hp.rfind("http://", 0) == 0) hp = hp.substr(7);
  if (!hp.empty() && hp.back() == '/') hp.pop_back();
  std::string sse_host, redis_host;
  int sse_port = 0, redis_port = 0;
  if (hp.find(':') == std::string::npos) hp += ":80";
  sockaddr_in sse_addr{}, redis_addr{};
  const bool consume = a.chat || a.mode == "consumer" || a.mode == "both";
  const bool produce = !a.chat && (a.mode == "producer" || a.mode == "both");
  if (consume && (!split_hostport(hp, &sse_host, &sse_port) || !resolve(sse_host, sse_port, &sse_addr))) {
    fprintf(stderr, "bad -sse %s\n", a.sse.c_str());
    return 2;
  }
  if (produce && (!split_hostport(a.redis, &redis_host, &redis_port) || !resolve(redis_host, redis_port, &redis_addr))) {
    fprintf(stderr, "bad -redis %s\n", a.redis.c_str());
    return 2;
  }
  const std::string prefix = a.id_prefix.empty() ? "loadtest-" + std::to_string(now_ns()) + "-" : a.id_prefix;
  std::vector<std::string> ids;
  for (int i = 0; i < a.conversations; ++i) ids.push_back(prefix + std::to_string(i));
  const int64_t deadline = now_ns() + (int64_t)(a.duration_s * 1e9);
  Stats st;
  std::vector<std::thread> threads;
  std::vector<std::unique_ptr<ConsumerThread>> cons;
  // -rate: one global Poisson arrival process (exponential gaps), dealt round-robin to the threads in order
  std::vector<int64_t> start_at;
  if (a.chat && a.rate > 0) {
    std::mt19937_64 rng(a.seed);
    std::exponential_distribution<double> gap(a.rate);
    double t = 0;
    const int64_t t0 = now_ns() + 100'000'000LL;
    for (int i = 0; i < a.conversations; ++i) {
      start_at.push_back(t0 + (int64_t)(t * 1e9));
      t += gap(rng);
    }
  }
  std::string long_msg;
  for (int i = 0; i < a.long_words; ++i) long_msg += (i ? " w" : "w") + std::to_string(i % 9973);
  if (consume) {
    for (int t = 0; t < a.threads; ++t) {
      std::vector<std::string> part;
      std::vector<int> idx;
      std::vector<int64_t> at;
      for (int i = t; i < a.conversations; i += a.threads) {
        part.push_back(ids[(size_t)i]);
        idx.push_back(i);
        if (!start_at.empty()) at.push_back(start_at[(size_t)i]);
      }
      cons.emplace_back(new ConsumerThread(a, sse_addr, hp, part, idx, &st, deadline, at,
                                           a.long_words > 0 ? &long_msg : nullptr));
    }
    for (auto& c : cons) threads.emplace_back([&c] { c->run(); });
    if (produce) {
      // main.go:162 waits a fixed 500 ms; at 10k connections that is not enough for every subscription to exist
      // before its producer starts (tokens published earlier are not delivered live: round-2 runs received
      // 416k-476k of 500k).  Wait for every consumer's response headers (the server subscribes first), at least
      // 500 ms and at most 60 s.
      std::this_thread::sleep_for(std::chrono::milliseconds(500));
      const int64_t until = now_ns() + 60'000'000'000LL;
      while (st.opened.load() + st.errors.load() < a.conversations && now_ns() < until)
        std::this_thread::sleep_for(std::chrono::milliseconds(10));
    }
  }
  bool prod_ok = true;
  if (produce) {
    const int pt = std::max(1, std::min(a.threads, a.conversations));
    std::vector<std::thread> pth;
    std::atomic<bool> ok{true};
    for (int t = 0; t < pt; ++t) {
      std::vector<std::string> part;
      for (int i = t; i < a.conversations; i += pt) part.push_back(ids[(size_t)i]);
      int pool = std::max(1, a.pool / pt);
      pth.emplace_back([&, part, pool, t] {
        ProducerThread p(a, redis_addr, part, &st, deadline, pool, 1234567ULL + (uint64_t)t);
        if (!p.run()) ok = false;
      });
    }
    for (auto& t : pth) t.join();
    prod_ok = ok;
  }
  for (auto& t : threads) t.join();

  std::vector<double> lat, gaps;
  auto& arr = st.arrivals;
  std::sort(arr.begin(), arr.end(), [](const Arrival& x, const Arrival& y) {
    return x.stream != y.stream ? x.stream < y.stream : x.recv_ns < y.recv_ns;
  });
  for (size_t i = 0; i < arr.size(); ++i) {
    if (arr[i].seq == 0) continue;  // a request's send record (-rate)
    if (arr[i].ts_ns > 1'000'000'000'000'000LL) lat.push_back((double)(arr[i].recv_ns - arr[i].ts_ns) / 1e6);
    if (i > 0 && arr[i].stream == arr[i - 1].stream && arr[i - 1].seq > 0)
      gaps.push_back((double)(arr[i].recv_ns - arr[i - 1].recv_ns) / 1e6);
  }
  if (!a.arrivals.empty()) {
    FILE* f = std::fopen(a.arrivals.c_str(), "wb");
    if (f) {
      std::fwrite(arr.data(), sizeof(Arrival), arr.size(), f);
      std::fclose(f);
    }
  }
  double avg = 0, mn = 0, mx = 0;
  if (!lat.empty()) {
    for (double v : lat) avg += v;
    avg /= (double)lat.size();
    mn = *std::min_element(lat.begin(), lat.end());
    mx = *std::max_element(lat.begin(), lat.end());
  }
  const double p50 = pct(lat, 50), p99 = pct(lat, 99), g50 = pct(gaps, 50), g99 = pct(gaps, 99);
  if (a.json) {
    printf("{\"tokens_published\":%lld,\"tokens_received\":%lld,\"connections_opened\":%lld,\"connections_closed\":%lld,"
           "\"errors\":%lld,\"avg_latency_ms\":%.4f,\"min_latency_ms\":%.4f,\"max_latency_ms\":%.4f,\"p50_latency_ms\":%.4f,"
           "\"p99_latency_ms\":%.4f,\"p50_inter_token_ms\":%.4f,\"p99_inter_token_ms\":%.4f}\n",
           (long long)st.published.load(), (long long)st.received.load(), (long long)st.opened.load(),
           (long long)st.closed.load(), (long long)st.errors.load(), avg, mn, mx, p50, p99, g50, g99);
  } else {
    printf("\n=== Load Test Statistics ===\n");
    printf("Tokens Published:    %lld\n", (long long)st.published.load());
    printf("Tokens Received:     %lld\n", (long long)st.received.load());
    printf("Connections Opened:  %lld\n", (long long)st.opened.load());
    printf("Connections Closed:  %lld\n", (long long)st.closed.load());
    printf("Errors:              %lld\n", (long long)st.errors.load());
    if (!lat.empty()) {
      printf("Avg Latency:         %.2f ms\n", avg);
      printf("Min Latency:         %.2f ms\n", mn);
      printf("Max Latency:         %.2f ms\n", mx);
      printf("P50 / P99 Latency:   %.2f / %.2f ms\n", p50, p99);
    }
    if (!gaps.empty()) printf("P50 / P99 ITL:       %.2f / %.2f ms\n", g50, g99);
    printf("============================\n");
  }
  fflush(stdout);
  return prod_ok ? 0 : 1;
}
