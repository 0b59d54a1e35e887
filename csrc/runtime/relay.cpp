#include "relay.h"

#include <fcntl.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/epoll.h>
#include <sys/eventfd.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <chrono>
#include <cstring>
#include <vector>

#include "json.h"
#include "metrics.h"
#include "util.h"

namespace dsse {

namespace {
int64_t mono_ms() {
  return std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}
}  // namespace

struct UpstreamRelay::Link {
  std::string conv;
  int fd = -1;
  std::string out;
  size_t out_off = 0;
  std::string in, body;
  bool headers_done = false, chunked = false;
  int64_t chunk_left = -1;
  int64_t last_seq = 0;
  bool done = false;
  int retries = 0;
  int64_t retry_at_ms = 0;   // > 0: waiting to reconnect
  int64_t idle_since_ms = 0;  // no local subscriber since (0 = has subscribers)
};

UpstreamRelay::UpstreamRelay(Bus& bus, std::string upstream_url, int max_retries)
    : bus_(bus), url_(std::move(upstream_url)), max_retries_(max_retries) {
  std::string u = url_;
  if (u.rfind("http://", 0) == 0) u = u.substr(7);
  while (!u.empty() && u.back() == '/') u.pop_back();
  const size_t slash = u.find('/');
  const std::string hostport = u.substr(0, slash);
  base_ = slash == std::string::npos ? "" : u.substr(slash);
  host_ = hostport;
  port_ = "80";
  if (hostport.find(':') != std::string::npos) {
    host_ = hostport.substr(0, hostport.find(':'));
    port_ = hostport.substr(hostport.find(':') + 1);
  }
}

UpstreamRelay::~UpstreamRelay() { stop(); }

bool UpstreamRelay::start(std::string* err) {
  ep_ = epoll_create1(EPOLL_CLOEXEC);
  evfd_ = eventfd(0, EFD_NONBLOCK | EFD_CLOEXEC);
  if (ep_ < 0 || evfd_ < 0) {
    if (err) *err = "relay: epoll/eventfd failed";
    return false;
  }
  epoll_event ev{};
  ev.events = EPOLLIN;
  ev.data.ptr = nullptr;
  epoll_ctl(ep_, EPOLL_CTL_ADD, evfd_, &ev);
  running_ = true;
  thread_ = std::thread([this] { run(); });
  return true;
}

void UpstreamRelay::stop() {
  if (!running_.exchange(false)) return;
  uint64_t one = 1;
  ssize_t r = ::write(evfd_, &one, sizeof one);
  (void)r;
  if (thread_.joinable()) thread_.join();
  for (auto& kv : links_)
    if (kv.second->fd >= 0) ::close(kv.second->fd);
  links_.clear();
  if (ep_ >= 0) ::close(ep_);
  if (evfd_ >= 0) ::close(evfd_);
  ep_ = evfd_ = -1;
}

void UpstreamRelay::ensure(const std::string& conv_id) {
  {
    std::lock_guard<std::mutex> g(mu_);
    wanted_.push_back(conv_id);
  }
  uint64_t one = 1;
  ssize_t r = ::write(evfd_, &one, sizeof one);
  (void)r;
}

size_t UpstreamRelay::active() { return n_active_.load(); }

bool UpstreamRelay::open_link(Link& l) {
  addrinfo hints{}, *res = nullptr;
  hints.ai_socktype = SOCK_STREAM;
  if (getaddrinfo(host_.c_str(), port_.c_str(), &hints, &res) != 0 || !res) return false;
  l.fd = socket(res->ai_family, SOCK_STREAM | SOCK_NONBLOCK | SOCK_CLOEXEC, 0);
  if (l.fd < 0) {
    freeaddrinfo(res);
    return false;
  }
  int one = 1;
  setsockopt(l.fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
  const int rc = connect(l.fd, res->ai_addr, res->ai_addrlen);
  freeaddrinfo(res);
  if (rc < 0 && errno != EINPROGRESS) {
    ::close(l.fd);
    l.fd = -1;
    return false;
  }
  l.out = "GET " + base_ + "/stream/" + l.conv + (l.last_seq > 0 ? "" : "?replay=1") + " HTTP/1.1\r\nHost: " + host_ +
          ":" + port_ + "\r\nUser-Agent: dsse-edge-relay\r\nAccept: text/event-stream\r\nCache-Control: no-cache\r\n";
  if (l.last_seq > 0) l.out += "Last-Event-ID: " + std::to_string(l.last_seq) + "\r\n";
  l.out += "\r\n";
  l.out_off = 0;
  l.in.clear();
  l.body.clear();
  l.headers_done = l.chunked = false;
  l.chunk_left = -1;
  epoll_event ev{};
  ev.events = EPOLLIN | EPOLLOUT | EPOLLRDHUP;
  ev.data.ptr = &l;
  epoll_ctl(ep_, EPOLL_CTL_ADD, l.fd, &ev);
  return true;
}

void UpstreamRelay::close_link(Link& l) {
  if (l.fd >= 0) {
    epoll_ctl(ep_, EPOLL_CTL_DEL, l.fd, nullptr);
    ::close(l.fd);
    l.fd = -1;
  }
}

bool UpstreamRelay::parse(Link& l) {
  if (!l.headers_done) {
    const size_t e = l.in.find("\r\n\r\n");
    if (e == std::string::npos) return true;
    std::string head = l.in.substr(0, e);
    l.in.erase(0, e + 4);
    const size_t sp = head.find(' ');
    const int status = sp == std::string::npos ? 0 : std::atoi(head.c_str() + sp + 1);
    std::transform(head.begin(), head.end(), head.begin(), ::tolower);
    l.chunked = head.find("transfer-encoding: chunked") != std::string::npos;
    l.headers_done = true;
    if (status != 200) return false;
  }
  bool ended = false;  // upstream ended the stream (events before the terminator are still relayed)
  if (l.chunked) {
    size_t p = 0;
    while (p < l.in.size()) {
      if (l.chunk_left < 0) {
        const size_t e = l.in.find("\r\n", p);
        if (e == std::string::npos) break;
        l.chunk_left = std::strtoll(l.in.c_str() + p, nullptr, 16);
        p = e + 2;
        if (l.chunk_left == 0) {
          ended = true;
          break;
        }
      } else if (l.chunk_left > 0) {
        const size_t take = std::min<size_t>((size_t)l.chunk_left, l.in.size() - p);
        l.body.append(l.in, p, take);
        p += take;
        l.chunk_left -= (int64_t)take;
      } else {  // chunk data complete: expect CRLF
        if (l.in.size() - p < 2) break;
        p += 2;
        l.chunk_left = -1;
      }
    }
    l.in.erase(0, p);
  } else {
    l.body += l.in;
    l.in.clear();
  }
  // SSE events: only `event: token` frames are relayed (comments and keep-alives are local)
  size_t p = 0;
  std::vector<FramePtr> frames;
  while (true) {
    const size_t e = l.body.find("\n\n", p);
    if (e == std::string::npos) break;
    std::string ev, data;
    size_t q = p;
    while (q < e) {
      size_t nl = l.body.find('\n', q);
      if (nl == std::string::npos || nl > e) nl = e;
      if (l.body.compare(q, 6, "event:") == 0) {
        ev = l.body.substr(q + 6, nl - q - 6);
        if (!ev.empty() && ev[0] == ' ') ev.erase(0, 1);
      } else if (l.body.compare(q, 5, "data:") == 0) {
        data = l.body.substr(q + 5, nl - q - 5);
        if (!data.empty() && data[0] == ' ') data.erase(0, 1);
      }
      q = nl + 1;
    }
    p = e + 2;
    if (ev != "token" || data.empty()) continue;
    TokenMessage m;
    if (!parse_token_message(data, m)) continue;
    if (m.sequence <= l.last_seq) continue;  // replay overlap after a reconnect
    l.last_seq = m.sequence;
    if (m.done) l.done = true;
    frames.push_back(Bus::make_frame(m));
  }
  l.body.erase(0, p);
  if (!frames.empty()) {
    bus_.publish_batch(frames);
    metrics().relay_frames_total.add((double)frames.size());
  }
  return !l.done && !ended;
}

void UpstreamRelay::on_readable(Link& l) {
  char buf[65536];
  bool alive = true;
  while (true) {
    const ssize_t n = recv(l.fd, buf, sizeof buf, 0);
    if (n > 0) {
      l.in.append(buf, (size_t)n);
      continue;
    }
    if (n == 0) alive = false;
    else if (errno != EAGAIN && errno != EWOULDBLOCK) alive = false;
    break;
  }
  const bool ok = parse(l) && alive;
  if (!ok) {
    close_link(l);
    if (!l.done) l.retry_at_ms = mono_ms() + 200 * (1 << std::min(l.retries, 4));
  }
}

void UpstreamRelay::run() {
  std::vector<epoll_event> evs(256);
  int64_t last_scan = mono_ms();
  while (running_) {
    const int n = epoll_wait(ep_, evs.data(), (int)evs.size(), 100);
    for (int i = 0; i < n; ++i) {
      if (evs[i].data.ptr == nullptr) {
        uint64_t v;
        ssize_t r = ::read(evfd_, &v, sizeof v);
        (void)r;
        continue;
      }
      Link& l = *static_cast<Link*>(evs[i].data.ptr);
      if (l.fd < 0) continue;
      if (evs[i].events & EPOLLOUT) {
        while (l.out_off < l.out.size()) {
          const ssize_t w = send(l.fd, l.out.data() + l.out_off, l.out.size() - l.out_off, MSG_NOSIGNAL);
          if (w <= 0) break;
          l.out_off += (size_t)w;
        }
        if (l.out_off == l.out.size()) {
          epoll_event ev{};
          ev.events = EPOLLIN | EPOLLRDHUP;
          ev.data.ptr = &l;
          epoll_ctl(ep_, EPOLL_CTL_MOD, l.fd, &ev);
        }
      }
      if (evs[i].events & (EPOLLIN | EPOLLHUP | EPOLLERR | EPOLLRDHUP)) on_readable(l);
    }
    std::deque<std::string> want;
    {
      std::lock_guard<std::mutex> g(mu_);
      want.swap(wanted_);
    }
    for (auto& c : want) {
      auto it = links_.find(c);
      if (it != links_.end() && (it->second->fd >= 0 || it->second->retry_at_ms > 0)) continue;
      auto l = std::make_unique<Link>();
      l->conv = c;
      if (it != links_.end()) l->last_seq = it->second->last_seq;  // finished earlier: continue after it
      Link& ref = *l;
      links_[c] = std::move(l);
      if (!open_link(ref)) ref.retry_at_ms = mono_ms() + 200;
    }
    const int64_t now = mono_ms();
    if (now - last_scan >= 100) {
      last_scan = now;
      size_t active = 0;
      for (auto it = links_.begin(); it != links_.end();) {
        Link& l = *it->second;
        const bool interested = bus_.subscriber_count(l.conv) > 0;
        if (!interested && l.idle_since_ms == 0) l.idle_since_ms = now;
        if (interested) l.idle_since_ms = 0;
        const bool give_up = l.retries > max_retries_;
        if (l.done || give_up || (l.idle_since_ms > 0 && now - l.idle_since_ms > 2000)) {
          if (give_up && !l.done) {
            TokenMessage m{l.conv, "[ERROR]", l.last_seq + 1, true, now_ns()};
            bus_.publish(m);
            log_json(LogLevel::kWarn, "upstream relay gave up", "\"conversation_id\":" + json_quote(l.conv));
          }
          close_link(l);
          it = links_.erase(it);
          continue;
        }
        if (l.fd < 0 && l.retry_at_ms > 0 && now >= l.retry_at_ms) {
          l.retries++;
          l.retry_at_ms = 0;
          if (!open_link(l)) l.retry_at_ms = now + 200 * (1 << std::min(l.retries, 4));
        }
        active += l.fd >= 0 ? 1 : 0;
        ++it;
      }
      n_active_ = active;
      metrics().relay_upstream_connections.set((double)active);
    }
  }
}

}  // namespace dsse
