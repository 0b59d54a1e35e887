#include "inspector.h"

#include <netdb.h>
#include <netinet/in.h>
#include <fcntl.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <cctype>
#include <cstring>
#include <map>

#include "json.h"
#include "util.h"

namespace dsse {

namespace {
const char* const kSensitive[] = {"password", "secret", "api_key", "credit_card"};
const char* const kInjection[] = {"ignore previous", "disregard above", "new instructions", "system prompt"};
}  // namespace

InspectionResult inspect_message(std::string_view content) {
  std::string lower(content);
  std::transform(lower.begin(), lower.end(), lower.begin(), [](unsigned char c) { return (char)std::tolower(c); });
  InspectionResult r;
  for (const char* p : kSensitive) {
    if (lower.find(p) != std::string::npos) {
      r.action = InspectAction::kRedact;
      r.reason = std::string("Contains sensitive pattern: ") + p;
      r.redacted_content = "[REDACTED]";
      return r;
    }
  }
  for (const char* p : kInjection) {
    if (lower.find(p) != std::string::npos) {
      r.action = InspectAction::kDrop;
      r.reason = std::string("Potential prompt injection: ") + p;
      return r;
    }
  }
  return r;
}

const char* action_name(InspectAction a) {
  switch (a) {
    case InspectAction::kAllow: return "allow";
    case InspectAction::kRedact: return "redact";
    case InspectAction::kDrop: return "drop";
  }
  return "allow";
}

std::string inspection_result_json(const InspectionResult& r) {
  std::string o = "{\"action\":";
  json_append_string(o, action_name(r.action));
  o += ",\"reason\":";
  if (r.reason.empty()) o += "null";
  else json_append_string(o, r.reason);
  o += ",\"redacted_content\":";
  if (r.action == InspectAction::kRedact) json_append_string(o, r.redacted_content);
  else o += "null";
  o += '}';
  return o;
}

InspectionMode parse_inspection_mode(std::string_view s) {
  if (s == "inline") return InspectionMode::kInline;
  if (s == "async") return InspectionMode::kAsync;
  if (s == "hybrid") return InspectionMode::kHybrid;
  return InspectionMode::kDisabled;
}

const char* inspection_mode_name(InspectionMode m) {
  switch (m) {
    case InspectionMode::kInline: return "inline";
    case InspectionMode::kAsync: return "async";
    case InspectionMode::kHybrid: return "hybrid";
    default: return "disabled";
  }
}

// ------------------------------------------------------------------ remote inspector client
RemoteInspector::RemoteInspector(const std::string& url, int timeout_ms) : timeout_ms_(timeout_ms) {
  std::string u = url;
  if (u.rfind("http://", 0) == 0) u = u.substr(7);
  else if (u.find("://") != std::string::npos) return;  // only plain HTTP (in-cluster sidecar / service)
  const size_t slash = u.find('/');
  const std::string hostport = u.substr(0, slash);
  path_ = slash == std::string::npos ? "/inspect" : u.substr(slash);
  const size_t colon = hostport.rfind(':');
  host_ = colon == std::string::npos ? hostport : hostport.substr(0, colon);
  port_ = colon == std::string::npos ? "80" : hostport.substr(colon + 1);
}

RemoteInspector::~RemoteInspector() {
  if (fd_ >= 0) ::close(fd_);
}

bool RemoteInspector::connect_() {
  if (fd_ >= 0) return true;
  if (mono_ns() < open_until_ns_) return false;  // circuit open after a failure: fail open without waiting
  addrinfo hints{}, *res = nullptr;
  hints.ai_socktype = SOCK_STREAM;
  if (getaddrinfo(host_.c_str(), port_.c_str(), &hints, &res) != 0 || !res) return false;
  // non-blocking connect bounded by timeout_ms: a black-holed endpoint must not stall the gate for the kernel's
  // SYN retry period (minutes)
  fd_ = socket(res->ai_family, SOCK_STREAM | SOCK_NONBLOCK | SOCK_CLOEXEC, 0);
  bool ok = fd_ >= 0;
  if (ok && ::connect(fd_, res->ai_addr, res->ai_addrlen) != 0) {
    ok = false;
    if (errno == EINPROGRESS) {
      pollfd pfd{fd_, POLLOUT, 0};
      int err = 0;
      socklen_t len = sizeof err;
      ok = ::poll(&pfd, 1, timeout_ms_) == 1 && getsockopt(fd_, SOL_SOCKET, SO_ERROR, &err, &len) == 0 && err == 0;
    }
  }
  freeaddrinfo(res);
  if (!ok) {
    if (fd_ >= 0) ::close(fd_);
    fd_ = -1;
    return false;
  }
  fcntl(fd_, F_SETFL, fcntl(fd_, F_GETFL) & ~O_NONBLOCK);
  const int one = 1;
  setsockopt(fd_, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
  timeval tv{timeout_ms_ / 1000, (timeout_ms_ % 1000) * 1000};
  setsockopt(fd_, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof tv);
  setsockopt(fd_, SOL_SOCKET, SO_SNDTIMEO, &tv, sizeof tv);
  return true;
}

void RemoteInspector::trip() {
  open_until_ns_ = mono_ns() + backoff_ms_ * 1000000LL;
  backoff_ms_ = std::min<int64_t>(backoff_ms_ * 2, kMaxBackoffMs);
}

// One request / response on the keep-alive connection (Content-Length or chunked body).
bool RemoteInspector::roundtrip(const std::string& req, std::string* body) {
  if (::send(fd_, req.data(), req.size(), MSG_NOSIGNAL) != (ssize_t)req.size()) return false;
  std::string in;
  char buf[4096];
  size_t hdr_end = std::string::npos;
  const int64_t deadline = mono_ns() + (int64_t)timeout_ms_ * 1000000;
  auto more = [&]() {
    if (mono_ns() > deadline) return false;
    const ssize_t n = ::recv(fd_, buf, sizeof buf, 0);
    if (n <= 0) return false;
    in.append(buf, (size_t)n);
    return true;
  };
  while ((hdr_end = in.find("\r\n\r\n")) == std::string::npos)
    if (!more()) return false;
  int code = 0;
  if (sscanf(in.c_str(), "HTTP/%*s %d", &code) != 1 || code != 200) return false;
  std::string head = in.substr(0, hdr_end);
  std::transform(head.begin(), head.end(), head.begin(), [](unsigned char c) { return (char)std::tolower(c); });
  size_t pos = hdr_end + 4;
  const size_t cl = head.find("content-length:");
  if (cl != std::string::npos) {
    const size_t len = std::strtoul(head.c_str() + cl + 15, nullptr, 10);
    while (in.size() < pos + len)
      if (!more()) return false;
    *body = in.substr(pos, len);
    return true;
  }
  if (head.find("transfer-encoding: chunked") == std::string::npos) return false;
  body->clear();
  while (true) {
    size_t eol;
    while ((eol = in.find("\r\n", pos)) == std::string::npos)
      if (!more()) return false;
    const size_t len = std::strtoul(in.c_str() + pos, nullptr, 16);
    pos = eol + 2;
    while (in.size() < pos + len + 2)
      if (!more()) return false;
    if (len == 0) return true;
    body->append(in, pos, len);
    pos += len + 2;
  }
}

bool RemoteInspector::inspect(const std::string& subject, std::string_view data, int64_t sequence, int64_t timestamp,
                              InspectionResult* out) {
  if (!valid()) return false;
  std::string payload = "{\"subject\":";
  json_append_string(payload, subject);
  payload += ",\"data\":";
  json_append_string(payload, data);
  payload += ",\"sequence\":" + std::to_string(sequence) + ",\"timestamp\":" + std::to_string(timestamp) + "}";
  const std::string req = "POST " + path_ + " HTTP/1.1\r\nHost: " + host_ + ":" + port_ +
                          "\r\nContent-Type: application/json\r\nConnection: keep-alive\r\nContent-Length: " +
                          std::to_string(payload.size()) + "\r\n\r\n" + payload;
  std::string body;
  bool ok = false;
  for (int attempt = 0; attempt < 2 && !ok; ++attempt) {  // one reconnect: the server may close idle sockets
    if (!connect_()) {
      if (mono_ns() >= open_until_ns_) trip();
      return false;
    }
    ok = roundtrip(req, &body);
    if (!ok) {
      ::close(fd_);
      fd_ = -1;
    }
  }
  if (!ok) {
    trip();
    return false;
  }
  backoff_ms_ = kMinBackoffMs;
  std::map<std::string, JsonValue> o;
  if (!parse_json_object(body, o)) return false;
  auto a = o.find("action");
  if (a == o.end() || a->second.kind != JsonValue::kString) return false;
  InspectionResult r;
  if (a->second.str == "redact") r.action = InspectAction::kRedact;
  else if (a->second.str == "drop") r.action = InspectAction::kDrop;
  else if (a->second.str != "allow") return false;
  auto rs = o.find("reason");
  if (rs != o.end() && rs->second.kind == JsonValue::kString) r.reason = rs->second.str;
  auto rc = o.find("redacted_content");
  if (rc != o.end() && rc->second.kind == JsonValue::kString) r.redacted_content = rc->second.str;
  else if (r.action == InspectAction::kRedact) r.redacted_content = "[REDACTED]";
  *out = std::move(r);
  return true;
}

}  // namespace dsse
