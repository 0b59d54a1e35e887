// Security inspection of streamed tokens (reference: src/spin-functions/nats-subscriber/src/lib.rs:57-102,
// docs/security-inspection-patterns.md; config src/sse-adapter/main.go:22-24,34-36).
//
// Rules: a sensitive keyword (password, secret, api_key, credit_card) -> redact to "[REDACTED]";
// a prompt-injection phrase (ignore previous, disregard above, new instructions, system prompt) ->
// drop; otherwise allow.  Matching is case-insensitive substring search.  Modes:
//   disabled (default) - no inspection
//   inline             - every token is inspected before it is written (drop / redact applied)
//   async              - tokens are delivered at once; a wildcard tap inspects them and a `drop`
//                        verdict kills the conversation (publishes on chat.<id>.control)
//   hybrid             - tokens are held for INSPECTION_BUFFER_MS while inspected, then released
#pragma once
#include <cstdint>
#include <string>
#include <string_view>

namespace dsse {

enum class InspectAction { kAllow, kRedact, kDrop };

struct InspectionResult {
  InspectAction action = InspectAction::kAllow;
  std::string reason;
  std::string redacted_content;
};

InspectionResult inspect_message(std::string_view content);
const char* action_name(InspectAction a);
std::string inspection_result_json(const InspectionResult& r);

enum class InspectionMode { kDisabled, kInline, kAsync, kHybrid };
InspectionMode parse_inspection_mode(std::string_view s);
const char* inspection_mode_name(InspectionMode m);

// Client of a remote inspector (INSPECTION_ENDPOINT, src/sse-adapter/main.go:36; the inline hook of
// src/sse-adapter/sse_handler.go:199-206 calls it per token): POSTs the reference's NatsMessage
// {"subject","data","sequence","timestamp"} to the endpoint URL (the Spin function's POST /inspect,
// src/spin-functions/nats-subscriber/src/lib.rs:34-54) and parses {"action","reason","redacted_content"}.
// Blocking HTTP/1.1 over one keep-alive connection (reconnected on error); one client per calling thread.
// Every wait is bounded by timeout_ms (connect included: non-blocking connect + poll), and a failure opens a
// circuit: for the next 1 s (doubling per consecutive failure, up to 30 s) inspect() fails at once, so the
// caller fails open instead of paying the timeout per token while the endpoint is down.
class RemoteInspector {
 public:
  explicit RemoteInspector(const std::string& url, int timeout_ms = 250);
  ~RemoteInspector();
  RemoteInspector(const RemoteInspector&) = delete;
  RemoteInspector& operator=(const RemoteInspector&) = delete;
  bool valid() const { return !host_.empty(); }
  // false on transport / protocol failure (the caller fails open)
  bool inspect(const std::string& subject, std::string_view data, int64_t sequence, int64_t timestamp,
               InspectionResult* out);

 private:
  bool connect_();
  bool roundtrip(const std::string& req, std::string* body);
  void trip();
  static constexpr int64_t kMinBackoffMs = 1000, kMaxBackoffMs = 30000;
  std::string host_, port_, path_;
  int timeout_ms_;
  int fd_ = -1;
  int64_t open_until_ns_ = 0;
  int64_t backoff_ms_ = kMinBackoffMs;
};

}  // namespace dsse
