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

}  // namespace dsse
