#include "inspector.h"

#include <algorithm>
#include <cctype>

#include "json.h"

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

}  // namespace dsse
