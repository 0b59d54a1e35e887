// Wire-format JSON for the token stream (TokenMessage) and the chat request bodies.
//
// TokenMessage field order and escaping follow Go's encoding/json, which the reference services
// use end to end (src/llm-stream-proxy/main.go:55-61,230-245; src/sse-adapter/sse_handler.go:46-52):
//   {"conversation_id":"<id>","token":"<text>","sequence":<int64>,"done":<bool>,"timestamp":<ns>}
// Strings are HTML-escaped like json.Marshal (<, >, & -> <, >, &; U+2028/U+2029
// escaped; invalid UTF-8 -> �), so byte-for-byte frames match the Go adapter.
#pragma once
#include <cstdint>
#include <map>
#include <optional>
#include <string>
#include <string_view>
#include <vector>

namespace dsse {

// Engine finish reason of a terminal message (not part of the wire JSON: it rides along in the Frame so the
// OpenAI surface can report vLLM's finish_reason / usage).
enum FinishReason : uint8_t { kFinishNone = 0, kFinishStop = 1, kFinishLength = 2, kFinishAbort = 3 };

struct TokenMessage {
  std::string conversation_id;
  std::string token;
  int64_t sequence = 0;
  bool done = false;
  int64_t timestamp = 0;
  uint8_t finish = kFinishNone;  // terminal messages from the engine
  int32_t prompt_tokens = -1;    // terminal messages from the engine: prompt length (-1 = unknown)
};

// Append a JSON string literal (with quotes) using Go json.Marshal escaping rules.
void json_append_string(std::string& out, std::string_view s);
std::string json_quote(std::string_view s);

void encode_token_message(std::string& out, const TokenMessage& m);
std::string encode_token_message(const TokenMessage& m);

// Minimal JSON value for flat request objects: strings, numbers, bools, null (nested values are
// parsed and skipped).
struct JsonValue {
  enum Kind { kNull, kBool, kNumber, kString, kObject, kArray } kind = kNull;
  bool b = false;
  double num = 0;
  int64_t i64 = 0;
  bool is_int = false;
  std::string str;
  std::string raw;  // exact JSON text of an object / array value
};

// Parse the first JSON value of `text` as an object of scalar fields.  Keys are stored lower-cased
// (encoding/json matches struct fields case-insensitively).  Returns false on malformed JSON or when
// the top-level value is not an object.
bool parse_json_object(std::string_view text, std::map<std::string, JsonValue>& out, size_t* consumed = nullptr);

// Parse a JSON array whose elements are all objects (e.g. OpenAI chat `messages`).  Returns false on
// malformed JSON or a non-object element.
bool parse_json_array_of_objects(std::string_view text, std::vector<std::map<std::string, JsonValue>>& out);

// Parse a TokenMessage (as published by the proxy / load generator).  Missing fields keep defaults.
bool parse_token_message(std::string_view text, TokenMessage& m);

}  // namespace dsse
