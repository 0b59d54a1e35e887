#include "json.h"

#include <cctype>
#include <cstring>
#include <cmath>
#include <cstdio>
#include <cstdlib>

namespace dsse {

namespace {

const char kHex[] = "0123456789abcdef";

void append_u(std::string& out, uint32_t cp) {
  out += "\\u";
  out += kHex[(cp >> 12) & 15];
  out += kHex[(cp >> 8) & 15];
  out += kHex[(cp >> 4) & 15];
  out += kHex[cp & 15];
}

// Decode one UTF-8 sequence at s[i]; returns its length, or 0 if invalid (Go emits � for
// each invalid byte).
size_t utf8_len(std::string_view s, size_t i, uint32_t& cp) {
  const unsigned char c = (unsigned char)s[i];
  auto cont = [&](size_t k) { return i + k < s.size() && ((unsigned char)s[i + k] & 0xC0) == 0x80; };
  if (c < 0x80) { cp = c; return 1; }
  if (c >= 0xC2 && c <= 0xDF && cont(1)) { cp = ((c & 0x1F) << 6) | (s[i + 1] & 0x3F); return 2; }
  if (c >= 0xE0 && c <= 0xEF && cont(1) && cont(2)) {
    cp = ((c & 0x0F) << 12) | ((s[i + 1] & 0x3F) << 6) | (s[i + 2] & 0x3F);
    if (cp < 0x800 || (cp >= 0xD800 && cp <= 0xDFFF)) return 0;
    return 3;
  }
  if (c >= 0xF0 && c <= 0xF4 && cont(1) && cont(2) && cont(3)) {
    cp = ((c & 0x07) << 18) | ((s[i + 1] & 0x3F) << 12) | ((s[i + 2] & 0x3F) << 6) | (s[i + 3] & 0x3F);
    if (cp < 0x10000 || cp > 0x10FFFF) return 0;
    return 4;
  }
  return 0;
}

}  // namespace

void json_append_string(std::string& out, std::string_view s) {
  out += '"';
  size_t i = 0;
  while (i < s.size()) {
    const unsigned char c = (unsigned char)s[i];
    if (c < 0x80) {
      switch (c) {
        case '"': out += "\\\""; break;
        case '\\': out += "\\\\"; break;
        case '\n': out += "\\n"; break;
        case '\r': out += "\\r"; break;
        case '\t': out += "\\t"; break;
        case '<': case '>': case '&': append_u(out, c); break;
        default:
          if (c < 0x20) append_u(out, c);
          else out += (char)c;
      }
      ++i;
      continue;
    }
    uint32_t cp = 0;
    const size_t n = utf8_len(s, i, cp);
    if (n == 0) {
      out += "\\ufffd";
      ++i;
      continue;
    }
    if (cp == 0x2028 || cp == 0x2029) append_u(out, cp);
    else out.append(s.data() + i, n);
    i += n;
  }
  out += '"';
}

std::string json_quote(std::string_view s) {
  std::string out;
  out.reserve(s.size() + 2);
  json_append_string(out, s);
  return out;
}

void encode_token_message(std::string& out, const TokenMessage& m) {
  char num[32];
  out += "{\"conversation_id\":";
  json_append_string(out, m.conversation_id);
  out += ",\"token\":";
  json_append_string(out, m.token);
  out += ",\"sequence\":";
  int n = snprintf(num, sizeof num, "%lld", (long long)m.sequence);
  out.append(num, n);
  out += m.done ? ",\"done\":true" : ",\"done\":false";
  out += ",\"timestamp\":";
  n = snprintf(num, sizeof num, "%lld", (long long)m.timestamp);
  out.append(num, n);
  out += '}';
}

std::string encode_token_message(const TokenMessage& m) {
  std::string s;
  s.reserve(96 + m.conversation_id.size() + m.token.size());
  encode_token_message(s, m);
  return s;
}

// ---------------------------------------------------------------- parser
namespace {

struct Parser {
  std::string_view t;
  size_t p = 0;
  int depth = 0;

  void ws() {
    while (p < t.size() && (t[p] == ' ' || t[p] == '\t' || t[p] == '\n' || t[p] == '\r')) ++p;
  }
  bool lit(const char* s) {
    size_t n = strlen(s);
    if (t.substr(p, n) != s) return false;
    p += n;
    return true;
  }
  static int hexv(char c) {
    if (c >= '0' && c <= '9') return c - '0';
    if (c >= 'a' && c <= 'f') return c - 'a' + 10;
    if (c >= 'A' && c <= 'F') return c - 'A' + 10;
    return -1;
  }
  static void put_utf8(std::string& o, uint32_t cp) {
    if (cp < 0x80) o += (char)cp;
    else if (cp < 0x800) { o += (char)(0xC0 | (cp >> 6)); o += (char)(0x80 | (cp & 0x3F)); }
    else if (cp < 0x10000) {
      o += (char)(0xE0 | (cp >> 12)); o += (char)(0x80 | ((cp >> 6) & 0x3F)); o += (char)(0x80 | (cp & 0x3F));
    } else {
      o += (char)(0xF0 | (cp >> 18)); o += (char)(0x80 | ((cp >> 12) & 0x3F));
      o += (char)(0x80 | ((cp >> 6) & 0x3F)); o += (char)(0x80 | (cp & 0x3F));
    }
  }
  bool hex4(uint32_t& v) {
    if (p + 4 > t.size()) return false;
    v = 0;
    for (int k = 0; k < 4; ++k) {
      int h = hexv(t[p + k]);
      if (h < 0) return false;
      v = (v << 4) | h;
    }
    p += 4;
    return true;
  }
  bool string(std::string& o) {
    if (p >= t.size() || t[p] != '"') return false;
    ++p;
    while (p < t.size()) {
      char c = t[p++];
      if (c == '"') return true;
      if ((unsigned char)c < 0x20) return false;
      if (c != '\\') { o += c; continue; }
      if (p >= t.size()) return false;
      char e = t[p++];
      switch (e) {
        case '"': o += '"'; break;
        case '\\': o += '\\'; break;
        case '/': o += '/'; break;
        case 'b': o += '\b'; break;
        case 'f': o += '\f'; break;
        case 'n': o += '\n'; break;
        case 'r': o += '\r'; break;
        case 't': o += '\t'; break;
        case 'u': {
          uint32_t cp;
          if (!hex4(cp)) return false;
          if (cp >= 0xD800 && cp <= 0xDBFF && p + 6 <= t.size() && t[p] == '\\' && t[p + 1] == 'u') {
            size_t save = p;
            p += 2;
            uint32_t lo;
            if (hex4(lo) && lo >= 0xDC00 && lo <= 0xDFFF) cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
            else { p = save; cp = 0xFFFD; }
          } else if (cp >= 0xD800 && cp <= 0xDFFF) {
            cp = 0xFFFD;
          }
          put_utf8(o, cp);
          break;
        }
        default: return false;
      }
    }
    return false;
  }
  bool number(JsonValue& v) {
    size_t s = p;
    if (p < t.size() && t[p] == '-') ++p;
    if (p >= t.size() || !isdigit((unsigned char)t[p])) return false;
    if (t[p] == '0') ++p;
    else while (p < t.size() && isdigit((unsigned char)t[p])) ++p;
    bool frac = false;
    if (p < t.size() && t[p] == '.') {
      frac = true;
      ++p;
      if (p >= t.size() || !isdigit((unsigned char)t[p])) return false;
      while (p < t.size() && isdigit((unsigned char)t[p])) ++p;
    }
    if (p < t.size() && (t[p] == 'e' || t[p] == 'E')) {
      frac = true;
      ++p;
      if (p < t.size() && (t[p] == '+' || t[p] == '-')) ++p;
      if (p >= t.size() || !isdigit((unsigned char)t[p])) return false;
      while (p < t.size() && isdigit((unsigned char)t[p])) ++p;
    }
    std::string num(t.substr(s, p - s));
    v.kind = JsonValue::kNumber;
    v.num = strtod(num.c_str(), nullptr);
    v.is_int = !frac;
    if (!frac) v.i64 = strtoll(num.c_str(), nullptr, 10);
    return true;
  }
  bool value(JsonValue& v) {
    if (++depth > 64) return false;
    ws();
    if (p >= t.size()) return false;
    bool ok = true;
    char c = t[p];
    const size_t s0 = p;
    if (c == '"') { v.kind = JsonValue::kString; ok = string(v.str); }
    else if (c == '{') { v.kind = JsonValue::kObject; std::map<std::string, JsonValue> skip; ok = object(skip); }
    else if (c == '[') { v.kind = JsonValue::kArray; ok = array(); }
    else if (c == 't') { v.kind = JsonValue::kBool; v.b = true; ok = lit("true"); }
    else if (c == 'f') { v.kind = JsonValue::kBool; v.b = false; ok = lit("false"); }
    else if (c == 'n') { v.kind = JsonValue::kNull; ok = lit("null"); }
    else ok = number(v);
    if (ok && (c == '{' || c == '[')) v.raw = std::string(t.substr(s0, p - s0));
    --depth;
    return ok;
  }
  bool array() {
    ++p;  // '['
    ws();
    if (p < t.size() && t[p] == ']') { ++p; return true; }
    while (true) {
      JsonValue v;
      if (!value(v)) return false;
      ws();
      if (p >= t.size()) return false;
      if (t[p] == ',') { ++p; continue; }
      if (t[p] == ']') { ++p; return true; }
      return false;
    }
  }
  bool object(std::map<std::string, JsonValue>& out) {
    if (p >= t.size() || t[p] != '{') return false;
    ++p;
    ws();
    if (p < t.size() && t[p] == '}') { ++p; return true; }
    while (true) {
      ws();
      std::string key;
      if (!string(key)) return false;
      ws();
      if (p >= t.size() || t[p] != ':') return false;
      ++p;
      JsonValue v;
      if (!value(v)) return false;
      for (auto& ch : key) ch = (char)tolower((unsigned char)ch);
      out[key] = std::move(v);
      ws();
      if (p >= t.size()) return false;
      if (t[p] == ',') { ++p; continue; }
      if (t[p] == '}') { ++p; return true; }
      return false;
    }
  }
};

}  // namespace

bool parse_json_array_of_objects(std::string_view text, std::vector<std::map<std::string, JsonValue>>& out) {
  Parser ps{text};
  ps.ws();
  if (ps.p >= text.size() || text[ps.p] != '[') return false;
  ++ps.p;
  ps.ws();
  if (ps.p < text.size() && text[ps.p] == ']') return true;
  while (true) {
    ps.ws();
    std::map<std::string, JsonValue> o;
    if (!ps.object(o)) return false;
    out.push_back(std::move(o));
    ps.ws();
    if (ps.p >= text.size()) return false;
    if (text[ps.p] == ',') { ++ps.p; continue; }
    if (text[ps.p] == ']') return true;
    return false;
  }
}

bool parse_json_object(std::string_view text, std::map<std::string, JsonValue>& out, size_t* consumed) {
  Parser ps{text};
  ps.ws();
  if (!ps.object(out)) return false;
  if (consumed) *consumed = ps.p;
  return true;
}

bool parse_token_message(std::string_view text, TokenMessage& m) {
  std::map<std::string, JsonValue> o;
  if (!parse_json_object(text, o)) return false;
  auto it = o.find("conversation_id");
  if (it != o.end()) {
    if (it->second.kind != JsonValue::kString) return false;
    m.conversation_id = it->second.str;
  }
  if ((it = o.find("token")) != o.end()) {
    if (it->second.kind != JsonValue::kString) return false;
    m.token = it->second.str;
  }
  if ((it = o.find("sequence")) != o.end()) {
    if (it->second.kind != JsonValue::kNumber || !it->second.is_int) return false;
    m.sequence = it->second.i64;
  }
  if ((it = o.find("done")) != o.end()) {
    if (it->second.kind != JsonValue::kBool) return false;
    m.done = it->second.b;
  }
  if ((it = o.find("timestamp")) != o.end()) {
    if (it->second.kind != JsonValue::kNumber || !it->second.is_int) return false;
    m.timestamp = it->second.i64;
  }
  return true;
}

}  // namespace dsse
