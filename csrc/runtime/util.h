// Small host-side helpers shared by the runtime: clocks, ids, env config, logging.
#pragma once
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <string>

namespace dsse {

inline int64_t now_ns() {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::system_clock::now().time_since_epoch())
      .count();
}
inline int64_t mono_ns() {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

// RFC 4122 version-4 UUID (what google/uuid.New().String() produces for the reference's ids).
inline std::string uuid4() {
  thread_local std::mt19937_64 rng{std::random_device{}() ^ (uint64_t)mono_ns()};
  uint64_t a = rng(), b = rng();
  a = (a & 0xFFFFFFFFFFFF0FFFULL) | 0x0000000000004000ULL;
  b = (b & 0x3FFFFFFFFFFFFFFFULL) | 0x8000000000000000ULL;
  char s[37];
  snprintf(s, sizeof s, "%08x-%04x-%04x-%04x-%012llx", (unsigned)(a >> 32), (unsigned)((a >> 16) & 0xFFFF),
           (unsigned)(a & 0xFFFF), (unsigned)(b >> 48), (unsigned long long)(b & 0xFFFFFFFFFFFFULL));
  return s;
}

inline std::string env_str(const char* k, const std::string& dflt) {
  const char* v = std::getenv(k);
  return (v && *v) ? std::string(v) : dflt;
}
inline long env_long(const char* k, long dflt) {
  const char* v = std::getenv(k);
  return (v && *v) ? std::strtol(v, nullptr, 10) : dflt;
}

enum class LogLevel { kDebug = 0, kInfo = 1, kWarn = 2, kError = 3 };
LogLevel& log_level();
void log_json(LogLevel lvl, const std::string& msg, const std::string& kv_json = "");

}  // namespace dsse
