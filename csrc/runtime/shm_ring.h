// Single-producer / single-consumer message ring in POSIX shared memory.
//
// The channel between the DP router (the process that owns the sockets and the bus) and one engine
// worker process per GPU ("8 processes with POSIX shared-memory SPSC rings into a host
// bus process").  Messages are length-prefixed byte strings; the producer never blocks the consumer
// and vice versa (head/tail are separate cache lines), and a blocked side sleeps on a process-shared
// futex instead of spinning, so an idle worker costs nothing and a token batch is seen within a
// wake-up (~10 µs) of being pushed.
#pragma once
#include <atomic>
#include <cstddef>
#include <cstdint>
#include <memory>
#include <string>

namespace dsse {

class ShmRing {
 public:
  // Create (and own: unlinked on destruction) a ring with `capacity` payload bytes (rounded up to a
  // power of two, >= 4 KiB).  Fails if the name exists and `replace` is false.
  static std::unique_ptr<ShmRing> create(const std::string& name, size_t capacity, bool replace = true,
                                         std::string* err = nullptr);
  // Attach to an existing ring, retrying until it exists or `timeout_ms` passes.
  static std::unique_ptr<ShmRing> open(const std::string& name, int timeout_ms, std::string* err = nullptr);
  ~ShmRing();

  // Producer side.  push() returns false when the message does not fit right now.
  bool push(const void* data, uint32_t len);
  bool push_wait(const void* data, uint32_t len, int timeout_ms);
  // Consumer side.  pop() is non-blocking; pop_wait() sleeps until a message arrives or timeout.
  bool pop(std::string* out);
  // spin_us > 0: poll for that long before sleeping on the futex (a latency-critical consumer, e.g. a TP
  // follower waiting for the leader's next step plan, skips the sleep/wake round trip).
  bool pop_wait(std::string* out, int timeout_ms, int spin_us = 0);

  // Either side may close; the other side sees closed() (pending messages can still be popped).
  void close();
  bool closed() const;
  size_t capacity() const;
  size_t used() const;
  const std::string& name() const { return name_; }

 private:
  struct Header;
  ShmRing() = default;
  Header* h_ = nullptr;
  uint8_t* data_ = nullptr;
  size_t map_bytes_ = 0;
  bool owner_ = false;
  std::string name_;
};

}  // namespace dsse
