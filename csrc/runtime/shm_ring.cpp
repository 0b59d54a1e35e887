#include "shm_ring.h"

#include <fcntl.h>
#include <linux/futex.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <sys/syscall.h>
#include <time.h>
#include <unistd.h>

#include <chrono>
#include <cstring>
#include <thread>

namespace dsse {

namespace {
constexpr uint64_t kMagic = 0x4453534552494E47ULL;  // "DSSERING"
constexpr uint32_t kWrap = 0xFFFFFFFFu;             // length marker: continue at offset 0

int futex_wait(std::atomic<uint32_t>* addr, uint32_t expected, int timeout_ms) {
  timespec ts{timeout_ms / 1000, (long)(timeout_ms % 1000) * 1000000L};
  return (int)syscall(SYS_futex, reinterpret_cast<uint32_t*>(addr), FUTEX_WAIT, expected, timeout_ms >= 0 ? &ts : nullptr,
                      nullptr, 0);
}
void futex_wake(std::atomic<uint32_t>* addr) {
  syscall(SYS_futex, reinterpret_cast<uint32_t*>(addr), FUTEX_WAKE, 1, nullptr, nullptr, 0);
}
size_t pad8(size_t n) { return (n + 7) & ~size_t(7); }
int64_t mono_ms() {
  return std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}
}  // namespace

struct ShmRing::Header {
  uint64_t magic;
  uint64_t cap;
  alignas(64) std::atomic<uint64_t> head;  // bytes written (producer)
  alignas(64) std::atomic<uint64_t> tail;  // bytes consumed (consumer)
  alignas(64) std::atomic<uint32_t> data_seq;   // bumped on push (consumer futex)
  std::atomic<uint32_t> space_seq;              // bumped on pop (producer futex)
  std::atomic<uint32_t> closed;
  std::atomic<uint32_t> ready;                  // set last by the creator
  // sleepers on data_seq / space_seq: a push or pop only pays the futex_wake syscall when the other side is
  // actually asleep (seq_cst on both sides: the sleeper registers, re-checks, sleeps; the waker bumps, then looks)
  alignas(64) std::atomic<uint32_t> data_waiters;
  std::atomic<uint32_t> space_waiters;
};

std::unique_ptr<ShmRing> ShmRing::create(const std::string& name, size_t capacity, bool replace, std::string* err) {
  size_t cap = 4096;
  while (cap < capacity) cap <<= 1;
  if (replace) shm_unlink(name.c_str());
  int fd = shm_open(name.c_str(), O_CREAT | O_EXCL | O_RDWR, 0600);
  if (fd < 0) {
    if (err) *err = "shm_open(" + name + "): " + std::strerror(errno);
    return nullptr;
  }
  const size_t bytes = sizeof(Header) + cap;
  if (ftruncate(fd, (off_t)bytes) != 0) {
    if (err) *err = std::string("ftruncate: ") + std::strerror(errno);
    ::close(fd);
    shm_unlink(name.c_str());
    return nullptr;
  }
  void* p = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  ::close(fd);
  if (p == MAP_FAILED) {
    if (err) *err = std::string("mmap: ") + std::strerror(errno);
    shm_unlink(name.c_str());
    return nullptr;
  }
  std::unique_ptr<ShmRing> r(new ShmRing());
  r->h_ = new (p) Header();
  r->h_->magic = kMagic;
  r->h_->cap = cap;
  r->h_->head.store(0);
  r->h_->tail.store(0);
  r->h_->data_seq.store(0);
  r->h_->space_seq.store(0);
  r->h_->closed.store(0);
  r->h_->data_waiters.store(0);
  r->h_->space_waiters.store(0);
  r->data_ = static_cast<uint8_t*>(p) + sizeof(Header);
  r->map_bytes_ = bytes;
  r->owner_ = true;
  r->name_ = name;
  r->h_->ready.store(1, std::memory_order_release);
  return r;
}

std::unique_ptr<ShmRing> ShmRing::open(const std::string& name, int timeout_ms, std::string* err) {
  const int64_t t_end = mono_ms() + timeout_ms;
  while (true) {
    int fd = shm_open(name.c_str(), O_RDWR, 0600);
    if (fd >= 0) {
      struct stat st{};
      if (fstat(fd, &st) == 0 && (size_t)st.st_size > sizeof(Header)) {
        void* p = mmap(nullptr, (size_t)st.st_size, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
        ::close(fd);
        if (p != MAP_FAILED) {
          auto* h = static_cast<Header*>(p);
          if (h->ready.load(std::memory_order_acquire) == 1 && h->magic == kMagic) {
            std::unique_ptr<ShmRing> r(new ShmRing());
            r->h_ = h;
            r->data_ = static_cast<uint8_t*>(p) + sizeof(Header);
            r->map_bytes_ = (size_t)st.st_size;
            r->name_ = name;
            return r;
          }
          munmap(p, (size_t)st.st_size);
        }
      } else {
        ::close(fd);
      }
    }
    if (mono_ms() >= t_end) {
      if (err) *err = "shm ring " + name + " did not appear";
      return nullptr;
    }
    std::this_thread::sleep_for(std::chrono::milliseconds(20));
  }
}

ShmRing::~ShmRing() {
  if (h_) {
    if (owner_) h_->closed.store(1);
    munmap(h_, map_bytes_);
  }
  if (owner_) shm_unlink(name_.c_str());
}

bool ShmRing::push(const void* data, uint32_t len) {
  const uint64_t cap = h_->cap;
  const size_t need = pad8(4 + (size_t)len);
  if (need > cap / 2) return false;  // never fits reliably
  uint64_t head = h_->head.load(std::memory_order_relaxed);
  const uint64_t tail = h_->tail.load(std::memory_order_acquire);
  uint64_t off = head & (cap - 1);
  uint64_t extra = 0;
  if (off + need > cap) extra = cap - off;  // wrap: skip to the start
  if (head + extra + need - tail > cap) return false;
  if (extra) {
    const uint32_t w = kWrap;
    std::memcpy(data_ + off, &w, 4);
    head += extra;
    off = 0;
  }
  std::memcpy(data_ + off, &len, 4);
  std::memcpy(data_ + off + 4, data, len);
  h_->head.store(head + need, std::memory_order_release);
  h_->data_seq.fetch_add(1, std::memory_order_seq_cst);
  if (h_->data_waiters.load(std::memory_order_seq_cst) != 0) futex_wake(&h_->data_seq);
  return true;
}

bool ShmRing::push_wait(const void* data, uint32_t len, int timeout_ms) {
  const int64_t t_end = mono_ms() + timeout_ms;
  while (true) {
    const uint32_t seq = h_->space_seq.load(std::memory_order_acquire);
    if (push(data, len)) return true;
    if (closed()) return false;
    const int64_t left = t_end - mono_ms();
    if (left <= 0) return false;
    h_->space_waiters.fetch_add(1, std::memory_order_seq_cst);
    if (h_->space_seq.load(std::memory_order_seq_cst) == seq)
      futex_wait(&h_->space_seq, seq, (int)std::min<int64_t>(left, 50));
    h_->space_waiters.fetch_sub(1, std::memory_order_seq_cst);
  }
}

bool ShmRing::pop(std::string* out) {
  const uint64_t cap = h_->cap;
  uint64_t tail = h_->tail.load(std::memory_order_relaxed);
  const uint64_t head = h_->head.load(std::memory_order_acquire);
  if (tail == head) return false;
  uint64_t off = tail & (cap - 1);
  uint32_t len;
  std::memcpy(&len, data_ + off, 4);
  if (len == kWrap) {
    tail += cap - off;
    off = 0;
    std::memcpy(&len, data_, 4);
  }
  out->assign(reinterpret_cast<const char*>(data_ + off + 4), len);
  h_->tail.store(tail + pad8(4 + (size_t)len), std::memory_order_release);
  h_->space_seq.fetch_add(1, std::memory_order_seq_cst);
  if (h_->space_waiters.load(std::memory_order_seq_cst) != 0) futex_wake(&h_->space_seq);
  return true;
}

bool ShmRing::pop_wait(std::string* out, int timeout_ms, int spin_us) {
  if (spin_us > 0) {  // a consumer expecting the next message within microseconds polls before it sleeps
    const auto t_spin = std::chrono::steady_clock::now() + std::chrono::microseconds(spin_us);
    do {
      if (pop(out)) return true;
      if (closed()) return false;
      __builtin_ia32_pause();
    } while (std::chrono::steady_clock::now() < t_spin);
  }
  const int64_t t_end = mono_ms() + timeout_ms;
  while (true) {
    const uint32_t seq = h_->data_seq.load(std::memory_order_acquire);
    if (pop(out)) return true;
    if (closed()) return false;
    const int64_t left = t_end - mono_ms();
    if (left <= 0) return false;
    h_->data_waiters.fetch_add(1, std::memory_order_seq_cst);
    if (h_->data_seq.load(std::memory_order_seq_cst) == seq)
      futex_wait(&h_->data_seq, seq, (int)std::min<int64_t>(left, 50));
    h_->data_waiters.fetch_sub(1, std::memory_order_seq_cst);
  }
}

void ShmRing::close() {
  h_->closed.store(1);
  h_->data_seq.fetch_add(1);
  h_->space_seq.fetch_add(1);
  futex_wake(&h_->data_seq);
  futex_wake(&h_->space_seq);
}
bool ShmRing::closed() const { return h_->closed.load() != 0; }
size_t ShmRing::capacity() const { return (size_t)h_->cap; }
size_t ShmRing::used() const { return (size_t)(h_->head.load() - h_->tail.load()); }

}  // namespace dsse
