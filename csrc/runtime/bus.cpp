#include "bus.h"

#include <algorithm>
#include <cstdio>
#include <unordered_set>

#include "metrics.h"
#include "util.h"

namespace dsse {

Bus::Bus(BusConfig cfg) : cfg_(cfg) {
  if (cfg_.shards < 1) cfg_.shards = 1;
  for (int i = 0; i < cfg_.shards; ++i) shards_.emplace_back(new Shard);
}

Bus::Shard& Bus::shard(const std::string& id) {
  return *shards_[std::hash<std::string>{}(id) % shards_.size()];
}

FramePtr Bus::make_frame(const TokenMessage& m) {
  auto f = std::make_shared<Frame>();
  f->conversation_id = m.conversation_id;
  f->seq = m.sequence;
  f->done = m.done;
  f->timestamp = m.timestamp;
  f->finish = m.finish;
  f->prompt_tokens = m.prompt_tokens;
  f->created_mono = mono_ns();
  char head[48];
  const int n = snprintf(head, sizeof head, "event: token\nid: %lld\ndata: ", (long long)m.sequence);
  f->bytes.reserve(n + 120 + 6 * (m.conversation_id.size() + m.token.size()) / 5);
  f->bytes.append(head, n);
  encode_token_message(f->bytes, m);
  f->json_off = (uint32_t)n;
  f->json_len = (uint32_t)(f->bytes.size() - n);
  f->bytes += "\n\n";
  return f;
}

void Bus::subscribe(const std::string& id, const SinkPtr& s, int64_t after_seq, std::vector<FramePtr>* replay) {
  Shard& sh = shard(id);
  std::lock_guard<std::mutex> g(sh.mu);
  auto [it, inserted] = sh.convs.try_emplace(id);
  if (inserted) n_convs_.fetch_add(1);
  Conv& c = it->second;
  if (replay && after_seq >= 0) {
    for (const auto& f : c.ring)
      if (f->seq > after_seq) replay->push_back(f);
    metrics().bus_replayed_total.add((double)replay->size());
  }
  auto subs = c.subs ? std::make_shared<SubList>(*c.subs) : std::make_shared<SubList>();
  subs->push_back(s);
  c.subs = std::move(subs);
}

void Bus::unsubscribe(const std::string& id, const SinkPtr& s) {
  Shard& sh = shard(id);
  std::lock_guard<std::mutex> g(sh.mu);
  auto it = sh.convs.find(id);
  if (it == sh.convs.end() || !it->second.subs) return;
  auto subs = std::make_shared<SubList>(*it->second.subs);
  subs->erase(std::remove(subs->begin(), subs->end(), s), subs->end());
  if (subs->empty()) it->second.subs.reset();
  else it->second.subs = std::move(subs);
}

void Bus::add_tap(const SinkPtr& s) {
  std::lock_guard<std::mutex> g(taps_mu_);
  taps_.push_back(s);
  have_taps_.store(true);
}

void Bus::remove_tap(const SinkPtr& s) {
  std::lock_guard<std::mutex> g(taps_mu_);
  taps_.erase(std::remove(taps_.begin(), taps_.end(), s), taps_.end());
  have_taps_.store(!taps_.empty());
}

void Bus::set_gate(std::shared_ptr<FrameGate> g) {
  std::lock_guard<std::mutex> lk(gate_mu_);
  gate_ = std::move(g);
  have_gate_.store(gate_ != nullptr);
}

// Duplicate / post-terminal frame of conversation `c` (shard lock held).  A terminal conversation that sees
// sequence 1 again starts a new stream (e.g. the next turn of a conversation id a client reuses) -- but only
// when that frame is NEWER than the terminal one (producer timestamp; without timestamps: the dedupe window
// has passed since the terminal frame).  A redelivered first token of the finished stream is a duplicate: it
// must not wipe the replay ring that Last-Event-ID reconnects read.
bool Bus::duplicate_locked(Conv& c, const Frame& f, int64_t now) {
  if (f.seq <= 0) return false;
  if (c.done) {
    if (f.seq == 1 && !f.done && c.done_seq > 1) {
      const bool newer = (f.timestamp > 0 && c.done_ts > 0)
                             ? f.timestamp > c.done_ts
                             : (cfg_.dedupe_window_s <= 0 || now - c.done_mono > cfg_.dedupe_window_s * 1000000000LL);
      if (!newer) return true;
      c.done = false;  // a new stream under the same conversation id
      c.ring.clear();
      c.last_seq = 0;
      return false;
    }
    if (f.seq >= c.done_seq) return true;  // the terminal frame again, or something after it
  }
  if (cfg_.dedupe_window_s <= 0 || f.seq > c.last_seq) return false;
  const int64_t horizon = now - cfg_.dedupe_window_s * 1000000000LL;
  for (auto it = c.ring.rbegin(); it != c.ring.rend(); ++it) {
    if ((*it)->created_mono < horizon) break;
    if ((*it)->seq == f.seq) return true;
  }
  return false;
}

int Bus::deliver(const FramePtr& f, std::vector<SinkPtr>* flush_list) {
  std::shared_ptr<const SubList> subs;
  {
    Shard& sh = shard(f->conversation_id);
    std::lock_guard<std::mutex> g(sh.mu);
    auto [it, inserted] = sh.convs.try_emplace(f->conversation_id);
    if (inserted) n_convs_.fetch_add(1);
    Conv& c = it->second;
    if (!inserted && duplicate_locked(c, *f, f->created_mono)) {
      metrics().bus_duplicates_dropped_total.inc();
      return 0;
    }
    c.ring.push_back(f);
    while (c.ring.size() > cfg_.replay_max) c.ring.pop_front();
    c.last_seq = std::max(c.last_seq, f->seq);
    if (f->done && !c.done) {
      c.done = true;
      c.done_seq = f->seq;
      c.done_ns = now_ns();
      c.done_ts = f->timestamp;
      c.done_mono = f->created_mono;
    }
    subs = c.subs;  // a reference to the current (immutable) list; pushes happen outside the shard lock
  }
  int n = 0;
  if (subs) {
    for (const auto& s : *subs) {
      if (!s->push(f)) metrics().bus_backpressure_events_total.inc();
      if (flush_list) flush_list->push_back(s);
      else s->flush();
      ++n;
    }
  }
  if (have_taps_.load(std::memory_order_relaxed)) {
    std::vector<SinkPtr> taps;
    {
      std::lock_guard<std::mutex> g(taps_mu_);
      taps = taps_;
    }
    for (const auto& s : taps) {
      s->push(f);
      if (flush_list) flush_list->push_back(s);
      else s->flush();
    }
  }
  metrics().bus_published_total.inc();
  return n;
}

int Bus::publish(const TokenMessage& m) { return publish(make_frame(m)); }

int Bus::publish(const FramePtr& f) {
  if (have_gate_.load(std::memory_order_relaxed)) {
    std::shared_ptr<FrameGate> g;
    {
      std::lock_guard<std::mutex> lk(gate_mu_);
      g = gate_;
    }
    if (g && g->admit(f)) return 0;
  }
  return deliver(f, nullptr);
}

void Bus::flush_all(std::vector<SinkPtr>& flush) {
  if (flush.size() == 1) {
    flush[0]->flush();
    return;
  }
  std::unordered_set<Sink*> seen;
  for (const auto& s : flush)
    if (seen.insert(s.get()).second) s->flush();
}

void Bus::publish_batch(const std::vector<FramePtr>& frames) {
  std::shared_ptr<FrameGate> g;
  if (have_gate_.load(std::memory_order_relaxed)) {
    std::lock_guard<std::mutex> lk(gate_mu_);
    g = gate_;
  }
  std::vector<SinkPtr> flush;
  flush.reserve(frames.size());
  for (const auto& f : frames)
    if (!(g && g->admit(f))) deliver(f, &flush);
  if (!flush.empty()) flush_all(flush);
}

void Bus::deliver_gated(const std::vector<FramePtr>& frames) {
  std::vector<SinkPtr> flush;
  flush.reserve(frames.size());
  for (const auto& f : frames) deliver(f, &flush);
  if (!flush.empty()) flush_all(flush);
}

bool Bus::terminate(const std::string& id, const std::string& token, uint8_t finish) {
  std::shared_ptr<const SubList> subs;
  FramePtr f;
  {
    Shard& sh = shard(id);
    std::lock_guard<std::mutex> g(sh.mu);
    auto [it, inserted] = sh.convs.try_emplace(id);
    if (inserted) n_convs_.fetch_add(1);
    Conv& c = it->second;
    if (c.done) return false;
    TokenMessage m{id, token, c.last_seq + 1, true, now_ns()};
    m.finish = finish;
    f = make_frame(m);
    c.ring.push_back(f);
    while (c.ring.size() > cfg_.replay_max) c.ring.pop_front();
    c.last_seq = f->seq;
    c.done = true;
    c.done_seq = f->seq;
    c.done_ns = now_ns();
    subs = c.subs;
  }
  std::vector<SinkPtr> flush;
  if (subs)
    for (const auto& s : *subs) {
      s->push(f);
      flush.push_back(s);
    }
  if (have_taps_.load(std::memory_order_relaxed)) {
    std::lock_guard<std::mutex> g(taps_mu_);
    for (const auto& s : taps_) {
      s->push(f);
      flush.push_back(s);
    }
  }
  if (!flush.empty()) flush_all(flush);
  metrics().bus_published_total.inc();
  return true;
}

size_t Bus::subscriber_count(const std::string& id) {
  Shard& sh = shard(id);
  std::lock_guard<std::mutex> g(sh.mu);
  auto it = sh.convs.find(id);
  return (it == sh.convs.end() || !it->second.subs) ? 0 : it->second.subs->size();
}

bool Bus::conversation_done(const std::string& id) {
  Shard& sh = shard(id);
  std::lock_guard<std::mutex> g(sh.mu);
  auto it = sh.convs.find(id);
  return it != sh.convs.end() && it->second.done;
}

int64_t Bus::last_sequence(const std::string& id) {
  Shard& sh = shard(id);
  std::lock_guard<std::mutex> g(sh.mu);
  auto it = sh.convs.find(id);
  return it == sh.convs.end() ? 0 : it->second.last_seq;
}

size_t Bus::gc(int64_t now_ns) {
  size_t removed = 0;
  const int64_t horizon = cfg_.retention_s * 1000000000LL;
  for (auto& shp : shards_) {
    std::lock_guard<std::mutex> g(shp->mu);
    for (auto it = shp->convs.begin(); it != shp->convs.end();) {
      const Conv& c = it->second;
      const bool no_subs = !c.subs || c.subs->empty();
      const bool expired = c.done && no_subs && now_ns - c.done_ns > horizon;
      const bool empty_idle = !c.done && no_subs && c.ring.empty();
      if (expired || empty_idle) {
        it = shp->convs.erase(it);
        ++removed;
      } else {
        ++it;
      }
    }
  }
  n_convs_.fetch_sub(removed);
  metrics().bus_conversations.set((double)n_convs_.load());
  return removed;
}

}  // namespace dsse
