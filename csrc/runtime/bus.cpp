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
  f->json.reserve(112 + m.conversation_id.size() + m.token.size());
  encode_token_message(f->json, m);
  char head[48];
  const int n = snprintf(head, sizeof head, "event: token\nid: %lld\ndata: ", (long long)m.sequence);
  f->bytes.reserve(n + f->json.size() + 2);
  f->bytes.append(head, n);
  f->bytes += f->json;
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
  c.subs.push_back(s);
}

void Bus::unsubscribe(const std::string& id, const SinkPtr& s) {
  Shard& sh = shard(id);
  std::lock_guard<std::mutex> g(sh.mu);
  auto it = sh.convs.find(id);
  if (it == sh.convs.end()) return;
  auto& v = it->second.subs;
  v.erase(std::remove(v.begin(), v.end(), s), v.end());
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

int Bus::deliver(const FramePtr& f, std::vector<SinkPtr>* flush_list) {
  int n = 0;
  std::vector<SinkPtr> subs;
  {
    Shard& sh = shard(f->conversation_id);
    std::lock_guard<std::mutex> g(sh.mu);
    auto [it, inserted] = sh.convs.try_emplace(f->conversation_id);
    if (inserted) n_convs_.fetch_add(1);
    Conv& c = it->second;
    c.ring.push_back(f);
    while (c.ring.size() > cfg_.replay_max) c.ring.pop_front();
    c.last_seq = std::max(c.last_seq, f->seq);
    if (f->done) {
      c.done = true;
      c.done_ns = now_ns();
    }
    subs = c.subs;  // snapshot; pushes happen outside the shard lock
  }
  for (const auto& s : subs) {
    if (!s->push(f)) metrics().bus_backpressure_events_total.inc();
    if (flush_list) flush_list->push_back(s);
    else s->flush();
    ++n;
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

int Bus::publish(const FramePtr& f) { return deliver(f, nullptr); }

void Bus::publish_batch(const std::vector<FramePtr>& frames) {
  std::vector<SinkPtr> flush;
  flush.reserve(frames.size());
  for (const auto& f : frames) deliver(f, &flush);
  std::unordered_set<Sink*> seen;
  for (const auto& s : flush)
    if (seen.insert(s.get()).second) s->flush();
}

size_t Bus::subscriber_count(const std::string& id) {
  Shard& sh = shard(id);
  std::lock_guard<std::mutex> g(sh.mu);
  auto it = sh.convs.find(id);
  return it == sh.convs.end() ? 0 : it->second.subs.size();
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
      const bool expired = c.done && c.subs.empty() && now_ns - c.done_ns > horizon;
      const bool empty_idle = !c.done && c.subs.empty() && c.ring.empty();
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
