// Runtime-decided keep / stream classes (see ogkm/spread.hpp).
#include "ogkm/spread.hpp"

#include <algorithm>

#include "ogkm/arena.hpp"
#include "ogkm/config.hpp"

namespace ogkm {

// Error diffusion over the use order: each range adds f x its bytes to the
// accumulator and is kept when the accumulator covers it - the keep class is
// f of the cycle's bytes, spread evenly over the cycle (a run of stream-class
// units is never longer than ~1/f units), like the static plan's evenly
// spread resident layers.
void SpreadPolicy::assign_locked(const std::function<ArenaView()>& view_fn) {
  const ArenaView view = view_fn();
  const double pct = std::clamp<double>((double)config().perf_spread_keep_pct, 0.0, 100.0) / 100.0;
  const uint64_t held = view.pinned + reserve_;
  const uint64_t usable = view.capacity > held ? view.capacity - held : 0;
  f_ = cycle_bytes_ ? std::min(1.0, pct * scale_ * (double)usable / (double)cycle_bytes_) : 1.0;
  acc_ = 0.0;
  for (uint64_t id : order_) {
    Entry& e = ranges_[id];
    const double nb = (double)e.bytes;
    acc_ += nb * f_;
    const bool keep = acc_ >= nb;
    if (keep) acc_ -= nb;
    e.cls = keep ? 0 : 1;
  }
  assigned_bytes_ = cycle_bytes_;
  assigned_reserve_ = reserve_;
  // Chunks keep the class flag of their last hint until their next use: the
  // pass after a (re)assignment moves data between the classes - its keep-class
  // evictions are the transition, not a sign the keep class does not fit.
  grace_until_ = passes_ + 3;
}

uint64_t SpreadPolicy::on_hint(uint64_t id, uint64_t bytes, const std::function<ArenaView()>& view) {
  std::lock_guard<std::mutex> g(m_);
  auto pit = pending_.find(id);
  if (pit != pending_.end()) {  // its use: it leaves the prefetch window
    pending_bytes_ -= pit->second.first;
    pending_.erase(pit);
  }
  max_range_bytes_ = std::max(max_range_bytes_, bytes);
  auto it = ranges_.find(id);
  if (it == ranges_.end()) {
    Entry e;
    e.bytes = bytes;
    e.order = (uint32_t)order_.size();
    it = ranges_.emplace(id, e).first;
    order_.push_back(id);
    cycle_bytes_ += bytes;
    // While the cycle is being discovered, re-diffuse whenever it grew 5 %
    // past the last assignment (a handful of times over the first pass).
    if (cycle_bytes_ > assigned_bytes_ + assigned_bytes_ / 20) assign_locked(view);
    else {  // appended to the current diffusion
      const double nb = (double)bytes;
      acc_ += nb * f_;
      const bool keep = acc_ >= nb;
      if (keep) acc_ -= nb;
      it->second.cls = keep ? 0 : 1;
    }
  } else if (it->second.order == 0) {
    // The first range of the cycle again: one pass done. Keep-class data
    // evicted during it means the keep class does not fit: shrink it.
    ++passes_;
    if (!ready_) {  // the first pass was the discovery: the whole cycle is known now
      ready_ = true;
      pass_keep_evictions_ = 0;
      assign_locked(view);  // exact cycle bytes (the interim assignments saw part of it)
    }
    const uint64_t keep_n = std::count_if(ranges_.begin(), ranges_.end(),
                                          [](const auto& kv) { return kv.second.cls == 0; });
    if (config().perf_spread_adapt && passes_ >= grace_until_ &&
        pass_keep_evictions_ > std::max<uint64_t>(1, keep_n / 50) && scale_ > 0.5) {
      scale_ *= 1.0 - (double)std::max<int64_t>(1, config().perf_spread_step_pct) / 100.0;
      ++adaptations_;
      assign_locked(view);
    }
    last_pass_keep_evictions_ = pass_keep_evictions_;
    pass_keep_evictions_ = 0;
    for (auto p = pending_.begin(); p != pending_.end();) {  // prefetched a pass ago, never used
      if (p->second.second + 1 < passes_) {
        pending_bytes_ -= p->second.first;
        p = pending_.erase(p);
      } else {
        ++p;
      }
    }
  }
  // The window grew past the reserve of the last assignment: re-diffuse.
  if (ready_ && reserve_ > assigned_reserve_ + max_range_bytes_) assign_locked(view);
  return it->second.cls == 1 ? kEvictFirst : 0;
}

void SpreadPolicy::on_prefetch(uint64_t id, uint64_t bytes) {
  std::lock_guard<std::mutex> g(m_);
  auto it = pending_.find(id);
  if (it == pending_.end()) {
    pending_.emplace(id, std::make_pair(bytes, passes_));
    pending_bytes_ += bytes;
  }
  max_range_bytes_ = std::max(max_range_bytes_, bytes);
  reserve_ = std::max(reserve_, pending_bytes_);  // (the unit about to be used is still pending)
}

void SpreadPolicy::on_evict(uint64_t id) {
  std::lock_guard<std::mutex> g(m_);
  auto it = ranges_.find(id);
  if (it != ranges_.end() && it->second.cls == 0) {
    ++keep_evictions_;
    ++pass_keep_evictions_;
  }
}

int SpreadPolicy::range_class(uint64_t id) {
  std::lock_guard<std::mutex> g(m_);
  auto it = ranges_.find(id);
  return it == ranges_.end() ? -1 : it->second.cls;
}

void SpreadPolicy::reset() {
  std::lock_guard<std::mutex> g(m_);
  ranges_.clear();
  order_.clear();
  cycle_bytes_ = assigned_bytes_ = 0;
  ready_ = false;
  f_ = 0.0;
  acc_ = 0.0;
  scale_ = 1.0;
  passes_ = keep_evictions_ = pass_keep_evictions_ = adaptations_ = 0;
  pending_.clear();
  pending_bytes_ = max_range_bytes_ = reserve_ = assigned_reserve_ = 0;
  grace_until_ = 0;
  last_pass_keep_evictions_ = 0;
}

SpreadPolicy::Stats SpreadPolicy::stats() {
  std::lock_guard<std::mutex> g(m_);
  Stats s;
  s.ready = ready_;
  s.ranges = ranges_.size();
  s.cycle_bytes = cycle_bytes_;
  for (auto& kv : ranges_)
    if (kv.second.cls == 0) {
      ++s.keep_ranges;
      s.keep_bytes += kv.second.bytes;
    }
  s.passes = passes_;
  s.keep_evictions = keep_evictions_;
  s.adaptations = adaptations_;
  s.keep_fraction = f_;
  s.window_reserve = reserve_;
  s.last_pass_keep_evictions = last_pass_keep_evictions_;
  return s;
}

}  // namespace ogkm
