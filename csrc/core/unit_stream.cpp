// Native per-unit protocol of a cyclic consumer (see ogkm/unit_stream.hpp).
#include "ogkm/unit_stream.hpp"

#include <algorithm>

#include "ogkm/arena.hpp"
#include "ogkm/config.hpp"
#include "ogkm/runtime.hpp"

namespace ogkm {

// Live streams, for Runtime::shutdown (detach_all).
static std::mutex g_streams_m;
static std::vector<UnitStream*> g_streams;

void UnitStream::detach_all(Runtime* rt) {
  std::lock_guard<std::mutex> g(g_streams_m);
  for (UnitStream* u : g_streams)
    if (u->rt_ == rt) u->detach(true);
}

// at_shutdown: the consumer's stream may be gone already (the runtime drains
// the device itself), so the leases go back without a stream fence.
void UnitStream::detach(bool at_shutdown) {
  if (!rt_) return;
  rt_->remove_pressure_handler(pressure_id_);
  std::lock_guard<std::recursive_mutex> g(m_);
  if (at_shutdown) {
    hold_on_stream_ = false;
    hold_stream_ = nullptr;
  }
  drop_holds(hold_stream_);
  for (Lease* l : pending_) (void)rt_->release(l, nullptr);
  pending_.clear();
  for (auto& f : ahead_) (void)f->wait();
  ahead_.clear();
  inflight_.clear();
  inflight_bytes_ = 0;
  rt_ = nullptr;
}

UnitStream::UnitStream(Runtime* rt, int dev, std::vector<Range*> ranges, uint64_t window_bytes, bool next_use,
                       uint32_t max_ahead)
    : rt_(rt), dev_(dev), ranges_(std::move(ranges)), window_(window_bytes), next_use_(next_use),
      max_ahead_(max_ahead) {
  for (uint32_t i = 0; i < ranges_.size(); ++i) pos_of_.emplace(ranges_[i], i);
  // Held leases are soft pins: an allocation that finds nothing else to evict
  // gets them back (from any thread; the owner's own acquire re-enters).
  pressure_id_ = rt_->add_pressure_handler(dev_, [this] {
    pressure_calls_.fetch_add(1, std::memory_order_relaxed);
    std::unique_lock<std::recursive_mutex> g(m_, std::try_to_lock);
    if (!g.owns_lock()) {  // the owner is mid-use on another thread: it drops them next
      drop_requested_.store(true);
      return false;
    }
    bool any = false;
    for (Lease* l : held_) any |= l != nullptr;
    drop_holds(hold_stream_);
    return any;
  });
  std::lock_guard<std::mutex> g(g_streams_m);
  g_streams.push_back(this);
}

UnitStream::~UnitStream() {
  std::lock_guard<std::mutex> g(g_streams_m);
  detach(false);
  g_streams.erase(std::remove(g_streams.begin(), g_streams.end(), this), g_streams.end());
}

uint64_t UnitStream::due(uint32_t pos) const {
  const uint64_t n = ranges_.size();
  return (pass_ + ((int64_t)pos <= last_pos_ ? 1 : 0)) * n + pos;
}

void UnitStream::prefetch_window() {
  std::lock_guard<std::recursive_mutex> g(m_);
  if (!rt_) return;
  const uint32_t n = (uint32_t)ranges_.size();
  const Loc gpu = Loc::gpu(dev_);
  while (inflight_.size() < n) {
    Range* r = ranges_[pf_next_];
    const uint64_t nb = r->size;
    if (!inflight_.empty() && inflight_bytes_ + nb > window_) break;
    const uint64_t t0 = now_ns();
    Tracker t;
    Status st;
    {
      // next-use mode: evict only data needed after this unit's own use
      VictimFloor vf(next_use_ ? due(pf_next_) : 0);
      st = rt_->prefetch(r, 0, r->size, gpu, &t, Cause::Prefetch);
    }
    st_.prefetch_ns += now_ns() - t0;
    if (st != Status::OK) {
      // refused by the floor (no victim needed later than it): left to its use
      ++st_.refused;
      pressure_ = true;
      pass_quiet_ = false;
      break;
    }
    inflight_.push_back(pf_next_);
    inflight_bytes_ += nb;
    ++st_.prefetched;
    pf_next_ = (pf_next_ + 1) % n;
  }
}

Status UnitStream::use(uint32_t pos, void* stream, Lease** out, bool on_stream) {
  if (pos >= ranges_.size()) return Status::INVALID_ARGUMENT;
  std::lock_guard<std::recursive_mutex> g(m_);
  if (!rt_) return Status::NOT_SUPPORTED;  // detached: the runtime was shut down
  if (drop_requested_.exchange(false)) drop_holds(stream);
  struct Clock {
    uint64_t& acc;
    uint64_t t0 = now_ns();
    ~Clock() { acc += now_ns() - t0; }
  } clock{st_.use_ns};
  const uint64_t n = ranges_.size();
  Range* r = ranges_[pos];
  const bool new_pass = (int64_t)pos <= cur_pos_;
  cur_pos_ = pos;
  if (new_pass) update_hold(stream);
  if (hold_ && !held_.empty() && held_[pos]) {
    // Held since its last use (no memory pressure): the same lease again - its
    // chunks stayed pinned and the stream already waited for them.
    if (hold_arena_ && hold_arena_->evictions() != hold_ev_) {
      drop_holds(stream);  // someone needed HBM meanwhile: back to leases per use
    } else if (r->mod_gen.load(std::memory_order_acquire) != held_gen_[pos]) {
      // written or migrated since it was kept: the held copy may be stale or
      // revoked - hand it back and lease the unit afresh (below)
      FenceRef f = hold_on_stream_ ? fence_record(rt_->be(), dev_, stream) : nullptr;
      (void)rt_->release(held_[pos], stream, f);
      held_[pos] = nullptr;
      ++st_.hold_drops;
    } else {
      if (next_use_) {
        if ((int64_t)pos <= last_pos_) ++pass_;
        last_pos_ = pos;
      }
      *out = held_[pos];
      held_[pos] = nullptr;
      ++st_.held;
      return Status::OK;
    }
  }
  if (!inflight_.empty() && inflight_.front() == pos) {
    inflight_.pop_front();
    inflight_bytes_ -= r->size;
  } else {
    // not in the window: a use out of the prefetch order (not by itself
    // pressure - a resident unit faults in for free; evictions tell)
    ++st_.demand;
    pressure_ = true;
  }
  if (next_use_) {  // the op clock moves to this use
    if ((int64_t)pos <= last_pos_) ++pass_;
    last_pos_ = pos;
    rt_->set_op_clock(dev_, pass_ * n + pos);
  }
  prefetch_window();
  const uint64_t t0 = now_ns();
  Status st = rt_->acquire(r, 0, r->size, dev_, Access::READ, out);
  st_.acquire_ns += now_ns() - t0;
  if (st != Status::OK) return st;
  // hinted once leased (before, the prefetches queued for this use would see it
  // as the furthest-needed unit and evict it): next used one pass later
  const uint64_t t1 = now_ns();
  if (next_use_) rt_->hint_next_use(*out, pass_ * n + pos + n);
  const uint64_t t2 = now_ns();
  st_.hint_ns += t2 - t1;
  // the consumer's stream waits GPU-side (no stream: the host waits)
  st = on_stream ? (*out)->ready.gpu_wait(rt_->be(), stream) : (*out)->ready.wait();
  st_.wait_ns += now_ns() - t2;
  if (st != Status::OK) {
    (void)rt_->release(*out, on_stream ? stream : nullptr);
    *out = nullptr;
  }
  return st;
}

Status UnitStream::release(Lease* l, void* stream, bool on_stream) {
  std::lock_guard<std::recursive_mutex> g(m_);
  if (!rt_) return Status::NOT_SUPPORTED;
  if (!on_stream || l->proc == kCpuProc) return rt_->release(l, nullptr);
  if (hold_ && l->offset == 0 && l->bytes == l->range->size) {
    auto it = pos_of_.find(l->range);
    if (it != pos_of_.end() && it->second < held_.size() && !held_[it->second]) {
      held_[it->second] = l;  // kept until its next use (or until pressure)
      held_gen_[it->second] = l->range->mod_gen.load(std::memory_order_acquire);
      hold_stream_ = stream;
      hold_on_stream_ = true;
      return Status::OK;
    }
  }
  // Released units are handed back in groups of unit_release_batch behind ONE
  // event recorded after the group's kernels: it is the runtime's reuse fence
  // of their chunks and the run-ahead bound below (every event record is a
  // barrier + release packet on the consumer's stream). A group closes early
  // when this use had to stream (a prefetch was refused or the unit faulted on
  // demand): then the chunks are needed back as victims right away.
  pending_.push_back(l);
  const uint32_t batch = (uint32_t)std::max<int64_t>(1, config().unit_release_batch);
  if (pending_.size() < batch && !pressure_) return Status::OK;
  return flush_released(stream);
}

Status UnitStream::flush_released(void* stream) {
  std::lock_guard<std::recursive_mutex> g(m_);
  if (!rt_) return Status::NOT_SUPPORTED;
  if (pending_.empty()) return Status::OK;
  FenceRef f = fence_record(rt_->be(), dev_, stream);
  Status st = Status::OK;
  for (Lease* x : pending_) {
    Status s = rt_->release(x, stream, f);
    if (st == Status::OK) st = s;
  }
  pending_.clear();
  pressure_ = false;
  if (!max_ahead_ || !f || !f->event) return st;
  // Bounded run-ahead: leases wait GPU-side, so without a bound the host would
  // prefetch a whole step ahead and the ring would evict (and wait on) chunks
  // whose readers are still queued - the copies then serialise behind compute.
  ahead_.push_back(std::move(f));
  const uint32_t batch = (uint32_t)std::max<int64_t>(1, config().unit_release_batch);
  const size_t keep = std::max<size_t>(1, (max_ahead_ + batch - 1) / batch);
  while (ahead_.size() > keep) {
    const uint64_t t0 = now_ns();
    (void)ahead_.front()->wait();
    st_.ahead_wait_ns += now_ns() - t0;
    ahead_.pop_front();
  }
  return st;
}

// Hold mode (config unit_hold): after a whole pass in which the arena evicted
// nothing and no use streamed (every unit resident - e.g. a model that fits),
// released units keep their leases until their next use: a use is then a
// lookup instead of a lease (pins, LRU touches, readiness, hints) and a release
// is no event record - the host cost of a resident decode step is what the
// static plan has. The first eviction the arena reports (another allocation
// needs HBM), a refused prefetch or a demand fault ends it: every held lease
// is released behind one fence and the next pass decides again.
void UnitStream::update_hold(void* stream) {
  ChunkArena* a = rt_->arena_for(Loc::gpu(dev_));
  const uint64_t ev = a ? a->evictions() : 0;
  const bool quiet = config().unit_hold && a && pass_quiet_ && ev == pass_ev0_;
  if (quiet) ++st_.quiet_passes;
  else if (!pass_quiet_) ++st_.loud_streaming;
  else if (ev != pass_ev0_) ++st_.loud_evictions;
  if (!quiet && hold_) drop_holds(stream);
  hold_ = quiet;
  hold_arena_ = a;
  hold_ev_ = ev;
  if (hold_ && held_.size() != ranges_.size()) {
    held_.assign(ranges_.size(), nullptr);
    held_gen_.assign(ranges_.size(), 0);
  }
  pass_ev0_ = ev;
  pass_quiet_ = true;
}

void UnitStream::drop_holds(void* stream) {
  hold_ = false;
  pass_quiet_ = false;
  bool any = false;
  for (Lease* l : held_) any |= l != nullptr;
  if (!any) return;
  FenceRef f = hold_on_stream_ ? fence_record(rt_->be(), dev_, stream) : nullptr;
  for (Lease*& l : held_)
    if (l) {
      (void)rt_->release(l, stream, f);
      l = nullptr;
    }
  ++st_.hold_drops;
}

}  // namespace ogkm
