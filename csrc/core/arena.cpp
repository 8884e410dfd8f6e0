// ChunkArena / HbmArena / HostArena implementation.
#include "ogkm/arena.hpp"
#include "ogkm/ledger.hpp"

#include <fcntl.h>
#include <numaif.h>
#include <sys/mman.h>
#include <unistd.h>

#include <algorithm>
#include <deque>
#include <sstream>

#include "ogkm/config.hpp"
#include "ogkm/events.hpp"
#include "ogkm/va_space.hpp"

namespace ogkm {

ChunkArena::ChunkArena(std::string name, Loc loc, LockOrder order) : name_(std::move(name)), loc_(loc), m_(order) {}
ChunkArena::~ChunkArena() = default;

void ChunkArena::init_chunks(uint64_t base, uint32_t n) {
  base_ = base;
  nchunks_ = n;
  chunks_.assign(n, ChunkInfo{});
  free_runs_.clear();
  if (n) free_runs_[0] = n;
  st_ = Stats{};
  st_.capacity = (uint64_t)n << kBlockShift;
  active_limit_ = (uint32_t)((uint64_t)n * (uint64_t)std::max<int64_t>(0, config().perf_workingset_active_pct) / 100);
}

int64_t ChunkArena::chunk_of(uint64_t addr) const {
  if (addr < base_ || addr >= base_ + ((uint64_t)nchunks_ << kBlockShift)) return -1;
  return (int64_t)((addr - base_) >> kBlockShift);
}

// ------------------------------------------------------------ free runs
void ChunkArena::take_run(uint32_t first, uint32_t n) {
  auto it = free_runs_.upper_bound(first);
  RT_ASSERT_RELEASE(it != free_runs_.begin());
  --it;
  uint32_t s = it->first, l = it->second;
  RT_ASSERT_RELEASE(s <= first && first + n <= s + l);
  free_runs_.erase(it);
  if (first > s) free_runs_[s] = first - s;
  if (first + n < s + l) free_runs_[first + n] = s + l - (first + n);
}

void ChunkArena::add_run(uint32_t first, uint32_t n) {
  uint32_t s = first, e = first + n;
  auto it = free_runs_.lower_bound(first);
  if (it != free_runs_.end() && it->first == e) {
    e += it->second;
    it = free_runs_.erase(it);
  }
  if (it != free_runs_.begin()) {
    auto pv = std::prev(it);
    if (pv->first + pv->second == s) {
      s = pv->first;
      free_runs_.erase(pv);
    }
  }
  free_runs_[s] = e - s;
}

// ------------------------------------------------------------ LRU lists
void ChunkArena::lru_remove(uint32_t i) {
  ChunkInfo& c = chunks_[i];
  if (!c.list) return;
  if (c.prev >= 0) chunks_[c.prev].next = c.next;
  else head_[c.list] = c.next;
  if (c.next >= 0) chunks_[c.next].prev = c.prev;
  else tail_[c.list] = c.prev;
  if (c.list == 1) st_.unused_list--;
  else st_.used_list--;
  c.prev = c.next = -1;
  c.list = 0;
}

void ChunkArena::lru_push_tail(uint32_t i, uint8_t list) {
  ChunkInfo& c = chunks_[i];
  c.list = list;
  c.prev = tail_[list];
  c.next = -1;
  if (tail_[list] >= 0) chunks_[tail_[list]].next = (int32_t)i;
  else head_[list] = (int32_t)i;
  tail_[list] = (int32_t)i;
  if (list == 1) st_.unused_list++;
  else st_.used_list++;
}

// ------------------------------------------------------------ allocation
Status ChunkArena::alloc(uint32_t n, Block* owner, int64_t hint, uint32_t* first, bool pin) {
  if (n == 0) return Status::INVALID_ARGUMENT;
  std::lock_guard<OrderedMutex> g(m_);
  int64_t pick = -1;
  // Honour the hint (keeps a range's blocks adjacent) when that window is free.
  if (hint >= 0 && hint + n <= nchunks_) {
    auto it = free_runs_.upper_bound((uint32_t)hint);
    if (it != free_runs_.begin()) {
      --it;
      if (it->first <= hint && hint + n <= (int64_t)it->first + it->second) pick = hint;
    }
  }
  if (pick < 0 && n == 1 && hint < 0) {
    // A single chunk: prefer one nobody is still using. A chunk freed a moment
    // ago usually still has a queued reader (the H2D fill that drained it); a
    // writer handed that chunk would wait for that copy - e.g. an eviction
    // copy-out serialised behind the previous fill. Idle chunks keep the two
    // copy directions overlapping.
    int scanned = 0;
    for (auto it = free_runs_.begin(); it != free_runs_.end() && scanned < 32 && pick < 0; ++it) {
      for (uint32_t k = 0; k < it->second && scanned < 32; ++k, ++scanned) {
        Tracker& t = chunks_[it->first + k].reuse_fence;
        if (t.query()) {
          pick = it->first + k;
          break;
        }
      }
    }
  }
  const int side = PlacementSide::value();
  if (pick < 0 && side == 1) {  // low end: first fit
    for (auto& r : free_runs_)
      if (r.second >= n) {
        pick = r.first;
        break;
      }
  } else if (pick < 0 && side == 2) {  // high end: the top n chunks of the highest run that fits
    for (auto it = free_runs_.rbegin(); it != free_runs_.rend(); ++it)
      if (it->second >= n) {
        pick = it->first + it->second - n;
        break;
      }
  }
  if (pick < 0) {
    // Best fit: smallest run that holds n chunks (limits fragmentation).
    uint32_t best = UINT32_MAX;
    for (auto& r : free_runs_)
      if (r.second >= n && r.second < best) {
        best = r.second;
        pick = r.first;
        if (best == n) break;
      }
  }
  if (pick < 0) return Status::NO_MEMORY;
  take_run((uint32_t)pick, n);
  for (uint32_t i = 0; i < n; ++i) {
    ChunkInfo& c = chunks_[pick + i];
    c.state = ChunkState::ALLOCATED;
    c.owner = owner;
    c.pin_count = pin ? 1 : 0;
    c.last_use = ++clock_;
    c.last_op = op_clock_;
    c.next_use = 0;
    lru_push_tail((uint32_t)pick + i, 1);
  }
  if (pin) st_.pinned += (uint64_t)n << kBlockShift;
  st_.allocated += (uint64_t)n << kBlockShift;
  st_.peak = std::max(st_.peak, st_.allocated);
  st_.allocs += n;
  *first = (uint32_t)pick;
  return Status::OK;
}

Status ChunkArena::reserve(uint32_t n, Reservation* r) {
  std::lock_guard<OrderedMutex> g(m_);
  if (n == 0 || n > nchunks_) return Status::NO_MEMORY;
  // Fast path: a free run.
  for (auto& fr : free_runs_)
    if (fr.second >= n) {
      r->first = fr.first;
      r->n = n;
      r->victims.clear();
      take_run(fr.first, n);
      for (uint32_t i = 0; i < n; ++i) chunks_[fr.first + i].state = ChunkState::RESERVED;
      st_.reservations++;
      return Status::OK;
    }
  if (n == 1) {
    int32_t best = pick_victim_locked();
    if (best < 0) return Status::NO_MEMORY;
    ChunkInfo& c = chunks_[best];
    lru_remove((uint32_t)best);
    c.state = ChunkState::EVICTING;
    r->first = best;
    r->n = 1;
    r->victims = {(uint32_t)best};
    r->list.clear();
    st_.reservations++;
    return Status::OK;
  }
  // Sliding window over [0, nchunks): every chunk must be FREE or evictable;
  // minimise the newest last_use in the window (evict the coldest data).
  int64_t best_first = -1;
  uint64_t best_cost = UINT64_MAX;
  std::deque<uint32_t> dq;  // monotone deque of last_use maxima
  uint32_t start = 0;
  // Cost of evicting a chunk: 0 if free, its recency otherwise; chunks on the
  // preferred list cost more than any ordinary chunk.
  const uint64_t floor = hinted_ ? VictimFloor::value() : 0;
  auto cost_of = [&](uint32_t i) -> uint64_t {
    const ChunkInfo& c = chunks_[i];
    if (c.state == ChunkState::FREE) return 0;
    if (hinted_) return ~victim_key_locked(c);  // a window of the furthest-needed data
    return c.last_use + (c.list == 3 ? (1ull << 62) : 0) + (c.active ? (1ull << 61) : 0);
  };
  // Costs first (one key per chunk; UINT64_MAX = not evictable), then the
  // monotone-deque window pass over the array.
  static thread_local std::vector<uint64_t> costs;
  costs.resize(nchunks_);
  for (uint32_t i = 0; i < nchunks_; ++i) {
    const ChunkInfo& c = chunks_[i];
    const bool ok = c.state == ChunkState::FREE ||
                    (c.state == ChunkState::ALLOCATED && c.pin_count == 0 && !floor_protects_locked(c, floor));
    costs[i] = ok ? cost_of(i) : UINT64_MAX;
  }
  for (uint32_t i = 0; i < nchunks_; ++i) {
    const uint64_t cost = costs[i];
    if (cost == UINT64_MAX) {
      start = i + 1;
      dq.clear();
      continue;
    }
    while (!dq.empty() && costs[dq.back()] <= cost) dq.pop_back();
    dq.push_back(i);
    if (i + 1 - start > n) {
      start = i + 1 - n;
      while (!dq.empty() && dq.front() < start) dq.pop_front();
    }
    if (i + 1 - start == n) {
      const uint64_t wcost = costs[dq.front()];
      if (wcost < best_cost || (wcost == best_cost && PlacementSide::value() == 2)) {  // (high end: the last tie)
        best_cost = wcost;
        best_first = start;
      }
    }
  }
  if (best_first < 0) return Status::NO_MEMORY;
  r->first = best_first;
  r->n = n;
  r->victims.clear();
  for (uint32_t i = 0; i < n; ++i) {
    uint32_t k = (uint32_t)best_first + i;
    ChunkInfo& c = chunks_[k];
    if (c.state == ChunkState::FREE) {
      take_run(k, 1);
      c.state = ChunkState::RESERVED;
    } else {
      lru_remove(k);
      c.state = ChunkState::EVICTING;
      r->victims.push_back(k);
    }
  }
  st_.reservations++;
  return Status::OK;
}

// Victim order: unused list head, then used LRU head (uvm_pmm_gpu.c:1460-1500),
// then chunks whose data prefers this tier.
// Within a list, the oldest few candidates compete on recency (prefetched
// chunks carry a recency bonus and lose to genuinely cold data).
// Workingset-protected (active) chunks go only when nothing inactive is left.
int32_t ChunkArena::pick_victim_locked() {
  if (hinted_) {
    std::vector<uint32_t> v;
    pick_victims_by_next_use_locked(1, &v);
    return v.empty() ? -1 : (int32_t)v[0];
  }
  for (int pass = 0; pass < 6; ++pass) {
    const int list = 1 + pass % 3;
    const bool allow_active = pass >= 3;
    int32_t best = -1;
    int scanned = 0;
    for (int32_t i = head_[list]; i >= 0 && scanned < 64; i = chunks_[i].next) {
      ChunkInfo& c = chunks_[i];
      if (c.state != ChunkState::ALLOCATED || c.pin_count != 0 || (c.active && !allow_active)) continue;
      ++scanned;
      if (best < 0 || c.last_use < chunks_[best].last_use) best = i;
    }
    if (best >= 0) return best;
  }
  return -1;
}

int& PlacementSide::value() {
  static thread_local int side = 0;
  return side;
}

uint64_t& VictimFloor::value() {
  static thread_local uint64_t floor = 0;
  return floor;
}

void ChunkArena::set_next_use_many(const uint32_t* idx, size_t n, uint64_t when) {
  std::lock_guard<OrderedMutex> g(m_);
  for (size_t k = 0; k < n; ++k) set_next_use_locked(idx[k], when);
}

void ChunkArena::set_next_use(uint32_t i, uint64_t when) {
  std::lock_guard<OrderedMutex> g(m_);
  set_next_use_locked(i, when);
}

void ChunkArena::set_next_use_locked(uint32_t i, uint64_t when) {
  if (i >= nchunks_ || chunks_[i].state != ChunkState::ALLOCATED) return;
  const bool track = vcache_valid_ && hinted_ && config().arena_victim_rerank;
  const uint64_t before = track ? victim_key_locked(chunks_[i]) : 0;
  chunks_[i].next_use = when;
  if (when && when != kDeadUse) hinted_ = true;
  // A new hint that raises the chunk's rank (data just used gets a far next
  // use, or the evict-first class) puts it past where the victim cache has
  // it: remember it, next_victims_locked ranks these ahead of the cache's
  // stale order. (Many at once - a whole op trace re-hinting - rebuild the
  // cache instead of sorting a long list on every victim query.)
  if (track && victim_key_locked(chunks_[i]) > before) {
    if (vrisen_.size() >= 256) {
      vcache_valid_ = false;
      vrisen_.clear();
    } else {
      vrisen_.push_back(i);
    }
  }
}

void ChunkArena::set_op_clock(uint64_t now) {
  std::lock_guard<OrderedMutex> g(m_);
  op_clock_ = std::max(op_clock_, now);
}

void ChunkArena::reset_op_clock() {
  std::lock_guard<OrderedMutex> g(m_);
  op_clock_ = 0;
  hinted_ = false;
  vcache_.clear();
  vcache_pos_ = 0;
  vcache_clock_ = 0;
  vcache_valid_ = false;
  vrisen_.clear();
  for (uint32_t i = 0; i < nchunks_; ++i) {
    ChunkInfo& c = chunks_[i];
    if (c.next_use != kDeadUse) c.next_use = 0;
    c.last_op = 0;
  }
}

// Larger = evicted sooner: dead data, then unhinted data by age, then hinted
// data by the distance to its next use. Unhinted data touched within the last
// two ops (an activation between its producer and consumer) ranks as needed
// next. Hints in the past (the trace moved on without a use) count as unknown.
uint64_t ChunkArena::base_key_locked(const ChunkInfo& c) const {
  if (c.next_use == kDeadUse) {
    // Freed data: nothing to copy out - but kernels queued before the free may
    // still read it, and a freed torch tensor is usually re-allocated (same
    // size, same stable VA) within a few ops: evicting it then costs a remap
    // that waits for those readers. Recently used dead data ranks as just used.
    const int64_t dc = config().arena_dead_cooldown;
    if (dc > 0 && c.last_op && op_clock_ >= c.last_op && op_clock_ - c.last_op < (uint64_t)dc) return 1;
    return kDeadUse;
  }
  // Just used: its readers may still be queued, so a copy into the chunk would
  // wait for them (the reuse fence) and the link would idle behind compute -
  // keep it for arena_reuse_cooldown op-clock steps (it is next needed a whole
  // pass later: evicting the data used a few steps earlier costs the same).
  const int64_t cool = config().arena_reuse_cooldown;
  if (cool > 0 && c.last_op && op_clock_ >= c.last_op && op_clock_ - c.last_op < (uint64_t)cool) return 1;
  const uint64_t nu = c.next_use & ~kEvictFirst;
  if (nu >= op_clock_) return nu - op_clock_;  // due now: 0, the last to go
  if (op_clock_ - c.last_op <= 2) return 1;
  return (1ull << 62) + (clock_ - std::min(clock_, c.last_use));
}

// Ranking key: the base key, hinted data flagged kEvictFirst (the "stream"
// class of a spread plan) ahead of every unflagged hinted chunk.
uint64_t ChunkArena::victim_key_locked(const ChunkInfo& c) const {
  const uint64_t k = base_key_locked(c);
  const bool first = c.next_use != kDeadUse && (c.next_use & kEvictFirst);
  return first && k < kEvictFirst ? k + kEvictFirst : k;
}

// The floor is an op-clock time: data whose next use comes no later is kept.
bool ChunkArena::floor_protects_locked(const ChunkInfo& c, uint64_t floor) const {
  if (!floor || !hinted_) return false;
  const uint64_t k = base_key_locked(c);  // the true next use, not the class bonus
  return k < (1ull << 62) && k + op_clock_ <= floor;
}

void ChunkArena::next_victims_locked(uint32_t want, uint64_t floor, std::vector<std::pair<uint64_t, uint32_t>>* out) {
  out->clear();
  if (!want) return;
  struct Clock {  // host cost of the victim search (stats victim_search_ns)
    uint64_t t0 = now_ns();
    ~Clock() { Tools::get().inc(Counter::VictimSearchNs, now_ns() - t0); }
  } clock;
  Tools::get().inc(Counter::VictimRisenSeen, vrisen_.size());
  const int64_t every = config().arena_victim_cache_ops;
  for (int pass = 0; pass < 2 && out->size() < want; ++pass) {
    const bool stale = !vcache_valid_ || vcache_pos_ >= vcache_.size() || every <= 0 ||
                       op_clock_ < vcache_clock_ || op_clock_ - vcache_clock_ > (uint64_t)every;
    if (pass == 1 || stale) {  // full scan: every evictable chunk, best first
      vcache_.clear();
      vrisen_.clear();
      for (uint32_t i = 0; i < nchunks_; ++i) {
        const ChunkInfo& c = chunks_[i];
        if (c.state != ChunkState::ALLOCATED || c.pin_count != 0) continue;
        vcache_.emplace_back(victim_key_locked(c), i);
      }
      auto better = [](const std::pair<uint64_t, uint32_t>& a, const std::pair<uint64_t, uint32_t>& b) {
        return a.first > b.first || (a.first == b.first && a.second < b.second);
      };
      // A periodic rebuild ranks only the best few thousand (a selection, then
      // a sort of those - the full sort of a 100+ GB arena's chunks on every
      // rebuild was most of a long-context step's prefetch time); the
      // fallback pass ranks everything, so no victim is ever missed.
      const int64_t rank_top = config().arena_victim_rank_top;
      const size_t top = pass == 0 && rank_top > 0 ? std::max<size_t>((size_t)rank_top, 8 * (size_t)want)
                                                   : vcache_.size();
      if (top < vcache_.size()) {
        std::nth_element(vcache_.begin(), vcache_.begin() + top, vcache_.end(), better);
        vcache_.resize(top);
      }
      std::sort(vcache_.begin(), vcache_.end(), better);
      vcache_pos_ = 0;
      vcache_clock_ = op_clock_;
      vcache_valid_ = true;
      out->clear();
    }
    const uint64_t shift = op_clock_ - vcache_clock_;  // every hinted key fell by this much since the build
    // Chunks re-hinted since the build, ranked now: those that outrank the
    // cache's current front go first.
    size_t nrisen = 0;
    if (!vrisen_.empty()) {
      std::vector<std::pair<uint64_t, uint32_t>> risen;
      for (uint32_t i : vrisen_) {
        const ChunkInfo& c = chunks_[i];
        if (c.state != ChunkState::ALLOCATED || c.pin_count != 0) continue;
        risen.emplace_back(victim_key_locked(c), i);
      }
      std::sort(risen.begin(), risen.end(), [](const auto& a, const auto& b) {
        return a.first > b.first || (a.first == b.first && a.second < b.second);
      });
      risen.erase(std::unique(risen.begin(), risen.end()), risen.end());
      uint64_t front_key = 0;  // the best cache entry still valid (the same test as the scan below)
      for (size_t k = vcache_pos_; k < vcache_.size(); ++k) {
        const ChunkInfo& c = chunks_[vcache_[k].second];
        const uint64_t key = victim_key_locked(c);
        const bool gone = c.state != ChunkState::ALLOCATED || c.pin_count != 0 ||
                          (key < (1ull << 62) && key + shift < vcache_[k].first && vcache_[k].first < (1ull << 62));
        if (!gone) {
          front_key = key;
          break;
        }
      }
      for (auto& e : risen) {
        if (out->size() >= want || e.first < front_key) break;
        if (floor_protects_locked(chunks_[e.second], floor)) continue;
        out->push_back(e);
      }
      nrisen = out->size();
    }
    auto taken = [&](uint32_t i) {
      for (size_t k = 0; k < nrisen; ++k)
        if ((*out)[k].second == i) return true;
      return false;
    };
    bool front = true;
    for (size_t k = vcache_pos_; k < vcache_.size() && out->size() < want; ++k) {
      if (nrisen && taken(vcache_[k].second)) continue;
      const ChunkInfo& c = chunks_[vcache_[k].second];
      const uint64_t key = victim_key_locked(c);
      const bool gone = c.state != ChunkState::ALLOCATED || c.pin_count != 0 ||
                        (key < (1ull << 62) && key + shift < vcache_[k].first && vcache_[k].first < (1ull << 62));
      if (gone) {
        if (front) vcache_pos_ = k + 1;  // never a candidate again before the next build
        continue;
      }
      front = false;
      if (floor_protects_locked(c, floor)) continue;
      out->emplace_back(key, vcache_[k].second);
    }
  }
}

void ChunkArena::pick_victims_by_next_use_locked(uint32_t n, std::vector<uint32_t>* out) {
  const uint64_t floor = VictimFloor::value();
  std::vector<std::pair<uint64_t, uint32_t>> cand;
  next_victims_locked(n, floor, &cand);
  static const bool dbg = getenv("OGKM_DEBUG_VICTIMS") != nullptr;
  static const bool dbg2 = getenv("OGKM_DEBUG_VICTIMS_ALL") != nullptr;
  if (dbg2) {
    for (uint32_t i = 0; i < nchunks_; ++i) {
      const ChunkInfo& c = chunks_[i];
      Block* ob = c.owner;
      fprintf(stderr, "  [chunk] %u state %d pin %u key %llu nu %llu owner %s\n", i, (int)c.state, c.pin_count,
              (unsigned long long)victim_key_locked(c), (unsigned long long)c.next_use,
              ob ? ob->range->name.c_str() : "-");
    }
    fprintf(stderr, "  [vcache] pos %zu size %zu valid %d clock %llu risen %zu\n", vcache_pos_, vcache_.size(),
            (int)vcache_valid_, (unsigned long long)vcache_clock_, vrisen_.size());
  }
  for (auto& c : cand) {
    if (dbg) {
      Block* ob = chunks_[c.second].owner;
      fprintf(stderr, "[victim] %s chunk %u key %llu next_use %llu clock %llu floor %llu owner %s/%llu\n",
              name_.c_str(), c.second, (unsigned long long)c.first, (unsigned long long)chunks_[c.second].next_use,
              (unsigned long long)op_clock_, (unsigned long long)floor, ob ? ob->range->name.c_str() : "-",
              ob ? (unsigned long long)ob->index : 0ull);
    }
    out->push_back(c.second);
  }
}

Status ChunkArena::reserve_for(const std::vector<int64_t>& want, std::vector<uint32_t>* got, Reservation* r) {
  std::lock_guard<OrderedMutex> g(m_);
  const uint32_t n = (uint32_t)want.size();
  constexpr uint32_t kNone = UINT32_MAX;
  got->assign(n, kNone);
  r->first = -1;
  r->n = n;
  r->victims.clear();
  r->list.clear();
  if (n == 0) return Status::OK;
  auto undo = [&]() {
    for (uint32_t k : r->list) {
      ChunkInfo& c = chunks_[k];
      if (c.state == ChunkState::RESERVED) {
        c.state = ChunkState::FREE;
        add_run(k, 1);
      } else {
        c.state = ChunkState::ALLOCATED;
        lru_push_tail(k, 2);
      }
    }
    r->list.clear();
    r->victims.clear();
    r->n = 0;
    got->assign(n, kNone);
    return Status::NO_MEMORY;
  };
  auto take_free = [&](uint32_t i, uint32_t k) {
    take_run(k, 1);
    chunks_[k].state = ChunkState::RESERVED;
    r->list.push_back(k);
    (*got)[i] = k;
  };
  auto take_victim = [&](uint32_t i, uint32_t k) {
    lru_remove(k);
    chunks_[k].state = ChunkState::EVICTING;
    r->list.push_back(k);
    r->victims.push_back(k);
    (*got)[i] = k;
  };
  // 1. free home chunks
  uint32_t left = n;
  for (uint32_t i = 0; i < n; ++i) {
    const int64_t h = want[i];
    if (h >= 0 && h < (int64_t)nchunks_ && chunks_[h].state == ChunkState::FREE) {
      take_free(i, (uint32_t)h);
      --left;
    }
  }
  uint64_t nfree = 0;
  for (auto& fr : free_runs_) nfree += fr.second;
  const uint32_t evict = left > nfree ? (uint32_t)(left - nfree) : 0;
  std::vector<std::pair<uint64_t, uint32_t>> cand;
  if (evict) {
    const uint64_t floor = VictimFloor::value();
    next_victims_locked(evict + n, floor, &cand);
    if (cand.size() < evict) return undo();
    uint64_t kthr = ~0ull;  // Belady's worst pick for `evict` victims
    for (uint32_t k = 0; k < evict; ++k) kthr = std::min(kthr, cand[k].first);
    // 2. home chunks that are as good a victim as Belady's own picks
    uint32_t used = 0;
    for (uint32_t i = 0; i < n && used < evict; ++i) {
      const int64_t h = want[i];
      if ((*got)[i] != kNone || h < 0 || h >= (int64_t)nchunks_) continue;
      const ChunkInfo& c = chunks_[h];
      if (c.state != ChunkState::ALLOCATED || c.pin_count != 0 || floor_protects_locked(c, floor)) continue;
      if (victim_key_locked(c) < kthr) continue;
      take_victim(i, (uint32_t)h);
      ++used;
      --left;
    }
    // 3. the rest of the evictions in next-use order
    size_t ci = 0;
    for (uint32_t i = 0; i < n && used < evict; ++i) {
      if ((*got)[i] != kNone) continue;
      while (ci < cand.size() && chunks_[cand[ci].second].state != ChunkState::ALLOCATED) ++ci;
      if (ci >= cand.size()) return undo();
      take_victim(i, cand[ci++].second);
      ++used;
      --left;
    }
  }
  // 4. free chunks for the others
  for (uint32_t i = 0; i < n && left; ++i) {
    if ((*got)[i] != kNone) continue;
    if (free_runs_.empty()) return undo();
    take_free(i, free_runs_.begin()->first);
    --left;
  }
  if (left) return undo();
  st_.reservations++;
  return Status::OK;
}

Status ChunkArena::reserve_scattered(uint32_t n, Reservation* r) {
  std::lock_guard<OrderedMutex> g(m_);
  if (n == 0 || n > nchunks_) return Status::NO_MEMORY;
  r->first = -1;
  r->n = n;
  r->victims.clear();
  r->list.clear();
  r->list.reserve(n);
  while (r->list.size() < n && !free_runs_.empty()) {
    uint32_t k = free_runs_.begin()->first;
    take_run(k, 1);
    chunks_[k].state = ChunkState::RESERVED;
    r->list.push_back(k);
  }
  if (hinted_ && r->list.size() < n) {
    std::vector<uint32_t> v;
    pick_victims_by_next_use_locked(n - (uint32_t)r->list.size(), &v);
    for (uint32_t k : v) {
      lru_remove(k);
      chunks_[k].state = ChunkState::EVICTING;
      r->list.push_back(k);
      r->victims.push_back(k);
    }
  }
  while (r->list.size() < n) {
    int32_t v = pick_victim_locked();
    if (v < 0) break;
    lru_remove((uint32_t)v);
    chunks_[v].state = ChunkState::EVICTING;
    r->list.push_back((uint32_t)v);
    r->victims.push_back((uint32_t)v);
  }
  if (r->list.size() < n) {  // not enough evictable memory: give everything back
    for (uint32_t k : r->list) {
      ChunkInfo& c = chunks_[k];
      if (c.state == ChunkState::RESERVED) {
        c.state = ChunkState::FREE;
        add_run(k, 1);
      } else {
        c.state = ChunkState::ALLOCATED;
        lru_push_tail(k, 2);
      }
    }
    r->list.clear();
    r->victims.clear();
    r->n = 0;
    return Status::NO_MEMORY;
  }
  st_.reservations++;
  return Status::OK;
}

void ChunkArena::evicted(uint32_t i) {
  std::lock_guard<OrderedMutex> g(m_);
  ChunkInfo& c = chunks_[i];
  RT_ASSERT_RELEASE(c.state == ChunkState::EVICTING);
  c.state = ChunkState::RESERVED;
  c.owner = nullptr;
  c.next_use = 0;
  deactivate(c);
  st_.allocated -= kBlockSize;
  st_.evictions++;
}

void ChunkArena::commit(const Reservation& r, bool pin) {
  std::lock_guard<OrderedMutex> g(m_);
  r.for_each([&](uint32_t k) {
    ChunkInfo& c = chunks_[k];
    RT_ASSERT_RELEASE(c.state == ChunkState::RESERVED);
    c.state = ChunkState::ALLOCATED;
    c.owner = nullptr;
    c.pin_count = pin ? 1 : 0;
    c.last_use = ++clock_;
    c.last_op = op_clock_;
    c.next_use = 0;
    lru_push_tail(k, 1);
  });
  if (pin) st_.pinned += (uint64_t)r.n << kBlockShift;
  st_.allocated += (uint64_t)r.n << kBlockShift;
  st_.peak = std::max(st_.peak, st_.allocated);
  st_.allocs += r.n;
}

void ChunkArena::cancel(const Reservation& r) {
  std::lock_guard<OrderedMutex> g(m_);
  r.for_each([&](uint32_t k) {
    ChunkInfo& c = chunks_[k];
    if (c.state == ChunkState::RESERVED) {
      c.state = ChunkState::FREE;
      c.owner = nullptr;
      add_run(k, 1);
    } else if (c.state == ChunkState::EVICTING) {
      // eviction failed: the owner keeps the chunk
      c.state = ChunkState::ALLOCATED;
      lru_push_tail(k, 2);
    }
  });
}

void ChunkArena::free(uint32_t first, uint32_t n) {
  std::lock_guard<OrderedMutex> g(m_);
  for (uint32_t i = 0; i < n; ++i) free_locked(first + i);
}

void ChunkArena::free_locked(uint32_t k) {
  ChunkInfo& c = chunks_[k];
  RT_ASSERT_RELEASE(c.state == ChunkState::ALLOCATED);
  lru_remove(k);
  if (c.pin_count) st_.pinned -= kBlockSize;
  c.state = ChunkState::FREE;
  c.owner = nullptr;
  c.pin_count = 0;
  c.next_use = 0;
  c.zeroed = false;
  c.doomed = false;
  deactivate(c);
  add_run(k, 1);
  st_.allocated -= kBlockSize;
  st_.frees++;
}

void ChunkArena::free_when_unpinned(uint32_t i) {
  std::lock_guard<OrderedMutex> g(m_);
  ChunkInfo& c = chunks_[i];
  if (c.pin_count == 0) {
    free_locked(i);
    return;
  }
  c.doomed = true;
  c.owner = nullptr;
  c.next_use = 0;
  lru_remove(i);  // not a victim candidate (pinned anyway) nor an LRU entry
}

void ChunkArena::unpinned_locked(uint32_t k) {
  st_.pinned -= kBlockSize;
  if (chunks_[k].doomed) free_locked(k);
}

void ChunkArena::set_owner(uint32_t i, Block* b) {
  std::lock_guard<OrderedMutex> g(m_);
  chunks_[i].owner = b;
}

Block* ChunkArena::owner(uint32_t i) {
  std::lock_guard<OrderedMutex> g(m_);
  return chunks_[i].owner;
}

void ChunkArena::touch(uint32_t i, bool has_data, bool preferred, bool prefetched, uint64_t refault_key,
                       uint64_t evicted_at, bool clean) {
  std::lock_guard<OrderedMutex> g(m_);
  touch_locked(i, has_data, preferred, prefetched, refault_key, evicted_at, clean);
}

bool ChunkArena::try_pin_many(const uint32_t* idx, size_t n) {
  std::lock_guard<OrderedMutex> g(m_);
  for (size_t k = 0; k < n; ++k)
    if (chunks_[idx[k]].state != ChunkState::ALLOCATED) return false;
  for (size_t k = 0; k < n; ++k)
    if (chunks_[idx[k]].pin_count++ == 0) st_.pinned += kBlockSize;
  return true;
}

void ChunkArena::touch_many(const TouchReq* r, size_t n) {
  std::lock_guard<OrderedMutex> g(m_);
  for (size_t k = 0; k < n; ++k) {
    const TouchReq& t = r[k];
    touch_locked(t.chunk, t.has_data, t.preferred, t.prefetched, t.refault_key, t.evicted_at, t.clean);
    if (t.next_use) set_next_use_locked(t.chunk, t.next_use);
  }
}

void ChunkArena::release_many(const uint32_t* idx, size_t n, const FenceRef& f) {
  std::lock_guard<OrderedMutex> g(m_);
  for (size_t k = 0; k < n; ++k) {
    ChunkInfo& c = chunks_[idx[k]];
    if (f) c.reuse_fence.add(f);
    RT_ASSERT_RELEASE(c.pin_count > 0);
    if (--c.pin_count == 0) {
      if (c.doomed) {
        unpinned_locked(idx[k]);
        continue;
      }
      st_.pinned -= kBlockSize;
    }
    touch_locked(idx[k], true, false, false, 0, 0, false);
  }
}

void ChunkArena::touch_locked(uint32_t i, bool has_data, bool preferred, bool prefetched, uint64_t refault_key,
                              uint64_t evicted_at, bool clean) {
  ChunkInfo& c = chunks_[i];
  if (c.state != ChunkState::ALLOCATED) return;
  c.last_use = ++clock_ + (prefetched ? kPrefetchBoost : 0);
  if (!prefetched) c.last_op = op_clock_;
  // A chunk keeps its preferred status until it loses its data.
  bool pref = has_data && (preferred || c.list == 3);
  if (!has_data) {
    deactivate(c);
  } else if (refault_key && preferred && !c.active && st_.active + (st_.pinned >> kBlockShift) < active_limit_) {
    // (pinned chunks - leased / allocator memory - count against the protected share)
    const uint64_t distance = st_.evictions > evicted_at ? st_.evictions - evicted_at : 0;
    const uint64_t ws = distance + nchunks_;  // estimated cyclic working set, in chunks
    const uint64_t h = (refault_key * 0x9E3779B97F4A7C15ull) >> 44;  // 20-bit bucket
    if (h * ws < ((uint64_t)active_limit_ << 20)) {
      c.active = true;
      st_.active++;
    }
  }
  lru_remove(i);
  lru_push_tail(i, !has_data ? 1 : (pref && !clean ? 3 : 2));
}

void ChunkArena::pin(uint32_t i) {
  std::lock_guard<OrderedMutex> g(m_);
  if (chunks_[i].pin_count++ == 0) st_.pinned += kBlockSize;
}

bool ChunkArena::try_pin(uint32_t i) {
  std::lock_guard<OrderedMutex> g(m_);
  if (chunks_[i].state != ChunkState::ALLOCATED) return false;
  if (chunks_[i].pin_count++ == 0) st_.pinned += kBlockSize;
  return true;
}

void ChunkArena::unpin(uint32_t i) {
  std::lock_guard<OrderedMutex> g(m_);
  RT_ASSERT_RELEASE(chunks_[i].pin_count > 0);
  if (--chunks_[i].pin_count == 0) unpinned_locked(i);
}

bool ChunkArena::pinned(uint32_t i) {
  std::lock_guard<OrderedMutex> g(m_);
  return chunks_[i].pin_count > 0;
}

void ChunkArena::add_reuse_fence(uint32_t i, const FenceRef& f) {
  std::lock_guard<OrderedMutex> g(m_);
  chunks_[i].reuse_fence.add(f);
}

// Every writer of a chunk waits for the chunk's reuse fence; the fence stays
// (completed fences are pruned) because one chunk can receive several writers
// on different rings - e.g. a D2D relocation of resident pages plus the H2D copy
// of the missing ones. Consuming the fence on the first writer let the second
// overwrite data the previous owner's kernels were still reading (the corrupt
// ANS chunks / ~47 s decoder spin of the 70B tp8 shard,
// profiles/r2_corrupt_chunk_hunt.md).
Tracker ChunkArena::reuse_fence(uint32_t i) {
  std::lock_guard<OrderedMutex> g(m_);
  chunks_[i].reuse_fence.prune();
  return chunks_[i].reuse_fence;
}

ChunkArena::Stats ChunkArena::stats() {
  std::lock_guard<OrderedMutex> g(m_);
  return st_;
}

uint32_t ChunkArena::free_chunks() {
  std::lock_guard<OrderedMutex> g(m_);
  uint32_t n = 0;
  for (auto& r : free_runs_) n += r.second;
  return n;
}

uint32_t ChunkArena::largest_free_run() {
  std::lock_guard<OrderedMutex> g(m_);
  uint32_t n = 0;
  for (auto& r : free_runs_) n = std::max(n, r.second);
  return n;
}

uint64_t ChunkArena::outstanding_bytes() {
  std::lock_guard<OrderedMutex> g(m_);
  return st_.allocated;
}

std::string ChunkArena::check() {
  std::lock_guard<OrderedMutex> g(m_);
  std::ostringstream os;
  uint32_t nfree = 0, nalloc = 0, nfree_state = 0, ndoomed = 0;
  std::vector<uint8_t> in_run(nchunks_, 0);
  uint32_t prev_end = 0;
  bool first = true;
  for (auto& r : free_runs_) {
    if (!first && r.first <= prev_end) os << "free runs overlap/adjacent at " << r.first << "; ";
    first = false;
    prev_end = r.first + r.second;
    for (uint32_t i = r.first; i < r.first + r.second; ++i) {
      if (i >= nchunks_) { os << "run past end; "; break; }
      in_run[i] = 1;
      if (chunks_[i].state != ChunkState::FREE) os << "chunk " << i << " in free run but not FREE; ";
    }
    nfree += r.second;
  }
  for (uint32_t i = 0; i < nchunks_; ++i) {
    if (chunks_[i].state == ChunkState::FREE && !in_run[i]) os << "FREE chunk " << i << " not in runs; ";
    if (chunks_[i].state == ChunkState::ALLOCATED) nalloc++;
    if (chunks_[i].state == ChunkState::ALLOCATED && chunks_[i].doomed) {
      ndoomed++;  // revoked under a lease: freed at its last unpin, off the LRU lists meanwhile
      if (chunks_[i].pin_count == 0) os << "doomed chunk " << i << " unpinned but not freed; ";
    }
    if (chunks_[i].state == ChunkState::FREE) nfree_state++;
  }
  if (nfree != nfree_state) os << "free runs hold " << nfree << " chunks but " << nfree_state << " are FREE; ";
  uint64_t n_on_lists = 0;
  for (int l : {1, 2, 3})
    for (int32_t i = head_[l]; i >= 0; i = chunks_[i].next) {
      n_on_lists++;
      if (chunks_[i].state != ChunkState::ALLOCATED) os << "non-allocated chunk " << i << " on LRU; ";
      if (n_on_lists > nchunks_) { os << "LRU cycle; "; break; }
    }
  if (n_on_lists + ndoomed != nalloc)
    os << "LRU holds " << n_on_lists << " (+" << ndoomed << " doomed) but " << nalloc << " allocated; ";
  if ((uint64_t)nalloc << kBlockShift != st_.allocated) os << "allocated bytes mismatch; ";
  return os.str();
}

// ------------------------------------------------------------ HBM arena
HbmArena::HbmArena(Backend* be, int dev, uint64_t budget, int provider)
    : ChunkArena("hbm" + std::to_string(dev), Loc::gpu(dev), LockOrder::HBM_ARENA), be_(be), dev_(dev) {
  uint32_t n = (uint32_t)(budget >> kBlockShift);
  bytes_ = (uint64_t)n << kBlockShift;
  if (n == 0) {
    init_chunks(0, 0);
    return;
  }
  if (provider == 1 && be->vmm_supported(dev)) {
    void* va = nullptr;
    init_ = be->va_reserve(bytes_, &va);
    if (init_ == Status::OK) {
      handles_.resize(n);
      for (uint32_t i = 0; i < n && init_ == Status::OK; ++i) {
        init_ = be->vmm_create(dev, kBlockSize, &handles_[i]);
        if (init_ == Status::OK) init_ = be->vmm_map((char*)va + ((uint64_t)i << kBlockShift), kBlockSize, handles_[i], dev);
        if (init_ != Status::OK) handles_.resize(i);
      }
      slab_ = va;
    }
  } else {
    init_ = be->hbm_alloc(dev, bytes_, &slab_);
  }
  if (init_ != Status::OK) {
    RT_ERR("HBM arena init on gpu %d (%llu MB) failed: %s", dev, (unsigned long long)(bytes_ >> 20), status_str(init_));
    init_chunks(0, 0);
    return;
  }
  init_chunks((uint64_t)slab_, n);
  RT_INFO("HBM arena gpu%d: %u x 2MB chunks at %p (%s)", dev, n, slab_, handles_.empty() ? "slab" : "vmm");
}

HbmArena::~HbmArena() {
  if (!slab_) return;
  if (!handles_.empty()) {
    for (size_t i = 0; i < handles_.size(); ++i) {
      be_->vmm_unmap((char*)slab_ + (i << kBlockShift), kBlockSize);
      be_->vmm_release(handles_[i]);
    }
    be_->va_free(slab_, bytes_);
  } else {
    be_->hbm_free(dev_, slab_, bytes_);
  }
}

// ------------------------------------------------------------ host / CXL arena
HostArena::HostArena(Backend* be, Tier tier, int node, uint64_t capacity)
    : ChunkArena(std::string(tier_str(tier)) + std::to_string(node), Loc{tier, (int16_t)node}, LockOrder::HOST_ARENA),
      be_(be),
      node_(node) {
  uint32_t n = (uint32_t)(capacity >> kBlockShift);
  bytes_ = (uint64_t)n << kBlockShift;
  fd_ = memfd_create(name_.c_str(), MFD_CLOEXEC);
  if (fd_ < 0 || ftruncate(fd_, bytes_) != 0) {
    init_ = Status::NO_MEMORY;
    init_chunks(0, 0);
    return;
  }
  view_ = mmap(nullptr, bytes_, PROT_READ | PROT_WRITE, MAP_SHARED, fd_, 0);
  if (view_ == MAP_FAILED) {
    view_ = nullptr;
    init_ = Status::NO_MEMORY;
    init_chunks(0, 0);
    return;
  }
  // Ask for transparent huge pages on the tier (honoured when shmem THP is
  // "advise"/"always"): fewer TLB entries for the DMA engines and the GPU's
  // remote reads, 2 MB pin granularity. hugetlbfs is not used: a
  // memfd past the reserved huge-page pool would SIGBUS on first touch.
  thp_advised_ = madvise(view_, bytes_, MADV_HUGEPAGE) == 0;
  // Bind the pages of this tier to its NUMA node (CXL.mem nodes are CPU-less
  // NUMA nodes). Shared (shmem) mappings keep the policy on the object.
  if (node >= 0 && node < 64) {
    unsigned long mask = 1ul << node;
    numa_bound_ = mbind(view_, bytes_, MPOL_BIND, &mask, 64, 0) == 0;
    if (!numa_bound_) RT_DBG("mbind to node %d failed (errno %d); pages use the default policy", node, errno);
  }
  if (config().host_segment_mb > 0) seg_ = std::max<uint64_t>(kBlockSize, (uint64_t)config().host_segment_mb << 20) / kBlockSize * kBlockSize;
  seg_registered_.assign((bytes_ + seg_ - 1) / seg_, 0);
  init_chunks((uint64_t)view_, n);
}

HostArena::~HostArena() {
  if (view_) {
    for (size_t s = 0; s < seg_registered_.size(); ++s)
      if (seg_registered_[s]) be_->host_unregister((char*)view_ + s * seg_);
    munmap(view_, bytes_);
  }
  NodeLedger& L = NodeLedger::get();
  if (ledger_bytes_ && L.epoch() == ledger_epoch_) L.release(node_, ledger_bytes_);
  if (fd_ >= 0) close(fd_);
}

Status HostArena::ensure_registered(uint32_t first, uint32_t n) {
  if (!view_) return Status::NO_MEMORY;
  uint64_t lo = (uint64_t)first << kBlockShift, hi = ((uint64_t)(first + n) << kBlockShift);
  std::lock_guard<std::mutex> g(seg_m_);
  NodeLedger& L = NodeLedger::get();
  for (uint64_t s = lo / seg_; s * seg_ < hi; ++s) {
    if (seg_registered_[s]) continue;
    char* p = (char*)view_ + s * seg_;
    uint64_t len = std::min<uint64_t>(seg_, bytes_ - s * seg_);
    // Node-wide budget first (every rank process on this node shares it): a
    // segment the node cannot back is refused here, before it is touched.
    if (!L.reserve(node_, len)) {
      ledger_refused() = true;
      Tools::get().inc(Counter::LedgerRefusals);
      RT_WARN("%s: node %d budget exhausted across processes (ledger %s: %llu of %llu MB reserved)", name_.c_str(),
              node_, L.path().c_str(), (unsigned long long)(L.view(node_).reserved >> 20),
              (unsigned long long)(L.view(node_).capacity >> 20));
      return Status::NO_MEMORY;
    }
    if (ledger_bytes_ && ledger_epoch_ != L.epoch()) ledger_bytes_ = 0;  // (reserved under an old attachment)
    ledger_epoch_ = L.epoch();
    // Populate first (fault in on the bound node), then pin for device DMA.
    if (madvise(p, len, MADV_POPULATE_WRITE) != 0) {
      for (uint64_t o = 0; o < len; o += kPageSize) ((volatile char*)p)[o] = 0;
    }
    Status st = be_->host_register(p, len);
    if (st != Status::OK) {
      L.release(node_, len);
      return st;
    }
    ledger_bytes_ += len;
    seg_registered_[s] = 1;
  }
  return Status::OK;
}

}  // namespace ogkm
