// Physical memory managers for every tier.
//
// ChunkArena is the common 2 MB root-chunk allocator (analog of the GPU PMM,
// uvm_pmm_gpu.c, and of the sysmem PMM, uvm_pmm_sysmem.c):
//   * chunks are 2 MB (UVM_CHUNK_SIZE_MAX, uvm_pmm_gpu.h:79) carved out of one
//     device-usable region (an HBM slab, or a NUMA-bound memfd mapping for
//     host / CXL tiers);
//   * contiguous extents are allocated from a free-run map (range allocator,
//     uvm_range_allocator.c:27-67) so a tensor's blocks can be viewed as one
//     contiguous device buffer;
//   * allocated chunks sit on an UNUSED or USED LRU list (uvm_pmm_gpu.c:99-112)
//     and victims are chosen free -> unused -> used-LRU
//     (pick_root_chunk_to_evict, uvm_pmm_gpu.c:1460-1500);
//   * eviction is a two-phase protocol: the arena *reserves* a window and marks
//     victims EVICTING under its own lock, drops the lock, the owner blocks are
//     evicted under their block locks, then the window is committed
//     (lock-order discipline of uvm_pmm_gpu.c:1181-1202);
//   * every chunk carries a reuse fence (Tracker) that the next writer waits on
//     GPU-side, so a clean chunk can be recycled without stalling the CPU.
#pragma once

#include <functional>
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "ogkm/backend.hpp"
#include "ogkm/common.hpp"
#include "ogkm/lock_order.hpp"
#include "ogkm/tracker.hpp"

namespace ogkm {

class Block;

enum class ChunkState : uint8_t { FREE = 0, RESERVED = 1, ALLOCATED = 2, EVICTING = 3 };

struct ChunkInfo {
  ChunkState state = ChunkState::FREE;
  uint8_t list = 0;      // 0 none, 1 unused, 2 used, 3 used + preferred here
  bool zeroed = false;
  bool doomed = false;   // freed by its owner while a lease pinned it: freed at the last unpin
  bool active = false;   // workingset-protected (a refaulted block's data): evicted after every inactive chunk
  uint32_t pin_count = 0;
  Block* owner = nullptr;
  int32_t prev = -1, next = -1;  // LRU links
  uint64_t last_use = 0;         // logical clock
  uint64_t next_use = 0;         // op clock of the owner's next use (0 = unknown, kDeadUse = never)
  uint64_t last_op = 0;          // op clock at the last touch
  Tracker reuse_fence;           // work that must finish before the chunk is overwritten
};

struct Reservation {
  int64_t first = -1;
  uint32_t n = 0;
  std::vector<uint32_t> victims;  // chunks that must be evicted before commit
  // Scattered reservation (reserve_scattered): exactly these chunks, in no
  // particular order; empty = the contiguous window [first, first + n).
  std::vector<uint32_t> list;
  template <class F>
  void for_each(F f) const {
    if (!list.empty())
      for (uint32_t k : list) f(k);
    else
      for (uint32_t i = 0; i < n; ++i) f((uint32_t)first + i);
  }
};

class ChunkArena {
 public:
  ChunkArena(std::string name, Loc loc, LockOrder order);
  virtual ~ChunkArena();

  const std::string& name() const { return name_; }
  Loc loc() const { return loc_; }
  uint64_t base() const { return base_; }          // device-usable address of chunk 0
  uint32_t nchunks() const { return nchunks_; }
  uint64_t chunk_addr(uint32_t i) const { return base_ + ((uint64_t)i << kBlockShift); }
  int64_t chunk_of(uint64_t addr) const;

  // Contiguous allocation of n chunks without eviction. `hint` = preferred first chunk.
  // `pin`: the chunks come back pinned (never eviction victims) so a caller that
  // hands them to their owners later cannot lose them to a concurrent reserve().
  Status alloc(uint32_t n, Block* owner_for_all, int64_t hint, uint32_t* first, bool pin = false);
  // Reserve a window of n contiguous chunks, possibly containing evictable chunks.
  Status reserve(uint32_t n, Reservation* r);
  // Reserve n chunks anywhere (stable-VA blocks are mapped one by one and need
  // no contiguity): free chunks first, then victims in reserve(1)'s order.
  // All or nothing.
  Status reserve_scattered(uint32_t n, Reservation* r);
  // Next-use mode: one chunk per requested block, honouring each block's home
  // chunk `want[i]` (the chunk its stable VA still maps, -1 = none) - free, or
  // an eviction victim as good as Belady's own choice (its next use no sooner
  // than the furthest-needed chunks that would be evicted otherwise). A block
  // back on its home chunk needs no VMM remap and no translation flush. The
  // rest: free chunks, then next-use victims. got[i] = the block's chunk; all
  // or nothing (NO_MEMORY).
  Status reserve_for(const std::vector<int64_t>& want, std::vector<uint32_t>* got, Reservation* r);
  void commit(const Reservation& r, bool pin = false);  // window -> ALLOCATED (owners set later)
  void cancel(const Reservation& r);                // give the window back
  void free(uint32_t first, uint32_t n);
  // Free chunk i now, or - while a lease still pins it (a reader that leased
  // the copy before a migration revoked it) - at its last unpin. Owner-less
  // from now on; never a victim meanwhile (pinned).
  void free_when_unpinned(uint32_t i);
  void set_owner(uint32_t i, Block* b);
  Block* owner(uint32_t i);
  // Evictor calls this once the owner has let go of an EVICTING chunk.
  void evicted(uint32_t i);

  // LRU bump. `preferred`: the owner's preferred location is this tier - such
  // chunks sit on their own list and are evicted only after every other
  // allocated chunk (protects the planned resident set from streaming traffic).
  // `prefetched`: the data was brought in ahead of its use - it ranks as newer than
  // every chunk that has actually been used until its first access (otherwise a
  // layer-ahead prefetch would be the LRU victim of the next prefetch).
  // `refault`: the owner block's data was evicted from this tier before and is
  // back - with `preferred`, the chunk joins the protected active set while that
  // set is below perf_workingset_active_pct of the arena (the refault-distance
  // workingset idea: a cyclic scan larger than the arena keeps a stable subset
  // resident instead of evicting every block just before its next use).
  //
  // Admission is spread over the scan: the refault distance (evictions since
  // the block left, + the arena size) estimates the cyclic working set W, and a
  // unit (`refault_key`, e.g. its range id - a unit is all in or all out) is
  // admitted when its hash falls in the first active_limit / W of the hash
  // space, so resident units interleave with streamed ones over the cycle (the
  // link keeps streaming behind them) instead of forming one long stretch.
  // clean: every page also has a valid copy elsewhere - evicting it costs no
  // copy-out, so it goes to the normal list even when preferred (dirty data,
  // which costs a copy-out and a refill, stays in the protected list).
  void touch(uint32_t i, bool has_data, bool preferred = false, bool prefetched = false, uint64_t refault_key = 0,
             uint64_t evicted_at = 0, bool clean = false);
  // Next-use (Belady) victim order. Once any chunk carries a hint the
  // evictable chunks are ranked by the op clock of their next use instead of
  // recency: dead data first, then unhinted data by age (data not seen for a few
  // ops; just-touched unhinted data counts as needed next), then hinted data
  // furthest in the future first - the optimal replacement order for a known
  // access sequence (a cyclic decode step under LRU evicts every block just
  // before its next use). Victims never have a next use before the thread's
  // VictimFloor (a prefetch must not evict data needed before its own).
  void set_next_use(uint32_t i, uint64_t when);
  void set_next_use_many(const uint32_t* idx, size_t n, uint64_t when);  // one lock for a range's chunks
  void set_op_clock(uint64_t now);
  // A new hint producer (another ogkm.managed() context, a new model) restarts
  // its op clock at 0: forget the old clock, every chunk's hint and the victim
  // cache, so the new hints are not read as lying in the past.
  void reset_op_clock();
  bool next_use_mode() {
    std::lock_guard<OrderedMutex> g(m_);
    return hinted_;
  }
  uint64_t evictions() {
    std::lock_guard<OrderedMutex> g(m_);
    return st_.evictions;
  }
  // Lease fast path (Runtime::acquire of a resident extent): pin every chunk
  // under one lock, or none (false) when any is no longer ALLOCATED; release
  // = reuse fence + unpin + LRU touch of each, under one lock.
  bool try_pin_many(const uint32_t* idx, size_t n);
  // Each chunk's LRU touch (and next-use hint when nonzero) under one lock:
  // the lease fast path's recency updates of a whole unit.
  struct TouchReq {
    uint32_t chunk;
    bool has_data, preferred, prefetched, clean;
    uint64_t refault_key, evicted_at, next_use;
  };
  void touch_many(const TouchReq* r, size_t n);
  void release_many(const uint32_t* idx, size_t n, const FenceRef& f);
  void pin(uint32_t i);
  // Pin only an ALLOCATED chunk: false when it is reserved for eviction (or
  // free) - a pin taken after another thread chose the chunk as a victim would
  // be overwritten by that reservation's commit.
  bool try_pin(uint32_t i);
  void unpin(uint32_t i);
  bool pinned(uint32_t i);
  void add_reuse_fence(uint32_t i, const FenceRef& f);
  Tracker reuse_fence(uint32_t i);                  // what the next writer must wait for (not consumed)

  struct Stats {
    uint64_t capacity = 0, allocated = 0, peak = 0, pinned = 0, evictions = 0, allocs = 0, frees = 0,
             used_list = 0, unused_list = 0, reservations = 0, active = 0;
  };
  Stats stats();
  uint32_t free_chunks();
  uint32_t largest_free_run();
  // Leak check (uvm_kvmalloc / UVM_TEST_PMM_CHECK_LEAK analog).
  uint64_t outstanding_bytes();
  // Consistency check used by tests; returns empty string when consistent.
  std::string check();

 protected:
  void init_chunks(uint64_t base, uint32_t n);
  std::string name_;
  Loc loc_;
  uint64_t base_ = 0;
  uint32_t nchunks_ = 0;

 private:
  void set_next_use_locked(uint32_t i, uint64_t when);
  void free_locked(uint32_t k);  // one ALLOCATED chunk back to the free runs
  void unpinned_locked(uint32_t k);  // pin count just reached 0
  void touch_locked(uint32_t i, bool has_data, bool preferred, bool prefetched, uint64_t refault_key,
                    uint64_t evicted_at, bool clean);
  int32_t pick_victim_locked();  // coldest evictable chunk (reserve(1) order), -1 = none
  uint64_t victim_key_locked(const ChunkInfo& c) const;  // next-use mode: larger = evict sooner
  uint64_t base_key_locked(const ChunkInfo& c) const;    // the same without the kEvictFirst class bonus
  bool floor_protects_locked(const ChunkInfo& c, uint64_t floor) const;
  // next-use mode: up to n evictable chunks with the largest keys above the floor
  void pick_victims_by_next_use_locked(uint32_t n, std::vector<uint32_t>* out);
  // The next `want` victims in next-use order, (current key, chunk), from a
  // ranked candidate list rebuilt by a full scan only when it runs dry or the
  // op clock moved arena_victim_cache_ops past its build (a full scan per
  // fault was ~1 s per 70B step over 40k chunks). Entries that left ALLOCATED,
  // got pinned or fell in rank (re-used for data needed sooner) are skipped.
  void next_victims_locked(uint32_t want, uint64_t floor, std::vector<std::pair<uint64_t, uint32_t>>* out);
  bool hinted_ = false;
  uint64_t op_clock_ = 0;
  std::vector<std::pair<uint64_t, uint32_t>> vcache_;  // (key at build, chunk), best first
  size_t vcache_pos_ = 0;
  uint64_t vcache_clock_ = 0;
  bool vcache_valid_ = false;
  std::vector<uint32_t> vrisen_;  // chunks re-hinted since the cache was built (set_next_use)
  void lru_remove(uint32_t i);
  void lru_push_tail(uint32_t i, uint8_t list);
  void take_run(uint32_t first, uint32_t n);  // remove [first,first+n) from free runs
  void add_run(uint32_t first, uint32_t n);   // insert + coalesce

  OrderedMutex m_;
  std::vector<ChunkInfo> chunks_;
  std::map<uint32_t, uint32_t> free_runs_;  // start -> len
  int32_t head_[4] = {-1, -1, -1, -1}, tail_[4] = {-1, -1, -1, -1};
  uint64_t clock_ = 0;
  uint32_t active_limit_ = 0;
  void deactivate(ChunkInfo& c) {
    if (c.active) {
      c.active = false;
      st_.active--;
    }
  }
  Stats st_;
};

// HBM of one GPU: a slab from the backend (hipMalloc) or VMM handles mapped
// contiguously at an alias VA (needed for stable-VA managed ranges).
class HbmArena : public ChunkArena {
 public:
  HbmArena(Backend* be, int dev, uint64_t budget_bytes, int provider);
  ~HbmArena() override;
  int dev() const { return dev_; }
  bool vmm() const { return !handles_.empty(); }
  uint64_t handle(uint32_t i) const { return handles_.empty() ? 0 : handles_[i]; }
  Status init_status() const { return init_; }

 private:
  Backend* be_;
  int dev_;
  void* slab_ = nullptr;
  uint64_t bytes_ = 0;
  std::vector<uint64_t> handles_;
  Status init_ = Status::OK;
};

constexpr uint64_t kHostSegment = 1ull << 30;  // default host_segment_mb

// Scoped placement side for the calling thread's arena allocations: 0 any
// (best fit), 1 low end (first fit), 2 high end (last fit). Data that stays
// (the keep class) packs at one end, data that cycles through (the stream
// class) at the other, so contiguous extents for the stream class are found
// among stream-class chunks instead of cutting into kept ones.
struct PlacementSide {
  static int& value();
  int saved;
  explicit PlacementSide(int side) : saved(value()) { value() = side; }
  ~PlacementSide() { value() = saved; }
  PlacementSide(const PlacementSide&) = delete;
  PlacementSide& operator=(const PlacementSide&) = delete;
};

// Host DRAM or CXL.mem of one NUMA node: a memfd mapped once (the arena view,
// device-registered segment by segment) and bound to the node with mbind.
// CPU views of managed ranges map the same memfd pages with MAP_FIXED, so the
// CPU VA of a block can be remapped without copying.
class HostArena : public ChunkArena {
 public:
  HostArena(Backend* be, Tier tier, int node, uint64_t capacity_bytes);
  ~HostArena() override;
  int fd() const { return fd_; }
  int node() const { return node_; }
  uint64_t file_offset(uint32_t chunk) const { return (uint64_t)chunk << kBlockShift; }
  // Ensure the segment(s) backing [first, first+n) are populated and registered.
  Status ensure_registered(uint32_t first, uint32_t n);
  Status init_status() const { return init_; }
  bool numa_bound() const { return numa_bound_; }
  bool thp_advised() const { return thp_advised_; }
  uint64_t ledger_bytes() const { return ledger_bytes_; }

 private:
  Backend* be_;
  int node_;
  int fd_ = -1;
  void* view_ = nullptr;
  uint64_t bytes_ = 0;
  std::vector<uint8_t> seg_registered_;  // per segment (host_segment_mb, default 1 GB)
  uint64_t seg_ = kHostSegment;
  std::mutex seg_m_;
  // Bytes reserved in the node-wide ledger (NodeLedger) for the populated
  // segments, and the ledger attachment they were reserved under.
  uint64_t ledger_bytes_ = 0;
  uint64_t ledger_epoch_ = 0;
  bool numa_bound_ = false;
  bool thp_advised_ = false;
  Status init_ = Status::OK;
};

constexpr uint64_t kDeadUse = ~0ull;  // ChunkInfo::next_use of dead data
// Flag bit of a next-use hint (hint_next_use(when | kEvictFirst)): among data
// with a known next use, flagged data is evicted first (a spread residency:
// the "stream" class); the floor still compares the true next use.
constexpr uint64_t kEvictFirst = 1ull << 61;

// Scoped lower bound on the next-use key of eviction victims for the calling
// thread (next-use mode only): a prefetch of data needed at op T evicts only
// data needed after T, or nothing.
struct VictimFloor {
  static uint64_t& value();
  uint64_t saved;
  explicit VictimFloor(uint64_t floor) : saved(value()) { value() = floor; }
  ~VictimFloor() { value() = saved; }
  VictimFloor(const VictimFloor&) = delete;
  VictimFloor& operator=(const VictimFloor&) = delete;
};

constexpr uint64_t kPrefetchBoost = 1ull << 40;  // recency bonus of not-yet-used prefetched chunks

}  // namespace ogkm
