// Per-unit fault / prefetch protocol of a cyclic consumer, in one native call.
//
// A decode step uses its weight units (and KV prefixes) in the same order
// every pass. Under runtime-decided residency (planner off) each use is: move
// the op clock to the unit, keep a byte window of the following units in
// flight on the migration ring (each prefetch evicting only data needed later
// than it - the victim floor), fault the unit in (a lease), let the consumer's
// stream wait for its copies GPU-side, hint its next use one pass later; and
// after its kernels are enqueued, release it fenced on the stream and keep the
// host at most `max_ahead` units ahead of the GPU. Done from Python that was
// ~100 us of host time per unit in round 4 (five calls, list bookkeeping),
// which made a fully resident 8B decode host-bound (10.8 vs 6.8 ms/step); here
// it is two calls per unit. The reference services a whole batch of faults per
// pass for the same reason (uvm_gpu_replayable_faults.c:2906 batch loop;
// multi-block migration uvm_migrate.c:456-553).
#pragma once

#include <cstdint>
#include <atomic>
#include <deque>
#include <unordered_map>
#include <mutex>
#include <vector>

#include "ogkm/common.hpp"
#include "ogkm/tracker.hpp"

namespace ogkm {

class Runtime;
class Range;
class ChunkArena;
struct Lease;

class UnitStream {
 public:
  struct Stats {
    uint64_t prefetched = 0, refused = 0, demand = 0, prefetch_ns = 0, acquire_ns = 0, ahead_wait_ns = 0, hint_ns = 0,
             wait_ns = 0, use_ns = 0, held = 0, hold_drops = 0, quiet_passes = 0, loud_streaming = 0,
             loud_evictions = 0, pressure_calls = 0;
  };
  // `ranges`: the units in use order; `window_bytes`: bytes of following units
  // kept in flight; `next_use`: hint next uses / floor prefetches (planner off);
  // `max_ahead`: released units whose kernels may still be queued before the
  // host waits (0 = unbounded).
  UnitStream(Runtime* rt, int dev, std::vector<Range*> ranges, uint64_t window_bytes, bool next_use,
             uint32_t max_ahead);
  ~UnitStream();
  // Unit `pos` is used now on `stream`: returns its lease (device pointer =
  // lease->dptr) with the stream already ordered after its copies.
  // on_stream: `stream` (nullptr = the null stream) waits GPU-side; false:
  // the host waits (fake backend, tools).
  Status use(uint32_t pos, void* stream, Lease** out, bool on_stream = true);
  // Its kernels are enqueued on `stream` (handed back in groups, see .cpp).
  Status release(Lease* l, void* stream, bool on_stream = true);
  // Hand back every unit released so far (a step's end).
  Status flush_released(void* stream);
  // Keep the window full (the step's start: nothing used yet).
  void prefetch_window();
  Stats stats() const {
    Stats s = st_;
    s.pressure_calls = pressure_calls_.load(std::memory_order_relaxed);
    return s;
  }
  void reset_stats() { st_ = Stats{}; }
  uint32_t size() const { return (uint32_t)ranges_.size(); }
  bool detached() const { return rt_ == nullptr; }
  // Runtime shutdown: every live stream hands back its holds and pending
  // leases and forgets the runtime (its own destructor - a Python object
  // collected later - then touches nothing the runtime owned; its calls fail
  // with NOT_INITIALIZED).
  static void detach_all(Runtime* rt);

 private:
  uint64_t due(uint32_t pos) const;
  void detach(bool at_shutdown);
  Runtime* rt_;
  int dev_;
  std::vector<Range*> ranges_;
  uint64_t window_;
  bool next_use_;
  uint32_t max_ahead_;
  uint32_t pf_next_ = 0;
  std::deque<uint32_t> inflight_;
  uint64_t inflight_bytes_ = 0;
  uint64_t pass_ = 0;
  int64_t last_pos_ = -1;
  std::deque<FenceRef> ahead_;  // fences of released groups (host bound)
  std::vector<Lease*> pending_; // released, not yet handed back
  bool pressure_ = false;       // this group's uses streamed (close it now)
  // hold mode (see update_hold)
  void update_hold(void* stream);
  void drop_holds(void* stream);
  std::vector<Lease*> held_;    // per unit: its lease, kept since its last release
  std::vector<uint64_t> held_gen_;  // per unit: its range's mod_gen when it was kept
  bool hold_ = false;
  bool pass_quiet_ = false;     // this pass: no demand fault, no refused prefetch
  uint64_t pass_ev0_ = ~0ull;   // arena evictions at the pass start
  ChunkArena* hold_arena_ = nullptr;
  uint64_t hold_ev_ = 0;
  void* hold_stream_ = nullptr;
  bool hold_on_stream_ = false;
  int64_t cur_pos_ = -1;        // the unit of the latest use
  std::unordered_map<const Range*, uint32_t> pos_of_;  // unit -> its position
  std::recursive_mutex m_;      // use / release / the pressure handler (any thread)
  std::atomic<bool> drop_requested_{false};
  uint64_t pressure_id_ = 0;
  std::atomic<uint64_t> pressure_calls_{0};
  Stats st_;
};

}  // namespace ogkm
