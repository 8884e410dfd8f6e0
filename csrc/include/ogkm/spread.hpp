// Keep / stream classes for cyclically reused data, decided by the runtime.
//
// Next-use (Belady) eviction alone keeps one contiguous run of a cyclic access
// sequence resident: the units used right after the current position are the
// ones needed soonest, so everything the arena can hold is the next stretch of
// the cycle, and while the compute crosses that stretch nothing streams - the
// link idles (126 ms of a 614 ms 70B step, profiles/r4_planner_off_diag.jsonl).
// Interleaving resident and streamed units over the cycle keeps the link busy
// the whole pass; the static plan did this by hand (evenly spread resident
// layers) and round 4's model computed "spread classes" itself.
//
// Here the runtime derives them from what it already sees: the next-use hints
// (their order is the use order, a range hinted twice closes the cycle), each
// hinted range's size, and its own HBM arena (capacity, pinned bytes). Once a
// cycle is known, a keep fraction f = keep_pct x (capacity - pinned) / (bytes
// of the cycle) is error-diffused over the ranges in use order - keep when the
// accumulated share covers the range's bytes - and the rest is the stream
// class: its chunks rank ahead of every keep-class chunk as victims (the arena's
// kEvictFirst flag); the victim floor still compares true next uses. Online
// adaptation: a pass in which keep-class data was evicted (a refault the class
// was meant to prevent) lowers f by perf_spread_step_pct and re-diffuses.
//
// Reference: the runtime, not the client, chooses residency from faults and
// policy (uvm_va_block.c:11560-11760 select_residency; root-chunk victim order
// uvm_pmm_gpu.c:1460-1500).
#pragma once

#include <cstdint>
#include <functional>
#include <mutex>
#include <unordered_map>
#include <vector>

namespace ogkm {

class SpreadPolicy {
 public:
  // Arena view at class assignment: usable bytes = capacity - pinned.
  struct ArenaView {
    uint64_t capacity = 0, pinned = 0;
  };
  // A next-use hint for range `id` of `bytes` at op-clock `now` (the hint's
  // time `when` > now). Returns the class flag to OR into the hint (0 or
  // kEvictFirst). `view` is consulted when classes are (re)assigned.
  uint64_t on_hint(uint64_t id, uint64_t bytes, const std::function<ArenaView()>& view);
  // An HBM chunk of range `id` was evicted.
  void on_evict(uint64_t id);
  // A prefetch of `bytes` of range `id` ahead of its use (a victim floor was
  // given): until its use is hinted the data occupies the prefetch window. The
  // peak window (+ the largest range, the one in use) is held back from the
  // keep class - the runtime's version of a planner's staging slots.
  void on_prefetch(uint64_t id, uint64_t bytes);
  void reset();
  int range_class(uint64_t id);  // -1 unknown, 0 keep, 1 stream
  // Introspection (stats / tests).
  struct Stats {
    bool ready = false;
    uint64_t ranges = 0, cycle_bytes = 0, keep_ranges = 0, keep_bytes = 0, passes = 0, keep_evictions = 0,
             adaptations = 0, window_reserve = 0, last_pass_keep_evictions = 0;
    double keep_fraction = 0.0;
  };
  Stats stats();

 private:
  struct Entry {
    uint64_t bytes = 0;
    uint32_t order = 0;
    int8_t cls = -1;  // -1 unassigned, 0 keep, 1 stream
  };
  void assign_locked(const std::function<ArenaView()>& view);
  std::mutex m_;
  std::unordered_map<uint64_t, Entry> ranges_;
  std::vector<uint64_t> order_;
  uint64_t cycle_bytes_ = 0;
  uint64_t assigned_bytes_ = 0;  // cycle bytes at the last assignment
  bool ready_ = false;
  double f_ = 0.0;
  double acc_ = 0.0;           // error-diffusion accumulator (continues for ranges appended later)
  double scale_ = 1.0;         // online adaptation factor on keep_pct
  uint64_t passes_ = 0, keep_evictions_ = 0, pass_keep_evictions_ = 0, adaptations_ = 0;
  std::unordered_map<uint64_t, std::pair<uint64_t, uint64_t>> pending_;  // prefetched, unused: id -> (bytes, pass)
  uint64_t pending_bytes_ = 0, max_range_bytes_ = 0;
  uint64_t reserve_ = 0, assigned_reserve_ = 0;
  uint64_t grace_until_ = 0;
  uint64_t last_pass_keep_evictions_ = 0;  // no adaptation before this pass (transition after an assignment)  // peak window + largest range; at the last assignment
};

}  // namespace ogkm
