// Performance heuristics: residency selection, bitmap-tree prefetch and
// thrashing detection.
//
//  * select_residency   - the rules of block_select_processor_residency,
//                         uvm_va_block.c:11560-11712 (read duplication, preferred
//                         location, thrashing pin, accessed_by, remote mapping).
//  * prefetch_hint      - uvm_perf_prefetch.c:102-250: prefetch the largest
//                         aligned subregion whose resident+faulted fraction exceeds
//                         perf_prefetch_threshold (51%).
//  * thrashing          - uvm_perf_thrashing.c:241-314: >= threshold migrations
//                         within `lapse` -> THROTTLE; >= pin_threshold throttles ->
//                         PIN (map remotely) for pin*lapse; epoch resets.
#include <algorithm>

#include "ogkm/runtime.hpp"

namespace ogkm {

static bool accessible(Runtime* rt, const Loc& l, int proc) {
  if (proc == kCpuProc) return !l.is_gpu();
  if (!l.is_gpu()) return true;  // registered host / CXL memory over PCIe
  if (l.id == proc) return true;
  for (auto& p : rt->vs().peer_pairs)
    if (p.first == proc && p.second == l.id) return !((rt->inject().peer_link_down.load() >> l.id) & 1);
  return false;
}

// Closest location holding any of `pages`: own memory, then peers, then host, then CXL.
static bool closest_resident(Runtime* rt, Block* b, int proc, const PageMask& pages, Loc* out) {
  Loc me = rt->proc_loc(proc);
  int best = 1 << 30;
  bool found = false;
  for (auto& r : b->res) {
    if (!r.resident.intersects(pages)) continue;
    int rank;
    if (r.loc == me) rank = 0;
    else if (r.loc.is_gpu()) rank = proc == kCpuProc ? 4 : 1;
    else if (r.loc.tier == Tier::HOST) rank = 2;
    else rank = 3;
    if (rank < best) {
      best = rank;
      *out = r.loc;
      found = true;
    }
  }
  return found;
}

ResidencyDecision select_residency(Runtime* rt, Block* b, int proc, Access access, const PageMask& pages) {
  ResidencyDecision d;
  Loc me = rt->proc_loc(proc);
  uint64_t now = now_ns();
  if (config().fault_force_sysmem) {
    d.dst = rt->cpu_loc();
    d.map_remote = proc != kCpuProc;
    return d;
  }
  Loc closest;
  bool have_closest = closest_resident(rt, b, proc, pages, &closest);
  // Frozen residency (non-migratable range group / user pin): access in place.
  if ((b->range->group && !b->range->group->migratable) || b->user_pins) {
    if (have_closest && accessible(rt, closest, proc)) {
      d.dst = closest;
      d.map_remote = !(closest == me);
      return d;
    }
  }
  bool pinned = thrash_pinned(b, now);
  bool may_dup = b->policy.read_dup && !pinned;
  if (may_dup) {
    d.dst = me;
    d.read_dup = access == Access::READ || access == Access::PREFETCH;
    return d;
  }
  const Policy& pol = b->policy;
  if (pol.has_preferred && pol.preferred == me) {
    d.dst = me;
    return d;
  }
  if (pinned && have_closest && accessible(rt, closest, proc)) {
    d.dst = closest;
    d.map_remote = !(closest == me);
    return d;
  }
  if (!have_closest) {
    if (pol.has_preferred && accessible(rt, pol.preferred, proc)) {
      d.dst = pol.preferred;
      d.map_remote = !(pol.preferred == me);
      return d;
    }
    d.dst = me;
    return d;
  }
  int pbit = proc == kCpuProc ? kCpuProc : proc;
  bool& hot = b->counters.promote[proc == kCpuProc ? kMaxGpus : proc];
  if (hot && proc != kCpuProc) {
    // Access counters found the remote mapping hot: migrate it here.
    hot = false;
    Tools::get().inc(Counter::AccessCounterMigrations);
    d.dst = me;
    return d;
  }
  if (((pol.accessed_by >> pbit) & 1) && accessible(rt, closest, proc)) {
    d.dst = closest;
    d.map_remote = !(closest == me);
    return d;
  }
  if (access == Access::ATOMIC && config().perf_map_remote_on_native_atomics_fault && accessible(rt, closest, proc)) {
    d.dst = closest;
    d.map_remote = !(closest == me);
    return d;
  }
  if (!(closest == me) && pol.has_preferred && accessible(rt, pol.preferred, proc)) {
    d.dst = pol.preferred;
    d.map_remote = !(pol.preferred == me);
    return d;
  }
  d.dst = me;
  return d;
}

PageMask prefetch_hint(const PageMask& resident_on_dst, const PageMask& faulted, uint32_t npages, uint32_t thr) {
  PageMask out;
  PageMask have = resident_on_dst | faulted;
  PageMask valid = PageMask::range(0, npages);
  uint32_t p = faulted.next_set(0);
  while (p < npages) {
    // A faulted page inside a region already chosen would choose that same
    // region (its larger ancestors did not qualify): skip it.
    if (!out.test(p)) {
      // Largest aligned region first (the root of the bitmap tree), then descend.
      for (int lvl = 9; lvl >= 0; --lvl) {
        uint32_t size = 1u << lvl;
        uint32_t start = p & ~(size - 1);
        if (start >= npages) continue;
        uint32_t len = std::min(size, npages - start);
        if (have.count_range(start, len) * 100 > thr * len) {
          out.set_range(start, len);
          p = start + len - 1;  // continue after the region
          break;
        }
      }
    }
    p = faulted.next_set(p + 1);
  }
  return out & valid;
}

ThrashHint thrash_on_migration(Block* b, int dst_slot, uint64_t now) {
  if (!config().perf_thrashing_enable) return ThrashHint::NONE;
  ThrashState& t = b->thrash;
  uint64_t lapse = (uint64_t)config().perf_thrashing_lapse_usec * 1000;
  if (t.epoch_start_ns == 0) t.epoch_start_ns = now;
  if (now - t.epoch_start_ns > lapse * (uint64_t)config().perf_thrashing_epoch) {
    if (t.resets < (uint32_t)config().perf_thrashing_max_resets) {
      t.resets++;
      t.events_in_window = 0;
      t.throttles = 0;
      t.detected = false;
    }
    t.epoch_start_ns = now;
  }
  ThrashHint h = ThrashHint::NONE;
  if (t.last_dst_slot >= 0 && t.last_dst_slot != dst_slot) {
    if (now - t.window_start_ns > lapse) {
      t.window_start_ns = now;
      t.events_in_window = 0;
    }
    t.events_in_window++;
    if (t.events_in_window >= (uint32_t)config().perf_thrashing_threshold) {
      if (!t.detected) Tools::get().inc(Counter::ThrashingDetected);
      t.detected = true;
      t.throttles++;
      h = ThrashHint::THROTTLE;
      Tools::get().inc(Counter::ThrottleEvents);
      tools_event(ToolsEventType::ThrashingDetected, Cause::Thrashing, Loc{}, Loc{}, 0, b->block_offset(), 0,
                  b->range->id);
      if (t.throttles >= (uint32_t)config().perf_thrashing_pin_threshold) {
        t.pinned_until_ns = now + lapse * (uint64_t)config().perf_thrashing_pin;
        t.throttles = 0;
        h = ThrashHint::PIN;
        Tools::get().inc(Counter::PinEvents);
      } else {
        // The processor that just pulled the block in naps: its next faults
        // on the block do not migrate it again until the nap ends.
        t.throttle_until_ns = now + lapse * (uint64_t)std::max<int64_t>(1, config().perf_thrashing_nap);
        t.throttle_slot = dst_slot;
        if (!t.throttling)
          tools_event(ToolsEventType::ThrottlingStart, Cause::Thrashing, Loc{}, Loc{}, dst_slot,
                      b->range->addr() + b->block_offset(), kBlockSize, b->range->id);
        t.throttling = true;
      }
    }
  }
  t.last_dst_slot = dst_slot;
  t.last_migration_ns = now;
  return h;
}

ThrashHint thrash_hint(Block* b, int slot, uint64_t now) {
  ThrashState& t = b->thrash;
  if (t.pinned_until_ns > now) return ThrashHint::PIN;
  if (t.throttling && now >= t.throttle_until_ns) {
    t.throttling = false;
    tools_event(ToolsEventType::ThrottlingEnd, Cause::Thrashing, Loc{}, Loc{}, t.throttle_slot,
                b->range->addr() + b->block_offset(), kBlockSize, b->range->id);
  }
  if (t.throttling && slot == t.throttle_slot) return ThrashHint::THROTTLE;
  return ThrashHint::NONE;
}

// ---------------------------------------------------------------- perf modules
// Thrashing module: consumes MIGRATION events (state update + hints on the
// block); prefetch module: consumes FAULT events (per-processor fault counts
// that gate the bitmap-tree prefetch). Callbacks run with the block lock held.
std::vector<int> perf_modules_register(PerfEventBus& bus) {
  std::vector<int> tok;
  tok.push_back(bus.subscribe(PerfEvent::MIGRATION, [](const PerfEventData& d) {
    auto* b = static_cast<Block*>(d.block);
    if (!b || !d.moved || d.cause == (int)Cause::Eviction) return;
    thrash_on_migration(b, d.dst.slot(), now_ns());
  }));
  tok.push_back(bus.subscribe(PerfEvent::FAULT, [](const PerfEventData& d) {
    auto* b = static_cast<Block*>(d.block);
    if (!b) return;
    b->faults_by_proc[d.processor == kCpuProc ? kMaxGpus : d.processor]++;
  }));
  return tok;
}

bool thrash_pinned(Block* b, uint64_t now) { return b->thrash.pinned_until_ns > now; }

}  // namespace ogkm
