// Lock-order checker (uvm_lock.c:75-145 semantics).
#include "ogkm/lock_order.hpp"

#include <cstdlib>

#include "ogkm/common.hpp"
#include "ogkm/config.hpp"

namespace ogkm {

const char* lock_order_name(LockOrder o) {
  static const char* n[] = {"GLOBAL_PM",  "GLOBAL",    "VA_SPACE",   "CXL_REGISTRY", "RANGE_GROUP",
                            "RANGE_PLACE", "VA_BLOCK", "PERF",       "HBM_ARENA",    "HOST_ARENA",
                            "STREAM_POOL", "RING",     "TOOLS",      "LEAF"};
  int i = (int)o;
  return i >= 0 && i < (int)LockOrder::COUNT ? n[i] : "?";
}

namespace lockcheck {
namespace {
thread_local uint32_t t_held = 0;        // bit per order currently held
thread_local uint32_t t_out_of_order = 0;  // held via trylock out of order
thread_local uint16_t t_depth[(int)LockOrder::COUNT] = {0};
std::atomic<uint64_t> g_violations{0};
std::atomic<int> g_enabled{-1};
}  // namespace

bool enabled() {
  int e = g_enabled.load(std::memory_order_relaxed);
  if (e < 0) {
    e = config().lock_check ? 1 : 0;
    g_enabled.store(e);
  }
  return e != 0;
}

void set_enabled(bool on) { g_enabled.store(on ? 1 : 0); }

void on_acquire(LockOrder o, bool trylock) {
  if (!enabled()) return;
  uint32_t bit = 1u << (int)o;
  // Any held lock of equal or deeper order is a violation (trylocks exempt).
  uint32_t deeper_or_equal = t_held & ~((bit)-1);
  if (deeper_or_equal & ~t_out_of_order) {
    if (trylock) {
      t_out_of_order |= bit;
    } else {
      g_violations.fetch_add(1);
      int worst = 31 - __builtin_clz(deeper_or_equal);
      RT_ERR("lock order violation: acquiring %s while holding %s", lock_order_name(o),
             lock_order_name((LockOrder)worst));
      static const bool abort_on = getenv("RT_LOCKCHECK_ABORT") != nullptr;  // debugging: stop at the culprit
      if (abort_on) abort();
    }
  }
  t_held |= bit;
  t_depth[(int)o]++;
}

void on_release(LockOrder o) {
  if (!enabled()) return;
  uint32_t bit = 1u << (int)o;
  if (t_depth[(int)o] > 0 && --t_depth[(int)o] == 0) {
    t_held &= ~bit;
    t_out_of_order &= ~bit;
  }
}

uint64_t violations() { return g_violations.load(); }
void reset_violations() { g_violations.store(0); }
uint32_t held_mask() { return t_held; }
}  // namespace lockcheck

}  // namespace ogkm
