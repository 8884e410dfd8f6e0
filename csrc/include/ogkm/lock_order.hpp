// Lock-order checker (analog of uvm_lock.c:75-145 / uvm_lock.h:504-546).
//
// Every runtime lock has an order. A thread may only acquire a lock whose order
// is strictly greater than every order it already holds; trylocks are exempt
// (recorded as out-of-order holders, as __uvm_record_lock does). Per-thread
// state lives in a thread_local bitmap (uvm_thread_context.h:36-98 analog).
// The checker is enabled by the `lock_check` knob; violations are counted,
// logged, and visible through rt.stats()["lock_violations"].
#pragma once

#include <atomic>
#include <cstdint>
#include <mutex>
#include <shared_mutex>

namespace ogkm {

enum class LockOrder : int {
  GLOBAL_PM = 0,   // checkpoint quiesce / resume
  GLOBAL = 1,      // runtime registry (va spaces, devices)
  VA_SPACE = 2,    // range tree (reader/writer)
  CXL_REGISTRY = 3,
  RANGE_GROUP = 4,
  RANGE_PLACE = 5, // per-range GPU extent placement (serialises concurrent acquires of one range)
  VA_BLOCK = 6,    // per 2 MB block state
  PERF = 7,        // thrashing / prefetch / access-counter state
  HBM_ARENA = 8,   // per-GPU chunk allocator (taken under a block lock)
  HOST_ARENA = 9,
  STREAM_POOL = 10,
  RING = 11,       // SQ/CQ ring
  TOOLS = 12,      // event queues
  LEAF = 13,
  COUNT = 14
};
const char* lock_order_name(LockOrder o);

namespace lockcheck {
bool enabled();
void set_enabled(bool on);
void on_acquire(LockOrder o, bool trylock);
void on_release(LockOrder o);
uint64_t violations();
void reset_violations();
uint32_t held_mask();  // current thread's held orders (for tests / asserts)
}  // namespace lockcheck

class OrderedMutex {
 public:
  explicit OrderedMutex(LockOrder o) : order_(o) {}
  void lock() { lockcheck::on_acquire(order_, false); m_.lock(); }
  bool try_lock() {
    if (!m_.try_lock()) return false;
    lockcheck::on_acquire(order_, true);
    return true;
  }
  void unlock() { m_.unlock(); lockcheck::on_release(order_); }
  LockOrder order() const { return order_; }

 private:
  std::mutex m_;
  LockOrder order_;
};

class OrderedRWLock {
 public:
  explicit OrderedRWLock(LockOrder o) : order_(o) {}
  void lock() { lockcheck::on_acquire(order_, false); m_.lock(); }
  void unlock() { m_.unlock(); lockcheck::on_release(order_); }
  void lock_shared() { lockcheck::on_acquire(order_, false); m_.lock_shared(); }
  void unlock_shared() { m_.unlock_shared(); lockcheck::on_release(order_); }
  bool try_lock_shared() {
    if (!m_.try_lock_shared()) return false;
    lockcheck::on_acquire(order_, true);
    return true;
  }

 private:
  std::shared_mutex m_;
  LockOrder order_;
};

}  // namespace ogkm
