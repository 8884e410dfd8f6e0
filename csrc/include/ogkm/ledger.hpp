// Node-wide host / CXL capacity ledger shared by every runtime process on the
// machine (one process per GPU: 8 ranks on 2 sockets).
//
// The reference keeps one global, spinlock-protected pin budget (90% of RAM)
// for every CXL buffer in the kernel (nv-p2p.c:1034-1111 cxl_pinned_tracker_t).
// A user-space runtime per GPU has no kernel to share state in: without a
// common ledger each rank sizes its host and CXL arenas from the whole
// machine's RAM and binds them to one node, so 8 ranks can commit several
// times a socket's memory and meet the OOM killer instead of a refusal.
//
// The ledger is a small shared-memory file (default /dev/shm/ogkm-node-ledger-
// <uid>; RT env OGKM_NODE_LEDGER overrides the path) holding, per NUMA node, a
// byte budget (the node's MemTotal x cxl_pin_budget_pct, or node_budget_mb)
// and the bytes reserved on it, plus one slot per attached process with its
// own reservations. Host arenas reserve a segment before they populate and pin
// it and return it when they are destroyed; reservations are lock-free CAS
// updates on the shared counters (clamped at zero on release); attach's
// liveness scan, reset and slot claim run under an flock on the file. A process that died without releasing is
// reclaimed by the next process whose reservation does not fit (its pid no
// longer exists).
#pragma once

#include <cstdint>
#include <mutex>
#include <string>

#include "ogkm/common.hpp"

namespace ogkm {

class NodeLedger {
 public:
  static NodeLedger& get();
  // Map (and on first use create) the shared ledger; idempotent. A failure
  // (no /dev/shm) leaves the ledger detached: reserve() then always succeeds.
  Status attach();
  void detach();  // return this process's reservations and slot
  bool attached() const { return sh_ != nullptr; }
  // Reserve `bytes` on `node`; false (and nothing reserved) when the node's
  // budget would be exceeded even after reclaiming dead processes' slots.
  bool reserve(int node, uint64_t bytes);
  void release(int node, uint64_t bytes);
  struct NodeView {
    uint64_t capacity = 0, reserved = 0, mine = 0;
  };
  NodeView view(int node);
  std::string path() const { return path_; }
  uint64_t refusals() const { return refusals_; }
  // Incremented by every attach: a reservation made under an earlier
  // attachment must not be released into a later one.
  uint64_t epoch() const { return epoch_; }

  static constexpr uint64_t kMagic = 0x4f474b4d4c444752ull;  // "OGKMLDGR"
  static constexpr uint32_t kSlots = 256;
  struct Slot {
    int32_t pid;
    uint32_t pad;
    uint64_t reserved[kMaxNodes];
  };
  struct Shared {
    uint64_t magic;      // kMagic once initialised (1 while the creator fills it in)
    uint32_t version;
    uint32_t nnodes;
    uint64_t capacity[kMaxNodes];
    uint64_t reserved[kMaxNodes];
    Slot slots[kSlots];
  };

 private:
  bool reclaim_dead();         // takes the file lock
  bool reclaim_dead_locked();  // caller holds it
  std::mutex m_;
  int lock_fd_ = -1;  // the ledger file: flock'ed around attach / reclaim
  Shared* sh_ = nullptr;
  Slot* mine_ = nullptr;
  std::string path_;
  uint64_t refusals_ = 0;
  uint64_t epoch_ = 0;
};

// Set by a host arena when the ledger refused a segment on the calling thread
// (cleared by the caller before the allocation it wants to judge).
inline bool& ledger_refused() {
  static thread_local bool refused = false;
  return refused;
}

// Bytes of memory on NUMA node `node` (sysfs MemTotal; 0 when unknown).
uint64_t node_mem_bytes(int node);
// The per-node budget: node_budget_mb when set, else the node's memory x
// cxl_pin_budget_pct (falls back to system RAM for a node sysfs does not list).
uint64_t node_budget_bytes(int node);

}  // namespace ogkm
