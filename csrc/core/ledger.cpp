// Node-wide capacity ledger (see ogkm/ledger.hpp).
#include "ogkm/ledger.hpp"

#include <fcntl.h>
#include <signal.h>
#include <sys/file.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>

#include "ogkm/config.hpp"
#include "ogkm/cxl.hpp"

namespace ogkm {

uint64_t node_mem_bytes(int node) {
  char path[96];
  snprintf(path, sizeof(path), "/sys/devices/system/node/node%d/meminfo", node);
  FILE* f = fopen(path, "r");
  if (!f) return 0;
  char line[256];
  uint64_t kb = 0;
  while (fgets(line, sizeof(line), f)) {
    const char* p = strstr(line, "MemTotal:");
    if (p) {
      kb = strtoull(p + 9, nullptr, 10);
      break;
    }
  }
  fclose(f);
  return kb << 10;
}

uint64_t node_budget_bytes(int node) {
  if (config().node_budget_mb > 0) return (uint64_t)config().node_budget_mb << 20;
  uint64_t mem = node_mem_bytes(node);
  if (!mem) mem = system_ram_bytes();
  return mem / 100 * (uint64_t)config().cxl_pin_budget_pct;
}

NodeLedger& NodeLedger::get() {
  static NodeLedger l;
  return l;
}

Status NodeLedger::attach() {
  std::lock_guard<std::mutex> g(m_);
  if (sh_) return Status::OK;
  if (!config().node_ledger) return Status::NOT_SUPPORTED;
  const char* env = getenv("OGKM_NODE_LEDGER");
  if (env && *env) {
    path_ = env;
  } else {
    char buf[96];
    snprintf(buf, sizeof(buf), "/dev/shm/ogkm-node-ledger-%u", (unsigned)getuid());
    path_ = buf;
  }
  int fd = open(path_.c_str(), O_RDWR | O_CREAT | O_CLOEXEC, 0600);
  if (fd < 0) {
    RT_WARN("node ledger %s unavailable (errno %d): host / CXL budgets are per process", path_.c_str(), errno);
    return Status::IO_ERROR;
  }
  // Every structural change of the ledger (first initialisation, the reset of
  // a file nobody uses any more, slot claims and dead-slot reclaims) happens
  // under an exclusive flock on the file: 8 ranks starting together on a file
  // left by a crashed job must not interleave "nobody is live" scans with
  // another rank's reset and claim (a reset after a claim would wipe the
  // claimer's reservations and let its releases underflow the node counter).
  // The kernel drops the lock with the descriptor, so a rank that dies inside
  // never blocks the others. Reservations themselves stay lock-free CAS.
  while (flock(fd, LOCK_EX) != 0) {
    if (errno != EINTR) {
      close(fd);
      return Status::IO_ERROR;
    }
  }
  struct stat st;
  if (fstat(fd, &st) != 0 || ((uint64_t)st.st_size < sizeof(Shared) && ftruncate(fd, sizeof(Shared)) != 0)) {
    close(fd);
    return Status::IO_ERROR;
  }
  void* p = mmap(nullptr, sizeof(Shared), PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  if (p == MAP_FAILED) {
    close(fd);
    return Status::IO_ERROR;
  }
  Shared* s = (Shared*)p;
  // A ledger nobody uses any more (never initialised, a creator that died
  // mid-way, or every slot free or its process gone) is (re-)initialised:
  // budgets from this process's configuration, nothing reserved - a file left
  // behind by an earlier job (or a test's budget) must not constrain this one.
  bool live = false;
  if (__atomic_load_n(&s->magic, __ATOMIC_ACQUIRE) == kMagic) {
    for (uint32_t i = 0; i < kSlots && !live; ++i) {
      const int32_t pid = __atomic_load_n(&s->slots[i].pid, __ATOMIC_ACQUIRE);
      live = pid != 0 && (pid < 0 || kill(pid, 0) == 0 || errno != ESRCH);
    }
  }
  // (test hook: widen the scan -> reset window, tests/test_node_ledger.py)
  if (const char* d = getenv("OGKM_LEDGER_TEST_DELAY_US"))
    std::this_thread::sleep_for(std::chrono::microseconds(atoi(d)));
  if (!live) {
    __atomic_store_n(&s->magic, 1ull, __ATOMIC_RELEASE);  // reserve() waits while this is not kMagic
    s->version = 1;
    s->nnodes = kMaxNodes;
    for (int n = 0; n < kMaxNodes; ++n) {
      s->capacity[n] = node_budget_bytes(n);
      __atomic_store_n(&s->reserved[n], 0ull, __ATOMIC_RELEASE);
    }
    for (uint32_t i = 0; i < kSlots; ++i) {
      s->slots[i].pid = 0;
      memset(s->slots[i].reserved, 0, sizeof(s->slots[i].reserved));
    }
    __atomic_store_n(&s->magic, kMagic, __ATOMIC_RELEASE);
  }
  sh_ = s;
  ++epoch_;
  const int32_t me = (int32_t)getpid();
  for (int pass = 0; pass < 2 && !mine_; ++pass) {
    for (uint32_t i = 0; i < kSlots; ++i) {
      int32_t free_pid = 0;
      if (__atomic_compare_exchange_n(&s->slots[i].pid, &free_pid, me, false, __ATOMIC_ACQ_REL, __ATOMIC_ACQUIRE)) {
        memset(s->slots[i].reserved, 0, sizeof(s->slots[i].reserved));
        mine_ = &s->slots[i];
        break;
      }
    }
    if (!mine_) reclaim_dead_locked();
  }
  lock_fd_ = fd;  // kept for reclaim_dead(); unlocked here
  flock(fd, LOCK_UN);
  if (!mine_) RT_WARN("node ledger %s: no free process slot (reservations are global only)", path_.c_str());
  return Status::OK;
}

// Subtract `b` from a shared counter, never below zero (a release that does not
// match a reservation - e.g. one made before a reset - must not wrap the
// counter to ~2^64 and make every later reservation on the node fail).
static void sub_clamped(uint64_t* c, uint64_t b) {
  uint64_t cur = __atomic_load_n(c, __ATOMIC_ACQUIRE);
  while (!__atomic_compare_exchange_n(c, &cur, cur > b ? cur - b : 0ull, true, __ATOMIC_ACQ_REL, __ATOMIC_ACQUIRE)) {
  }
}

bool NodeLedger::reclaim_dead() {
  if (lock_fd_ < 0) return reclaim_dead_locked();
  while (flock(lock_fd_, LOCK_EX) != 0 && errno == EINTR) {
  }
  const bool any = reclaim_dead_locked();
  flock(lock_fd_, LOCK_UN);
  return any;
}

// Slots of processes that no longer exist: their reservations go back to the
// nodes (caller holds the file lock).
bool NodeLedger::reclaim_dead_locked() {
  bool any = false;
  for (uint32_t i = 0; i < kSlots; ++i) {
    Slot& sl = sh_->slots[i];
    int32_t pid = __atomic_load_n(&sl.pid, __ATOMIC_ACQUIRE);
    if (pid <= 0 || pid == (int32_t)getpid()) continue;
    if (kill(pid, 0) == 0 || errno != ESRCH) continue;
    // Claim the dead slot (-pid marks it being reclaimed), return its bytes, free it.
    if (!__atomic_compare_exchange_n(&sl.pid, &pid, -pid, false, __ATOMIC_ACQ_REL, __ATOMIC_ACQUIRE)) continue;
    for (int n = 0; n < kMaxNodes; ++n) {
      uint64_t b = __atomic_exchange_n(&sl.reserved[n], 0ull, __ATOMIC_ACQ_REL);
      if (b) sub_clamped(&sh_->reserved[n], b);
    }
    __atomic_store_n(&sl.pid, 0, __ATOMIC_RELEASE);
    any = true;
    RT_INFO("node ledger: reclaimed the reservations of exited process %d", (int)pid);
  }
  return any;
}

bool NodeLedger::reserve(int node, uint64_t bytes) {
  if (!sh_ || node < 0 || node >= kMaxNodes || !bytes) return true;
  // (a re-initialisation in progress - only ever of a ledger without live
  // slots, i.e. this process has none - finishes first)
  while (__atomic_load_n(&sh_->magic, __ATOMIC_ACQUIRE) != kMagic) std::this_thread::yield();
  for (int attempt = 0; attempt < 2; ++attempt) {
    uint64_t cur = __atomic_load_n(&sh_->reserved[node], __ATOMIC_ACQUIRE);
    const uint64_t cap = sh_->capacity[node];
    bool fits = true;
    while (true) {
      if (cur + bytes > cap) {
        fits = false;
        break;
      }
      if (__atomic_compare_exchange_n(&sh_->reserved[node], &cur, cur + bytes, true, __ATOMIC_ACQ_REL,
                                      __ATOMIC_ACQUIRE))
        break;
    }
    if (fits) {
      if (mine_) __atomic_fetch_add(&mine_->reserved[node], bytes, __ATOMIC_ACQ_REL);
      return true;
    }
    if (attempt == 0 && !reclaim_dead()) break;
  }
  ++refusals_;
  return false;
}

void NodeLedger::release(int node, uint64_t bytes) {
  if (!sh_ || node < 0 || node >= kMaxNodes || !bytes) return;
  sub_clamped(&sh_->reserved[node], bytes);
  if (mine_) sub_clamped(&mine_->reserved[node], bytes);
}

NodeLedger::NodeView NodeLedger::view(int node) {
  NodeView v;
  if (!sh_ || node < 0 || node >= kMaxNodes) return v;
  v.capacity = sh_->capacity[node];
  v.reserved = __atomic_load_n(&sh_->reserved[node], __ATOMIC_ACQUIRE);
  v.mine = mine_ ? __atomic_load_n(&mine_->reserved[node], __ATOMIC_ACQUIRE) : 0;
  return v;
}

void NodeLedger::detach() {
  std::lock_guard<std::mutex> g(m_);
  if (!sh_) return;
  if (mine_) {
    for (int n = 0; n < kMaxNodes; ++n) {
      uint64_t b = __atomic_exchange_n(&mine_->reserved[n], 0ull, __ATOMIC_ACQ_REL);
      if (b) sub_clamped(&sh_->reserved[n], b);
    }
    __atomic_store_n(&mine_->pid, 0, __ATOMIC_RELEASE);
    mine_ = nullptr;
  }
  munmap(sh_, sizeof(Shared));
  sh_ = nullptr;
  if (lock_fd_ >= 0) close(lock_fd_);
  lock_fd_ = -1;
}

}  // namespace ogkm
