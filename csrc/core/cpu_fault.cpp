// CPU faults on managed CPU views (the UVM CPU-fault path: uvm_vm_fault,
// uvm.c:576 -> uvm_va_space_cpu_fault, uvm_va_space.c:2482-2590), made
// async-signal-safe.
//
// A CPU view is a PROT_NONE reservation whose 2 MB windows are mapped onto host
// / CXL arena pages on demand; touching a page that is not mapped for the access
// raises SIGSEGV. Servicing a fault takes runtime locks, allocates and calls
// mmap / mprotect - none of which may run inside a signal handler (a fault taken
// while the thread holds a runtime lock or is inside malloc would deadlock). So:
//
//   * the handler only (1) finds out, lock-free, whether the address belongs to
//     a CPU view (an immutable sorted table published with release/acquire and
//     replaced, never edited, when ranges come and go), (2) posts the fault into
//     a slot of a static array, (3) wakes the service thread and sleeps on the
//     slot with futex - raw syscalls and atomics only;
//   * the CPU-fault service thread (the analog of the bottom half that services
//     a fault batch outside the interrupt context) runs Runtime::cpu_fault()
//     for the slot, publishes the result and wakes the faulting thread, which
//     returns from the handler and re-executes the access.
//
// A fault on an address outside every view, or one the runtime cannot service,
// is passed to the previously installed handler (or the default action).
#include <linux/futex.h>
#include <signal.h>
#include <sys/syscall.h>
#include <time.h>
#include <ucontext.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

#include "ogkm/runtime.hpp"

namespace ogkm {

namespace {

// ---------------------------------------------------------------- view index
struct ViewTable {
  size_t n = 0;
  std::vector<uint64_t> start, end;  // sorted by start
};
std::atomic<const ViewTable*> g_views{nullptr};
std::mutex g_views_m;                              // writers only
std::vector<const ViewTable*> g_retired;           // old tables (a handler may still read one)
std::atomic<int> g_readers{0};                     // handlers between entering and leaving in_view

// Retired tables are freed once no handler is inside in_view: a handler that
// enters later loads the table already published (seq_cst on both sides).
void reclaim_locked() {
  if (g_readers.load(std::memory_order_seq_cst) != 0) return;
  for (const ViewTable* t : g_retired) delete t;
  g_retired.clear();
}

bool in_view(uint64_t a) {
  g_readers.fetch_add(1, std::memory_order_seq_cst);
  const ViewTable* t = g_views.load(std::memory_order_seq_cst);
  bool hit = false;
  if (t && t->n) {
    size_t lo = 0, hi = t->n;
    while (lo < hi) {  // first start > a
      size_t mid = (lo + hi) / 2;
      if (t->start[mid] <= a) lo = mid + 1;
      else hi = mid;
    }
    hit = lo > 0 && a < t->end[lo - 1];
  }
  g_readers.fetch_sub(1, std::memory_order_seq_cst);
  return hit;
}

// ---------------------------------------------------------------- fault slots
constexpr int kSlots = 256;
// FREE -> CLAIMED (handler) -> POSTED (handler) -> SERVICING (service thread,
// CAS) -> DONE (service) -> FREE (handler). A BUSY slot goes SERVICING -> POSTED
// again with a not-before time, so it is retried in a LATER batch and never
// holds up the other posted faults.
enum : int { SLOT_FREE = 0, SLOT_CLAIMED = 1, SLOT_POSTED = 2, SLOT_SERVICING = 3, SLOT_DONE = 4 };
struct alignas(64) FaultSlot {
  std::atomic<int> state{SLOT_FREE};
  uint64_t addr = 0;
  int write = 0;
  int result = 0;
  // service thread only
  uint64_t retry_at_ns = 0;
  int busy_tries = 0;
};
FaultSlot g_slots[kSlots];
std::atomic<int> g_posted{0};  // futex word of the service thread: number of posts ever made
std::atomic<bool> g_service_up{false};
std::atomic<pid_t> g_service_tid{0};
std::atomic<uint64_t> g_serviced{0}, g_passed_on{0};
constexpr int kBusyTries = 20000;  // ~10 s of BUSY retries (20 us, then 500 us apart)

long futex(std::atomic<int>* w, int op, int val, const struct timespec* ts = nullptr) {
  return syscall(SYS_futex, reinterpret_cast<int*>(w), op, val, ts, nullptr, 0);
}

uint64_t mono_ns() {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return (uint64_t)t.tv_sec * 1000000000ull + (uint64_t)t.tv_nsec;
}

std::atomic<bool> g_service_stop{false};
// Heap-held so a process that exits without shutting the runtime down does not
// destroy a joinable std::thread (std::terminate) in static destructors.
std::thread* g_service = nullptr;

void complete(FaultSlot& s, Status st) {
  s.result = (int)st;
  g_serviced.fetch_add(1, std::memory_order_relaxed);
  s.state.store(SLOT_DONE, std::memory_order_release);
  futex(&s.state, FUTEX_WAKE_PRIVATE, 1);
}

// Bottom half: every posted fault is serviced in ONE batch (one
// service_faults call: coalescing, one copy submission, one wait), then the
// faulting threads are woken - the batch service of
// uvm_gpu_replayable_faults.c:2906 applied to CPU faults.
void service_loop() {
  g_service_tid.store((pid_t)syscall(SYS_gettid));
  int seen = 0;
  uint64_t next_retry = 0;  // earliest not-before time of a BUSY slot (0 = none)
  std::vector<FaultSlot*> batch;
  std::vector<std::pair<uint64_t, bool>> req;
  std::vector<Status> res;
  while (!g_service_stop.load(std::memory_order_acquire)) {
    int now = g_posted.load(std::memory_order_acquire);
    const uint64_t t = mono_ns();
    if (now == seen && (!next_retry || t < next_retry)) {
      if (next_retry) {
        struct timespec ts{0, (long)std::min<uint64_t>(next_retry - t, 1000000)};
        futex(&g_posted, FUTEX_WAIT_PRIVATE, seen, &ts);
      } else {
        futex(&g_posted, FUTEX_WAIT_PRIVATE, seen);
      }
      continue;
    }
    seen = now;
    next_retry = 0;
    batch.clear();
    req.clear();
    for (auto& s : g_slots) {
      if (s.state.load(std::memory_order_acquire) != SLOT_POSTED) continue;
      if (s.busy_tries && s.retry_at_ns > t) {
        next_retry = next_retry ? std::min(next_retry, s.retry_at_ns) : s.retry_at_ns;
        continue;
      }
      int expect = SLOT_POSTED;  // the handler may take a slot back once the service is down
      if (!s.state.compare_exchange_strong(expect, SLOT_SERVICING, std::memory_order_acq_rel)) continue;
      batch.push_back(&s);
      req.emplace_back(s.addr, s.write != 0);
    }
    if (batch.empty()) continue;
    Runtime* rt = Runtime::get();
    res.assign(batch.size(), Status::NOT_FOUND);
    if (rt) rt->cpu_fault_batch(req, &res);
    const uint64_t t1 = mono_ns();
    for (size_t k = 0; k < batch.size(); ++k) {
      FaultSlot& s = *batch[k];
      Status st = res[k];
      // BUSY: a GPU lease pins the only copy (the GPU may be writing it); the
      // CPU access waits for the release, like a CPU fault on a block whose GPU
      // mapping cannot be revoked yet (uvm_va_space.c:2540-2590 retries) - in a
      // later batch, so the rest of this one completes now.
      if (rt && st == Status::BUSY && s.busy_tries < kBusyTries) {
        s.retry_at_ns = t1 + (s.busy_tries < 100 ? 20000ull : 500000ull);
        s.busy_tries++;
        next_retry = next_retry ? std::min(next_retry, s.retry_at_ns) : s.retry_at_ns;
        s.state.store(SLOT_POSTED, std::memory_order_release);
        continue;
      }
      s.busy_tries = 0;
      complete(s, st);
    }
  }
  // Stopping: complete every fault still posted (NOT_FOUND -> the handler passes
  // it on) so no faulting thread sleeps forever on its slot.
  for (auto& s : g_slots) {
    int expect = SLOT_POSTED;
    if (s.state.compare_exchange_strong(expect, SLOT_SERVICING, std::memory_order_acq_rel)) {
      s.busy_tries = 0;
      complete(s, Status::NOT_FOUND);
    }
  }
}

struct sigaction g_prev_segv;
std::atomic<bool> g_handler_installed{false};

void pass_on(int sig, siginfo_t* si, void* uc) {
  g_passed_on.fetch_add(1, std::memory_order_relaxed);
  if (g_prev_segv.sa_flags & SA_SIGINFO) {
    if (g_prev_segv.sa_sigaction) {
      g_prev_segv.sa_sigaction(sig, si, uc);
      return;
    }
  } else if (g_prev_segv.sa_handler != SIG_DFL && g_prev_segv.sa_handler != SIG_IGN) {
    g_prev_segv.sa_handler(sig);
    return;
  }
  // Default action: reset and return; the access faults again and terminates.
  struct sigaction dfl;
  memset(&dfl, 0, sizeof dfl);
  dfl.sa_handler = SIG_DFL;
  sigaction(SIGSEGV, &dfl, nullptr);
}

// Async-signal-safe: atomics and raw syscalls only.
void segv_handler(int sig, siginfo_t* si, void* uc) {
  uint64_t addr = (uint64_t)si->si_addr;
  pid_t me = (pid_t)syscall(SYS_gettid);
  if (!in_view(addr) || !g_service_up.load(std::memory_order_acquire) || me == g_service_tid.load()) {
    pass_on(sig, si, uc);
    return;
  }
  bool write = false;
#if defined(__x86_64__)
  write = (((ucontext_t*)uc)->uc_mcontext.gregs[REG_ERR] & 2) != 0;
#endif
  FaultSlot* slot = nullptr;
  for (int spin = 0; !slot; ++spin) {
    for (auto& s : g_slots) {
      int f = SLOT_FREE;
      if (s.state.compare_exchange_strong(f, SLOT_CLAIMED, std::memory_order_acquire)) {
        slot = &s;
        break;
      }
    }
    if (!slot) syscall(SYS_sched_yield);  // more than kSlots threads faulting at once
  }
  slot->addr = addr;
  slot->write = write;
  slot->state.store(SLOT_POSTED, std::memory_order_release);
  g_posted.fetch_add(1, std::memory_order_acq_rel);
  futex(&g_posted, FUTEX_WAKE_PRIVATE, 1);
  // Bounded sleeps: if the service stopped after this thread passed the
  // g_service_up check (and after its final sweep), take the slot back and pass
  // the fault on instead of sleeping forever.
  for (;;) {
    int st = slot->state.load(std::memory_order_acquire);
    if (st == SLOT_DONE) break;
    struct timespec ts{0, 20 * 1000 * 1000};
    futex(&slot->state, FUTEX_WAIT_PRIVATE, st, &ts);
    if (!g_service_up.load(std::memory_order_acquire) && !g_service_tid.load()) {
      int expect = SLOT_POSTED;
      if (slot->state.compare_exchange_strong(expect, SLOT_FREE, std::memory_order_acq_rel)) {
        pass_on(sig, si, uc);
        return;
      }
    }
  }
  int result = slot->result;
  slot->state.store(SLOT_FREE, std::memory_order_release);
  if (result != (int)Status::OK) pass_on(sig, si, uc);
  // else: return and re-execute the access, now mapped.
}

}  // namespace

void cpu_views_add(uint64_t start, uint64_t bytes) {
  std::lock_guard<std::mutex> g(g_views_m);
  auto* t = new ViewTable();
  if (const ViewTable* old = g_views.load()) {
    t->start = old->start;
    t->end = old->end;
  }
  auto it = std::upper_bound(t->start.begin(), t->start.end(), start);
  size_t i = it - t->start.begin();
  t->start.insert(t->start.begin() + i, start);
  t->end.insert(t->end.begin() + i, start + bytes);
  t->n = t->start.size();
  if (const ViewTable* old = g_views.exchange(t, std::memory_order_seq_cst)) g_retired.push_back(old);
  reclaim_locked();
}

void cpu_views_remove(uint64_t start) {
  std::lock_guard<std::mutex> g(g_views_m);
  const ViewTable* old = g_views.load();
  if (!old) return;
  auto* t = new ViewTable();
  for (size_t i = 0; i < old->n; ++i)
    if (old->start[i] != start) {
      t->start.push_back(old->start[i]);
      t->end.push_back(old->end[i]);
    }
  t->n = t->start.size();
  if (t->n == 0) {  // no views left: nothing for a handler to read
    delete t;
    t = nullptr;
  }
  g_views.store(t, std::memory_order_seq_cst);
  g_retired.push_back(old);
  reclaim_locked();
}

void cpu_fault_stats(uint64_t* serviced, uint64_t* passed_on) {
  *serviced = g_serviced.load();
  *passed_on = g_passed_on.load();
}

// The service thread lives as long as a runtime does (Runtime::init /
// ~Runtime); faults outside that window are not ours to service.
void start_cpu_fault_service() {
  if (g_service) return;
  g_service_stop.store(false);
  g_service_tid.store(0);
  g_service = new std::thread(service_loop);
  while (!g_service_tid.load()) std::this_thread::yield();
  g_service_up.store(true, std::memory_order_release);
}

void stop_cpu_fault_service() {
  if (!g_service) return;
  g_service_up.store(false, std::memory_order_release);
  g_service_stop.store(true, std::memory_order_release);
  g_posted.fetch_add(1, std::memory_order_acq_rel);
  futex(&g_posted, FUTEX_WAKE_PRIVATE, 1);
  g_service->join();
  delete g_service;
  g_service = nullptr;
  g_service_tid.store(0);
}

void install_cpu_fault_handler() {
  bool expected = false;
  if (!g_handler_installed.compare_exchange_strong(expected, true)) return;
  struct sigaction sa;
  memset(&sa, 0, sizeof sa);
  sa.sa_sigaction = segv_handler;
  sa.sa_flags = SA_SIGINFO | SA_ONSTACK;
  sigemptyset(&sa.sa_mask);
  sigaction(SIGSEGV, &sa, &g_prev_segv);
}

}  // namespace ogkm

namespace ogkm {

// Host-side producer of the device fault-buffer protocol (ogkm/fault_abi.hpp).
bool fault_buf_produce(FaultBufHeader* h, DeviceFaultRecord* recs, uint32_t entries, DeviceFaultRecord rec,
                       bool may_drop) {
  if (may_drop && __atomic_load_n(&h->put, __ATOMIC_RELAXED) - __atomic_load_n(&h->get, __ATOMIC_ACQUIRE) >= entries) {
    __atomic_fetch_add(&h->overflow, 1u, __ATOMIC_RELAXED);
    return false;
  }
  const uint32_t p = __atomic_fetch_add(&h->put, 1u, __ATOMIC_RELAXED);
  auto t0 = std::chrono::steady_clock::now();
  while (p - __atomic_load_n(&h->get, __ATOMIC_ACQUIRE) >= entries) {
    if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(1)) {
      __atomic_fetch_add(&h->overflow, 1u, __ATOMIC_RELAXED);  // overwrite: the old record counts as lost
      break;
    }
    std::this_thread::yield();
  }
  DeviceFaultRecord* slot = &recs[p & (entries - 1)];
  slot->range_id = rec.range_id;
  slot->block = rec.block;
  slot->page = rec.page;
  slot->access = rec.access;
  slot->kind = rec.kind;
  slot->proc = rec.proc;
  __atomic_store_n(&slot->seq, p + 1, __ATOMIC_RELEASE);
  return true;
}

}  // namespace ogkm
