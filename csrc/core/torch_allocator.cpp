// HBM allocator for PyTorch's pluggable-allocator interface
// (torch.cuda.memory.CUDAPluggableAllocator). Allocations are carved out of the
// runtime's per-GPU HBM arena, so the framework and the model share one budget
// and managed-range eviction can make room for tensors:
//   * size <= 1 MB: power-of-two size classes (512 B .. 1 MB) sub-allocated from
//     2 MB arena chunks (a slab per class, chunks returned when empty);
//   * size  > 1 MB: a contiguous extent of 2 MB chunks, evicting cold managed
//     data through the arena's reservation protocol when the budget is full.
//
// Stream ordering (the caching-allocator contract torch expects, and what the
// reference's PMM gets from its trackers, uvm_pmm_gpu.c free-with-tracker):
//   * free(ptr, stream) records a fence on the freeing stream; the memory is
//     reusable at once, but every later user waits for that fence GPU-side;
//   * alloc(size, stream) makes the allocating stream wait (hipStreamWaitEvent,
//     no host stall) for the fences of the slot / chunks it hands out - the
//     previous tensor's kernels and any ring copy that last touched the chunk.
//   * chunks are taken from the arena already pinned and returned while still
//     pinned (one critical section each): an allocator chunk is never an
//     eviction victim, and never visible to reserve() between two steps.
//
// Managed mode (torch_alloc_managed_min_mb > 0, hbm_provider=1): allocations at
// least that large are not arena extents but managed ranges with a stable device
// VA (HIP VMM): the tensor's pointer never changes while its 2 MB blocks move.
// Such a tensor is "active" (leased: resident in HBM, pinned) from allocation
// until torch_park(); a parked tensor is an ordinary preferred-GPU managed range
// that the arena LRU may evict to host DRAM under pressure (its VA is unmapped),
// and torch_unpark() makes it resident again at the same VA (the stream waits
// GPU-side for the copies). Torch tensors thereby oversubscribe HBM - the
// cudaMallocManaged + cudaMemPrefetchAsync pattern the reference serves with
// uvm_migrate.c, with explicit park points instead of replayable GPU faults
// (a kernel touching a parked, evicted tensor would hit an unmapped VA).
// Frees of managed tensors are deferred until the freeing stream's fence
// completes (no host stall in free).
// The C entry points ogkm_torch_alloc / ogkm_torch_free are what
// CUDAPluggableAllocator dlsym()s.
#include <cstdlib>
#include <deque>
#include <mutex>
#include <unordered_map>
#include <vector>

#include "ogkm/runtime.hpp"

namespace ogkm {

namespace {

constexpr uint64_t kMinClass = 512;
constexpr int kNumClasses = 12;  // 512 B .. 1 MB

struct Slot {
  uint32_t index;
  Tracker fence;  // uses of the previous tensor in this slot
};

struct Slab {
  uint32_t chunk;
  uint32_t used = 0;
  std::vector<Slot> free_slots;
};

struct DevAlloc {
  std::mutex m;
  std::vector<Slab> slabs[kNumClasses];
  struct Entry {
    int cls;           // -1 = extent
    uint32_t chunk;    // extent first chunk / slab chunk
    uint32_t n;        // extent length
    uint64_t size;
  };
  std::unordered_map<uint64_t, Entry> live;
  struct Managed {
    Range* r;
    Lease* lease;      // nullptr while parked (no holds)
    uint64_t size;
    uint32_t holds = 0;       // allocation hold + op holds (the lease lives while > 0)
    bool alloc_hold = false;  // the allocation's own hold (dropped by park / the end of the allocating op)
    bool read_mostly = false;
    // Long-lived (parameters, buffers, caches): held by two ops at least
    // torch_persistent_ops ops apart. Activations are consumed within a few ops
    // and get a new address every pass; the transparent mode's prefetcher keys
    // its trace on persistent operands only.
    bool persistent = false;
    bool held_once = false;
    uint64_t last_hold_op = 0;
  };
  std::unordered_map<uint64_t, Managed> managed;   // stable VA -> range
  std::vector<std::pair<Range*, Tracker>> deferred;  // freed, waiting for their stream fence
  // Freed managed ranges kept for reuse by an allocation of the same size
  // (oldest first): the range keeps its stable VA, its blocks their chunks
  // and mappings, so a reuse costs no VA reservation, no remap and no
  // translation flush. Bounded by torch_alloc_cache_mb; the oldest go to
  // `deferred` beyond it. The fence orders the next owner after the last uses.
  std::deque<std::pair<Range*, Tracker>> cache;
  uint64_t cache_bytes = 0, cache_hits = 0;
  uint64_t allocated = 0, peak = 0, nallocs = 0, stream_waits = 0;
  uint64_t managed_bytes = 0, parks = 0, unparks = 0, op_holds = 0;
  uint64_t op_seq = 0;  // dispatched ops that held managed operands (the persistence clock)
};

std::mutex g_m;
std::vector<std::unique_ptr<DevAlloc>> g_devs;

DevAlloc* dev_alloc(int d) {
  std::lock_guard<std::mutex> g(g_m);
  if ((int)g_devs.size() <= d) g_devs.resize(d + 1);
  if (!g_devs[d]) g_devs[d] = std::make_unique<DevAlloc>();
  return g_devs[d].get();
}

int class_of(uint64_t size) {
  uint64_t c = kMinClass;
  for (int i = 0; i < kNumClasses; ++i, c <<= 1)
    if (size <= c) return i;
  return -1;
}

// n pinned chunks from the arena (evicting cold managed data if needed).
bool take_chunks(Runtime* rt, ChunkArena* a, uint32_t n, uint32_t* first) {
  if (rt->alloc_chunks(a, n, -1, first, nullptr, true) == Status::OK) return true;
  Reservation r;
  if (rt->ensure_capacity(a, n, &r, true) != Status::OK) return false;
  *first = (uint32_t)r.first;
  return true;
}

// The allocating stream waits for everything that last used the memory -
// except the uses queued on that same stream, which stream order already puts
// before anything the new owner enqueues (the caching-allocator rule: reuse on
// the freeing stream costs no wait).
void order_after(Runtime* rt, DevAlloc* da, Tracker t, void* stream) {
  t.prune();
  if (t.empty()) return;
  bool foreign = false;
  for (auto& f : t.fences())
    if (f->ring || f->stream != stream) foreign = true;
  if (!foreign) return;
  Tracker other;
  for (auto& f : t.fences())
    if (f->ring || f->stream != stream) other.add(f);
  t = std::move(other);
  if (t.gpu_wait(rt->be(), stream) != Status::OK) t.wait();
  da->stream_waits++;
}

// Free managed ranges whose last uses have completed (da->m held).
void reap_deferred(Runtime* rt, DevAlloc* da) {
  for (size_t i = 0; i < da->deferred.size();) {
    if (!da->deferred[i].second.query()) {
      ++i;
      continue;
    }
    rt->free_range(da->deferred[i].first);
    da->deferred[i] = std::move(da->deferred.back());
    da->deferred.pop_back();
  }
}

// Lease the whole range on `device` (resident in HBM at its stable VA, pinned)
// and make `stream` wait for the copies that bring it there.
Status lease_on(Runtime* rt, DevAlloc* da, DevAlloc::Managed& m, int device, void* stream, Access access) {
  Lease* L = nullptr;
  Status st = rt->acquire(m.r, 0, m.size, device, access, &L);
  if (st != Status::OK) return st;
  if (L->remote) {  // thrashing / accessed-by chose a zero-copy mapping: the stable VA would not map it
    rt->release(L, stream);
    return Status::BUSY;
  }
  order_after(rt, da, L->ready, stream);
  m.lease = L;
  return Status::OK;
}

void* managed_alloc(Runtime* rt, DevAlloc* da, size_t size, int device, void* stream) {
  Range* r = nullptr;
  uint64_t bytes = align_up((uint64_t)size, kBlockSize);
  // newest cached range of this size first (likeliest still resident)
  for (size_t i = da->cache.size(); i-- > 0;) {
    if (da->cache[i].first->size != bytes) continue;
    r = da->cache[i].first;
    order_after(rt, da, da->cache[i].second, stream);
    da->cache_bytes -= bytes;
    da->cache.erase(da->cache.begin() + (ptrdiff_t)i);
    da->cache_hits++;
    break;
  }
  if (!r) {
    if (rt->malloc_managed(bytes, RANGE_STABLE_VA | RANGE_NO_CPU_VIEW | RANGE_NO_ZERO_FILL, "torch", &r, device) !=
        Status::OK)
      return nullptr;
    rt->mem_advise(r, 0, bytes, Advice::SET_PREFERRED_LOCATION, Loc::gpu(device), device);
  }
  DevAlloc::Managed m{r, nullptr, bytes};
  m.holds = 1;
  m.alloc_hold = true;
  if (lease_on(rt, da, m, device, stream, Access::WRITE) != Status::OK) {
    rt->free_range(r);
    return nullptr;
  }
  uint64_t addr = (uint64_t)r->dev_va;
  da->managed[addr] = m;
  da->managed_bytes += bytes;
  da->allocated += bytes;
  return (void*)addr;
}

}  // namespace

// Out of arena memory: free every deferred managed range now (host-waiting
// for the streams that last used them) - the caching-allocator move of freeing
// its cache and synchronizing before reporting OOM. da->m held.
static bool drain_deferred(Runtime* rt, DevAlloc* da) {
  for (auto& c : da->cache) da->deferred.push_back(std::move(c));
  da->cache.clear();
  da->cache_bytes = 0;
  if (da->deferred.empty()) return false;
  for (auto& d : da->deferred) {
    (void)d.second.wait();
    rt->free_range(d.first);
  }
  da->deferred.clear();
  return true;
}

static void* torch_alloc_locked(Runtime* rt, ChunkArena* a, DevAlloc* da, size_t size, int device, void* stream);


void* torch_alloc(size_t size, int device, void* stream) {
  Runtime* rt = Runtime::get();
  if (!rt || !rt->is_local(device)) return nullptr;
  ChunkArena* a = rt->arena_for(Loc::gpu(device));
  if (!a) return nullptr;
  if (size == 0) size = 1;
  DevAlloc* da = dev_alloc(device);
  std::lock_guard<std::mutex> g(da->m);
  if (!da->deferred.empty()) reap_deferred(rt, da);
  void* p = torch_alloc_locked(rt, a, da, size, device, stream);
  if (!p && drain_deferred(rt, da)) p = torch_alloc_locked(rt, a, da, size, device, stream);
  return p;
}


static void* torch_alloc_locked(Runtime* rt, ChunkArena* a, DevAlloc* da, size_t size, int device, void* stream) {
  int cls = class_of(size);
  const int64_t mmin = config().torch_alloc_managed_min_mb;
  if (mmin > 0 && size >= ((uint64_t)mmin << 20) && static_cast<HbmArena*>(a)->vmm()) {
    void* p = managed_alloc(rt, da, size, device, stream);
    if (p) {
      da->nallocs++;
      da->peak = std::max(da->peak, da->allocated);
    }
    return p;
  }
  uint64_t addr = 0;
  if (cls >= 0) {
    uint64_t csz = kMinClass << cls;
    Slab* s = nullptr;
    // A slot whose previous tensor is done beats one still in flight.
    for (int pass = 0; pass < 2 && !s; ++pass)
      for (auto& x : da->slabs[cls]) {
        if (x.free_slots.empty()) continue;
        if (pass == 0 && !x.free_slots.back().fence.query()) continue;
        s = &x;
        break;
      }
    if (!s) {
      uint32_t ch;
      if (!take_chunks(rt, a, 1, &ch)) return nullptr;
      order_after(rt, da, a->reuse_fence(ch), stream);
      Slab ns;
      ns.chunk = ch;
      uint32_t nslots = (uint32_t)(kBlockSize / csz);
      for (uint32_t i = nslots; i-- > 0;) ns.free_slots.push_back(Slot{i, Tracker{}});
      da->slabs[cls].push_back(std::move(ns));
      s = &da->slabs[cls].back();
    }
    Slot slot = std::move(s->free_slots.back());
    s->free_slots.pop_back();
    s->used++;
    order_after(rt, da, slot.fence, stream);
    addr = a->chunk_addr(s->chunk) + (uint64_t)slot.index * csz;
    da->live[addr] = DevAlloc::Entry{cls, s->chunk, 0, csz};
    da->allocated += csz;
  } else {
    uint32_t n = (uint32_t)((size + kBlockSize - 1) >> kBlockShift);
    uint32_t first;
    if (!take_chunks(rt, a, n, &first)) return nullptr;
    Tracker t;
    for (uint32_t i = 0; i < n; ++i) t.merge(a->reuse_fence(first + i));
    order_after(rt, da, t, stream);
    addr = a->chunk_addr(first);
    da->live[addr] = DevAlloc::Entry{-1, first, n, (uint64_t)n << kBlockShift};
    da->allocated += (uint64_t)n << kBlockShift;
  }
  da->nallocs++;
  da->peak = std::max(da->peak, da->allocated);
  return (void*)addr;
}


void torch_free(void* p, int device, void* stream) {
  Runtime* rt = Runtime::get();
  if (!rt || !p || !rt->is_local(device)) return;
  ChunkArena* a = rt->arena_for(Loc::gpu(device));
  DevAlloc* da = dev_alloc(device);
  // The freeing stream's queued work may still use the memory.
  FenceRef f = fence_record(rt->be(), device, stream);
  std::lock_guard<std::mutex> g(da->m);
  auto mt = da->managed.find((uint64_t)p);
  if (mt != da->managed.end()) {
    DevAlloc::Managed m = mt->second;
    da->managed.erase(mt);
    da->allocated -= m.size;
    da->managed_bytes -= m.size;
    if (m.lease) rt->release(m.lease, stream);
    Tracker t;
    if (f) t.add(f);
    const uint64_t cap = (uint64_t)std::max<int64_t>(0, config().torch_alloc_cache_mb) << 20;
    if (m.size <= cap) {
      da->cache.emplace_back(m.r, std::move(t));
      da->cache_bytes += m.size;
      while (da->cache_bytes > cap) {  // the oldest leave the cache: freed once their uses completed
        da->cache_bytes -= da->cache.front().first->size;
        da->deferred.push_back(std::move(da->cache.front()));
        da->cache.pop_front();
      }
    } else {
      da->deferred.emplace_back(m.r, std::move(t));
    }
    reap_deferred(rt, da);
    return;
  }
  auto it = da->live.find((uint64_t)p);
  if (it == da->live.end()) return;
  DevAlloc::Entry e = it->second;
  da->live.erase(it);
  da->allocated -= e.size;
  if (e.cls < 0) {
    for (uint32_t i = 0; i < e.n; ++i)
      if (f) a->add_reuse_fence(e.chunk + i, f);
    a->free(e.chunk, e.n);  // still pinned: free() drops the pin atomically
    return;
  }
  auto& slabs = da->slabs[e.cls];
  for (size_t i = 0; i < slabs.size(); ++i) {
    if (slabs[i].chunk != e.chunk) continue;
    uint64_t csz = kMinClass << e.cls;
    Slot slot{(uint32_t)(((uint64_t)p - a->chunk_addr(e.chunk)) / csz), Tracker{}};
    if (f) slot.fence.add(f);
    slabs[i].free_slots.push_back(std::move(slot));
    if (--slabs[i].used == 0) {
      for (auto& s : slabs[i].free_slots)
        for (auto& x : s.fence.fences()) a->add_reuse_fence(e.chunk, x);
      a->free(e.chunk, 1);
      slabs.erase(slabs.begin() + i);
    }
    return;
  }
}

// Runtime teardown: forget every slab / live entry (their fences reference
// the backend being destroyed). Tensors still alive after shutdown dangle, as
// any device memory does once its context is gone.
void torch_alloc_reset() {
  std::lock_guard<std::mutex> g(g_m);
  g_devs.clear();
}

// Drop one hold of a managed tensor; the last one releases its lease (the
// stream's queued uses fence any eviction). da->m held.
Status drop_hold(Runtime* rt, DevAlloc* da, DevAlloc::Managed& m, void* stream) {
  if (m.holds == 0) return Status::OK;
  if (--m.holds > 0 || !m.lease) return Status::OK;
  Status st = rt->release(m.lease, stream);
  m.lease = nullptr;
  da->parks++;
  return st;
}

// Add one hold; the first one leases the tensor (resident at its VA, pinned;
// the stream waits GPU-side for the copies). da->m held.
Status add_hold(Runtime* rt, DevAlloc* da, DevAlloc::Managed& m, int device, void* stream, Access access) {
  if (m.holds++ > 0 && m.lease) return Status::OK;
  Status st = lease_on(rt, da, m, device, stream, m.read_mostly && access == Access::READ ? Access::READ : access);
  if (st != Status::OK) {
    m.holds--;
    return st;
  }
  da->unparks++;
  return Status::OK;
}

// Park / unpark a managed tensor (see the header comment): park drops the
// allocation's hold, unpark takes it again. Returns NOT_FOUND for a pointer
// that is not a managed allocation's base.
Status torch_park(void* p, int device, void* stream) {
  Runtime* rt = Runtime::get();
  if (!rt || !rt->is_local(device)) return Status::INVALID_ARGUMENT;
  DevAlloc* da = dev_alloc(device);
  std::lock_guard<std::mutex> g(da->m);
  auto it = da->managed.find((uint64_t)p);
  if (it == da->managed.end()) return Status::NOT_FOUND;
  if (!it->second.alloc_hold) return Status::OK;
  it->second.alloc_hold = false;
  return drop_hold(rt, da, it->second, stream);
}

Status torch_unpark(void* p, int device, void* stream) {
  Runtime* rt = Runtime::get();
  if (!rt || !rt->is_local(device)) return Status::INVALID_ARGUMENT;
  DevAlloc* da = dev_alloc(device);
  std::lock_guard<std::mutex> g(da->m);
  auto it = da->managed.find((uint64_t)p);
  if (it == da->managed.end()) return Status::NOT_FOUND;
  if (it->second.alloc_hold) return Status::OK;
  Status st = add_hold(rt, da, it->second, device, stream, Access::WRITE);
  if (st == Status::OK) it->second.alloc_hold = true;
  return st;
}

// Drop the allocation hold of every managed tensor of `device` (entering the
// transparent mode: from then on only op holds keep tensors resident).
void torch_park_all(int device, void* stream) {
  Runtime* rt = Runtime::get();
  if (!rt || !rt->is_local(device)) return;
  DevAlloc* da = dev_alloc(device);
  std::lock_guard<std::mutex> g(da->m);
  for (auto& kv : da->managed) {
    if (kv.second.alloc_hold) {
      kv.second.alloc_hold = false;
      (void)drop_hold(rt, da, kv.second, stream);
    }
  }
}

// Tensor-granular software faults for one dispatched op (the transparent mode,
// open-gpu-kernel-modules_amd/managed.py): every managed storage the op reads
// or writes gets an op hold - made resident at its stable VA, pinned, the
// stream ordered after the copies - before the op is enqueued. Non-managed
// pointers are ignored. Returns the pointers that were held (for op_end).
// Reference: the fault -> service -> replay path of
// uvm_gpu_replayable_faults.c:2906 at tensor granularity, with the operands
// declared by the dispatcher instead of reported by the MMU.
Status torch_op_begin(const std::vector<std::pair<uint64_t, bool>>& ptrs, int device, void* stream,
                      std::vector<uint64_t>* held, std::vector<uint64_t>* persistent) {
  Runtime* rt = Runtime::get();
  if (!rt || !rt->is_local(device)) return Status::INVALID_ARGUMENT;
  DevAlloc* da = dev_alloc(device);
  std::lock_guard<std::mutex> g(da->m);
  if (da->managed.empty()) return Status::OK;
  // Writers first: a tensor both read and written is leased for writing.
  std::vector<std::pair<uint64_t, bool>> v;
  for (auto& pw : ptrs) {
    if (!da->managed.count(pw.first)) continue;
    bool dup = false;
    for (auto& x : v)
      if (x.first == pw.first) {
        x.second |= pw.second;
        dup = true;
      }
    if (!dup) v.push_back(pw);
  }
  if (!v.empty()) da->op_seq++;
  for (auto& pw : v) {
    auto& m = da->managed[pw.first];
    Status st = add_hold(rt, da, m, device, stream, pw.second ? Access::WRITE : Access::READ);
    if (st != Status::OK) {
      for (uint64_t p : *held) (void)drop_hold(rt, da, da->managed[p], stream);
      held->clear();
      return st;
    }
    held->push_back(pw.first);
    if (m.held_once && da->op_seq - m.last_hold_op >= (uint64_t)std::max<int64_t>(1, config().torch_persistent_ops))
      m.persistent = true;
    m.held_once = true;
    m.last_hold_op = da->op_seq;
    if (m.persistent) persistent->push_back(pw.first);
    da->op_holds++;
  }
  return Status::OK;
}

// End of a dispatched op: drop the op holds of `held`, and the allocation hold
// of every managed operand and output (from its first use as an operand on,
// a tensor is resident only while an op holds it; a tensor never passed to an
// op - a library workspace used behind the dispatcher's back - keeps its
// allocation hold and is never evicted).
Status torch_op_end(const std::vector<uint64_t>& held, const std::vector<uint64_t>& outs, int device, void* stream) {
  Runtime* rt = Runtime::get();
  if (!rt || !rt->is_local(device)) return Status::INVALID_ARGUMENT;
  DevAlloc* da = dev_alloc(device);
  std::lock_guard<std::mutex> g(da->m);
  Status res = Status::OK;
  auto drop_alloc = [&](uint64_t p) {
    auto it = da->managed.find(p);
    if (it == da->managed.end() || !it->second.alloc_hold) return;
    it->second.alloc_hold = false;
    Status st = drop_hold(rt, da, it->second, stream);
    if (res == Status::OK) res = st;
  };
  for (uint64_t p : outs) drop_alloc(p);
  for (uint64_t p : held) drop_alloc(p);
  for (uint64_t p : held) {
    auto it = da->managed.find(p);
    if (it == da->managed.end()) continue;  // freed inside the op (its free already released the lease)
    Status st = drop_hold(rt, da, it->second, stream);
    if (res == Status::OK) res = st;
  }
  return res;
}

// Keep host copies of a managed tensor when it is only read (READ_MOSTLY:
// evicting a clean duplicate then costs no copy-out).
Status torch_set_read_mostly(void* p, int device, bool on) {
  Runtime* rt = Runtime::get();
  if (!rt || !rt->is_local(device)) return Status::INVALID_ARGUMENT;
  DevAlloc* da = dev_alloc(device);
  std::lock_guard<std::mutex> g(da->m);
  auto it = da->managed.find((uint64_t)p);
  if (it == da->managed.end()) return Status::NOT_FOUND;
  it->second.read_mostly = on;
  return rt->mem_advise(it->second.r, 0, it->second.size, on ? Advice::SET_READ_MOSTLY : Advice::UNSET_READ_MOSTLY,
                        Loc::gpu(device), device);
}

// Layer-ahead prefetch of managed tensors not currently held: queue their
// H2D copies (no lease, no stream wait; a later op hold finds them resident or
// waits for the copies). Returns how many prefetches were queued.
size_t torch_prefetch(const std::vector<uint64_t>& ptrs, int device) {
  Runtime* rt = Runtime::get();
  if (!rt || !rt->is_local(device)) return 0;
  DevAlloc* da = dev_alloc(device);
  std::lock_guard<std::mutex> g(da->m);
  size_t n = 0;
  for (uint64_t p : ptrs) {
    auto it = da->managed.find(p);
    if (it == da->managed.end() || it->second.holds) continue;
    Tracker t;
    if (rt->prefetch(it->second.r, 0, it->second.size, Loc::gpu(device), &t, Cause::Prefetch) == Status::OK) ++n;
  }
  return n;
}

uint64_t torch_managed_size(void* p, int device) {
  DevAlloc* da = dev_alloc(device);
  std::lock_guard<std::mutex> g(da->m);
  auto it = da->managed.find((uint64_t)p);
  return it == da->managed.end() ? 0 : it->second.size;
}

bool torch_is_managed(void* p, int device) {
  DevAlloc* da = dev_alloc(device);
  std::lock_guard<std::mutex> g(da->m);
  return da->managed.count((uint64_t)p) != 0;
}

// (active, parked bytes, parks, unparks) of the managed tensors.
void torch_managed_stats(int device, uint64_t* active, uint64_t* parked, uint64_t* parks, uint64_t* unparks) {
  DevAlloc* da = dev_alloc(device);
  std::lock_guard<std::mutex> g(da->m);
  *active = *parked = 0;
  for (auto& kv : da->managed) (kv.second.holds ? *active : *parked) += kv.second.size;
  *parks = da->parks;
  *unparks = da->unparks;
}

void torch_alloc_stats(int device, uint64_t* allocated, uint64_t* peak, uint64_t* nallocs, uint64_t* stream_waits) {
  DevAlloc* da = dev_alloc(device);
  std::lock_guard<std::mutex> g(da->m);
  *allocated = da->allocated;
  *peak = da->peak;
  *nallocs = da->nallocs;
  *stream_waits = da->stream_waits;
}

}  // namespace ogkm

extern "C" {
__attribute__((visibility("default"))) void* ogkm_torch_alloc(size_t size, int device, void* stream) {
  void* p = ogkm::torch_alloc(size, device, stream);
  if (!p && size) {
    // torch's pluggable-allocator path does not check for null: a null
    // tensor would reach a kernel and fault the GPU. Fail loudly on the CPU.
    ogkm::Runtime* rt = ogkm::Runtime::get();
    ogkm::ChunkArena* a = rt ? rt->arena_for(ogkm::Loc::gpu(device)) : nullptr;
    ogkm::ChunkArena::Stats st = a ? a->stats() : ogkm::ChunkArena::Stats{};
    RT_ERR("torch allocation of %zu bytes on gpu %d failed: HBM arena %llu MB, allocated %llu MB, pinned %llu MB "
           "(pinned = leased / held tensors + allocator slabs + tensors never used as an operand, e.g. library "
           "workspaces). Raise the HBM budget or lower the working set of one op; aborting instead of returning "
           "a null device pointer.",
           size, device, (unsigned long long)(st.capacity >> 20), (unsigned long long)(st.allocated >> 20),
           (unsigned long long)(st.pinned >> 20));
    std::abort();
  }
  return p;
}
__attribute__((visibility("default"))) void ogkm_torch_free(void* ptr, size_t /*size*/, int device, void* stream) {
  ogkm::torch_free(ptr, device, stream);
}
}
