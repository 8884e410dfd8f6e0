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
    Lease* lease;      // nullptr while parked
    uint64_t size;
  };
  std::unordered_map<uint64_t, Managed> managed;   // stable VA -> range
  std::vector<std::pair<Range*, Tracker>> deferred;  // freed, waiting for their stream fence
  uint64_t allocated = 0, peak = 0, nallocs = 0, stream_waits = 0;
  uint64_t managed_bytes = 0, parks = 0, unparks = 0;
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
Status lease_on(Runtime* rt, DevAlloc* da, DevAlloc::Managed& m, int device, void* stream) {
  Lease* L = nullptr;
  Status st = rt->acquire(m.r, 0, m.size, device, Access::WRITE, &L);
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
  if (rt->malloc_managed(bytes, RANGE_STABLE_VA | RANGE_NO_CPU_VIEW, "torch", &r, device) != Status::OK)
    return nullptr;
  rt->mem_advise(r, 0, bytes, Advice::SET_PREFERRED_LOCATION, Loc::gpu(device), device);
  DevAlloc::Managed m{r, nullptr, bytes};
  if (lease_on(rt, da, m, device, stream) != Status::OK) {
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

void* torch_alloc(size_t size, int device, void* stream) {
  Runtime* rt = Runtime::get();
  if (!rt || !rt->is_local(device)) return nullptr;
  ChunkArena* a = rt->arena_for(Loc::gpu(device));
  if (!a) return nullptr;
  if (size == 0) size = 1;
  DevAlloc* da = dev_alloc(device);
  int cls = class_of(size);
  std::lock_guard<std::mutex> g(da->m);
  if (!da->deferred.empty()) reap_deferred(rt, da);
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
    da->deferred.emplace_back(m.r, std::move(t));
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

// Park / unpark a managed tensor (see the header comment). Returns NOT_FOUND
// for a pointer that is not a managed allocation's base.
Status torch_park(void* p, int device, void* stream) {
  Runtime* rt = Runtime::get();
  if (!rt || !rt->is_local(device)) return Status::INVALID_ARGUMENT;
  DevAlloc* da = dev_alloc(device);
  std::lock_guard<std::mutex> g(da->m);
  auto it = da->managed.find((uint64_t)p);
  if (it == da->managed.end()) return Status::NOT_FOUND;
  if (!it->second.lease) return Status::OK;
  Status st = rt->release(it->second.lease, stream);  // the stream's queued uses fence the eviction
  it->second.lease = nullptr;
  da->parks++;
  return st;
}

Status torch_unpark(void* p, int device, void* stream) {
  Runtime* rt = Runtime::get();
  if (!rt || !rt->is_local(device)) return Status::INVALID_ARGUMENT;
  DevAlloc* da = dev_alloc(device);
  std::lock_guard<std::mutex> g(da->m);
  auto it = da->managed.find((uint64_t)p);
  if (it == da->managed.end()) return Status::NOT_FOUND;
  if (it->second.lease) return Status::OK;
  Status st = lease_on(rt, da, it->second, device, stream);
  if (st == Status::OK) da->unparks++;
  return st;
}

// (active, parked bytes, parks, unparks) of the managed tensors.
void torch_managed_stats(int device, uint64_t* active, uint64_t* parked, uint64_t* parks, uint64_t* unparks) {
  DevAlloc* da = dev_alloc(device);
  std::lock_guard<std::mutex> g(da->m);
  *active = *parked = 0;
  for (auto& kv : da->managed) (kv.second.lease ? *active : *parked) += kv.second.size;
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
  return ogkm::torch_alloc(size, device, stream);
}
__attribute__((visibility("default"))) void ogkm_torch_free(void* ptr, size_t /*size*/, int device, void* stream) {
  ogkm::torch_free(ptr, device, stream);
}
}
