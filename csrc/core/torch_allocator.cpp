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
//   * free(ptr, stream) tags the slot / extent with the freeing stream and
//     records nothing: reuse by an allocation on the SAME stream needs no
//     fence (stream order already puts the old tensor's kernels first), which
//     is the common case of a decode step (hundreds of frees per step);
//   * a reuse from another stream, or the memory going back to the runtime's
//     arena (where ring copies and other users may take it), records the fence
//     on the freeing stream at that moment (later than the free: conservative,
//     never early) and the allocating stream waits for it GPU-side
//     (hipStreamWaitEvent, no host stall) - with any ring copy that last
//     touched the chunk.
//   * freed extents (> 1 MB) stay in a small per-device cache for same-size
//     reuse; the runtime's pressure handler hands them back to the arena when
//     it needs chunks.
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
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <deque>
#include <mutex>
#include <thread>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>

#include "ogkm/runtime.hpp"
#include "ogkm/torch_alloc.hpp"

namespace ogkm {

namespace {

constexpr uint64_t kMinClass = 512;
constexpr int kNumClasses = 12;  // 512 B .. 1 MB

struct Slot {
  uint32_t index;
  Tracker fence;  // uses of the previous tensor in this slot (recorded lazily, see settle)
  void* free_stream = nullptr;  // the stream that freed it (fence not yet recorded)
  bool tagged = false;
};

// A freed extent kept for same-size reuse (DevAlloc::extents).
struct ExtentFree {
  uint32_t first, n;
  void* free_stream;
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
  std::vector<ExtentFree> extents;  // freed extents, oldest first (torch_alloc_extent_cache_mb)
  uint64_t extent_bytes = 0, extent_hits = 0, lazy_fences = 0;
  uint64_t pressure_id = 0;
  bool pressure_registered = false;
  struct Managed {
    Range* r;
    Lease* lease;      // nullptr while parked (no holds)
    uint64_t size;
    uint32_t holds = 0;       // allocation hold + op holds (the lease lives while > 0)
    bool alloc_hold = false;  // the allocation's own hold (dropped by park / the end of the allocating op)
    // The lease's extent: the whole allocation for the allocation hold, the
    // pages of the op's views for an op hold.
    uint64_t lease_off = 0, lease_len = 0;
    uint64_t next_use = 0;    // last next-use hint applied (op clock)
    // Long-lived (parameters, buffers, caches): held again at least
    // torch_persistent_ops ops after its first hold. Activations die within a
    // layer (a residual stream lives ~35 ops) and their recycled addresses come
    // back every layer - keyed on them, the transparent mode's op trace would
    // see its first repeat inside the first layer; it keys on persistent
    // operands only.
    bool persistent = false;
    bool held_once = false;
    uint64_t first_hold_op = 0;
    uint32_t prefetching = 0;  // the prefetch worker is placing it (a free waits for it)
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
  std::string last_error;  // last allocation failure (surfaced by ogkm_torch_alloc)
  // Asynchronous op-trace prefetch (torch_async_prefetch): the dispatching
  // thread queues (tensor, op-clock time needed); a worker places them.
  struct PrefetchReq {
    uint64_t ptr, when;
  };
  std::deque<PrefetchReq> pq;
  std::condition_variable pq_cv, pf_done_cv;
  std::thread worker;
  bool stop = false;
  uint64_t pf_queued = 0, pf_done = 0, pf_skipped = 0;
  void stop_worker() {
    if (!worker.joinable()) return;
    {
      std::lock_guard<std::mutex> g(m);
      stop = true;
    }
    pq_cv.notify_all();
    worker.join();
  }
  ~DevAlloc() { stop_worker(); }  // process exit without a runtime shutdown
};

std::mutex g_m;
std::vector<std::unique_ptr<DevAlloc>> g_devs;
thread_local int t_in_alloc = 0;  // this thread holds a DevAlloc lock (pressure handler re-entry)
struct InAlloc {
  InAlloc() { ++t_in_alloc; }
  ~InAlloc() { --t_in_alloc; }
};

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

// A tagged slot's fence, recorded now on the stream that freed it (later than
// the free itself: it covers the old tensor's kernels and possibly more).
void settle(Runtime* rt, DevAlloc* da, int device, Slot& s) {
  if (!s.tagged) return;
  s.tagged = false;
  if (FenceRef f = fence_record(rt->be(), device, s.free_stream)) s.fence.add(f);
  da->lazy_fences++;
}

// An extent leaves the cache for the arena: its reuse fence is recorded on the
// stream that freed it, then the (still pinned) chunks are freed.
void extent_to_arena(Runtime* rt, DevAlloc* da, ChunkArena* a, int device, const ExtentFree& e) {
  FenceRef f = fence_record(rt->be(), device, e.free_stream);
  da->lazy_fences++;
  for (uint32_t i = 0; i < e.n; ++i)
    if (f) a->add_reuse_fence(e.first + i, f);
  a->free(e.first, e.n);
}

bool flush_extents(Runtime* rt, DevAlloc* da, ChunkArena* a, int device) {
  if (da->extents.empty()) return false;
  for (const ExtentFree& e : da->extents) extent_to_arena(rt, da, a, device, e);
  da->extents.clear();
  da->extent_bytes = 0;
  return true;
}

// An empty slab goes back to the arena: one fence per stream that freed a slot
// in it (recorded now), the chunk's reuse fences.
void slab_to_arena(Runtime* rt, DevAlloc* da, ChunkArena* a, int device, std::vector<Slab>& slabs, size_t i) {
  std::vector<std::pair<void*, FenceRef>> per_stream;
  for (auto& s : slabs[i].free_slots) {
    if (s.tagged) {
      FenceRef fr;
      for (auto& ps : per_stream)
        if (ps.first == s.free_stream) fr = ps.second;
      if (!fr) {
        fr = fence_record(rt->be(), device, s.free_stream);
        da->lazy_fences++;
        per_stream.emplace_back(s.free_stream, fr);
      }
      if (fr) s.fence.add(fr);
      s.tagged = false;
    }
    for (auto& x : s.fence.fences()) a->add_reuse_fence(slabs[i].chunk, x);
  }
  a->free(slabs[i].chunk, 1);
  slabs.erase(slabs.begin() + (ptrdiff_t)i);
}

// Cached extents and empty slabs back to the arena (pressure, re-init).
bool trim_locked(Runtime* rt, DevAlloc* da, ChunkArena* a, int device) {
  bool any = flush_extents(rt, da, a, device);
  for (auto& slabs : da->slabs)
    for (size_t i = slabs.size(); i-- > 0;)
      if (slabs[i].used == 0) {
        slab_to_arena(rt, da, a, device, slabs, i);
        any = true;
      }
  return any;
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

// Lease [off, off + len) of the range on `device` (resident in HBM at its
// stable VA, pinned) and make `stream` wait for the copies that bring it there.
// A zero-copy decision (thrashing pin, accessed_by) is served by a local copy:
// the stable VA maps HBM only (acquire(allow_remote = false)).
Status lease_on(Runtime* rt, DevAlloc* da, DevAlloc::Managed& m, int device, void* stream, Access access,
                uint64_t off, uint64_t len) {
  Lease* L = nullptr;
  Status st = rt->acquire(m.r, off, len, device, access, &L, false);
  if (st != Status::OK) return st;
  if (L->remote) {  // cannot happen with allow_remote = false; never hand out a VA that maps nothing
    rt->release(L, stream);
    return Status::NOT_SUPPORTED;
  }
  order_after(rt, da, L->ready, stream);
  m.lease = L;
  m.lease_off = off;
  m.lease_len = len;
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
    rt->set_dead(r, false);
    break;
  }
  if (!r) {
    Status st = rt->malloc_managed(bytes, RANGE_STABLE_VA | RANGE_NO_CPU_VIEW | RANGE_NO_ZERO_FILL, "torch", &r,
                                   device);
    if (st != Status::OK) {
      da->last_error = std::string("managed range of ") + std::to_string(bytes) + " bytes: " + status_str(st);
      return nullptr;
    }
    rt->mem_advise(r, 0, bytes, Advice::SET_PREFERRED_LOCATION, Loc::gpu(device), device);
    // Reads duplicate (the host copy of evicted data stays valid), writes
    // revoke only the pages they write: an eviction copies out only pages
    // written since the tensor last came back (TorchOperand::written).
    rt->mem_advise(r, 0, bytes, Advice::SET_READ_MOSTLY, Loc::gpu(device), device);
  }
  DevAlloc::Managed m{r, nullptr, bytes};
  m.holds = 1;
  m.alloc_hold = true;
  if (Status st = lease_on(rt, da, m, device, stream, Access::WRITE, 0, bytes); st != Status::OK) {
    da->last_error = std::string("lease of a ") + std::to_string(bytes >> 20) + " MB managed tensor: " + status_str(st);
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
  InAlloc in_alloc;
  da->last_error.clear();
  if (!da->deferred.empty()) reap_deferred(rt, da);
  void* p = torch_alloc_locked(rt, a, da, size, device, stream);
  if (!p && drain_deferred(rt, da)) p = torch_alloc_locked(rt, a, da, size, device, stream);
  if (!p && da->last_error.empty()) da->last_error = "no free or evictable HBM chunks";
  return p;
}


static void* torch_alloc_locked(Runtime* rt, ChunkArena* a, DevAlloc* da, size_t size, int device, void* stream) {
  int cls = class_of(size);
  const int64_t mmin = config().torch_alloc_managed_min_mb;
  // Managed (stable-VA) tensors need a VMM arena whose remaps passed the
  // translation self-test; otherwise the tensor is an ordinary arena extent
  // (it cannot oversubscribe, but it is never read through a stale mapping).
  if (mmin > 0 && size >= ((uint64_t)mmin << 20) && static_cast<HbmArena*>(a)->vmm() &&
      rt->dev(device).vmm_test.ok) {
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
    // A slot freed on this very stream (no fence at all) beats one whose
    // previous tensor is done, which beats one still in flight.
    for (int pass = 0; pass < 3 && !s; ++pass)
      for (auto& x : da->slabs[cls]) {
        if (x.free_slots.empty()) continue;
        const Slot& b = x.free_slots.back();
        if (pass == 0 && !(b.tagged && b.free_stream == stream)) continue;
        if (pass == 1 && (b.tagged || !const_cast<Tracker&>(b.fence).query())) continue;
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
    if (slot.tagged && slot.free_stream != stream) settle(rt, da, device, slot);
    order_after(rt, da, slot.fence, stream);
    addr = a->chunk_addr(s->chunk) + (uint64_t)slot.index * csz;
    da->live[addr] = DevAlloc::Entry{cls, s->chunk, 0, csz};
    da->allocated += csz;
  } else {
    uint32_t n = (uint32_t)((size + kBlockSize - 1) >> kBlockShift);
    uint32_t first = 0;
    bool reused = false;
    // a cached extent of this size: freed on this stream first (no fence), newest first
    for (int pass = 0; pass < 2 && !reused; ++pass)
      for (size_t i = da->extents.size(); i-- > 0;) {
        const ExtentFree e = da->extents[i];
        if (e.n != n || (pass == 0 && e.free_stream != stream)) continue;
        da->extents.erase(da->extents.begin() + (ptrdiff_t)i);
        da->extent_bytes -= (uint64_t)n << kBlockShift;
        da->extent_hits++;
        first = e.first;
        if (e.free_stream != stream) {
          Tracker t;
          t.add(fence_record(rt->be(), device, e.free_stream));
          da->lazy_fences++;
          order_after(rt, da, t, stream);
        }
        reused = true;
        break;
      }
    if (!reused) {
      if (!take_chunks(rt, a, n, &first)) {
        if (!trim_locked(rt, da, a, device) || !take_chunks(rt, a, n, &first)) return nullptr;
      }
      Tracker t;
      for (uint32_t i = 0; i < n; ++i) t.merge(a->reuse_fence(first + i));
      order_after(rt, da, t, stream);
    }
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
  std::unique_lock<std::mutex> g(da->m);
  InAlloc in_alloc;
  auto mt = da->managed.find((uint64_t)p);
  if (mt != da->managed.end() && mt->second.prefetching) {
    // the worker is placing it right now: let that finish before the range goes
    da->pf_done_cv.wait(g, [&] {
      auto it = da->managed.find((uint64_t)p);
      return it == da->managed.end() || !it->second.prefetching;
    });
    mt = da->managed.find((uint64_t)p);
  }
  if (mt != da->managed.end()) {
    DevAlloc::Managed m = mt->second;
    da->managed.erase(mt);
    da->allocated -= m.size;
    da->managed_bytes -= m.size;
    if (m.lease) rt->release(m.lease, stream);
    rt->set_dead(m.r, true);  // evicting it now copies nothing out; off-GPU copies are dropped
    // The freeing stream's queued work may still use the memory.
    FenceRef f = fence_record(rt->be(), device, stream);
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
    // kept for same-size reuse (no fence yet: the freeing stream's order is
    // the fence for its own next allocation), the oldest go back to the arena
    const uint64_t cap = (uint64_t)std::max<int64_t>(0, config().torch_alloc_extent_cache_mb) << 20;
    da->extents.push_back(ExtentFree{e.chunk, e.n, stream});
    da->extent_bytes += (uint64_t)e.n << kBlockShift;
    while (da->extent_bytes > cap && !da->extents.empty()) {
      extent_to_arena(rt, da, a, device, da->extents.front());  // still pinned: free() drops the pin
      da->extent_bytes -= (uint64_t)da->extents.front().n << kBlockShift;
      da->extents.erase(da->extents.begin());
    }
    if (!da->pressure_registered) {
      // the runtime needs chunks (nothing else evictable): the cached extents go back
      da->pressure_registered = true;
      da->pressure_id = rt->add_pressure_handler(device, [rt, da, a, device] {
        if (t_in_alloc) return false;  // the allocator itself is the one asking (it flushes)
        std::unique_lock<std::mutex> pg(da->m, std::try_to_lock);
        if (!pg.owns_lock()) return false;
        return trim_locked(rt, da, a, device);
      });
    }
    return;
  }
  auto& slabs = da->slabs[e.cls];
  for (size_t i = 0; i < slabs.size(); ++i) {
    if (slabs[i].chunk != e.chunk) continue;
    uint64_t csz = kMinClass << e.cls;
    Slot slot{(uint32_t)(((uint64_t)p - a->chunk_addr(e.chunk)) / csz), Tracker{}, stream, true};
    slabs[i].free_slots.push_back(std::move(slot));
    if (--slabs[i].used == 0) {
      // an empty slab stays for the next allocations of its class (up to
      // torch_alloc_empty_slabs of them); the others go back to the arena
      uint32_t empty = 0;
      for (auto& x : slabs)
        if (x.used == 0) ++empty;
      if ((int64_t)empty > std::max<int64_t>(0, config().torch_alloc_empty_slabs)) slab_to_arena(rt, da, a, device, slabs, i);
    }
    return;
  }
}

// Runtime teardown: forget every slab / live entry (their fences reference
// the backend being destroyed). Tensors still alive after shutdown dangle, as
// any device memory does once its context is gone.
void torch_alloc_trim(int device) {
  Runtime* rt = Runtime::get();
  if (!rt || !rt->is_local(device)) return;
  // Never through arena_for: on a device with no arena yet that would create
  // the default half-of-HBM arena just to trim it (and init_device then tears
  // it down again) - per-init that churn hung the GPU test sequence.
  ChunkArena* a = rt->hbm_arena_if_any(device);
  if (!a) return;
  DevAlloc* da = dev_alloc(device);
  std::lock_guard<std::mutex> g(da->m);
  InAlloc in_alloc;
  trim_locked(rt, da, a, device);
}

void torch_alloc_reset() {
  std::lock_guard<std::mutex> g(g_m);
  Runtime* rt = Runtime::get();
  for (auto& d : g_devs)
    if (d) {
      d->stop_worker();
      if (d->pressure_registered && rt) rt->remove_pressure_handler(d->pressure_id);
    }
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

// Add one hold of [off, off + len); the first one leases it (resident at its
// VA, pinned; the stream waits GPU-side for the copies). A hold beyond the
// current lease's extent re-leases the whole allocation. da->m held.
Status add_hold(Runtime* rt, DevAlloc* da, DevAlloc::Managed& m, int device, void* stream, Access access,
                uint64_t off, uint64_t len) {
  if (m.holds > 0 && m.lease) {
    if (off >= m.lease_off && off + len <= m.lease_off + m.lease_len) {
      m.holds++;
      return Status::OK;
    }
    Lease* old = m.lease;
    Status st = lease_on(rt, da, m, device, stream, access, 0, m.size);
    if (st != Status::OK) {
      m.lease = old;
      return st;
    }
    rt->release(old, stream);
    m.holds++;
    return Status::OK;
  }
  m.holds++;
  Status st = lease_on(rt, da, m, device, stream, access, off, len);
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
  Status st = add_hold(rt, da, it->second, device, stream, Access::WRITE, 0, it->second.size);
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

// Software faults for one dispatched op (the transparent mode,
// open-gpu-kernel-modules_amd/managed.py): every managed storage the op reads
// or writes gets an op hold over the pages its views span - made resident at
// its stable VA (reads duplicate: host copies stay valid), pinned, the stream
// ordered after the copies - before the op is enqueued. For a written operand
// the other copies of exactly the written pages are revoked, so the tensor's
// dirty set is what the op wrote, not the whole allocation (a KV-cache row
// append dirties 4 KB pages, not the cache). Non-managed pointers are ignored.
// Returns the pointers that were held (for op_end).
// Reference: the fault -> service -> replay path of
// uvm_gpu_replayable_faults.c:2906 with the faulted pages declared by the
// dispatcher instead of reported by the MMU; per-page residency / dirty state
// as uvm_va_block.h:101-230.
Status torch_op_begin(const std::vector<TorchOperand>& ops, int device, void* stream, std::vector<uint64_t>* held,
                      std::vector<uint64_t>* persistent) {
  Runtime* rt = Runtime::get();
  if (!rt || !rt->is_local(device)) return Status::INVALID_ARGUMENT;
  DevAlloc* da = dev_alloc(device);
  std::lock_guard<std::mutex> g(da->m);
  if (da->managed.empty()) return Status::OK;
  // One entry per storage: extents unioned, written intervals collected.
  std::vector<TorchOperand> v;
  for (auto& o : ops) {
    auto mt = da->managed.find(o.ptr);
    if (mt == da->managed.end()) continue;
    const uint64_t size = mt->second.size;
    uint64_t lo = o.hi ? std::min(o.lo, size) : 0, hi = o.hi ? std::min(o.hi, size) : size;
    if (hi <= lo) continue;  // an empty view touches nothing
    TorchOperand* x = nullptr;
    for (auto& y : v)
      if (y.ptr == o.ptr) x = &y;
    if (!x) {
      v.push_back(TorchOperand{o.ptr, false, lo, hi, {}});
      x = &v.back();
    } else {
      x->lo = std::min(x->lo, lo);
      x->hi = std::max(x->hi, hi);
    }
    if (o.write) {
      x->write = true;
      if (o.written.empty())
        x->written.emplace_back(lo, hi);
      else
        x->written.insert(x->written.end(), o.written.begin(), o.written.end());
    }
  }
  if (!v.empty()) da->op_seq++;
  auto undo = [&](Status st) {
    for (uint64_t p : *held) (void)drop_hold(rt, da, da->managed[p], stream);
    held->clear();
    persistent->clear();
    return st;
  };
  for (auto& o : v) {
    auto& m = da->managed[o.ptr];
    const uint64_t lo = align_down(o.lo, kPageSize), hi = std::min(align_up(o.hi, kPageSize), m.size);
    Status st = add_hold(rt, da, m, device, stream, Access::READ, lo, hi - lo);
    if (st != Status::OK) return undo(st);
    held->push_back(o.ptr);
    if (o.write) {
      st = rt->invalidate_others(m.r, o.written, device);
      if (st != Status::OK) return undo(st);
    }
    if (!m.held_once) {
      m.held_once = true;
      m.first_hold_op = da->op_seq;
    } else if (da->op_seq - m.first_hold_op >= (uint64_t)std::max<int64_t>(1, config().torch_persistent_ops)) {
      m.persistent = true;
    }
    if (m.persistent) persistent->push_back(o.ptr);
    da->op_holds++;
  }
  return Status::OK;
}

// End of a dispatched op: apply the trace's next-use hints of its operands,
// then drop the op holds of `held`, and the allocation hold of every managed
// operand and output (from its first use as an operand on, a tensor is
// resident only while an op holds it; a tensor never passed to an op - a
// library workspace used behind the dispatcher's back - keeps its allocation
// hold and is never evicted).
Status torch_op_end(const std::vector<uint64_t>& held, const std::vector<uint64_t>& outs, int device, void* stream,
                    const std::vector<std::pair<uint64_t, uint64_t>>& hints, uint64_t now) {
  Runtime* rt = Runtime::get();
  if (!rt || !rt->is_local(device)) return Status::INVALID_ARGUMENT;
  DevAlloc* da = dev_alloc(device);
  std::lock_guard<std::mutex> g(da->m);
  Status res = Status::OK;
  if (now) rt->set_op_clock(device, now);
  for (auto& h : hints) {
    auto it = da->managed.find(h.first);
    if (it == da->managed.end() || it->second.next_use == h.second) continue;
    it->second.next_use = h.second;
    rt->hint_next_use(it->second.r, h.second);
  }
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
  return rt->mem_advise(it->second.r, 0, it->second.size, on ? Advice::SET_READ_MOSTLY : Advice::UNSET_READ_MOSTLY,
                        Loc::gpu(device), device);
}

// cudaMemAdvise on a managed tensor (advice / location / processor as
// rt.mem_advise: loc_kind 0 gpu, 1 host node, 2 cxl node).
Status torch_advise(void* p, int device, int advice, int loc_kind, int loc_id, int proc) {
  Runtime* rt = Runtime::get();
  if (!rt || !rt->is_local(device)) return Status::INVALID_ARGUMENT;
  DevAlloc* da = dev_alloc(device);
  std::lock_guard<std::mutex> g(da->m);
  auto it = da->managed.find((uint64_t)p);
  if (it == da->managed.end()) return Status::NOT_FOUND;
  Loc loc = loc_kind == 0 ? Loc::gpu(loc_id) : loc_kind == 1 ? Loc::host(loc_id) : Loc::cxl(loc_id);
  return rt->mem_advise(it->second.r, 0, it->second.size, (Advice)advice, loc, proc);
}

// One prefetch: hint the tensor's next use and place it on the GPU, evicting
// only data needed after `when` (VictimFloor). da->m NOT held.
static bool prefetch_one(Runtime* rt, Range* r, uint64_t size, int device, uint64_t when) {
  VictimFloor floor(when);
  Tracker t;
  return rt->prefetch(r, 0, size, Loc::gpu(device), &t, Cause::Prefetch) == Status::OK;
}

// Prefetch worker of one GPU: places queued tensors in FIFO order. A tensor
// that an op holds by now is skipped (its op faulted it in); a tensor being
// placed is marked so that a concurrent free waits for it.
static void prefetch_worker(DevAlloc* da, int device) {
  std::unique_lock<std::mutex> g(da->m);
  InAlloc in_alloc;
  for (;;) {
    da->pq_cv.wait(g, [&] { return da->stop || !da->pq.empty(); });
    if (da->stop) return;
    DevAlloc::PrefetchReq q = da->pq.front();
    da->pq.pop_front();
    auto it = da->managed.find(q.ptr);
    Runtime* rt = Runtime::get();
    if (!rt || it == da->managed.end() || it->second.holds) {
      da->pf_skipped++;
      da->pf_done_cv.notify_all();
      continue;
    }
    it->second.prefetching++;
    Range* r = it->second.r;
    const uint64_t size = it->second.size;
    g.unlock();
    prefetch_one(rt, r, size, device, q.when);
    g.lock();
    auto jt = da->managed.find(q.ptr);
    if (jt != da->managed.end() && jt->second.prefetching) jt->second.prefetching--;
    da->pf_done++;
    da->pf_done_cv.notify_all();
  }
}

// Layer-ahead prefetch of managed tensors not currently held: queue their
// H2D copies (no lease, no stream wait; a later op hold finds them resident or
// waits for the copies). Each comes with the op-clock time it is needed at:
// with next-use hints the prefetch evicts only data needed later than that,
// or is dropped (VictimFloor) - a window never pushes out what it will need
// first. With torch_async_prefetch the placement itself (evictions, stable-VA
// remaps, translation flushes: most of the host time of a streaming step)
// runs on the GPU's prefetch worker, beside the dispatching thread. Returns
// how many prefetches were queued / done.
size_t torch_prefetch(const std::vector<std::pair<uint64_t, uint64_t>>& ptrs, int device) {
  Runtime* rt = Runtime::get();
  if (!rt || !rt->is_local(device)) return 0;
  DevAlloc* da = dev_alloc(device);
  std::unique_lock<std::mutex> g(da->m);
  InAlloc in_alloc;
  size_t n = 0;
  const bool async = config().torch_async_prefetch != 0;
  for (auto& pw : ptrs) {
    auto it = da->managed.find(pw.first);
    if (it == da->managed.end() || it->second.holds) continue;
    if (pw.second && it->second.next_use != pw.second) {
      it->second.next_use = pw.second;
      rt->hint_next_use(it->second.r, pw.second);
    }
    if (async) {
      da->pq.push_back(DevAlloc::PrefetchReq{pw.first, pw.second});
      da->pf_queued++;
      ++n;
      continue;
    }
    if (prefetch_one(rt, it->second.r, it->second.size, device, pw.second)) ++n;
  }
  if (async && n) {
    if (!da->worker.joinable()) da->worker = std::thread(prefetch_worker, da, device);
    da->pq_cv.notify_one();
  }
  return n;
}

// Wait until every queued prefetch of `device` has been placed (or skipped).
void torch_prefetch_wait(int device) {
  DevAlloc* da = dev_alloc(device);
  std::unique_lock<std::mutex> g(da->m);
  InAlloc in_alloc;
  da->pf_done_cv.wait(g, [&] { return da->pq.empty() && da->pf_done + da->pf_skipped >= da->pf_queued; });
}

const char* torch_last_error(int device) {
  DevAlloc* da = dev_alloc(device);
  std::lock_guard<std::mutex> g(da->m);
  static thread_local std::string copy;
  copy = da->last_error;
  return copy.c_str();
}

uint64_t torch_managed_size(void* p, int device) {
  DevAlloc* da = dev_alloc(device);
  std::lock_guard<std::mutex> g(da->m);
  auto it = da->managed.find((uint64_t)p);
  return it == da->managed.end() ? 0 : it->second.size;
}

uint64_t torch_managed_range_id(void* p, int device) {
  DevAlloc* da = dev_alloc(device);
  std::lock_guard<std::mutex> g(da->m);
  auto it = da->managed.find((uint64_t)p);
  return it == da->managed.end() ? 0 : it->second.r->id;
}

uint64_t torch_resident_bytes(void* p, int device) {
  Runtime* rt = Runtime::get();
  Range* r = nullptr;
  {
    DevAlloc* da = dev_alloc(device);
    std::lock_guard<std::mutex> g(da->m);
    auto it = da->managed.find((uint64_t)p);
    if (!rt || it == da->managed.end()) return 0;
    r = it->second.r;
  }
  uint64_t n = 0;
  for (uint64_t bi = 0; bi < r->nblocks; ++bi) {
    ResidencyInfo ri;
    if (rt->residency_info(r, bi << kBlockShift, &ri) != Status::OK) continue;
    for (size_t k = 0; k < ri.resident_on.size(); ++k)
      if (ri.resident_on[k] == Loc::gpu(device)) n += (uint64_t)ri.pages[k] << kPageShift;
  }
  return n;
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

void torch_alloc_stats(int device, uint64_t* allocated, uint64_t* peak, uint64_t* nallocs, uint64_t* stream_waits,
                       uint64_t* lazy_fences, uint64_t* extent_hits) {
  DevAlloc* da = dev_alloc(device);
  std::lock_guard<std::mutex> g(da->m);
  *allocated = da->allocated;
  *peak = da->peak;
  *nallocs = da->nallocs;
  *stream_waits = da->stream_waits;
  if (lazy_fences) *lazy_fences = da->lazy_fences;
  if (extent_hits) *extent_hits = da->extent_hits;
}

}  // namespace ogkm

extern "C" {
// torch's pluggable-allocator path does not check for null (a null tensor
// would reach a kernel and fault the GPU), so a failed allocation throws: the
// exception unwinds through torch's allocator call into the aten op, and the
// Python caller gets a RuntimeError naming the HBM arena's state (catchable -
// e.g. free tensors and retry - instead of the process aborting).
__attribute__((visibility("default"))) void* ogkm_torch_alloc(size_t size, int device, void* stream) {
  void* p = ogkm::torch_alloc(size, device, stream);
  if (!p && size) {
    ogkm::Runtime* rt = ogkm::Runtime::get();
    ogkm::ChunkArena* a = rt ? rt->arena_for(ogkm::Loc::gpu(device)) : nullptr;
    ogkm::ChunkArena::Stats st = a ? a->stats() : ogkm::ChunkArena::Stats{};
    char msg[768];
    snprintf(msg, sizeof(msg),
             "ogkm: out of memory: torch allocation of %zu bytes on gpu %d failed (%s). HBM arena %llu MB, "
             "allocated %llu MB, pinned %llu MB (pinned = leased / held tensors + allocator slabs + tensors never "
             "used as an operand, e.g. library workspaces). Raise the HBM budget or lower the working set of one op.",
             size, device, ogkm::torch_last_error(device), (unsigned long long)(st.capacity >> 20),
             (unsigned long long)(st.allocated >> 20), (unsigned long long)(st.pinned >> 20));
    RT_ERR("%s", msg);
    throw std::runtime_error(msg);
  }
  return p;
}
__attribute__((visibility("default"))) void ogkm_torch_free(void* ptr, size_t /*size*/, int device, void* stream) {
  ogkm::torch_free(ptr, device, stream);
}
}
