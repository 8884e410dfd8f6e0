// HBM allocator for PyTorch's pluggable-allocator interface
// (torch.cuda.memory.CUDAPluggableAllocator). Allocations are carved out of the
// runtime's per-GPU HBM arena, so the framework and the model share one budget
// and managed-range eviction can make room for tensors:
//   * size <= 1 MB: power-of-two size classes (512 B .. 1 MB) sub-allocated from
//     2 MB arena chunks (a slab per class, chunks returned when empty);
//   * size  > 1 MB: a contiguous extent of 2 MB chunks, evicting cold managed
//     data through the arena's reservation protocol when the budget is full.
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

struct Slab {
  uint32_t chunk;
  uint32_t used = 0;
  std::vector<uint32_t> free_slots;
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
  uint64_t allocated = 0, peak = 0, nallocs = 0;
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

}  // namespace

void* torch_alloc(size_t size, int device) {
  Runtime* rt = Runtime::get();
  if (!rt || device < 0 || device >= rt->ndev()) return nullptr;
  ChunkArena* a = rt->arena_for(Loc::gpu(device));
  if (!a) return nullptr;
  if (size == 0) size = 1;
  DevAlloc* da = dev_alloc(device);
  int cls = class_of(size);
  std::lock_guard<std::mutex> g(da->m);
  uint64_t addr = 0;
  if (cls >= 0) {
    uint64_t csz = kMinClass << cls;
    Slab* s = nullptr;
    for (auto& x : da->slabs[cls])
      if (!x.free_slots.empty()) {
        s = &x;
        break;
      }
    if (!s) {
      uint32_t ch;
      if (rt->alloc_chunks(a, 1, -1, &ch) != Status::OK) {
        Reservation r;
        if (rt->ensure_capacity(a, 1, &r) != Status::OK) return nullptr;
        ch = (uint32_t)r.first;
      }
      a->pin(ch);  // allocator chunks are never eviction victims
      Slab ns;
      ns.chunk = ch;
      uint32_t nslots = (uint32_t)(kBlockSize / csz);
      for (uint32_t i = nslots; i-- > 0;) ns.free_slots.push_back(i);
      da->slabs[cls].push_back(std::move(ns));
      s = &da->slabs[cls].back();
    }
    uint32_t slot = s->free_slots.back();
    s->free_slots.pop_back();
    s->used++;
    addr = a->chunk_addr(s->chunk) + (uint64_t)slot * csz;
    da->live[addr] = DevAlloc::Entry{cls, s->chunk, 0, csz};
    da->allocated += csz;
  } else {
    uint32_t n = (uint32_t)((size + kBlockSize - 1) >> kBlockShift);
    uint32_t first;
    if (rt->alloc_chunks(a, n, -1, &first) != Status::OK) {
      Reservation r;
      if (rt->ensure_capacity(a, n, &r) != Status::OK) return nullptr;
      first = (uint32_t)r.first;
    }
    for (uint32_t i = 0; i < n; ++i) a->pin(first + i);
    addr = a->chunk_addr(first);
    da->live[addr] = DevAlloc::Entry{-1, first, n, (uint64_t)n << kBlockShift};
    da->allocated += (uint64_t)n << kBlockShift;
  }
  da->nallocs++;
  da->peak = std::max(da->peak, da->allocated);
  return (void*)addr;
}

void torch_free(void* p, int device) {
  Runtime* rt = Runtime::get();
  if (!rt || !p || device < 0 || device >= rt->ndev()) return;
  ChunkArena* a = rt->arena_for(Loc::gpu(device));
  DevAlloc* da = dev_alloc(device);
  std::lock_guard<std::mutex> g(da->m);
  auto it = da->live.find((uint64_t)p);
  if (it == da->live.end()) return;
  DevAlloc::Entry e = it->second;
  da->live.erase(it);
  da->allocated -= e.size;
  if (e.cls < 0) {
    for (uint32_t i = 0; i < e.n; ++i) a->unpin(e.chunk + i);
    a->free(e.chunk, e.n);
    return;
  }
  auto& slabs = da->slabs[e.cls];
  for (size_t i = 0; i < slabs.size(); ++i) {
    if (slabs[i].chunk != e.chunk) continue;
    uint64_t csz = kMinClass << e.cls;
    slabs[i].free_slots.push_back((uint32_t)(((uint64_t)p - a->chunk_addr(e.chunk)) / csz));
    if (--slabs[i].used == 0) {
      a->unpin(e.chunk);
      a->free(e.chunk, 1);
      slabs.erase(slabs.begin() + i);
    }
    return;
  }
}

void torch_alloc_stats(int device, uint64_t* allocated, uint64_t* peak, uint64_t* nallocs) {
  DevAlloc* da = dev_alloc(device);
  std::lock_guard<std::mutex> g(da->m);
  *allocated = da->allocated;
  *peak = da->peak;
  *nallocs = da->nallocs;
}

}  // namespace ogkm

extern "C" {
__attribute__((visibility("default"))) void* ogkm_torch_alloc(size_t size, int device, void* /*stream*/) {
  return ogkm::torch_alloc(size, device);
}
__attribute__((visibility("default"))) void ogkm_torch_free(void* ptr, size_t /*size*/, int device,
                                                            void* /*stream*/) {
  ogkm::torch_free(ptr, device);
}
}
