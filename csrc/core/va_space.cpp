// Block / Range / VaSpace basics.
#include "ogkm/va_space.hpp"

#include <sys/mman.h>

namespace ogkm {

const char* range_type_str(RangeType t) {
  switch (t) {
    case RangeType::MANAGED: return "managed";
    case RangeType::EXTERNAL: return "external";
    case RangeType::CXL: return "cxl";
    case RangeType::DEVICE_P2P: return "device_p2p";
  }
  return "?";
}

Residency* Block::find(const Loc& l) {
  for (auto& r : res)
    if (r.loc == l) return &r;
  return nullptr;
}

Residency* Block::find_slot(int slot) {
  for (auto& r : res)
    if (r.slot == slot) return &r;
  return nullptr;
}

Residency& Block::get_or_add(const Loc& l) {
  if (Residency* r = find(l)) return *r;
  Residency r;
  r.slot = l.slot();
  r.loc = l;
  res.push_back(r);
  return res.back();
}

void Block::drop(const Loc& l) {
  for (size_t i = 0; i < res.size(); ++i)
    if (res[i].loc == l) {
      // The chunk is about to be freed or handed to another block: a CPU view
      // that still maps it must lose the mapping first, or a concurrent CPU
      // access would read (or write) the chunk's next owner.
      if (cpu_arena && cpu_arena == res[i].arena && cpu_chunk == res[i].chunk && range->cpu_view) {
        mmap(range->cpu_view + block_offset(), kBlockSize, PROT_NONE, MAP_PRIVATE | MAP_ANONYMOUS | MAP_FIXED | MAP_NORESERVE,
             -1, 0);
        cpu_arena = nullptr;
        cpu_chunk = -1;
        cpu_ro.zero();
        cpu_rw.zero();
      }
      res.erase(res.begin() + i);
      return;
    }
}

PageMask Block::resident_anywhere() const {
  PageMask m;
  for (auto& r : res) m |= r.resident;
  return m;
}

LocMask Block::resident_locs(const PageMask& pages) const {
  LocMask m = 0;
  for (auto& r : res)
    if (r.resident.intersects(pages)) m |= loc_bit(r.loc);
  return m;
}

Range::Range(VaSpace* v, uint64_t i, RangeType t, uint64_t sz, uint32_t fl, std::string nm, uint64_t want_view)
    : vs(v), id(i), type(t), size(sz), flags(fl), name(std::move(nm)) {
  nblocks = (sz + kBlockSize - 1) >> kBlockShift;
  cpu_view_bytes = nblocks << kBlockShift;
  if (t == RangeType::MANAGED && !(fl & RANGE_NO_CPU_VIEW) && want_view) {
    void* m = mmap((void*)want_view, cpu_view_bytes, PROT_NONE,
                   MAP_PRIVATE | MAP_ANONYMOUS | MAP_NORESERVE | MAP_FIXED_NOREPLACE, -1, 0);
    if (m == (void*)want_view) cpu_view = (uint8_t*)m;
    else if (m != MAP_FAILED) munmap(m, cpu_view_bytes);
  } else if (t == RangeType::MANAGED && !(fl & RANGE_NO_CPU_VIEW)) {
    // Reserve a 2 MB-aligned CPU window (PROT_NONE until blocks become
    // CPU-resident): over-reserve and trim.
    uint64_t want = cpu_view_bytes + kBlockSize;
    void* m = mmap(nullptr, want, PROT_NONE, MAP_PRIVATE | MAP_ANONYMOUS | MAP_NORESERVE, -1, 0);
    if (m != MAP_FAILED) {
      uint64_t a = align_up((uint64_t)m, kBlockSize);
      if (a > (uint64_t)m) munmap(m, a - (uint64_t)m);
      uint64_t end = (uint64_t)m + want, aend = a + cpu_view_bytes;
      if (end > aend) munmap((void*)aend, end - aend);
      cpu_view = (uint8_t*)a;
    }
  }
  blocks.reserve(nblocks);
  for (uint64_t b = 0; b < nblocks; ++b) {
    uint64_t bytes = b + 1 == nblocks ? sz - (b << kBlockShift) : kBlockSize;
    uint32_t np = (uint32_t)((bytes + kPageSize - 1) >> kPageShift);
    blocks.emplace_back(new Block(this, b, np));
  }
}

Range::~Range() {
  if (cpu_view) munmap(cpu_view, cpu_view_bytes);
}

Range* VaSpace::find_locked(uint64_t addr) {
  auto it = tree.upper_bound(addr);
  if (it == tree.begin()) return nullptr;
  --it;
  Range* r = it->second;
  if (addr >= it->first && addr < it->first + r->cpu_view_bytes) return r;
  return nullptr;
}

Range* VaSpace::by_id_locked(uint64_t id) {
  auto it = ranges.find(id);
  return it == ranges.end() ? nullptr : it->second.get();
}

}  // namespace ogkm
