// Migration engine: make_resident / populate / evict / acquire / prefetch /
// fault service / CPU faults.
//
// Reference call stacks mirrored here:
//   service_fault_batch_block_locked  uvm_gpu_replayable_faults.c:1375
//     -> uvm_perf_thrashing_get_hint  uvm_perf_thrashing.c:1615
//     -> uvm_va_block_select_residency uvm_va_block.c:11762
//     -> uvm_va_block_service_locked  uvm_va_block.c:12307 (prefetch hint, copy, finish)
//   block_populate_pages              uvm_va_block.c:3099   (alloc-retry protocol :2060-2108)
//   block_copy_resident_pages_between uvm_va_block.c:4069   (run coalescing :4278-4326)
//   uvm_va_block_evict_chunks         uvm_va_block.c:12999
//   uvm_migrate                       uvm_migrate.c:635     (two-pass)
//
// Lock discipline: VA space (shared) -> one block at a time -> arena -> ring.
// Eviction never runs with a block lock held: the caller drops its block lock,
// evicts (locking each victim block individually), and retries - the
// MORE_PROCESSING_REQUIRED protocol.
#include <sys/mman.h>

#include <algorithm>
#include <chrono>
#include <cstring>
#include <mutex>
#include <shared_mutex>
#include <thread>

#include "ogkm/codec.hpp"
#include "ogkm/runtime.hpp"
#include "ogkm/ledger.hpp"

namespace ogkm {

namespace {

inline uint64_t page_addr(ChunkArena* a, int64_t chunk, uint32_t page) {
  // (a residency without a chunk must never become a copy address)
  RT_ASSERT_RELEASE(chunk >= 0 && (uint64_t)chunk < a->nchunks() && page < kPagesPerBlock);
  return a->chunk_addr((uint32_t)chunk) + ((uint64_t)page << kPageShift);
}

Counter xfer_counter(const Loc& s, const Loc& d) {
  if (s.is_gpu() && d.is_gpu()) return Counter::BytesXferDtD;
  if (!s.is_gpu() && d.is_gpu()) return s.tier == Tier::CXL ? Counter::BytesXferCtD : Counter::BytesXferHtD;
  if (s.is_gpu() && !d.is_gpu()) return d.tier == Tier::CXL ? Counter::BytesXferDtC : Counter::BytesXferDtH;
  if (d.tier == Tier::CXL) return Counter::BytesXferHtC;
  return Counter::BytesXferCtH;
}

}  // namespace

// ------------------------------------------------------------------ helpers
// Where evicted data goes when `full` cannot take it: the tier below it, then
// host memory of the other NUMA nodes this process knows (its GPUs' nodes and
// its host node), nearest node first.
std::vector<Loc> Runtime::fallback_targets(const Loc& full) {
  std::vector<Loc> out;
  if (full.tier == Tier::HOST) {
    Loc d = demotion_target(full);
    if (d.id >= 0) out.push_back(d);
  }
  std::vector<int> nodes{host_node_};
  for (auto& d : devs_) nodes.push_back(d->numa);
  std::sort(nodes.begin(), nodes.end());
  nodes.erase(std::unique(nodes.begin(), nodes.end()), nodes.end());
  std::sort(nodes.begin(), nodes.end(), [&](int a, int b) { return std::abs(a - full.id) < std::abs(b - full.id); });
  for (int n : nodes)
    if (!(full.tier == Tier::HOST && n == full.id) && n >= 0) out.push_back(Loc::host(n));
  return out;
}

Loc Runtime::demotion_target(const Loc& from) {
  if (from.is_gpu()) {
    // Evicted HBM data goes to host DRAM; a CXL preferred location is honoured
    // by the caller through the block policy.
    return cpu_loc();
  }
  if (from.tier == Tier::HOST) {
    // The CXL pool nearest the host node the data leaves (SLIT distance), as
    // block_select_node_residency picks the node closest to the processor
    // (uvm_va_block.c:11714-11760): with one runtime per GPU, each rank's host
    // tier is its GPU's socket, so every rank demotes to its own socket's pool.
    int n = cxl_topo_.nearest_node(from.id);
    if (n >= 0) return Loc::cxl(n);
  }
  return Loc{Tier::HOST, -1};  // nowhere to go
}

Status Runtime::alloc_chunks(ChunkArena* a, uint32_t n, int64_t hint, uint32_t* first, Block* owner, bool pin) {
  if (a->loc().is_gpu()) {
    int64_t left = inject_.alloc_fail_after.load();
    if (left == 0) {
      Tools::get().inc(Counter::InjectedErrors);
      return Status::NO_MEMORY;
    }
    if (left > 0) inject_.alloc_fail_after.fetch_sub(1);
  } else if (inject_.host_alloc_error.load() > 0 && inject_.host_alloc_error.fetch_sub(1) > 0) {
    Tools::get().inc(Counter::InjectedErrors);
    return Status::INJECTED_ERROR;
  }
  Status st = a->alloc(n, owner, hint, first, pin);
  if (st == Status::OK && !a->loc().is_gpu()) {
    st = static_cast<HostArena*>(a)->ensure_registered(*first, n);
    if (st != Status::OK) a->free(*first, n);
  }
  return st;
}

uint64_t Runtime::add_pressure_handler(int dev, PressureFn f) {
  std::lock_guard<std::mutex> g(pressure_m_);
  pressure_.emplace_back(pressure_next_, dev, std::move(f));
  return pressure_next_++;
}

void Runtime::remove_pressure_handler(uint64_t id) {
  std::lock_guard<std::mutex> g(pressure_m_);
  pressure_.erase(std::remove_if(pressure_.begin(), pressure_.end(),
                                 [id](const auto& h) { return std::get<0>(h) == id; }),
                  pressure_.end());
}

bool Runtime::relieve_pressure(const Loc& l) {
  if (!l.is_gpu()) return false;
  std::vector<PressureFn> fs;
  {
    std::lock_guard<std::mutex> g(pressure_m_);
    for (auto& h : pressure_)
      if (std::get<1>(h) == l.id) fs.push_back(std::get<2>(h));
  }
  bool any = false;
  for (auto& f : fs) any |= f();
  if (any) Tools::get().inc(Counter::PressureReliefs);
  return any;
}

// Reserve n contiguous chunks, evicting victims (no block lock may be held).
Status Runtime::ensure_capacity(ChunkArena* a, uint32_t n, Reservation* r, bool pin) {
  if (a->loc().is_gpu() && !config().global_oversubscription) return Status::NO_MEMORY;
  if (a->loc().is_gpu() && inject_.alloc_fail_after.load() == 0) {
    Tools::get().inc(Counter::InjectedErrors);
    return Status::NO_MEMORY;  // injected allocation failure: eviction cannot help either
  }
  Status st = Status::OK, es = Status::OK;
  bool relieved = false;
  for (int attempt = 0;; ++attempt) {
    st = a->reserve(n, r);
    if (st == Status::NO_MEMORY && !relieved) {  // soft pins (held leases) let go, once
      relieved = true;
      if (relieve_pressure(a->loc())) continue;
    }
    if (st != Status::OK) return st;
    es = evict_batch(a, r->victims);
    if (es == Status::OK) break;
    a->cancel(*r);  // evicted victims come back free, the busy one stays with its user
    // BUSY: a victim was leased / pinned after the reservation chose it
    // (another thread's lease): choose again.
    if (es != Status::BUSY || attempt >= 8) return es;
    std::this_thread::yield();
  }
  if (!a->loc().is_gpu()) {
    st = static_cast<HostArena*>(a)->ensure_registered((uint32_t)r->first, r->n);
    if (st != Status::OK) {
      a->cancel(*r);
      return st;
    }
  }
  a->commit(*r, pin);
  Tools::get().inc(Counter::AllocRetries);
  return Status::OK;
}

// LRU bump of a block's chunk at one location: data-less chunks go to the
// unused list, chunks whose data prefers this location to the protected list.
// What touch_residency tells the arena about residency r of block b (lock held).
static ChunkArena::TouchReq touch_req(Block* b, Residency* r, bool prefetched) {
  ChunkArena::TouchReq t{};
  t.chunk = (uint32_t)r->chunk;
  t.preferred = b->policy.has_preferred && b->policy.preferred == r->loc;
  t.has_data = !r->resident.empty();
  t.prefetched = prefetched;
  const bool refault = r->loc.is_gpu() && b->gpu_evictions > 0;
  t.refault_key = refault ? b->range->id + 1 : 0;
  t.evicted_at = b->gpu_evicted_at;
  if (r->loc.is_gpu() && config().evict_clean_first) {
    PageMask others;
    for (auto& x : b->res)
      if (&x != r) others |= x.resident;
    t.clean = r->resident.andnot(others).empty();
  }
  if (r->loc.is_gpu())
    t.next_use = b->range->dead.load(std::memory_order_relaxed) ? kDeadUse : b->range->next_use.load();
  return t;
}

void Runtime::touch_residency(Block* b, Residency* r, bool prefetched) {
  if (!r || r->chunk < 0) return;
  const ChunkArena::TouchReq t = touch_req(b, r, prefetched);
  r->arena->touch(t.chunk, t.has_data, t.preferred, t.prefetched, t.refault_key, t.evicted_at, t.clean);
  if (t.next_use) r->arena->set_next_use(t.chunk, t.next_use);
}

// Next-use hint of a whole range (the transparent mode's op trace): stored on
// the range for chunks it gets later, and set on the HBM chunks it holds now.
void Runtime::hint_next_use(Range* r, uint64_t when) {
  when = classify_hint(r, when);
  r->next_use.store(when);
  std::shared_lock<OrderedRWLock> vg(vs_.lock);
  // The range's HBM chunks, collected under their block locks, hinted under one
  // arena lock per arena (a 118-block unit: one arena lock instead of 118).
  std::vector<uint32_t> idx;
  ChunkArena* arena = nullptr;
  for (auto& bp : r->blocks) {
    Block* b = bp.get();
    std::lock_guard<OrderedMutex> g(b->lock);
    for (auto& x : b->res) {
      if (!x.loc.is_gpu() || x.chunk < 0) continue;
      if (arena && x.arena != arena) {
        arena->set_next_use_many(idx.data(), idx.size(), when);
        idx.clear();
      }
      arena = x.arena;
      idx.push_back((uint32_t)x.chunk);
    }
  }
  if (arena && !idx.empty()) arena->set_next_use_many(idx.data(), idx.size(), when);
}

void Runtime::hint_next_use(Lease* l, uint64_t when) {
  Range* r = l->range;
  // a partial or remote lease does not hold every HBM chunk of the range
  if (l->offset != 0 || l->bytes != r->size || l->remote || l->proc == kCpuProc ||
      l->pinned_chunks.size() != r->blocks.size()) {
    hint_next_use(r, when);
    return;
  }
  when = classify_hint(r, when);
  r->next_use.store(when);
  std::vector<uint32_t> idx;
  ChunkArena* arena = nullptr;
  for (auto& pc : l->pinned_chunks) {
    if (arena && pc.first != arena) {
      arena->set_next_use_many(idx.data(), idx.size(), when);
      idx.clear();
    }
    arena = pc.first;
    idx.push_back(pc.second);
  }
  if (arena && !idx.empty()) arena->set_next_use_many(idx.data(), idx.size(), when);
}

void Runtime::reset_op_clock(int dev) {
  if (ChunkArena* a = arena_for(Loc::gpu(dev))) a->reset_op_clock();
  if (is_local(dev)) devs_[dev]->spread.reset();
}

// The GPU whose arena a range's hints order: its stable-VA device, else its
// preferred GPU, else the first local GPU.
uint64_t Runtime::classify_hint(Range* r, uint64_t when) {
  if (!config().perf_spread_enable || !when || when == kDeadUse || (when & kEvictFirst)) return when;
  int dev = r->stable_dev;
  if (dev < 0 && !r->blocks.empty()) {
    Block* b0 = r->blocks[0].get();
    std::lock_guard<OrderedMutex> g(b0->lock);
    if (b0->policy.has_preferred && b0->policy.preferred.is_gpu()) dev = b0->policy.preferred.id;
  }
  if (dev < 0) {
    for (auto& d : devs_)
      if (d->local) {
        dev = d->id;
        break;
      }
  }
  if (!is_local(dev)) return when;
  ChunkArena* a = arena_for(Loc::gpu(dev));
  if (!a) return when;
  const uint64_t flag = devs_[dev]->spread.on_hint(r->id, r->size, [a] {
    auto st = a->stats();
    return SpreadPolicy::ArenaView{st.capacity, st.pinned};
  });
  r->spread_cls.store(flag ? 1 : 0, std::memory_order_relaxed);
  return when | flag;
}

SpreadPolicy::Stats Runtime::spread_stats(int dev) {
  return is_local(dev) ? devs_[dev]->spread.stats() : SpreadPolicy::Stats{};
}

void Runtime::set_op_clock(int dev, uint64_t now) {
  if (ChunkArena* a = arena_for(Loc::gpu(dev))) a->set_op_clock(now);
}

// The range's contents are dead (`dead`: a freed torch allocation) or live
// again. Dead: every copy off the GPU is dropped now (a later reuse must not
// copy garbage back) and evicting its HBM chunks copies nothing out; the
// chunks rank first among victims. Live again: the next writes repopulate it.
void Runtime::set_dead(Range* r, bool dead) {
  r->dead.store(dead);
  r->next_use.store(0);
  std::shared_lock<OrderedRWLock> vg(vs_.lock);
  Ctx c;
  for (auto& bp : r->blocks) {
    Block* b = bp.get();
    std::lock_guard<OrderedMutex> g(b->lock);
    if (dead) {
      std::vector<Loc> off_gpu;
      for (auto& x : b->res)
        if (!x.loc.is_gpu()) off_gpu.push_back(x.loc);
      for (auto& l : off_gpu) drop_copy(c, b, l);
    }
    for (auto& x : b->res)
      if (x.loc.is_gpu() && x.chunk >= 0) x.arena->set_next_use((uint32_t)x.chunk, dead ? kDeadUse : 0);
  }
  finish_ctx(c, nullptr);
}

// The GPU copy of `pages` (byte intervals of r) is about to be written by
// `gpu`: every other copy of those pages is revoked, the rest of each block
// keeps its duplicates - so an eviction copies out only what was written
// since the data was last duplicated (per-page dirty tracking,
// uvm_va_block.h:101-230 resident masks; block_copy_resident_pages copies
// only the pages it needs, uvm_va_block.c:4143-4326). The pages must be
// resident on `gpu` (a lease holds them); others are made resident first.
Status Runtime::invalidate_others(Range* r, const std::vector<std::pair<uint64_t, uint64_t>>& bytes, int gpu) {
  if (!r || !is_local(gpu)) return Status::INVALID_ARGUMENT;
  std::map<uint64_t, PageMask> per_block;
  for (auto& iv : bytes) {
    uint64_t lo = std::min(iv.first, r->size), hi = std::min(iv.second, r->size);
    if (hi <= lo) continue;
    for (uint64_t p = lo >> kPageShift, pe = (hi - 1) >> kPageShift; p <= pe;) {
      const uint64_t bi = p >> (kBlockShift - kPageShift);
      const uint32_t p0 = (uint32_t)(p & ((kBlockSize >> kPageShift) - 1));
      const uint64_t last_in_block = ((bi + 1) << (kBlockShift - kPageShift)) - 1;
      const uint64_t q = std::min(pe, last_in_block);
      per_block[bi] |= PageMask::range(p0, (uint32_t)(q - p + 1));
      p = q + 1;
    }
  }
  std::shared_lock<OrderedRWLock> vg(vs_.lock);
  Ctx c;
  Status st = Status::OK;
  const Loc dst = Loc::gpu(gpu);
  for (auto& kv : per_block) {
    Block* b = r->block(kv.first);
    if (!b) continue;
    std::lock_guard<OrderedMutex> g(b->lock);
    bool others = false;
    for (auto& x : b->res)
      if (!(x.loc == dst) && x.resident.intersects(kv.second)) others = true;
    if (!others) continue;
    st = make_resident(c, b, kv.second, dst, false, Cause::User);
    if (st != Status::OK) break;
    Tools::get().inc(Counter::WriteInvalidations);
  }
  Status fs = finish_ctx(c, nullptr);
  return st != Status::OK ? st : fs;
}

// Populate: give block b a chunk at location dst (block lock held).
Status Runtime::populate(Ctx& c, Block* b, Loc dst, int64_t hint, Residency** out) {
  if (Residency* r = b->find(dst)) {
    *out = r;
    return Status::OK;
  }
  if (inject_.populate_error.load() > 0 && inject_.populate_error.fetch_sub(1) > 0) {
    Tools::get().inc(Counter::InjectedErrors);
    return Status::INJECTED_ERROR;
  }
  ChunkArena* a = arena_for(dst);
  if (!a) return Status::INVALID_ARGUMENT;
  uint32_t chunk = 0;
  ledger_refused() = false;
  Status st = alloc_chunks(a, 1, hint, &chunk, b);
  if (st == Status::NO_MEMORY && !dst.is_gpu() && ledger_refused()) {
    // The node's budget is spent by the ranks that share it (NodeLedger), not
    // by this arena: evicting our own data would not make room. The data rests
    // on the next tier / node instead (nearest first).
    for (const Loc& alt : fallback_targets(dst)) {
      if (Residency* x = b->find(alt)) {
        *out = x;
        return Status::OK;
      }
      ChunkArena* a2 = arena_for(alt);
      if (a2 && alloc_chunks(a2, 1, -1, &chunk, b) == Status::OK) {
        Tools::get().inc(Counter::DemotionFallbacks);
        dst = alt;
        a = a2;
        st = Status::OK;
        break;
      }
    }
  }
  if (st == Status::NO_MEMORY) {
    c.need_arena = a;
    c.need_n = 1;
    return Status::MORE_PROCESSING_REQUIRED;
  }
  if (st != Status::OK) return st;
  Residency& r = b->get_or_add(dst);
  r.arena = a;
  r.chunk = chunk;
  r.resident.zero();
  *out = &r;
  return Status::OK;
}

static Ring* ring_for(Runtime* rt, const Loc& s, const Loc& d) {
  if (d.is_gpu() && !s.is_gpu()) return rt->ring(d.id, RingKind::CPU_TO_GPU);
  if (s.is_gpu() && !d.is_gpu()) return rt->ring(s.id, RingKind::GPU_TO_CPU);
  if (s.is_gpu() && d.is_gpu()) return s.id == d.id ? rt->ring(s.id, RingKind::GPU_INTERNAL)
                                                    : rt->ring(s.id, RingKind::GPU_TO_GPU);
  if (config().block_cpu_to_cpu_copy_with_ce)
    for (int d : rt->local_devices()) return rt->ring(d, RingKind::CPU_TO_GPU);
  return nullptr;
}

// Queue copies of `pages` from residency `from` to residency `to` of block b.
static Status copy_pages(Runtime* rt, Runtime::Ctx& c, Block* b, Residency* from, Residency* to,
                         const PageMask& pages) {
  if (pages.empty()) return Status::OK;
  // The source is one of this block's residencies (a stale Residency* after
  // b->res changed would fail here; the destination may be a relocation's
  // temporary, place_extent), and an HBM destination chunk is owned by the
  // block: a copy never lands in a chunk another block holds.
  auto owned = [&](const Residency* x) {
    for (const auto& y : b->res)
      if (&y == x) return true;
    return false;
  };
  RT_ASSERT_RELEASE(owned(from) && from != to);
  if (config().debug_check_copy_owner && to->loc.is_gpu() && to->chunk >= 0)
    RT_ASSERT_RELEASE(to->arena->owner((uint32_t)to->chunk) == b);
  // A packed copy that lost pages since (a write elsewhere revoked them) is no
  // whole-block source any more: back to raw pages first.
  if (from->fmt == 2 && !(from->resident == b->valid_pages())) {
    Status st = rt->expand_packed(b, from);
    if (st != Status::OK) return st;
  }
  // A segmented copy as the source: a packed segment is decoded whole, so one
  // only partly requested (or any, towards a CPU tier) is expanded on the host
  // first and moves as raw pages.
  uint32_t seg_dec = 0;  // packed segments decoded into the destination by the ring
  if (from->fmt == 3 && from->seg) {
    const uint32_t req = segs_of(pages) & from->seg->packed;
    const uint32_t part = to->loc.is_gpu() ? (req & ~segs_full(pages)) : req;
    if (part) {
      Status st = rt->expand_segments(b, from, part);
      if (st != Status::OK) return st;
    }
    if (from->seg && to->loc.is_gpu()) seg_dec = req & from->seg->packed;
  }
  const bool whole_enc = from->fmt == 1 || from->fmt == 2;  // an encoded block moves whole
  if (to->fmt == 2 && !whole_enc) {  // raw pages into a packed copy (a write-back)
    if (pages == b->valid_pages()) {
      // every page is overwritten (after the chunk's queued readers, below)
      to->fmt = 0;
      to->enc_bytes = 0;
    } else {
      Status st = rt->expand_packed(b, to);  // raw first, then the pages land
      if (st != Status::OK) return st;
    }
  }
  const bool write_back = from->loc.is_gpu() && !to->loc.is_gpu();
  if (write_back) {
    // written pages reach the host copy: note its written segments (a
    // segmented copy expands only those; the untouched ones may pack, below)
    Status st = rt->note_host_write(b, to, pages, pages);
    if (st != Status::OK) return st;
  } else if (to->fmt == 3 && !whole_enc) {
    Status st = rt->expand_segments(b, to, segs_of(pages), segs_full(pages));
    if (st != Status::OK) return st;
  }
  Ring* ring = ring_for(rt, from->loc, to->loc);
  Counter ctr = xfer_counter(from->loc, to->loc);
  // Bytes that actually cross the link (an encoded block moves its encoded size).
  PageMask raw_pages = pages;
  uint64_t bytes = 0;
  if (whole_enc) {
    bytes = from->enc_bytes;
  } else {
    for (uint32_t sg = 0; sg < kSegsPerBlock; ++sg)
      if ((seg_dec >> sg) & 1u) {
        bytes += from->seg->len[sg];
        raw_pages = raw_pages.andnot(seg_pages(sg));
      }
    bytes += (uint64_t)raw_pages.count() << kPageShift;
  }
  Tools::get().inc(ctr, bytes);
  if (whole_enc && to->loc.is_gpu()) Tools::get().inc(Counter::DecodedBytes, (uint64_t)b->npages << kPageShift);
  if (seg_dec) Tools::get().inc(Counter::DecodedBytes, (uint64_t)__builtin_popcount(seg_dec) * kSegBytes);
  if (c.cause == Cause::Prefetch) {
    if (to->loc.is_gpu()) Tools::get().inc(Counter::PrefetchBytesXferHtD, bytes);
    else Tools::get().inc(Counter::PrefetchBytesXferDtH, bytes);
  }
  uint64_t t0 = now_ns();
  bool peer_down = from->loc.is_gpu() && to->loc.is_gpu() && from->loc.id != to->loc.id &&
                   (((rt->inject().peer_link_down.load() >> from->loc.id) & 1) ||
                    !rt->be()->can_access_peer(to->loc.id, from->loc.id));
  if (peer_down) {
    // No peer path: stage GPU->GPU through host memory (uvm_va_block.c:4703-4836).
    Residency* bounce = nullptr;
    Loc h = rt->cpu_loc();
    Status st = rt->populate(c, b, h, -1, &bounce);
    if (st != Status::OK) return st;
    PageMask need = pages.andnot(bounce->resident);
    if (!need.empty()) {
      st = copy_pages(rt, c, b, from, bounce, need);
      if (st != Status::OK) return st;
      Ring* d2h = rt->ring(from->loc.id, RingKind::GPU_TO_CPU);
      FenceRef f = d2h->submit();
      b->tracker.add(f);
      bounce->resident |= need;
    }
    return copy_pages(rt, c, b, bounce, to, pages);
  }
  // The writer waits for readers of the destination chunk's previous contents
  // and for pending writes into this block issued on other rings.
  Tracker reuse = to->arena->reuse_fence((uint32_t)to->chunk);
  Tracker pend = b->tracker;
  pend.prune();
  if (!ring) {
    // CPU <-> CPU (host / CXL tiers): synchronous memcpy.
    reuse.wait();
    pend.wait();
    if (whole_enc) {
      memcpy((void*)page_addr(to->arena, to->chunk, 0), (const void*)page_addr(from->arena, from->chunk, 0),
             from->enc_bytes);
      to->fmt = from->fmt;
      to->enc_bytes = from->enc_bytes;
    } else {
      pages.for_each_run([&](uint32_t p, uint32_t n) {
        memcpy((void*)page_addr(to->arena, to->chunk, p), (const void*)page_addr(from->arena, from->chunk, p),
               (uint64_t)n << kPageShift);
      });
    }
    tools_event(ToolsEventType::Migration, c.cause, from->loc, to->loc, kCpuProc, b->range->addr() + b->block_offset(),
                bytes, b->range->id, t0, now_ns());
    return Status::OK;
  }
  if (const int64_t dw = config().debug_copy_host_wait; dw == 2 || (dw == 1 && to->loc.is_gpu())) {
    // (diagnostics) dependencies met on the host before anything is queued
    for (auto& f : reuse.fences())
      if (f->ring != ring) (void)f->wait();
    for (auto& f : pend.fences())
      if (f->ring != ring) (void)f->wait();
  }
  for (auto& f : reuse.fences()) {
    if (f->ring == ring || f->done.load(std::memory_order_relaxed) || !c.first_wait(ring, f)) continue;
    ring->push_wait(f);
  }
  for (auto& f : pend.fences()) {
    if (f->ring == ring || f->done.load(std::memory_order_relaxed) || !c.first_wait(ring, f)) continue;
    ring->push_wait(f);
  }
  if (seg_dec) {
    // Packed segments of a segmented copy: each its own ANS1 chunk, back to
    // back in the sidecar - ONE ring op for the block: one staging copy of the
    // span holding them, one decode descriptor per segment.
    const SegDir& d = *from->seg;
    uint32_t lo = ~0u, hi = 0;
    for (uint32_t sg = 0; sg < kSegsPerBlock; ++sg)
      if ((seg_dec >> sg) & 1u) {
        lo = std::min(lo, d.off[sg]);
        hi = std::max(hi, d.off[sg] + d.len[sg]);
      }
    Sqe s;
    s.op = SqeOp::DECODE_SEGS;
    s.dst = page_addr(to->arena, to->chunk, 0);
    s.src = (uint64_t)d.arena->chunk_addr((uint32_t)d.chunk) + lo;
    s.bytes = hi - lo;
    for (uint32_t sg = 0; sg < kSegsPerBlock; ++sg)
      if ((seg_dec >> sg) & 1u) {
        s.idx.push_back(sg | (d.len[sg] << 5));
        s.idx.push_back(d.off[sg] - lo);
      }
    s.user_data = b->range->id;
    s.file = __FILE__;
    s.line = __LINE__;
    ring->push(std::move(s));
    Tools::get().inc(Counter::SegDecodes, (uint64_t)__builtin_popcount(seg_dec));
    c.chunk_uses.push_back({ring, d.arena, (uint32_t)d.chunk, false});
  }
  if (whole_enc) {
    // Encoded source: the whole block decoded into HBM - BF12 by one fused
    // copy+decode kernel, ANS1 packed bytes staged by SDMA and decoded in HBM
    // (Ring DECODE_ANS) - or a verbatim copy of the encoded bytes into another
    // host / CXL chunk.
    Sqe s;
    s.op = !to->loc.is_gpu() ? SqeOp::COPY : (from->fmt == 1 ? SqeOp::DECODE_BF12 : SqeOp::DECODE_ANS);
    s.dst = page_addr(to->arena, to->chunk, 0);
    s.src = page_addr(from->arena, from->chunk, 0);
    s.bytes = from->enc_bytes;  // encoded bytes read (the output is n_values bf16)
    s.n_values = b->npages << (kPageShift - 1);
    s.user_data = b->range->id;
    s.file = __FILE__;
    s.line = __LINE__;
    ring->push(std::move(s));
    if (!to->loc.is_gpu()) {
      to->fmt = from->fmt;
      to->enc_bytes = from->enc_bytes;
    }
  } else if (raw_pages.empty()) {
    // (every requested page comes from packed segments)
  } else if (!seg_dec && raw_pages.runs() >= (uint32_t)std::max<int64_t>(2, config().copy_page_list_min_runs)) {
    // (a segmented copy's raw segments go as engine copies: a page-list kernel
    // would read the host over PCIe from the CUs and drain the ring's staged
    // decodes around it)
    // Fragmented mask: one page-list kernel (LDS-staged) instead of one copy
    // per run - the staged pack of uvm_va_block.c:4278-4326 / 3673-3860.
    Sqe s;
    s.op = SqeOp::PAGE_COPY;
    s.dst = page_addr(to->arena, to->chunk, 0);
    s.src = page_addr(from->arena, from->chunk, 0);
    s.bytes = (uint64_t)raw_pages.count() << kPageShift;
    s.idx.reserve(raw_pages.count());
    raw_pages.for_each_run([&](uint32_t p, uint32_t n) {
      for (uint32_t k = 0; k < n; ++k) s.idx.push_back(p + k);
    });
    s.user_data = b->range->id;
    s.file = __FILE__;
    s.line = __LINE__;
    ring->push(std::move(s));
    Tools::get().inc(Counter::PageListCopies);
  } else {
    raw_pages.for_each_run([&](uint32_t p, uint32_t n) {
      Sqe s;
      s.op = SqeOp::COPY;
      s.dst = page_addr(to->arena, to->chunk, p);
      s.src = page_addr(from->arena, from->chunk, p);
      s.bytes = (uint64_t)n << kPageShift;
      s.user_data = b->range->id;
      s.file = __FILE__;
      s.line = __LINE__;
      if (from->loc.is_gpu() && to->loc.is_gpu() && from->loc.id != to->loc.id) s.dst_dev = to->loc.id;
      if (log_level() >= LogLevel::DEBUG)
        s.desc = "range " + std::to_string(b->range->id) + " block " + std::to_string(b->index) + " " +
                 from->loc.str() + "->" + to->loc.str();
      ring->push(std::move(s));
    });
  }
  c.use_ring(ring);
  c.touched.push_back({ring, b});
  b->unpublished++;
  // The pages count as resident from now on: another thread that sources them
  // before this operation publishes its fence must still wait for the copy.
  b->tracker.add(ring_fence(ring, ring->pushed_seq()));
  c.chunk_uses.push_back({ring, from->arena, (uint32_t)from->chunk, false});
  tools_event(ToolsEventType::Migration, c.cause, from->loc, to->loc, to->loc.is_gpu() ? to->loc.id : kCpuProc,
              b->range->addr() + b->block_offset(), bytes, b->range->id, t0, 0, ring->pushed_seq());
  if (write_back) rt->seg_pack_enqueue(b);  // (the job waits until the write-back has landed)
  return Status::OK;
}

static Status zero_pages(Runtime* rt, Runtime::Ctx& c, Block* b, Residency* to, const PageMask& pages) {
  if (pages.empty()) return Status::OK;
  if (!to->loc.is_gpu()) {
    Tracker reuse = to->arena->reuse_fence((uint32_t)to->chunk);
    reuse.wait();
    pages.for_each_run([&](uint32_t p, uint32_t n) {
      memset((void*)page_addr(to->arena, to->chunk, p), 0, (uint64_t)n << kPageShift);
    });
    return Status::OK;
  }
  Ring* ring = rt->ring(to->loc.id, RingKind::CPU_TO_GPU);
  if (log_level() >= LogLevel::DEBUG) {
    std::string where;
    for (auto& x : b->res) where += " " + x.loc.str() + ":" + std::to_string(x.resident.count());
    RT_DBG("GPU zero-fill: range %llu '%s' block %llu pages %u (first %u) residencies%s",
           (unsigned long long)b->range->id, b->range->name.c_str(), (unsigned long long)b->index, pages.count(),
           pages.next_set(0), where.c_str());
  }
  Tracker reuse = to->arena->reuse_fence((uint32_t)to->chunk);
  for (auto& f : reuse.fences()) {
    if (f->ring == ring || f->done.load(std::memory_order_relaxed) || !c.first_wait(ring, f)) continue;
    ring->push_wait(f);
  }
  pages.for_each_run([&](uint32_t p, uint32_t n) {
    Sqe s;
    s.op = SqeOp::MEMSET;
    s.dst = page_addr(to->arena, to->chunk, p);
    s.bytes = (uint64_t)n << kPageShift;
    s.pattern = 0;
    s.file = __FILE__;
    s.line = __LINE__;
    ring->push(std::move(s));
  });
  c.use_ring(ring);
  c.touched.push_back({ring, b});
  b->unpublished++;
  b->tracker.add(ring_fence(ring, ring->pushed_seq()));
  return Status::OK;
}

// Release a residency whose pages are all gone (chunk freed after queued readers).
static void drop_residency(Runtime::Ctx& c, Block* b, const Loc& l) {
  Residency* r = b->find(l);
  if (!r) return;
  if (r->chunk >= 0) {
    Runtime::get()->shootdown(b, r);
    bool queued = false;
    for (auto& u : c.chunk_uses)
      if (u.arena == r->arena && u.chunk == (uint32_t)r->chunk) {
        u.free_after = true;
        queued = true;
        break;
      }
    if (queued) {
      // Still read by a queued copy: detach and pin (not an eviction victim)
      // until finish_ctx frees it behind the copy's fence.
      r->arena->set_owner((uint32_t)r->chunk, nullptr);
      r->arena->pin((uint32_t)r->chunk);
    } else {
      Tracker t = b->tracker;  // pending writers into the chunk
      for (auto& f : t.fences()) r->arena->add_reuse_fence((uint32_t)r->chunk, f);
      r->arena->free_when_unpinned((uint32_t)r->chunk);  // (a lease may still read it)
    }
  }
  Runtime::get()->free_sidecar(b, r);
  b->drop(l);
}

// Make `pages` of block b resident at dst (block lock held).
Status Runtime::make_resident(Ctx& c, Block* b, const PageMask& pages_in, Loc dst, bool read_dup, Cause cause) {
  PageMask pages = pages_in & b->valid_pages();
  if (pages.empty()) return Status::OK;
  if (b->range->flags & RANGE_COMPRESS_BF16) {
    // Encoded blocks move whole, and GPU copies are read-only duplicates.
    bool encoded_src = false;
    for (auto& r : b->res)
      if (r.fmt == 1) encoded_src = true;
    if (encoded_src) pages = b->valid_pages();
    if (dst.is_gpu()) read_dup = true;
  }
  c.cause = cause;
  if (!read_dup && b->lease_pins) {
    // A leased device pointer cannot be revoked under the holder: migrating
    // these pages away from a pinned copy must wait for the lease to end.
    for (auto& r : b->res)
      if (!(r.loc == dst) && r.chunk >= 0 && r.resident.intersects(pages) && r.arena->pinned((uint32_t)r.chunk))
        return Status::BUSY;
  }
  Residency* to = nullptr;
  int64_t hint = -1;
  // Keep a range's blocks adjacent in the destination arena.
  if (b->index > 0) {
    Block* prev = b->range->block(b->index - 1);
    // A hint only: skip it when the neighbour is busy (trylock keeps the lock
    // order - two block locks are never waited for at once).
    if (prev && prev->lock.try_lock()) {
      for (auto& r : prev->res)
        if (r.loc == dst && r.chunk >= 0) hint = r.chunk + 1;
      prev->lock.unlock();
    }
  }
  Status st = populate(c, b, dst, hint, &to);
  if (st != Status::OK) return st;
  PageMask missing = pages.andnot(to->resident);
  if (missing.empty() && dst.is_gpu()) {
    // Already resident here (the common case of a lease on a unit that stayed
    // in HBM): nothing moves, so no copies, no events, no CPU-view / table
    // refresh and no perf-module migration notice - only a write must still
    // revoke the other copies of these pages, and a stale stable-VA mapping
    // is still refreshed.
    bool others = false;
    if (!read_dup)
      for (auto& r : b->res)
        if (&r != to && r.resident.intersects(pages)) others = true;
    if (!others) {
      touch_residency(b, to, cause == Cause::Prefetch);
      b->last_access_ns = now_ns();
      if (b->range->dev_va && (b->stable_chunk.load() != to->chunk || b->stale_mapping.load()))
        c.cpu_refresh.push_back(b);
      return Status::OK;
    }
  }
  bool copied = false;
  // Raw pages are about to land in an encoded chunk, or a CPU consumer needs a
  // packed host copy's pages: expand it in place first. (A migration / prefetch
  // / eviction between CPU tiers keeps the packed form.)
  const bool cpu_use = !dst.is_gpu() && (cause == Cause::User || cause == Cause::Coherence);
  if (to->fmt == 3) {
    // segmented: raw pages landing expand only their segments (copy_pages); a
    // CPU consumer needs the segments of its pages raw (the CPU view maps the
    // raw segments)
    if (cpu_use) st = expand_segments(b, to, segs_of(pages));
    if (st != Status::OK) return st;
  } else if (to->fmt && (!missing.empty() || (to->fmt == 2 && cpu_use))) {
    st = expand_packed(b, to);
    if (st != Status::OK) return st;
  }
  if (!missing.empty()) {
    // Source = closest resident copy per page: same tier first, then HBM peers,
    // then host, then CXL.
    std::vector<Residency*> srcs;
    for (auto& r : b->res)
      if (&r != to) srcs.push_back(&r);
    auto rank = [&](Residency* r) {
      if (r->loc.is_gpu()) return r->loc.id == dst.id && dst.is_gpu() ? 0 : 1;
      return r->loc.tier == Tier::HOST ? 2 : 3;
    };
    std::sort(srcs.begin(), srcs.end(), [&](Residency* a, Residency* x) { return rank(a) < rank(x); });
    // A complete packed copy is a whole-block source: used alone (its decode
    // writes every page of the chunk - all of them become resident; the other
    // copies of a complete packed block are clean duplicates) unless the raw
    // copies hold every missing page.
    Residency* packed = nullptr;
    PageMask raw_cover;
    for (Residency* x : srcs) {
      if (x->fmt == 2 && x->resident == b->valid_pages()) {
        if (!packed) packed = x;
      } else if (!x->fmt) {
        raw_cover |= x->resident;
      }
    }
    if (packed && cpu_use) {
      // the CPU reads the destination: raw pages
      st = expand_packed(b, packed);
      if (st != Status::OK) return st;
      packed = nullptr;
    }
    if (packed) {
      if (missing.andnot(raw_cover).empty()) {
        srcs.erase(std::remove(srcs.begin(), srcs.end(), packed), srcs.end());
      } else {
        srcs.assign(1, packed);
        missing = b->valid_pages().andnot(to->resident);
      }
    }
    PageMask left = missing;
    for (Residency* s : srcs) {
      PageMask from_here = left & s->resident;
      if (from_here.empty()) continue;
      st = copy_pages(this, c, b, s, to, from_here);
      if (st != Status::OK) return st;
      copied = true;
      left = left.andnot(from_here);
      if (left.empty()) break;
    }
    // Never-populated pages are zero-filled (uvm_va_block.c:2863). Without the
    // fill (RANGE_NO_ZERO_FILL) nothing writes the chunk before its new owner
    // does, so the owner must still wait for the chunk's previous users (an
    // eviction copy-out may still be reading it): its reuse fence joins the
    // block's tracker, which every lease's ready-tracker includes.
    if (!left.empty() && (b->range->flags & RANGE_NO_ZERO_FILL) && to->chunk >= 0)
      b->tracker.merge(to->arena->reuse_fence((uint32_t)to->chunk));
    if (!left.empty() && !(b->range->flags & RANGE_NO_ZERO_FILL)) {
      st = zero_pages(this, c, b, to, left);
      if (st != Status::OK) return st;
    }
    to->resident |= missing;
  }
  bool moved = false;
  if (!read_dup) {
    for (auto& r : b->res)
      if (!(r.loc == dst) && r.resident.intersects(pages)) moved = true;
    if (copied) {
      // Sources stay valid until the replacing copies are submitted (finish_ctx).
      c.invals.push_back(Ctx::Inval{b, dst, pages});
      goto done;
    }
    {
    // Migration: invalidate every other copy of these pages (revocation).
    std::vector<Loc> empty_locs;
    for (auto& r : b->res) {
      if (&r == to) continue;
      if (r.resident.intersects(pages)) {
        Tools::get().inc(Counter::Revocations);
        if (b->policy.read_dup)
          tools_event(ToolsEventType::ReadDuplicateInvalidate, Cause::Coherence, r.loc, dst, kCpuProc,
                      b->range->addr() + b->block_offset(), (uint64_t)(r.resident & pages).count() << kPageShift,
                      b->range->id);
        r.resident = r.resident.andnot(pages);
        b->range->mod_gen.fetch_add(1, std::memory_order_acq_rel);
        if (r.resident.empty()) empty_locs.push_back(r.loc);
      }
    }
    // `to` may move when residencies are dropped: remember by location.
    for (auto& l : empty_locs) drop_residency(c, b, l);
    }
  } else {
    Tools::get().inc(Counter::ReadDuplications);
    tools_event(ToolsEventType::ReadDuplicate, cause, Loc::host(0), dst, dst.is_gpu() ? dst.id : kCpuProc,
                b->range->addr() + b->block_offset(), (uint64_t)pages.count() << kPageShift, b->range->id);
  }
done:
  if (Residency* t = b->find(dst)) touch_residency(b, t, cause == Cause::Prefetch);
  b->last_access_ns = now_ns();
  c.cpu_refresh.push_back(b);
  {
    // Perf modules (thrashing) see every migration through the bus.
    PerfEventData ev{PerfEvent::MIGRATION, b->range->id, b->index, Loc{}, dst, 0,
                     (uint64_t)pages.count() << kPageShift, (int)cause, 0, 0, false};
    ev.moved = moved;
    ev.block = b;
    Tools::get().bus().notify(ev);
  }
  return Status::OK;
}

// Snapshot of a block's tracker once every queued copy into it has published
// its fence (another thread may be between make_resident and finish_ctx).
Tracker Runtime::published_tracker(Block* b) {
  for (;;) {
    {
      std::lock_guard<OrderedMutex> g(b->lock);
      if (b->unpublished == 0) return b->tracker;
    }
    std::this_thread::yield();
  }
}

// Free the chunk behind residency `r` once every pending writer/reader of the
// block has finished (block lock held), and forget the residency.
static void release_residency_now(Block* b, const Loc& l) {
  Residency* r = b->find(l);
  if (!r) return;
  if (r->chunk >= 0) {
    Runtime::get()->shootdown(b, r);
    for (auto& f : b->tracker.fences()) r->arena->add_reuse_fence((uint32_t)r->chunk, f);
    // A reader may have leased this copy while the migration that revokes it
    // was in flight (the revocation lands at finish_ctx): the chunk is freed
    // when that lease ends, never under it.
    r->arena->free_when_unpinned((uint32_t)r->chunk);
  }
  Runtime::get()->free_sidecar(b, r);
  b->drop(l);
}

// Submit every ring used by the context, publish fences to blocks / chunks and
// apply (or, on a failed submission, reverse) the deferred invalidations.
Status Runtime::finish_ctx(Ctx& c, Tracker* out) {
  TraceRange tr(be_.get(), "ogkm:finish_ctx", 2);
  std::vector<std::pair<Ring*, FenceRef>> fences;
  std::vector<Ring*> failed;
  Status result = Status::OK;
  for (Ring* r : c.rings) {
    fences.emplace_back(r, r->submit());
    if (r->error() != Status::OK) {
      failed.push_back(r);
      if (result == Status::OK) result = r->error();
    }
  }
  auto fence_of = [&](Ring* r) -> FenceRef {
    for (auto& f : fences)
      if (f.first == r) return f.second;
    return nullptr;
  };
  for (auto& t : c.touched) {
    FenceRef f = fence_of(t.ring);
    std::lock_guard<OrderedMutex> g(t.block->lock);
    if (f) t.block->tracker.add(f);
    if (t.block->unpublished) t.block->unpublished--;
  }
  // Every reader's fence lands on its chunk before any chunk is freed: a chunk
  // read on two rings must not be handed out between the two fences.
  for (auto& u : c.chunk_uses)
    if (FenceRef f = fence_of(u.ring)) u.arena->add_reuse_fence(u.chunk, f);
  // Freed while still pinned (free() drops the pin in the same critical
  // section): an unpin first would let a concurrent reserve() take the
  // owner-less chunk as an eviction victim before the free.
  for (auto& u : c.chunk_uses)
    if (u.free_after) u.arena->free(u.chunk, 1);
  for (auto& iv : c.invals) {
    bool bad = false;
    for (auto& t : c.touched)
      if (t.block == iv.b && std::find(failed.begin(), failed.end(), t.ring) != failed.end()) bad = true;
    std::lock_guard<OrderedMutex> g(iv.b->lock);
    std::vector<Loc> empty;
    // Only pages the destination still holds retire their other copies: a
    // concurrent operation may have revoked (migrated away) some of them since
    // the copy was queued, and then the source is the copy that must stay.
    PageMask pages = iv.pages;
    if (!bad) {
      Residency* d = iv.b->find(iv.dst);
      pages = d ? (pages & d->resident) : PageMask{};
    }
    for (auto& r : iv.b->res) {
      bool is_dst = r.loc == iv.dst;
      if (bad ? !is_dst : is_dst) continue;  // failed copy: the destination is what becomes invalid
      if (!r.resident.intersects(pages)) continue;
      if (!bad) Tools::get().inc(Counter::Revocations);
      r.resident = r.resident.andnot(pages);
      iv.b->range->mod_gen.fetch_add(1, std::memory_order_acq_rel);
      if (r.resident.empty()) empty.push_back(r.loc);
    }
    for (auto& l : empty) release_residency_now(iv.b, l);
    c.cpu_refresh.push_back(iv.b);
  }
  if (out)
    for (auto& f : fences) out->add(f.second);
  for (Block* b : c.cpu_refresh) {
    std::lock_guard<OrderedMutex> g(b->lock);
    cpu_map_block(b);
    update_device_table(b);
    if (b->range->dev_va) stable_map_block(b);
  }
  // A caller that remaps several groups flushes once at its end (place_stable).
  if (!c.defer_flush && (thread_tlb_need() || tlb_dirty_.load(std::memory_order_relaxed))) flush_translations();
  // The context is spent; what the caller still needs for its retry (the
  // arena to evict from on MORE_PROCESSING_REQUIRED) survives the reset.
  ChunkArena* need_arena = c.need_arena;
  uint32_t need_n = c.need_n;
  Cause cause = c.cause;
  bool defer = c.defer_flush;
  c = Ctx{};
  c.need_arena = need_arena;
  c.need_n = need_n;
  c.cause = cause;
  c.defer_flush = defer;
  return result;
}

// ------------------------------------------------------------------ eviction
// Detach EVICTING chunk `i` of arena `a` from its owner block, queueing the
// copy-out of the pages only it holds into context `c` (no block lock may be
// held on entry). *detached is set when the chunk no longer belongs to a block
// (then its reuse fence must cover c's copies, see seal_evictions). Returns
// MORE_PROCESSING_REQUIRED with c.need_* set when the demotion tier is full.
Status Runtime::evict_one(Ctx& c, ChunkArena* a, uint32_t i, bool* detached) {
  TraceRange tr(be_.get(), "ogkm:evict_one", 2);
  *detached = false;
  if (inject_.evict_fail.load() > 0 && inject_.evict_fail.fetch_sub(1) > 0) {
    Tools::get().inc(Counter::InjectedErrors);
    return Status::INJECTED_ERROR;
  }
  Block* b = a->owner(i);
  if (!b) {
    *detached = true;
    return Status::OK;
  }
  std::lock_guard<OrderedMutex> g(b->lock);
  Residency* r = nullptr;
  for (auto& x : b->res)
    if (x.arena == a && x.chunk == (int64_t)i) r = &x;
  if (!r) {
    *detached = true;
    return Status::OK;
  }
  // Leased / pinned since the reservation chose it (a concurrent lease or
  // placement): not a victim after all.
  if (b->lease_pins || b->user_pins || a->pinned(i)) return Status::BUSY;
  PageMask others;
  for (auto& x : b->res)
    if (&x != r) others |= x.resident;
  PageMask only_here = r->resident.andnot(others);
  if (b->range->dead.load(std::memory_order_relaxed)) only_here.zero();  // nothing worth keeping
  Loc from = r->loc;
  uint64_t bytes = (uint64_t)r->resident.count() << kPageShift;
  if (!only_here.empty()) {
    Loc dst = demotion_target(from);
    // Honour a host/CXL preferred location for evicted HBM data.
    if (from.is_gpu() && b->policy.has_preferred && !b->policy.preferred.is_gpu()) dst = b->policy.preferred;
    if (dst.id < 0) return Status::NO_MEMORY;
    Residency* to = nullptr;
    Status st = populate(c, b, dst, -1, &to);
    if (st != Status::OK) return st;
    r = nullptr;
    for (auto& x : b->res)
      if (x.arena == a && x.chunk == (int64_t)i) r = &x;
    // Written pages going back into a packed host copy: with every page here,
    // the whole block is copied out raw over it (a D2H of the block instead of
    // a host-side decode of the packed copy to merge a few pages into).
    if (to->fmt == 2 && r->resident == b->valid_pages()) only_here = b->valid_pages();
    st = copy_pages(this, c, b, r, to, only_here);
    if (st != Status::OK) return st;
    to->resident |= only_here;
    c.cpu_refresh.push_back(b);
  }
  // Detach the chunk from the block; the arena keeps it reserved for the
  // evicting allocator, fenced on the copy-out.
  Tracker pend = b->tracker;
  shootdown(b, r);
  if (from.is_gpu()) {
    b->gpu_evictions++;
    b->gpu_evicted_at = a->evictions();
    // dropped without a copy-out: a clean read duplicate (read-mostly data);
    // a written copy restarts the count (a KV cache gets a row in every block
    // each step: packing it would only buy expansions)
    b->clean_evictions = only_here.empty() ? b->clean_evictions + 1 : 0;
    pack_enqueue(b);
    if (only_here.empty() && b->seg_written) {  // written segments cooled down: they may pack too
      b->seg_written = 0;
      seg_pack_enqueue(b);
    }
    if (is_local(from.id)) devs_[from.id]->spread.on_evict(b->range->id);
    // Users of the stable VA's mapping of this chunk (see Block::stable_users).
    if (b->range->dev_va && b->stable_chunk.load() == (int64_t)i) {
      std::lock_guard<std::mutex> sg(stable_m_);
      b->stable_users.merge(pend);
    }
  }
  b->drop(from);
  c.cpu_refresh.push_back(b);
  for (auto& f : pend.fences()) a->add_reuse_fence(i, f);
  *detached = true;
  Tools::get().inc(Counter::Evictions);
  Tools::get().inc(Counter::EvictedBytes, bytes);
  tools_event(ToolsEventType::Eviction, Cause::Eviction, from, demotion_target(from), kCpuProc,
              b->range->addr() + b->block_offset(), bytes, b->range->id);
  Tools::get().bus().notify(PerfEventData{PerfEvent::MIGRATION, b->range->id, b->index, from, demotion_target(from),
                                          kCpuProc, bytes, (int)Cause::Eviction});
  return Status::OK;
}

// Submit the copy-outs of context `c` (ONE submission per ring for every
// victim) and hand the detached chunks to the reserver: each victim's reuse
// fence covers the copies that read it; the chunks are not freed.
void Runtime::seal_evictions(Ctx& c, ChunkArena* a, const std::vector<uint32_t>& victims) {
  TraceRange tr(be_.get(), "ogkm:seal_evictions", 2);
  std::vector<std::pair<Ring*, FenceRef>> fs;
  for (Ring* rr : c.rings) fs.emplace_back(rr, rr->submit());
  for (uint32_t i : victims)
    for (auto& f : fs) a->add_reuse_fence(i, f.second);
  for (auto& u : c.chunk_uses)
    if (u.arena == a && std::find(victims.begin(), victims.end(), u.chunk) != victims.end())
      u.arena = nullptr;  // an evicted chunk is not freed
  c.chunk_uses.erase(std::remove_if(c.chunk_uses.begin(), c.chunk_uses.end(),
                                    [](const Ctx::ChunkUse& u) { return u.arena == nullptr; }),
                     c.chunk_uses.end());
  for (uint32_t i : victims) a->evicted(i);
  c.defer_flush = true;  // evictions only unmap stable VAs: nothing to flush
  finish_ctx(c, nullptr);
}

// Evict chunk `i` of arena `a` (EVICTING state). No block lock may be held.
Status Runtime::evict_chunk(ChunkArena* a, uint32_t i) { return evict_batch(a, {i}); }

// Evict a set of EVICTING chunks with one copy-out submission per ring
// (uvm_pmm_gpu.c evict_root_chunk, batched the way pick_root_chunk_to_evict's
// callers free a PMA batch). Victims whose owner is pinned are left EVICTING
// (the caller's cancel() gives them back) and BUSY is returned.
Status Runtime::evict_batch(ChunkArena* a, const std::vector<uint32_t>& victims) {
  if (victims.empty()) return Status::OK;
  TraceRange tr(be_.get(), "ogkm:evict_batch");
  Ctx c;
  c.cause = Cause::Eviction;
  std::vector<uint32_t> sealed;
  Status result = Status::OK;
  int retries = 0;
  for (size_t k = 0; k < victims.size() && result == Status::OK;) {
    bool detached = false;
    Status st = evict_one(c, a, victims[k], &detached);
    if (st == Status::OK) {
      if (detached) sealed.push_back(victims[k]);
      ++k;
      retries = 0;
      continue;
    }
    ChunkArena* na = c.need_arena;
    uint32_t nn = c.need_n ? c.need_n : 1;
    // Submit what is queued before waiting for anything.
    seal_evictions(c, a, sealed);
    sealed.clear();
    c = Ctx{};
    c.cause = Cause::Eviction;
    if (st != Status::MORE_PROCESSING_REQUIRED || ++retries > 4) {
      result = st == Status::MORE_PROCESSING_REQUIRED ? Status::NO_MEMORY : st;
      break;
    }
    // The demotion tier is full: make room there (a deeper eviction), retry.
    if (!na) na = arena_for(demotion_target(a->loc()));
    if (!na) {
      result = Status::NO_MEMORY;
      break;
    }
    Reservation rr;
    Status es = ensure_capacity(na, nn, &rr);
    if (es != Status::OK) {
      result = es;
      break;
    }
    na->free((uint32_t)rr.first, rr.n);
  }
  seal_evictions(c, a, sealed);
  return result;
}

// ------------------------------------------------------------------ prefetch / migrate
Status Runtime::prefetch(Range* r, uint64_t off, uint64_t len, Loc dst, Tracker* out, Cause cause) {
  if (global_status() != Status::OK) return global_status();
  if (quiesced_.load()) return Status::BUSY;  // checkpoint in progress: residency is frozen
  if (!r || off + len > r->size || len == 0) return Status::INVALID_ARGUMENT;
  if (r->type != RangeType::MANAGED) return Status::NOT_SUPPORTED;
  if (!arena_for(dst)) return Status::INVALID_ARGUMENT;
  TraceRange tr(be_.get(), "ogkm:prefetch");
  std::shared_lock<OrderedRWLock> vg(vs_.lock);
  if (r->group && !r->group->migratable) return Status::BUSY;
  if (cause == Cause::Prefetch || cause == Cause::ApiMigrate)
    tools_event(ToolsEventType::Prefetch, cause, Loc{}, dst, dst.is_gpu() ? dst.id : kCpuProc, r->addr() + off, len,
                r->id);
  if (dst.is_gpu()) {
    // GPU destinations are laid out as one contiguous extent so a later
    // acquire() finds the span in place (no relocation).
    for (uint64_t bi = off >> kBlockShift; bi <= (off + len - 1) >> kBlockShift; ++bi)
      if (r->block(bi)->user_pins) return Status::BUSY;
    // a prefetch ahead of a known use (next-use mode): it sits in the window
    if (VictimFloor::value() && is_local(dst.id) && config().perf_spread_enable)
      devs_[dst.id]->spread.on_prefetch(r->id, len);
    // already resident in one contiguous extent (a kept unit): an LRU touch
    if (config().lease_fast_path && !(r->dev_va && r->stable_dev == dst.id) && resident_extent(r, off, len, dst.id))
      return Status::OK;
    return gpu_extent_resident(r, off, len, dst.id, {}, nullptr, out, cause);
  }
  uint64_t b0 = off >> kBlockShift, b1 = (off + len - 1) >> kBlockShift;
  Ctx c;
  c.cause = cause;
  Status st = Status::OK;
  for (uint64_t bi = b0; bi <= b1 && st == Status::OK; ++bi) {
    Block* b = r->block(bi);
    uint64_t lo = std::max(off, bi << kBlockShift) - (bi << kBlockShift);
    uint64_t hi = std::min(off + len, (bi + 1) << kBlockShift) - (bi << kBlockShift);
    PageMask pages = PageMask::range((uint32_t)(lo >> kPageShift), (uint32_t)((hi + kPageSize - 1 - lo) >> kPageShift));
    for (int attempt = 0; attempt < 8; ++attempt) {
      {
        std::lock_guard<OrderedMutex> g(b->lock);
        if (b->user_pins) {
          st = Status::BUSY;
          break;
        }
        bool dup = b->policy.read_dup;
        st = make_resident(c, b, pages, dst, dup, cause);
      }
      if (st != Status::MORE_PROCESSING_REQUIRED) break;
      // Submit what we have so far, then evict outside the block lock.
      finish_ctx(c, out);
      Reservation rr;
      Status es = ensure_capacity(c.need_arena ? c.need_arena : arena_for(dst), c.need_n ? c.need_n : 1, &rr);
      if (es != Status::OK) {
        st = es;
        break;
      }
      ChunkArena* a = c.need_arena ? c.need_arena : arena_for(dst);
      a->free((uint32_t)rr.first, rr.n);
      c.need_arena = nullptr;
    }
  }
  Status fs = finish_ctx(c, out);
  return st != Status::OK ? st : fs;
}

Status Runtime::migrate_sync(Range* r, uint64_t off, uint64_t len, Loc dst) {
  // Two-pass scheme (uvm_migrate.c:674-722): pass 1 queues every block's copy,
  // pass 2 waits and establishes mappings.
  Tracker t;
  Status st = prefetch(r, off, len, dst, &t, Cause::ApiMigrate);
  Status w = t.wait();
  if (st == Status::OK) st = w;
  if (st == Status::OK) {
    std::shared_lock<OrderedRWLock> vg(vs_.lock);
    uint64_t b0 = off >> kBlockShift, b1 = (off + len - 1) >> kBlockShift;
    for (uint64_t bi = b0; bi <= b1; ++bi) {
      Block* b = r->block(bi);
      std::lock_guard<OrderedMutex> g(b->lock);
      b->tracker.prune();
      cpu_map_block(b);
    }
  }
  return st;
}

Status Runtime::evict_range(Range* r, Loc from) {
  if (!r) return Status::INVALID_ARGUMENT;
  ChunkArena* a = arena_for(from);
  if (!a) return Status::INVALID_ARGUMENT;
  std::vector<uint32_t> chunks;
  {
    std::shared_lock<OrderedRWLock> vg(vs_.lock);
    for (auto& bp : r->blocks) {
      std::lock_guard<OrderedMutex> g(bp->lock);
      if (Residency* x = bp->find(from))
        if (x->chunk >= 0) chunks.push_back((uint32_t)x->chunk);
    }
  }
  std::shared_lock<OrderedRWLock> vg(vs_.lock);
  for (uint32_t ch : chunks) {
    // Re-check through the reservation path: move the chunk to EVICTING.
    Reservation rr;
    rr.first = ch;
    rr.n = 1;
    // Explicit eviction: evict the owner block's data, then free the chunk.
    Block* b = a->owner(ch);
    if (!b) continue;
    Ctx c;
    c.cause = Cause::Eviction;
    Status st;
    {
      std::lock_guard<OrderedMutex> g(b->lock);
      if (b->lease_pins || b->user_pins) return Status::BUSY;
      Residency* x = b->find(from);
      if (!x || x->chunk != (int64_t)ch) continue;
      PageMask others;
      for (auto& y : b->res)
        if (&y != x) others |= y.resident;
      PageMask only_here = x->resident.andnot(others);
      if (!only_here.empty()) {
        Loc dst = demotion_target(from);
        if (from.is_gpu() && b->policy.has_preferred && !b->policy.preferred.is_gpu()) dst = b->policy.preferred;
        if (dst.id < 0) return Status::NO_MEMORY;
        // Written pages of a block whose host copy is packed, every page here:
        // drop the packed copy and write the whole block back raw (no host-side
        // decode to merge the written pages into it).
        if (Residency* h = b->find(dst); h && h->fmt == 2 && x->resident == b->valid_pages()) {
          drop_residency(c, b, dst);
          x = b->find(from);
          only_here = x->resident;
        }
        st = make_resident(c, b, only_here, dst, false, Cause::Eviction);
        if (st != Status::OK) {
          finish_ctx(c, nullptr);
          return st;
        }
      }
      // Any pages still only at `from` have been migrated; drop the rest (duplicates).
      if (b->find(from)) {
        Residency* y = b->find(from);
        y->resident.zero();
        drop_residency(c, b, from);
      }
      Tools::get().inc(Counter::Evictions);
      if (from.is_gpu()) {
        b->clean_evictions = only_here.empty() ? b->clean_evictions + 1 : 0;
        pack_enqueue(b);
      }
    }
    finish_ctx(c, nullptr);
  }
  return Status::OK;
}

// ------------------------------------------------------------------ GPU extents
// Make [off, off+len) of r resident on `gpu` in n CONSECUTIVE HBM chunks, so the
// span is one contiguous device buffer (what a kernel / torch view needs).
// Blocks already laid out in place only fetch missing pages; otherwise a fresh
// extent is allocated (evicting cold chunks through the reservation protocol)
// and resident pages are relocated D2D. With a lease, chunks are pinned.
Status Runtime::gpu_extent_resident(Range* r, uint64_t off, uint64_t len, int gpu, const std::vector<bool>& read_dup,
                                    Lease* L, Tracker* out, Cause cause) {
  // A stable-VA range on its own GPU is addressed through its VMM mapping: no
  // contiguous extent (and no relocation) is ever needed.
  if (r->dev_va && gpu == r->stable_dev) return place_stable(r, off, len, gpu, read_dup, L, out, cause);
  // An extent found in place can lose a block to a concurrent eviction between
  // the check and the copies (its chunk may already back another block): the
  // placement then starts over and relocates the span into a fresh extent.
  Status st = Status::OK;
  for (int round = 0; round < 8; ++round) {
    bool conflict = false;
    st = place_extent(r, off, len, gpu, read_dup, L, out, cause, &conflict);
    if (!conflict) return st;
    Tools::get().inc(Counter::AllocRetries);
  }
  return st;
}

Status Runtime::place_extent(Range* r, uint64_t off, uint64_t len, int gpu, const std::vector<bool>& read_dup,
                             Lease* L, Tracker* out, Cause cause, bool* conflict) {
  Loc dst = Loc::gpu(gpu);
  ChunkArena* ga = arena_for(dst);
  if (!ga) return Status::INVALID_ARGUMENT;
  uint64_t b0 = off >> kBlockShift, b1 = (off + len - 1) >> kBlockShift;
  uint32_t n = (uint32_t)(b1 - b0 + 1);
  auto pages_of = [&](uint64_t bi) {
    uint64_t lo = std::max(off, bi << kBlockShift) - (bi << kBlockShift);
    uint64_t hi = std::min(off + len, (bi + 1) << kBlockShift) - (bi << kBlockShift);
    uint32_t p0 = (uint32_t)(lo >> kPageShift), p1 = (uint32_t)((hi + kPageSize - 1) >> kPageShift);
    return PageMask::range(p0, p1 - p0);
  };
  // Concurrent acquires of one range must agree on one extent.
  std::lock_guard<OrderedMutex> placement(r->place_lock);
  Ctx c;
  c.cause = cause;
  Status st = Status::OK;
  int64_t first = -1;
  bool in_place = true;
  {
    int64_t c0 = -1;
    for (uint32_t k = 0; k < n && in_place; ++k) {
      Block* b = r->block(b0 + k);
      std::lock_guard<OrderedMutex> g(b->lock);
      Residency* x = b->find(dst);
      if (!x) in_place = false;
      else if (k == 0) c0 = x->chunk;
      else if (x->chunk != c0 + k) in_place = false;
    }
    if (in_place) first = c0;
  }
  if (!in_place) {
    const int cls = config().arena_class_sides ? r->spread_cls.load(std::memory_order_relaxed) : -1;
    PlacementSide side(cls < 0 ? 0 : cls == 0 ? 1 : 2);
    // The fresh extent stays pinned until the end of this call: its chunks have
    // no owner until each block takes its chunk, and an unpinned owner-less
    // chunk is a free eviction victim for a concurrent reserve() (two blocks
    // would end up sharing one HBM chunk).
    uint32_t f = 0;
    st = alloc_chunks(ga, n, -1, &f, nullptr, true);
    if (st == Status::OK) {
      first = f;
    } else if (st == Status::NO_MEMORY) {
      Reservation rv;
      st = ensure_capacity(ga, n, &rv, true);
      first = rv.first;
    }
    if (st != Status::OK) return st;
  }
  std::vector<Block*> done;
  // Extent chunks handed to their block: from then on the block owns (and may
  // drop) the chunk, so the allocation pin is released at hand-over, under the
  // block lock; chunks never handed over are freed (still pinned) at the end.
  std::vector<uint8_t> handed(n, 0);
  auto hand_over = [&](uint32_t k) {
    handed[k] = 1;
    ga->unpin((uint32_t)(first + k));
  };
  for (uint32_t k = 0; k < n && st == Status::OK; ++k) {
    Block* b = r->block(b0 + k);
    uint32_t target = (uint32_t)(first + k);
    for (int attempt = 0; attempt < 8; ++attempt) {
      {
        std::lock_guard<OrderedMutex> g(b->lock);
        Residency* x = b->find(dst);
        if ((in_place || handed[k]) && (!x || x->chunk != (int64_t)target)) {
          // Evicted since the in-place check (or since it was handed over, on a
          // MORE_PROCESSING_REQUIRED retry): `target` is not ours any more.
          *conflict = true;
          st = Status::BUSY;
        } else if (x && x->chunk != (int64_t)target && b->lease_pins) {
          st = Status::BUSY;  // another lease pins this block's chunk: it cannot move
        } else if (x && x->chunk != (int64_t)target) {
          // Relocate: copy the resident pages into the new extent (D2D).
          ga->set_owner(target, b);
          Residency tmp;
          tmp.slot = x->slot;
          tmp.loc = dst;
          tmp.arena = ga;
          tmp.chunk = target;
          st = copy_pages(this, c, b, x, &tmp, x->resident);
          if (st == Status::OK) {
            shootdown(b, x);
            bool queued = false;
            for (auto& u : c.chunk_uses)
              if (u.arena == x->arena && u.chunk == (uint32_t)x->chunk && !u.free_after) {
                u.free_after = true;
                x->arena->set_owner((uint32_t)x->chunk, nullptr);
                x->arena->pin((uint32_t)x->chunk);
                queued = true;
                break;
              }
            if (!queued) x->arena->free((uint32_t)x->chunk, 1);
            x->chunk = target;
            x->arena = ga;
            hand_over(k);
          } else {
            ga->set_owner(target, nullptr);
          }
        } else if (!x) {
          ga->set_owner(target, b);
          Residency& nr = b->get_or_add(dst);
          nr.arena = ga;
          nr.chunk = target;
          nr.resident.zero();
          if (!in_place) hand_over(k);
        }
        if (st == Status::OK) {
          PageMask want = pages_of(b0 + k);
          // Prefetch hint: grow the request inside the block (51% rule).
          if (config().perf_prefetch_enable) {
            Residency* y = b->find(dst);
            PageMask hint = prefetch_hint(y->resident, want, b->npages, (uint32_t)config().perf_prefetch_threshold);
            want |= (hint & b->resident_anywhere());
          }
          st = make_resident(c, b, want, dst, read_dup.empty() ? b->policy.read_dup : read_dup[k], cause);
        }
        if (st == Status::OK) {
          Residency* y = b->find(dst);
          touch_residency(b, y, cause == Cause::Prefetch && !L);
          if (L) {
            b->lease_pins++;
            y->arena->pin((uint32_t)y->chunk);
            L->pinned_chunks.emplace_back(y->arena, (uint32_t)y->chunk);
            L->blocks.push_back(b);
          }
          done.push_back(b);
        }
      }
      if (st != Status::MORE_PROCESSING_REQUIRED) break;
      finish_ctx(c, out);
      Reservation rr;
      Status es = ensure_capacity(c.need_arena, c.need_n, &rr);
      if (es != Status::OK) {
        st = es;
        break;
      }
      c.need_arena->free((uint32_t)rr.first, rr.n);
      c.need_arena = nullptr;
    }
  }
  if (!in_place)
    for (uint32_t k = 0; k < n; ++k)
      if (!handed[k]) ga->free((uint32_t)(first + k), 1);  // error path: never handed over
  Status fs = finish_ctx(c, out);
  if (st == Status::OK) st = fs;
  if (r->dev_va) {
    // A stable VA follows every block to its (possibly relocated) chunk: a
    // relocation queues no invalidation, so finish_ctx does not remap it.
    for (Block* b : done) {
      std::lock_guard<OrderedMutex> g(b->lock);
      stable_map_block(b);
    }
    if (thread_tlb_need() || tlb_dirty_.load(std::memory_order_relaxed)) flush_translations();
  }
  if (st != Status::OK) {
    if (L) {
      for (auto& pc : L->pinned_chunks) pc.first->unpin(pc.second);
      for (Block* b : L->blocks) {
        std::lock_guard<OrderedMutex> g(b->lock);
        b->lease_pins--;
      }
      L->pinned_chunks.clear();
      L->blocks.clear();
    }
    return st;
  }
  if (L) {
    for (Block* b : L->blocks) L->ready.merge(published_tracker(b));
    L->dptr = ga->chunk_addr((uint32_t)first) + (off - (b0 << kBlockShift));
  }
  return Status::OK;
}

// Stable-VA placement, in groups of `stable_batch_blocks` blocks and two
// passes so the two SDMA directions overlap:
//  A) for every group: the missing blocks get chunks - a block's previous
//     chunk when it is free again (its VMM mapping is then still right: no
//     remap), else any free chunk, else LRU victims evicted as ONE copy-out
//     submission per group. The D2H engine starts on group 0 while the host
//     evicts group 1. Blocks of the range that are already resident are
//     pinned for the call, so a later group never evicts an earlier one.
//  B) for every group: hand the chunks over and queue its fills as ONE H2D
//     submission that waits only for that group's copy-outs (H2D of group g
//     runs while D2H of group g+1 drains), then remap the group's VAs while
//     the copies fly. One translation flush covers every remap of the call.
Status Runtime::place_stable(Range* r, uint64_t off, uint64_t len, int gpu, const std::vector<bool>& read_dup,
                             Lease* L, Tracker* out, Cause cause) {
  TraceRange tr(be_.get(), "ogkm:place_stable");
  struct Clock {
    uint64_t t0 = now_ns();
    ~Clock() { Tools::get().inc(Counter::PlaceStableNs, now_ns() - t0); }
  } clock;
  Loc dst = Loc::gpu(gpu);
  ChunkArena* ga = arena_for(dst);
  if (!ga) return Status::INVALID_ARGUMENT;
  const uint64_t b0 = off >> kBlockShift, b1 = (off + len - 1) >> kBlockShift;
  auto pages_of = [&](uint64_t bi) {
    uint64_t lo = std::max(off, bi << kBlockShift) - (bi << kBlockShift);
    uint64_t hi = std::min(off + len, (bi + 1) << kBlockShift) - (bi << kBlockShift);
    uint32_t p0 = (uint32_t)(lo >> kPageShift), p1 = (uint32_t)((hi + kPageSize - 1) >> kPageShift);
    return PageMask::range(p0, p1 - p0);
  };
  // At least ~4 groups per call (so a tensor's own D2H and H2D overlap), of
  // 4 .. stable_batch_blocks blocks.
  const uint64_t cap = (uint64_t)std::max<int64_t>(1, config().stable_batch_blocks);
  const uint64_t group = std::min(cap, std::max<uint64_t>(std::min<uint64_t>(4, cap), (b1 - b0 + 1 + 3) / 4));
  std::lock_guard<OrderedMutex> placement(r->place_lock);
  Status st = Status::OK;
  struct Group {
    uint64_t g0, g1;
    std::vector<uint64_t> need;   // blocks without an HBM residency
    std::vector<uint32_t> chunks; // their chunks (pinned until handed over)
    size_t used = 0;              // chunks handed over (or given back)
  };
  std::vector<Group> groups;
  std::vector<uint32_t> kept;  // resident chunks of the range pinned for the call
  // ---- pass A: chunks (and the copy-outs they cost) for every group
  for (uint64_t g0 = b0; g0 <= b1 && st == Status::OK; g0 += group) {
    Group G{g0, std::min(b1, g0 + group - 1), {}, {}, 0};
    std::vector<int64_t> hints;
    for (uint64_t bi = G.g0; bi <= G.g1; ++bi) {
      Block* b = r->block(bi);
      for (int spin = 0;; ++spin) {
        std::unique_lock<OrderedMutex> g(b->lock);
        Residency* x = b->find(dst);
        if (!x) {
          G.need.push_back(bi);
          hints.push_back(b->stable_chunk.load());
        } else if (x->chunk >= 0) {
          if (!ga->try_pin((uint32_t)x->chunk)) {
            // Another thread chose this chunk as an eviction victim: it needs
            // the block lock to detach it - let it, then place the block anew.
            g.unlock();
            std::this_thread::yield();
            continue;
          }
          kept.push_back((uint32_t)x->chunk);
        }
        break;
      }
    }
    if (!G.need.empty() && ga->next_use_mode() && config().global_oversubscription &&
        inject_.alloc_fail_after.load() < 0) {
      // Next-use mode: every block back on its home chunk when that is free or
      // an eviction victim as good as any (ChunkArena::reserve_for) - a block
      // whose stable VA still maps its chunk needs no remap and no flush.
      std::vector<uint32_t> got;
      Reservation rv;
      st = ga->reserve_for(hints, &got, &rv);
      if (st == Status::NO_MEMORY && relieve_pressure(dst)) st = ga->reserve_for(hints, &got, &rv);
      for (int attempt = 0; st == Status::OK; ++attempt) {
        st = evict_batch(ga, rv.victims);
        if (st == Status::OK) break;
        ga->cancel(rv);
        if (st != Status::BUSY || attempt >= 8) break;
        std::this_thread::yield();
        rv = Reservation{};
        st = ga->reserve_for(hints, &got, &rv);
      }
      if (st == Status::OK) {
        ga->commit(rv, true);
        if (!rv.victims.empty()) Tools::get().inc(Counter::AllocRetries);
        G.chunks.assign(got.begin(), got.end());
      }
      groups.push_back(std::move(G));
      continue;
    }
    for (size_t k = 0; k < G.need.size(); ++k) {
      uint32_t ch = 0;
      if (alloc_chunks(ga, 1, hints[k], &ch, nullptr, true) != Status::OK) break;
      G.chunks.push_back(ch);
    }
    if (G.chunks.size() < G.need.size()) {
      Reservation rv;
      const uint32_t m = (uint32_t)(G.need.size() - G.chunks.size());
      if (!config().global_oversubscription) {
        st = Status::NO_MEMORY;
      } else if (inject_.alloc_fail_after.load() == 0) {
        Tools::get().inc(Counter::InjectedErrors);
        st = Status::NO_MEMORY;
      } else {
        st = ga->reserve_scattered(m, &rv);
        if (st == Status::NO_MEMORY && relieve_pressure(dst)) st = ga->reserve_scattered(m, &rv);
      }
      for (int attempt = 0; st == Status::OK; ++attempt) {
        st = evict_batch(ga, rv.victims);
        if (st == Status::OK) break;
        ga->cancel(rv);
        // BUSY: a victim was leased meanwhile (another thread): choose again
        if (st != Status::BUSY || attempt >= 8) break;
        std::this_thread::yield();
        rv = Reservation{};
        st = ga->reserve_scattered(m, &rv);
      }
      if (st == Status::OK) {
        ga->commit(rv, true);
        Tools::get().inc(Counter::AllocRetries);
        G.chunks.insert(G.chunks.end(), rv.list.begin(), rv.list.end());
      }
    }
    groups.push_back(std::move(G));
  }
  // ---- pass B: hand over, fill and remap group by group
  std::vector<Block*> leased;  // blocks this call pinned for L (undone on failure)
  for (size_t gi = 0; gi < groups.size() && st == Status::OK; ++gi) {
    Group& G = groups[gi];
    TraceRange trf(be_.get(), "ogkm:fill_group", 2);
    Ctx c;
    c.cause = cause;
    c.defer_flush = true;
    for (uint64_t bi = G.g0; bi <= G.g1 && st == Status::OK; ++bi) {
      Block* b = r->block(bi);
      for (int attempt = 0; attempt < 8; ++attempt) {
        {
          std::lock_guard<OrderedMutex> g(b->lock);
          Residency* x = b->find(dst);
          if (G.used < G.need.size() && G.need[G.used] == bi) {
            uint32_t ch = G.chunks[G.used++];
            if (x) {
              ga->free(ch, 1);  // populated concurrently (a prefetch): keep theirs
            } else {
              ga->set_owner(ch, b);
              Residency& nr = b->get_or_add(dst);
              nr.arena = ga;
              nr.chunk = ch;
              nr.resident.zero();
              ga->unpin(ch);
            }
          }
          PageMask want = pages_of(bi);
          const bool dup = read_dup.empty() ? b->policy.read_dup : read_dup[bi - b0];
          Residency* y = b->find(dst);
          // Fast path (the common case of a leased tensor that stayed resident):
          // every page here, mapped at the stable VA, no other copy to revoke.
          bool fast = y && want.andnot(y->resident).empty() && b->stable_chunk == y->chunk && !b->unpublished;
          if (fast && !dup)
            for (auto& o : b->res)
              if (&o != y && o.resident.intersects(want)) fast = false;
          if (!fast && config().perf_prefetch_enable) {
            PageMask hint = prefetch_hint(y ? y->resident : PageMask{}, want, b->npages,
                                          (uint32_t)config().perf_prefetch_threshold);
            want |= (hint & b->resident_anywhere());
          }
          st = fast ? Status::OK : make_resident(c, b, want, dst, dup, cause);
          if (st == Status::OK) {
            y = b->find(dst);
            touch_residency(b, y, cause == Cause::Prefetch && !L);
            // Mapped by another thread whose translation flush has not
            // completed yet: this lease flushes too before any use.
            if (b->map_seq != ~0ull && tlb_done_[gpu].load() <= b->map_seq) thread_tlb_need() |= 1u << gpu;
            if (L) {
              b->lease_pins++;
              y->arena->pin((uint32_t)y->chunk);
              L->pinned_chunks.emplace_back(y->arena, (uint32_t)y->chunk);
              L->blocks.push_back(b);
              leased.push_back(b);
            }
          }
        }
        if (st != Status::MORE_PROCESSING_REQUIRED) break;
        finish_ctx(c, out);
        Reservation rr;
        Status es = ensure_capacity(c.need_arena, c.need_n, &rr);
        if (es != Status::OK) {
          st = es;
          break;
        }
        c.need_arena->free((uint32_t)rr.first, rr.n);
        c.need_arena = nullptr;
      }
    }
    // submit the group; finish_ctx remaps the group's VAs (no flush yet)
    Status fs = finish_ctx(c, out);
    if (st == Status::OK) st = fs;
  }
  // chunks never handed over (an error part-way) go back; call pins end
  for (auto& G : groups)
    while (G.used < G.chunks.size()) ga->free(G.chunks[G.used++], 1);
  for (uint32_t ch : kept) ga->unpin(ch);
  // Blocks whose chunk did not change since they were last mapped are already
  // right; every other one was remapped above: one flush before any use.
  if (thread_tlb_need() || tlb_dirty_.load(std::memory_order_relaxed)) flush_translations();
  if (st != Status::OK) {
    if (L) {
      for (auto& pc : L->pinned_chunks) pc.first->unpin(pc.second);
      for (Block* b : leased) {
        std::lock_guard<OrderedMutex> g(b->lock);
        b->lease_pins--;
      }
      L->pinned_chunks.clear();
      L->blocks.clear();
    }
    return st;
  }
  if (L) {
    for (Block* b : L->blocks) L->ready.merge(published_tracker(b));
    L->dptr = (uint64_t)r->dev_va + off;
  }
  return Status::OK;
}

// ------------------------------------------------------------------ leases
Status Runtime::acquire(Range* r, uint64_t off, uint64_t len, int proc, Access access, Lease** out,
                        bool allow_remote) {
  TraceRange tr(be_.get(), "ogkm:acquire");
  if (global_status() != Status::OK) return global_status();
  if (quiesced_.load()) return Status::BUSY;
  if (!r || len == 0 || off + len > r->size) return Status::INVALID_ARGUMENT;
  if (proc != kCpuProc && !is_local(proc)) return Status::INVALID_ARGUMENT;
  auto L = std::make_unique<Lease>();
  L->range = r;
  L->offset = off;
  L->bytes = len;
  L->proc = proc;
  const bool packed = (r->flags & RANGE_COMPRESS_BF16) != 0;
  if (packed && (proc == kCpuProc || access == Access::WRITE || access == Access::ATOMIC))
    return Status::NOT_SUPPORTED;  // packed ranges are GPU-read-only (the host copy is encoded)
  if (r->type == RangeType::EXTERNAL || r->type == RangeType::DEVICE_P2P) {
    // Foreign / device-P2P memory never migrates: lease the original pointer.
    L->dptr = r->ext_ptr + off;
    L->remote = r->ext_dev != proc;
  } else {
    std::shared_lock<OrderedRWLock> vg(vs_.lock);
    uint64_t b0 = off >> kBlockShift, b1 = (off + len - 1) >> kBlockShift;
    uint32_t n = (uint32_t)(b1 - b0 + 1);
    Tools::get().inc(proc == kCpuProc ? Counter::CpuPageFaultCount : Counter::GpuPageFaultCount, n);
    auto pages_of = [&](uint64_t bi) {
      uint64_t lo = std::max(off, bi << kBlockShift) - (bi << kBlockShift);
      uint64_t hi = std::min(off + len, (bi + 1) << kBlockShift) - (bi << kBlockShift);
      return PageMask::range((uint32_t)(lo >> kPageShift), (uint32_t)((hi - lo + kPageSize - 1 + (lo & (kPageSize - 1))) >> kPageShift));
    };
    Loc dst = proc_loc(proc);
    // 0) fast path: a GPU read of data already resident in one contiguous
    // extent of this GPU's arena (the common streamed-or-kept unit at its use).
    // Every decision below would keep it where it is; only the pins, the LRU /
    // next-use touch and the readiness fences are needed - one arena lock for
    // all chunks instead of a placement pass (config lease_fast_path).
    if (proc != kCpuProc && access == Access::READ && !packed && !(r->dev_va && r->stable_dev == proc) &&
        config().lease_fast_path && fast_lease(r, off, len, proc, L.get())) {
      Tools::get().inc(Counter::LeaseFastPaths);
      r->views.fetch_add(1);
      std::lock_guard<std::mutex> g(leases_m_);
      L->id = next_lease_++;
      *out = L.get();
      leases_[L->id] = std::move(L);
      return Status::OK;
    }
    // 1) residency decisions
    bool all_remote = proc != kCpuProc;
    std::vector<ResidencyDecision> dec(n);
    for (uint32_t k = 0; k < n; ++k) {
      Block* b = r->block(b0 + k);
      std::lock_guard<OrderedMutex> g(b->lock);
      dec[k] = select_residency(this, b, proc, access, pages_of(b0 + k));
      if (packed) {  // encoded bytes cannot be read remotely: always decode into HBM
        dec[k].map_remote = false;
        dec[k].dst = dst;
        dec[k].read_dup = true;
      }
      // Readers never revoke another processor's leased copy: duplicate instead.
      if (access == Access::READ && b->lease_pins) dec[k].read_dup = true;
      if (!allow_remote && dec[k].map_remote && proc != kCpuProc) {
        // The caller needs the data at its own device address: a local copy
        // instead of the zero-copy mapping. A reader keeps the remote copy
        // (duplicate), so a thrash-pinned block is not pulled back and forth.
        dec[k].map_remote = false;
        dec[k].dst = dst;
        dec[k].read_dup = access == Access::READ || access == Access::PREFETCH;
        Tools::get().inc(Counter::RemoteFallbacks);
        // Software access counters on this path too (the transparent mode's op
        // holds): each such access is one the reference would count as a
        // remote access (uvm_gpu_access_counters.c:1617); at the threshold the
        // block is promoted - its next decision migrates it to this GPU
        // instead of serving another duplicate of the remote copy.
        Tools::get().inc(Counter::AccessCounterNotifications);
        uint32_t& cnt = b->counters.remote_hits[proc];
        if (++cnt >= (uint64_t)std::max<int64_t>(1, config().perf_access_counter_threshold)) {
          cnt = 0;
          if (config().perf_access_counter_migration_enable) b->counters.promote[proc] = true;
          tools_event(ToolsEventType::AccessCounter, Cause::AccessCounters, Loc{}, Loc::gpu(proc), proc,
                      r->addr() + b->block_offset(), kBlockSize, r->id);
        }
      }
      if (!dec[k].map_remote) all_remote = false;
    }
    Ctx c;
    Status st = Status::OK;
    if (proc == kCpuProc) {
      // CPU lease: the CPU view is the pointer; make pages resident on a
      // CPU-accessible tier and map them.
      for (uint32_t k = 0; k < n && st == Status::OK; ++k) {
        Block* b = r->block(b0 + k);
        for (int attempt = 0; attempt < 8; ++attempt) {
          {
            std::lock_guard<OrderedMutex> g(b->lock);
            Loc d = dec[k].map_remote ? dec[k].dst : (dec[k].dst.is_gpu() ? cpu_loc() : dec[k].dst);
            st = make_resident(c, b, pages_of(b0 + k), d, dec[k].read_dup, Cause::User);
            if (st == Status::OK) b->lease_pins++;
          }
          if (st != Status::MORE_PROCESSING_REQUIRED) break;
          finish_ctx(c, nullptr);
          Reservation rr;
          Status es = ensure_capacity(c.need_arena, c.need_n, &rr);
          if (es != Status::OK) {
            st = es;
            break;
          }
          c.need_arena->free((uint32_t)rr.first, rr.n);
        }
        if (st == Status::OK) L->blocks.push_back(b);
      }
      Status fs = finish_ctx(c, &L->ready);
      if (st == Status::OK) st = fs;
      L->ready.wait();
      for (Block* b : L->blocks) {
        published_tracker(b).wait();
        std::lock_guard<OrderedMutex> g(b->lock);
        b->tracker.prune();
        cpu_map_block(b);
      }
      L->dptr = r->addr() + off;
      if (st != Status::OK) {
        for (Block* b : L->blocks) {
          std::lock_guard<OrderedMutex> g(b->lock);
          b->lease_pins--;
        }
        return st;
      }
    } else if (all_remote) {
      // Remote (zero-copy) lease: the data stays where it is and the GPU reads it
      // over PCIe/xGMI. Requires the remote copy to be contiguous.
      int64_t first = -1;
      ChunkArena* ra = nullptr;
      bool contiguous = true;
      for (uint32_t k = 0; k < n && st == Status::OK; ++k) {
        Block* b = r->block(b0 + k);
        for (int attempt = 0; attempt < 8; ++attempt) {
          {
            std::lock_guard<OrderedMutex> g(b->lock);
            int64_t hint = first >= 0 ? first + k : -1;
            Residency* x = b->find(dec[k].dst);
            // read in place: raw pages (a segmented copy: the leased pages' segments)
            if (x && x->fmt == 3) st = expand_segments(b, x, segs_of(pages_of(b0 + k)));
            else if (x && x->fmt) st = expand_packed(b, x);
            if (st != Status::OK) break;
            if (!x) {
              st = populate(c, b, dec[k].dst, hint, &x);
              if (st == Status::OK) {
                c.cpu_refresh.push_back(b);
              }
            }
            if (st == Status::OK) {
              PageMask need = pages_of(b0 + k).andnot(x->resident);
              if (!need.empty()) st = make_resident(c, b, need, dec[k].dst, true, Cause::User);
              x = b->find(dec[k].dst);
            }
            if (st == Status::OK) {
              if (k == 0) {
                first = x->chunk;
                ra = x->arena;
              } else if (x->arena != ra || x->chunk != first + k) {
                contiguous = false;
              }
              b->lease_pins++;
              x->arena->pin((uint32_t)x->chunk);
              L->pinned_chunks.emplace_back(x->arena, (uint32_t)x->chunk);
              L->blocks.push_back(b);
              if (b->thrash.detected) Tools::get().inc(Counter::MapRemote);
            }
          }
          if (st != Status::MORE_PROCESSING_REQUIRED) break;
          finish_ctx(c, nullptr);
          Reservation rr;
          Status es = ensure_capacity(c.need_arena, c.need_n, &rr);
          if (es != Status::OK) {
            st = es;
            break;
          }
          c.need_arena->free((uint32_t)rr.first, rr.n);
        }
      }
      Status fs = finish_ctx(c, &L->ready);
      if (st == Status::OK) st = fs;
      if (st == Status::OK && !contiguous) {
        // Fall back to a local copy.
        for (auto& pc : L->pinned_chunks) pc.first->unpin(pc.second);
        for (Block* b : L->blocks) {
          std::lock_guard<OrderedMutex> g(b->lock);
          b->lease_pins--;
        }
        L->pinned_chunks.clear();
        L->blocks.clear();
        all_remote = false;
        for (auto& d : dec) d.map_remote = false;
      } else if (st == Status::OK) {
        L->remote = true;
        L->dptr = ra->chunk_addr((uint32_t)first) + (off - (b0 << kBlockShift));
        for (Block* b : L->blocks) L->ready.merge(published_tracker(b));
        Tools::get().inc(Counter::MapRemote, n);
        // Software access counters on real traffic: a remote lease is the GPU
        // reading the block over the link; hot blocks are promoted (their next
        // decision migrates them to the GPU).
        const int64_t thr = std::max<int64_t>(1, config().perf_access_counter_threshold);
        for (Block* b : L->blocks) {
          std::lock_guard<OrderedMutex> g(b->lock);
          Tools::get().inc(Counter::AccessCounterNotifications);
          tools_event(ToolsEventType::AccessCounter, Cause::AccessCounters, Loc{}, Loc::gpu(proc), proc,
                      r->addr() + b->block_offset(), kBlockSize, r->id);
          uint32_t& cnt = b->counters.remote_hits[proc];
          if (++cnt >= (uint64_t)thr) {
            cnt = 0;
            if (config().perf_access_counter_migration_enable) b->counters.promote[proc] = true;
          }
        }
      } else {
        for (auto& pc : L->pinned_chunks) pc.first->unpin(pc.second);
        for (Block* b : L->blocks) {
          std::lock_guard<OrderedMutex> g(b->lock);
          b->lease_pins--;
        }
        return st;
      }
    }
    if (proc != kCpuProc && !all_remote) {
      std::vector<bool> dup(n);
      for (uint32_t k = 0; k < n; ++k) dup[k] = dec[k].read_dup;
      st = gpu_extent_resident(r, off, len, proc, dup, L.get(), &L->ready, Cause::User);
      if (st != Status::OK) return st;
    }
  }
  r->views.fetch_add(1);
  std::lock_guard<std::mutex> g(leases_m_);
  L->id = next_lease_++;
  *out = L.get();
  leases_[L->id] = std::move(L);
  return Status::OK;
}

bool Runtime::resident_extent(Range* r, uint64_t off, uint64_t len, int gpu) {
  const Loc me = Loc::gpu(gpu);
  ChunkArena* ga = arena_for(me);
  if (!ga) return false;
  const uint64_t b0 = off >> kBlockShift, b1 = (off + len - 1) >> kBlockShift;
  int64_t first = -1;
  for (uint64_t bi = b0; bi <= b1; ++bi) {
    Block* b = r->block(bi);
    const uint64_t lo = std::max(off, bi << kBlockShift) - (bi << kBlockShift);
    const uint64_t hi = std::min(off + len, (bi + 1) << kBlockShift) - (bi << kBlockShift);
    const PageMask want = PageMask::range((uint32_t)(lo >> kPageShift),
                                          (uint32_t)((hi + kPageSize - 1) >> kPageShift) - (uint32_t)(lo >> kPageShift));
    std::lock_guard<OrderedMutex> g(b->lock);
    Residency* x = b->find(me);
    if (!x || x->chunk < 0 || x->arena != ga || (bi > b0 && x->chunk != first + (int64_t)(bi - b0)) ||
        b->unpublished || !want.andnot(x->resident).empty())
      return false;
    if (bi == b0) first = x->chunk;
    touch_residency(b, x, true);
  }
  return true;
}

bool Runtime::fast_lease(Range* r, uint64_t off, uint64_t len, int proc, Lease* L) {
  const Loc me = Loc::gpu(proc);
  ChunkArena* ga = arena_for(me);
  if (!ga || (r->group && !r->group->migratable)) return false;
  const uint64_t b0 = off >> kBlockShift, b1 = (off + len - 1) >> kBlockShift;
  const uint32_t n = (uint32_t)(b1 - b0 + 1);
  std::vector<Block*> bl;
  std::vector<uint32_t> ch;
  std::vector<ChunkArena::TouchReq> tr;
  bl.reserve(n);
  ch.reserve(n);
  tr.reserve(n);
  Tracker ready;
  bool ok = true;
  for (uint32_t k = 0; k < n && ok; ++k) {
    Block* b = r->block(b0 + k);
    const uint64_t bi = b0 + k;
    const uint64_t lo = std::max(off, bi << kBlockShift) - (bi << kBlockShift);
    const uint64_t hi = std::min(off + len, (bi + 1) << kBlockShift) - (bi << kBlockShift);
    const PageMask want = PageMask::range((uint32_t)(lo >> kPageShift),
                                          (uint32_t)((hi + kPageSize - 1) >> kPageShift) - (uint32_t)(lo >> kPageShift));
    std::lock_guard<OrderedMutex> g(b->lock);
    Residency* x = b->find(me);
    if (!x || x->chunk < 0 || x->arena != ga || (k && x->chunk != (int64_t)ch[0] + k) || b->unpublished ||
        b->user_pins || !want.andnot(x->resident).empty()) {
      ok = false;
      break;
    }
    // The chunk is pinned with the block lock held, together with lease_pins:
    // a migration that checks for leased copies (make_resident) must never see
    // the lease count without the pin (it would revoke and free the copy).
    if (!ga->try_pin((uint32_t)x->chunk)) {
      ok = false;
      break;
    }
    b->lease_pins++;
    bl.push_back(b);
    ch.push_back((uint32_t)x->chunk);
    tr.push_back(touch_req(b, x, false));
    ready.merge(b->tracker);
  }
  if (!ok) {
    for (size_t k = 0; k < bl.size(); ++k) {
      std::lock_guard<OrderedMutex> g(bl[k]->lock);
      bl[k]->lease_pins--;
      ga->unpin(ch[k]);
    }
    return false;
  }
  // LRU / next-use touches of every chunk under one arena lock
  ga->touch_many(tr.data(), tr.size());
  L->blocks = std::move(bl);
  L->pinned_chunks.reserve(ch.size());
  for (uint32_t c : ch) L->pinned_chunks.emplace_back(ga, c);
  L->ready = std::move(ready);
  L->dptr = ga->chunk_addr(ch[0]) + (off - (b0 << kBlockShift));
  return true;
}

Status Runtime::release(Lease* l, void* stream, const FenceRef& use) {
  if (!l) return Status::INVALID_ARGUMENT;
  std::unique_ptr<Lease> own;
  {
    std::lock_guard<std::mutex> g(leases_m_);
    auto it = leases_.find(l->id);
    if (it == leases_.end()) return Status::NOT_FOUND;
    own = std::move(it->second);
    leases_.erase(it);
  }
  FenceRef f;
  if (l->proc != kCpuProc && !l->pinned_chunks.empty()) f = use ? use : fence_record(be_.get(), l->proc, stream);
  // Chunks of one arena: fence + unpin + LRU touch under one arena lock.
  std::vector<uint32_t> idx;
  ChunkArena* cur = nullptr;
  auto flush = [&] {
    if (cur && !idx.empty()) cur->release_many(idx.data(), idx.size(), f);
    idx.clear();
  };
  for (auto& pc : l->pinned_chunks) {
    if (pc.first != cur) {
      flush();
      cur = pc.first;
    }
    idx.push_back(pc.second);
  }
  flush();
  // (no VA-space lock: the lease keeps its range alive - free_range refuses a
  // range with views - and a memory-pressure handler releases leases from
  // inside a placement that holds it already)
  for (Block* b : l->blocks) {
    std::lock_guard<OrderedMutex> g(b->lock);
    if (b->lease_pins) b->lease_pins--;
    if (f && l->proc != kCpuProc) {
      // GPU readers of this block: a later migration away must wait for them.
      b->tracker.add(f);
    }
  }
  l->range->views.fetch_sub(1);
  return Status::OK;
}

Lease* Runtime::lease_by_id(uint64_t id) {
  std::lock_guard<std::mutex> g(leases_m_);
  auto it = leases_.find(id);
  return it == leases_.end() ? nullptr : it->second.get();
}

// ------------------------------------------------------------------ fault batches
// Batch service (uvm_parent_gpu_service_replayable_faults, :2906): preprocess
// (sort by range, block, access; coalesce duplicates), then service per block
// with thrashing hints, residency selection and prefetch expansion.
Status Runtime::service_faults(std::vector<FaultEntry>& faults, Tracker* out) {
  if (faults.empty()) return Status::OK;
  TraceRange tr(be_.get(), "ogkm:service_faults");
  if (global_status() != Status::OK) return global_status();
  Tools::get().inc(Counter::FaultBatches);
  for (auto& f : faults) {
    f.block = f.offset >> kBlockShift;
    f.first_page = (uint32_t)((f.offset & (kBlockSize - 1)) >> kPageShift);
    uint64_t end = std::min<uint64_t>(f.offset + std::max<uint64_t>(f.bytes, 1), (f.block + 1) << kBlockShift);
    f.npages = (uint32_t)((end - (f.block << kBlockShift) + kPageSize - 1) >> kPageShift) - f.first_page;
  }
  std::sort(faults.begin(), faults.end(), [](const FaultEntry& a, const FaultEntry& b) {
    if (a.range_id != b.range_id) return a.range_id < b.range_id;
    if (a.block != b.block) return a.block < b.block;
    if (a.proc != b.proc) return a.proc < b.proc;
    if (a.first_page != b.first_page) return a.first_page < b.first_page;
    if (a.npages != b.npages) return a.npages < b.npages;
    return (int)a.access > (int)b.access;  // writes first: the highest access wins
  });
  uint64_t coalesced = 0;
  if (config().perf_fault_coalesce) {
    for (size_t i = 1; i < faults.size(); ++i) {
      FaultEntry& p = faults[i - 1];
      FaultEntry& f = faults[i];
      if (f.range_id == p.range_id && f.block == p.block && f.proc == p.proc && f.first_page == p.first_page &&
          f.npages == p.npages) {
        f.duplicate = true;
        coalesced++;
      }
    }
  }
  Tools::get().inc(Counter::FaultsCoalesced, coalesced);
  std::shared_lock<OrderedRWLock> vg(vs_.lock);
  Ctx c;
  c.cause = Cause::User;
  Status result = Status::OK;
  size_t i = 0;
  uint64_t nap_until = 0;
  while (i < faults.size()) {
    // Group: same (range, block, proc)
    size_t j = i;
    PageMask pages;
    Access acc = Access::READ;
    while (j < faults.size() && faults[j].range_id == faults[i].range_id && faults[j].block == faults[i].block &&
           faults[j].proc == faults[i].proc) {
      if (!faults[j].duplicate) {
        pages.set_range(faults[j].first_page, faults[j].npages);
        if ((int)faults[j].access > (int)acc && faults[j].access != Access::PREFETCH) acc = faults[j].access;
      }
      ++j;
    }
    Range* r = vs_.by_id_locked(faults[i].range_id);
    int proc = faults[i].proc;
    if (!r || faults[i].block >= r->nblocks || r->type != RangeType::MANAGED) {
      result = Status::INVALID_ARGUMENT;  // fatal fault: cancelled
      tools_event(ToolsEventType::FatalFault, Cause::User, Loc{}, Loc{}, proc, faults[i].offset, 0, faults[i].range_id);
      for (size_t k = i; k < j; ++k) faults[k].status = Status::INVALID_ARGUMENT;
      i = j;
      continue;
    }
    Block* b = r->block(faults[i].block);
    Status st = Status::OK;
    for (int attempt = 0; attempt < 8; ++attempt) {
      {
        std::lock_guard<OrderedMutex> g(b->lock);
        if (attempt == 0) {
          PerfEventData fe{PerfEvent::FAULT, r->id, b->index, Loc{}, proc_loc(proc), proc,
                           (uint64_t)pages.count() << kPageShift, (int)Cause::User, pages.next_set(0),
                           (uint32_t)pages.count(), acc == Access::WRITE};
          fe.block = b;
          Tools::get().bus().notify(fe);  // prefetch module: per-processor fault counts
        }
        tools_event(proc == kCpuProc ? ToolsEventType::CpuFault : ToolsEventType::GpuFault, Cause::User, Loc{}, Loc{},
                    proc, r->addr() + b->block_offset(), (uint64_t)pages.count() << kPageShift, r->id);
        ResidencyDecision d = select_residency(this, b, proc, acc, pages);
        // THROTTLE (consumed as at uvm_va_block.c:12528): the processor naps on
        // this block - map the closest copy remotely when it can reach it,
        // else come back once the nap ends.
        if (thrash_hint(b, proc_loc(proc).slot(), now_ns()) == ThrashHint::THROTTLE && !d.map_remote) {
          Loc closest;
          bool found = false;
          for (auto& x : b->res)
            if (x.resident.intersects(pages) && !x.loc.is_gpu()) {  // host / CXL: reachable by every processor
              closest = x.loc;
              found = true;
              break;
            }
          Tools::get().inc(Counter::ThrottleEvents);
          if (found && !(closest == proc_loc(proc))) {
            d.dst = closest;
            d.map_remote = true;
            d.read_dup = false;
            Tools::get().inc(Counter::MapRemote);
            tools_event(ToolsEventType::MapRemote, Cause::Thrashing, closest, proc_loc(proc), proc,
                        r->addr() + b->block_offset(), (uint64_t)pages.count() << kPageShift, r->id);
          } else {
            nap_until = b->thrash.throttle_until_ns;
          }
        }
        if (nap_until) {
          // serviced after the nap (below, outside the block lock)
        } else if (d.map_remote) {
          // Keep in place; make sure the pages exist somewhere reachable.
          PageMask have = b->resident_anywhere();
          PageMask need = pages.andnot(have);
          if (!need.empty()) st = make_resident(c, b, need, d.dst, false, Cause::User);
        } else {
          PageMask want = pages;
          Residency* y = b->find(d.dst);
          if (config().perf_prefetch_enable &&
              b->faults_by_proc[proc == kCpuProc ? kMaxGpus : proc] >= (uint32_t)config().perf_prefetch_min_faults) {
            PageMask hint = prefetch_hint(y ? y->resident : PageMask{}, pages, b->npages,
                                          (uint32_t)config().perf_prefetch_threshold);
            want |= hint & b->resident_anywhere();
          }
          st = make_resident(c, b, want, d.dst, d.read_dup, Cause::User);
        }
      }
      if (nap_until) {
        // The faulting processor naps (a CPU thread sleeps; a GPU's fault is
        // replayed later): at most one nap per group, then it is serviced.
        uint64_t now = now_ns();
        if (nap_until > now) std::this_thread::sleep_for(std::chrono::nanoseconds(nap_until - now));
        nap_until = 0;
        continue;
      }
      if (st != Status::MORE_PROCESSING_REQUIRED) break;
      finish_ctx(c, out);
      Reservation rr;
      Status es = ensure_capacity(c.need_arena, c.need_n, &rr);
      if (es != Status::OK) {
        st = es;
        break;
      }
      c.need_arena->free((uint32_t)rr.first, rr.n);
      c.need_arena = nullptr;
    }
    if (st != Status::OK && result == Status::OK) result = st;
    for (size_t k = i; k < j; ++k) faults[k].status = st;
    i = j;
  }
  Status fs = finish_ctx(c, out);
  if (result == Status::OK) result = fs;
  // Replay: with BATCH_FLUSH the waiting processors resume once every copy of the
  // batch has landed (the caller waits on `out`).
  tools_event(ToolsEventType::GpuFaultReplay, Cause::User, Loc{}, Loc{}, 0, 0, faults.size(), 0);
  return result;
}

// ------------------------------------------------------------------ CPU faults
void Runtime::cpu_fault_batch(const std::vector<std::pair<uint64_t, bool>>& faults, std::vector<Status>* out) {
  out->assign(faults.size(), Status::NOT_FOUND);
  if (faults.size() == 1) {
    (*out)[0] = cpu_fault(faults[0].first, faults[0].second);
    return;
  }
  TraceRange tr(be_.get(), "ogkm:cpu_fault_batch");
  std::vector<FaultEntry> fe;
  std::vector<Range*> ranges(faults.size(), nullptr);
  {
    std::shared_lock<OrderedRWLock> vg(vs_.lock);
    for (size_t i = 0; i < faults.size(); ++i) {
      Range* r = vs_.find_locked(faults[i].first);
      if (!r || r->type != RangeType::MANAGED) continue;
      uint64_t off = faults[i].first - r->addr();
      if (off >= r->cpu_view_bytes) continue;
      if (off >= align_up(r->size, kPageSize)) {
        (*out)[i] = Status::INVALID_ARGUMENT;
        continue;
      }
      ranges[i] = r;
      FaultEntry f;
      f.range_id = r->id;
      f.offset = align_down(off, kPageSize);
      f.bytes = kPageSize;
      f.proc = kCpuProc;
      f.access = faults[i].second ? Access::WRITE : Access::READ;
      f.ts_ns = now_ns();
      fe.push_back(f);
    }
  }
  Tools::get().inc(Counter::CpuPageFaultCount, fe.size());
  Tracker t;
  Status st = fe.empty() ? Status::OK : service_faults(fe, &t);
  t.wait();
  for (size_t i = 0; i < faults.size(); ++i) {
    if (!ranges[i]) continue;
    if (st != Status::OK) {
      (*out)[i] = cpu_fault(faults[i].first, faults[i].second);  // per-fault path (retries, BUSY)
      continue;
    }
    // Map (and, for writes, collapse duplicates) exactly as the single path does.
    (*out)[i] = cpu_fault_finish(ranges[i], faults[i].first, faults[i].second);
  }
}

Status Runtime::cpu_fault(uint64_t addr, bool write) {
  TraceRange tr(be_.get(), "ogkm:cpu_fault");
  Range* r = nullptr;
  {
    std::shared_lock<OrderedRWLock> vg(vs_.lock);
    r = vs_.find_locked(addr);
  }
  if (!r || r->type != RangeType::MANAGED) return Status::NOT_FOUND;
  uint64_t off = addr - r->addr();
  if (off >= r->cpu_view_bytes) return Status::NOT_FOUND;
  if (off >= align_up(r->size, kPageSize)) return Status::INVALID_ARGUMENT;  // past the allocation
  Tools::get().inc(Counter::CpuPageFaultCount);
  std::vector<FaultEntry> f(1);
  f[0].range_id = r->id;
  f[0].offset = align_down(off, kPageSize);
  f[0].bytes = kPageSize;
  f[0].proc = kCpuProc;
  f[0].access = write ? Access::WRITE : Access::READ;
  f[0].ts_ns = now_ns();
  Tracker t;
  Status st = service_faults(f, &t);
  t.wait();
  Status ms = cpu_fault_finish(r, addr, write);
  return st != Status::OK ? st : ms;
}

// After servicing: wait for every copy into the block, collapse duplicates of a
// written page, map the CPU view (block lock held only here).
Status Runtime::cpu_fault_finish(Range* r, uint64_t addr, bool write) {
  uint64_t off = addr - r->addr();
  std::shared_lock<OrderedRWLock> vg(vs_.lock);
  Block* b = r->block(off >> kBlockShift);
  // Concurrent faults (e.g. a multi-threaded memcpy over the CPU view) may still
  // be publishing copies into this block: wait for all of them, not just ours.
  published_tracker(b).wait();
  std::lock_guard<OrderedMutex> g(b->lock);
  b->tracker.prune();
  uint32_t page = (uint32_t)((off & (kBlockSize - 1)) >> kPageShift);
  if (write) {
    // A CPU write collapses read duplication: revoke every other copy of the page.
    Residency* cpu_res = nullptr;
    for (auto& x : b->res)
      if (!x.loc.is_gpu() && x.resident.test(page)) cpu_res = &x;
    if (cpu_res) {
      Ctx c;
      PageMask one;
      one.set(page);
      Loc keep = cpu_res->loc;
      std::vector<Loc> drop;
      for (auto& x : b->res)
        if (!(x.loc == keep) && x.resident.test(page)) {
          x.resident.clear(page);
          Tools::get().inc(Counter::Revocations);
          tools_event(ToolsEventType::ReadDuplicateInvalidate, Cause::Coherence, x.loc, keep, kCpuProc, addr,
                      kPageSize, r->id);
          if (x.resident.empty()) drop.push_back(x.loc);
        }
      for (auto& l : drop) drop_residency(c, b, l);
    }
  }
  cpu_map_block(b);
  update_device_table(b);
  if (r->dev_va) stable_map_block(b);
  return Status::OK;
}

// ------------------------------------------------------------------ device faults
size_t Runtime::drain_fault_records(int dev, std::vector<DeviceFaultRecord>* out, size_t max) {
  if (!is_local(dev)) return 0;
  DeviceFaultBuffer& fb = devs_[dev]->fault_buf;
  if (!fb.hdr) return 0;
  FaultBufHeader* h = fb.hdr;
  uint32_t ov = __atomic_load_n(&h->overflow, __ATOMIC_RELAXED);
  if (ov != fb.overflow_seen) {
    uint32_t lost = ov - fb.overflow_seen;
    fb.overflow_seen = ov;
    fb.overflows += lost;
    tools_event(ToolsEventType::FaultBufferOverflow, Cause::User, Loc{}, Loc{}, dev, 0, lost, 0);
  }
  uint32_t get = __atomic_load_n(&h->get, __ATOMIC_RELAXED);  // only the host writes GET
  const uint32_t put = __atomic_load_n(&h->put, __ATOMIC_ACQUIRE);
  size_t n = 0;
  uint64_t lost = 0;
  while (get != put && n < max) {
    const DeviceFaultRecord* rec = &fb.recs[get & (fb.entries - 1)];
    // A reserved slot becomes valid when its producer stores the sequence
    // number; a producer between the two steps is waited for briefly, else the
    // rest is left for the next poll (GET stops at the first unpublished slot).
    // A later lap's seq means a producer that gave up waiting overwrote it.
    int state = 0;  // 1 valid, 2 overwritten
    for (int spin = 0; spin < 20000 && !state; ++spin) {
      uint32_t seq = __atomic_load_n(&rec->seq, __ATOMIC_ACQUIRE);
      if (seq == get + 1) state = 1;
      else if ((int32_t)(seq - (get + 1)) > 0) state = 2;
      else if (spin > 64) std::this_thread::yield();
    }
    if (!state) break;
    if (state == 1) {
      DeviceFaultRecord copy = *rec;
      if (__atomic_load_n(&rec->seq, __ATOMIC_ACQUIRE) == get + 1) out->push_back(copy);
      else ++lost;
    } else {
      ++lost;
    }
    ++get;
    ++n;
  }
  (void)lost;  // an overwriting producer already counted it in hdr->overflow
  __atomic_store_n(&h->get, get, __ATOMIC_RELEASE);  // hands the slots back to producers
  Tools::get().inc(Counter::FaultRecordsConsumed, n);
  return n;
}

size_t Runtime::poll_device_faults(int dev) {
  if (!is_local(dev)) return 0;
  TraceRange tr(be_.get(), "ogkm:device_fault_batch");
  DeviceFaultBuffer& fb = devs_[dev]->fault_buf;
  if (!fb.hdr) return 0;
  refresh_device_tables();
  std::unique_lock<std::mutex> pg(poll_m_);  // the service thread and API callers drain one at a time
  std::vector<DeviceFaultRecord> recs;
  size_t n = drain_fault_records(dev, &recs, fb.entries);
  std::vector<FaultEntry> faults;
  std::vector<std::pair<uint64_t, uint32_t>> remote_hits;
  // Per-channel attribution (record.proc = dev | channel << 16) and the
  // precise cancel of faults no service can satisfy.
  std::vector<std::pair<uint16_t, int>> per_channel;  // (channel, 0 fault / 1 remote / 2 fatal)
  for (const DeviceFaultRecord& rec : recs) {
    const uint16_t ch = (uint16_t)(rec.proc >> 16);
    if (rec.kind == 1) {
      remote_hits.emplace_back(rec.range_id, rec.block);
      if (ch) per_channel.emplace_back(ch, 1);
      continue;
    }
    bool valid;
    {
      std::shared_lock<OrderedRWLock> vg(vs_.lock);
      Range* r = vs_.by_id_locked(rec.range_id);
      valid = r && r->type == RangeType::MANAGED && rec.block < r->nblocks;
    }
    if (!valid) {
      // A fault on a freed range / past its end: fatal for the faulting
      // channel, not serviced (the kernel's gate times out or is cancelled).
      if (ch) per_channel.emplace_back(ch, 2);
      tools_event(ToolsEventType::FatalFault, Cause::User, Loc{}, Loc::gpu(dev), dev, 0, 0, rec.range_id);
      continue;
    }
    FaultEntry f;
    f.range_id = rec.range_id;
    const bool whole = rec.page == kFaultWholeBlock;  // a gate needs the whole block in HBM
    f.offset = ((uint64_t)rec.block << kBlockShift) + (whole ? 0 : ((uint64_t)rec.page << kPageShift));
    f.bytes = whole ? kBlockSize : kPageSize;
    f.proc = (int)(rec.proc & 0xffff);
    f.channel = ch;
    f.access = rec.access == 2 ? Access::WRITE : Access::READ;
    faults.push_back(f);
    if (ch) per_channel.emplace_back(ch, 0);
  }
  if (!per_channel.empty()) {
    std::lock_guard<std::mutex> g(channels_m_);
    for (auto& pc : per_channel) {
      if (pc.first > channels_.size() || !channels_[pc.first - 1].id) continue;
      Channel& c = channels_[pc.first - 1];
      if (pc.second == 0) c.faults++;
      else if (pc.second == 1) c.remote_accesses++;
      else {
        c.fatal_faults++;
        c.error = Status::INVALID_ARGUMENT;
      }
    }
  }
  Tools::get().inc(Counter::GpuPageFaultCount, faults.size());
  // Access counters (uvm_gpu_access_counters.c:1617): migrate hot remote blocks.
  int64_t mig = config().perf_access_counter_migration_enable;
  if (!remote_hits.empty()) {
    std::vector<std::pair<Range*, uint64_t>> hot;
    {
      std::shared_lock<OrderedRWLock> vg(vs_.lock);
      for (auto& h : remote_hits) {
        Range* r = vs_.by_id_locked(h.first);
        if (!r || h.second >= r->nblocks) continue;
        Block* b = r->block(h.second);
        std::lock_guard<OrderedMutex> g(b->lock);
        Tools::get().inc(Counter::AccessCounterNotifications);
        tools_event(ToolsEventType::AccessCounter, Cause::AccessCounters, Loc{}, Loc::gpu(dev), dev,
                    r->addr() + b->block_offset(), kBlockSize, r->id);
        uint32_t& cnt = b->counters.remote_hits[dev];
        if (++cnt >= (uint64_t)config().perf_access_counter_threshold) {
          cnt = 0;
          if (mig != 0) hot.emplace_back(r, h.second);
        }
      }
    }
    for (auto& h : hot) {
      Tracker t;
      if (prefetch(h.first, h.second << kBlockShift,
                   std::min<uint64_t>(kBlockSize, h.first->size - (h.second << kBlockShift)), Loc::gpu(dev), &t,
                   Cause::AccessCounters) == Status::OK)
        Tools::get().inc(Counter::AccessCounterMigrations);
    }
  }
  // Precise cancel (cancel_faults_precise, uvm_gpu_replayable_faults.c:2863):
  // channels whose faults cannot be serviced are marked errored and their
  // gates released with kGateCancelled instead of being replayed blindly.
  std::vector<std::pair<uint16_t, Status>> cancel;
  for (auto& pc : per_channel)
    if (pc.second == 2) cancel.emplace_back(pc.first, Status::INVALID_ARGUMENT);
  if (!faults.empty()) {
    Tracker t;
    Status sst = service_faults(faults, &t);
    Status wst = t.wait();
    for (auto& f : faults) {
      Status fst = f.status != Status::OK ? f.status : wst;
      if (fst != Status::OK) cancel.emplace_back(f.channel, fst);
    }
    if (sst != Status::OK)
      RT_WARN("device fault batch on GPU %d: service failed (%s), %zu fault(s) cancelled", dev, status_str(sst),
              cancel.size());
    // The batch has landed: publish the new residency to the device tables
    // (entries stay 0 while copies are in flight), then replay - kernels
    // stalled in k_fault_gate re-check and proceed (BATCH_FLUSH policy).
    {
      std::shared_lock<OrderedRWLock> vg(vs_.lock);
      for (auto& f : faults) {
        Range* r = vs_.by_id_locked(f.range_id);
        if (!r || f.block >= r->nblocks) continue;
        Block* b = r->block(f.block);
        published_tracker(b).wait();
        std::lock_guard<OrderedMutex> g(b->lock);
        b->tracker.prune();
        update_device_table(b);
      }
    }
  }
  if (!cancel.empty()) {
    // Mark the channels errored, then bump their cancel words BEFORE the replay
    // token: a woken gate sees the cancel, never a bare replay of a fault that
    // will not be serviced.
    std::sort(cancel.begin(), cancel.end(),
              [](const std::pair<uint16_t, Status>& a, const std::pair<uint16_t, Status>& b) { return a.first < b.first; });
    uint16_t last = 0xffff;
    for (auto& cc : cancel) {
      if (cc.first == last) continue;
      last = cc.first;
      {
        std::lock_guard<std::mutex> g(channels_m_);
        if (cc.first && cc.first <= channels_.size() && channels_[cc.first - 1].id) {
          Channel& ch = channels_[cc.first - 1];
          if (ch.error == Status::OK) ch.error = cc.second;
          ch.cancelled_faults++;
        }
      }
      // Unattributed faults (channel 0) are never cancelled: their gates fall
      // back to the replay / timeout path (a cancel word shared by every
      // unregistered stream would cancel gates whose faults were serviced).
      if (!cc.first || cc.first >= kFaultCancelSlots) continue;
      __atomic_fetch_add(&fb.hdr->cancel[cc.first], 1u, __ATOMIC_RELEASE);
      Tools::get().inc(Counter::FaultsCancelled);
    }
  }
  if (!faults.empty() || !cancel.empty()) {
    __atomic_fetch_add(&fb.hdr->replay, 1, __ATOMIC_RELEASE);
    Tools::get().inc(Counter::FaultReplays);
    tools_event(ToolsEventType::GpuFaultReplay, Cause::User, Loc{}, Loc::gpu(dev), dev, 0, faults.size(), 0);
  }
  return n;
}

}  // namespace ogkm

namespace ogkm {
void Runtime::drop_copy(Ctx& c, Block* b, const Loc& l) { drop_residency(c, b, l); }
Status Runtime::queue_copy(Ctx& c, Block* b, Residency* from, Residency* to, const PageMask& pages) {
  return copy_pages(this, c, b, from, to, pages);
}
}  // namespace ogkm
