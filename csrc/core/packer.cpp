// Packed host copies of read-mostly managed blocks (Residency::fmt 2).
//
// A block whose HBM copy keeps being dropped without a copy-out (a clean read
// duplicate: weights under the transparent mode; once is enough for a range
// advised SET_READ_MOSTLY) gets its complete raw host / CXL copy rewritten in place as
// one lossless ANS1 chunk (codec.hpp: rANS over the bf16 exponents, ~0.66 of
// the bytes for weight-like data). From then on every H2D refill moves only the
// packed bytes: the CPU->GPU ring lands them in an HBM staging buffer by SDMA
// and one k_ans_blocks launch decodes a whole batch of blocks into their HBM
// chunks (Ring DECODE_ANS). Nothing else changes for the consumer - the chunk
// it leases holds raw pages - so this works for any torch tensor.
//
// The packed copy is a read-only duplicate: a CPU mapping, a CPU consumer or
// raw pages landing in it expand it back first (expand_packed), a copy that
// lost pages to a write elsewhere is expanded before it serves as a source
// again, and the CPU view never maps it.
//
// Packing runs on pack_threads host workers, off every hot path:
//   1. under the block lock: check the copy (complete, raw, nothing pending,
//      not leased) and snapshot it;
//   2. unlocked: encode the snapshot (kept only when it saves
//      pack_min_saving_pct);
//   3. under the block lock again: same copy, still quiet, no queued reader of
//      its chunk; revoke the CPU view, compare the chunk with the snapshot
//      (a CPU store between 1 and 3 shows up here and cancels), write the
//      packed bytes over it.
// Reference parity: the staged pack-through-buffer copies of
// uvm_va_block.c:3673-3760 (there: a GPU copy engine through a staging page;
// here: SDMA into HBM staging + an LDS-table rANS decode kernel).
#include <chrono>
#include <cstring>
#include <thread>
#include <vector>

#include "ogkm/codec.hpp"
#include "ogkm/runtime.hpp"

namespace ogkm {

namespace {

// The complete raw host / CXL copy packing would rewrite (host tier first).
Residency* pack_candidate(Block* b) {
  Residency* best = nullptr;
  for (auto& x : b->res) {
    if (x.loc.is_gpu() || x.chunk < 0 || x.fmt != 0 || !(x.resident == b->valid_pages())) continue;
    if (!best || (x.loc.tier == Tier::HOST && best->loc.tier != Tier::HOST)) best = &x;
  }
  return best;
}

}  // namespace

Status Runtime::expand_packed(Block* b, Residency* r) {
  if (!r || r->fmt == 0 || r->chunk < 0) return Status::OK;
  if (r->fmt == 3) return expand_segments(b, r, ~0u);
  // Queued readers of the packed bytes (decodes, verbatim copies) and queued
  // writers into the block finish first: the chunk is rewritten in place.
  Tracker rf = r->arena->reuse_fence((uint32_t)r->chunk);
  Status st = rf.wait();
  if (st == Status::OK) {
    Tracker t = b->tracker;
    st = t.wait();
  }
  if (st != Status::OK) return st;
  const uint32_t nv = b->npages << (kPageShift - 1);
  std::vector<uint16_t> tmp(nv);
  uint8_t* base = (uint8_t*)r->arena->chunk_addr((uint32_t)r->chunk);
  if (!block_decode(r->fmt, base, tmp.data(), nv)) return Status::IO_ERROR;
  memcpy(base, tmp.data(), (size_t)nv * 2);
  if (r->fmt == 2) Tools::get().inc(Counter::PackExpansions);
  r->fmt = 0;
  r->enc_bytes = 0;
  b->pack_skip = false;
  b->clean_evictions = 0;
  return Status::OK;
}

// ------------------------------------------------------------ segmented copies (fmt 3)

void Runtime::free_sidecar(Block* b, Residency* r) {
  if (!r->seg) return;
  SegDir& d = *r->seg;
  if (d.chunk >= 0) {
    // queued staging copies of the packed segments hold ring fences in the
    // block's tracker (copy_pages): the sidecar is handed out again after them
    Tracker t = b->tracker;
    for (auto& f : t.fences()) d.arena->add_reuse_fence((uint32_t)d.chunk, f);
    d.arena->free_when_unpinned((uint32_t)d.chunk);
  }
  r->seg.reset();
  if (r->fmt == 3) r->fmt = 0;
}

Status Runtime::expand_segments(Block* b, Residency* r, uint32_t segs, uint32_t overwrite) {
  if (!r || r->fmt != 3 || !r->seg) return Status::OK;
  SegDir& d = *r->seg;
  segs &= d.packed;
  if (!segs) return Status::OK;
  const uint32_t dec = segs & ~overwrite;
  if (dec) {
    // The stale raw pages of these segments are rewritten in place: queued
    // writers into the block (and readers of the chunk) finish first.
    Tracker rf = r->arena->reuse_fence((uint32_t)r->chunk);
    Status st = rf.wait();
    if (st == Status::OK) {
      Tracker t = b->tracker;
      st = t.wait();
    }
    if (st != Status::OK) return st;
    uint8_t* base = (uint8_t*)r->arena->chunk_addr((uint32_t)r->chunk);
    const uint8_t* side = (const uint8_t*)d.arena->chunk_addr((uint32_t)d.chunk);
    for (uint32_t s = 0; s < kSegsPerBlock; ++s) {
      if (!((dec >> s) & 1u)) continue;
      if (!ans_decode(side + d.off[s], (uint16_t*)(base + (uint64_t)s * kSegBytes), kSegBytes / 2))
        return Status::IO_ERROR;
      Tools::get().inc(Counter::SegExpansions);
    }
  }
  d.packed &= ~segs;
  if (!d.packed) free_sidecar(b, r);
  b->pack_skip = false;
  return Status::OK;
}

Status Runtime::note_host_write(Block* b, Residency* r, const PageMask& pages, const PageMask& full) {
  const uint32_t touched = segs_of(pages);
  b->seg_written = touched;
  b->seg_gen++;
  if (r && r->fmt == 3) return expand_segments(b, r, touched, segs_full(full));
  return Status::OK;
}

namespace {

// The complete host / CXL copy segment packing would work on (raw, or already
// segmented) and its candidate segments: whole segments inside the block, not
// packed yet, untouched by the latest write-back.
// (`complete` false: the write-back that makes it complete may still be on its
// way - seg_pack_enqueue runs while it is being queued.)
Residency* seg_candidate(Block* b, uint32_t* cand, bool complete = true) {
  Residency* best = nullptr;
  for (auto& x : b->res) {
    if (x.loc.is_gpu() || x.chunk < 0 || (x.fmt != 0 && x.fmt != 3)) continue;
    if (complete && !(x.resident == b->valid_pages())) continue;
    if (!best || (x.loc.tier == Tier::HOST && best->loc.tier != Tier::HOST)) best = &x;
  }
  *cand = 0;
  if (!best) return nullptr;
  const uint32_t whole = b->npages / kSegPages;  // segments fully inside the block
  uint32_t c = whole >= 32 ? ~0u : ((1u << whole) - 1u);
  c &= ~b->seg_written;
  if (best->fmt == 3 && best->seg) c &= ~best->seg->packed;
  *cand = c;
  return best;
}

}  // namespace

void Runtime::seg_pack_enqueue(Block* b) {
  if (!config().pack_host_copies || !config().pack_segments || b->seg_pack_queued || b->pack_queued) return;
  Range* r = b->range;
  if (r->type != RangeType::MANAGED || (r->flags & RANGE_COMPRESS_BF16) || r->dead.load(std::memory_order_relaxed))
    return;
  if (!b->policy.read_dup) return;  // read-mostly data (reads dominate its few writes)
  uint32_t cand = 0;
  if (!seg_candidate(b, &cand, false) ||
      (int64_t)__builtin_popcount(cand) < std::max<int64_t>(1, config().pack_seg_min))
    return;
  b->seg_pack_queued = true;
  {
    std::lock_guard<std::mutex> g(pack_m_);
    if (pack_stop_) {
      b->seg_pack_queued = false;
      return;
    }
    pack_q_.push_back(PackJob{r->id, b->index, 0, true});
    if (pack_threads_.empty()) {
      const int n = (int)std::max<int64_t>(1, config().pack_threads);
      for (int i = 0; i < n; ++i) pack_threads_.emplace_back([this] { pack_worker(); });
    }
  }
  pack_cv_.notify_one();
}

// Segment packing, phases as pack_block: snapshot the candidate segments
// (locked), encode each as its own ANS1 chunk (unlocked), install them in the
// sidecar (locked, only if no write-back touched the block meanwhile). The raw
// chunk is never modified - packed segments' raw pages just become stale - so
// readers of it in flight need no wait. True: deferred.
bool Runtime::pack_segments(uint64_t range_id, uint64_t bi, uint16_t* raw, uint8_t* enc) {
  ChunkArena* arena = nullptr;
  int64_t chunk = -1;
  uint32_t cand = 0;
  uint64_t gen = 0;
  {  // 1) snapshot
    std::shared_lock<OrderedRWLock> vg(vs_.lock);
    Range* r = vs_.by_id_locked(range_id);
    if (!r || bi >= r->nblocks) return false;
    {
      std::lock_guard<std::mutex> g(dev_tables_m_);
      if (dev_tables_.count(range_id)) return false;
    }
    Block* b = r->block(bi);
    std::lock_guard<OrderedMutex> g(b->lock);
    if (b->unpublished) return true;  // the write-back that completes the copy is still being queued
    Residency* x = seg_candidate(b, &cand);
    if (!x || !cand || r->dead.load() || b->user_pins) {
      b->seg_pack_queued = false;
      return false;
    }
    if (x->arena->pinned((uint32_t)x->chunk)) return true;
    if (b->unpublished || !b->tracker.query()) return true;  // the write-back is still landing
    arena = x->arena;
    chunk = x->chunk;
    gen = b->seg_gen;
    const uint8_t* base = (const uint8_t*)arena->chunk_addr((uint32_t)chunk);
    for (uint32_t s = 0; s < kSegsPerBlock; ++s)
      if ((cand >> s) & 1u) memcpy((uint8_t*)raw + (uint64_t)s * kSegBytes, base + (uint64_t)s * kSegBytes, kSegBytes);
  }
  // 2) encode, unlocked: segment s -> enc + s * kSegBytes (its own ANS1 chunk)
  uint32_t len[kSegsPerBlock] = {0};
  const uint64_t cap = (uint64_t)kSegBytes * (uint64_t)std::max<int64_t>(0, 100 - config().pack_min_saving_pct) / 100;
  uint32_t ok = 0;
  for (uint32_t s = 0; s < kSegsPerBlock; ++s) {
    if (!((cand >> s) & 1u)) continue;
    const uint64_t e = ans_encode(raw + (uint64_t)s * (kSegBytes / 2), kSegBytes / 2, enc + (uint64_t)s * kSegBytes, cap);
    if (e) {
      len[s] = (uint32_t)e;
      ok |= 1u << s;
    }
  }
  // 3) install
  std::shared_lock<OrderedRWLock> vg(vs_.lock);
  Range* r = vs_.by_id_locked(range_id);
  if (!r || bi >= r->nblocks) return false;
  Block* b = r->block(bi);
  std::lock_guard<OrderedMutex> g(b->lock);
  Residency* y = nullptr;
  for (auto& x : b->res)
    if (x.arena == arena && x.chunk == chunk) y = &x;
  if (!y || (y->fmt != 0 && y->fmt != 3) || !(y->resident == b->valid_pages()) || r->dead.load() || b->user_pins) {
    b->seg_pack_queued = false;
    return false;
  }
  if (b->seg_gen != gen) {  // written back meanwhile: look again with the new mask
    b->seg_pack_queued = false;
    seg_pack_enqueue(b);
    return false;
  }
  if (arena->pinned((uint32_t)chunk)) return true;
  if (b->unpublished || !b->tracker.query()) return true;
  if (y->fmt == 3 && y->seg) ok &= ~y->seg->packed;
  if (!ok) {
    b->seg_pack_queued = false;
    return false;
  }
  // The CPU view stops mapping these segments before the check (a store
  // through it between 1 and 3 shows up as a difference and cancels).
  const uint8_t old_fmt = y->fmt;
  std::shared_ptr<SegDir> d = y->seg ? y->seg : std::make_shared<SegDir>();
  const uint32_t old_packed = d->packed;
  y->seg = d;
  y->fmt = 3;
  d->packed |= ok;  // (no reader until the block lock is released: the sidecar is written below)
  cpu_map_block(b);
  const uint8_t* base = (const uint8_t*)arena->chunk_addr((uint32_t)chunk);
  for (uint32_t s = 0; s < kSegsPerBlock; ++s)
    if (((ok >> s) & 1u) && memcmp(base + (uint64_t)s * kSegBytes, (const uint8_t*)raw + (uint64_t)s * kSegBytes, kSegBytes)) {
      d->packed = old_packed;
      y->fmt = old_fmt;
      if (old_fmt != 3) y->seg.reset();
      cpu_map_block(b);
      b->seg_pack_queued = false;
      return false;
    }
  d->packed = old_packed;
  // sidecar layout: the packed segments back to back (256-B aligned); when the
  // new ones do not fit behind the used bytes, a fresh sidecar is written
  // compactly and the old one goes after its readers
  auto al = [](uint64_t v) { return (v + 255) & ~255ull; };
  uint64_t need = 0;
  for (uint32_t s = 0; s < kSegsPerBlock; ++s)
    if ((ok >> s) & 1u) need += al(len[s]);
  const bool fresh = d->chunk < 0 || al(d->used) + need > kBlockSize;
  uint32_t nch = 0;
  if (fresh) {
    if (alloc_chunks(arena, 1, -1, &nch, nullptr, false) != Status::OK) {
      y->fmt = old_fmt;
      if (old_fmt != 3) y->seg.reset();
      cpu_map_block(b);
      b->seg_pack_queued = false;
      return false;
    }
    uint8_t* side = (uint8_t*)arena->chunk_addr(nch);
    uint64_t at = 0;
    if (d->chunk >= 0) {  // carry the segments already packed over
      const uint8_t* old = (const uint8_t*)d->arena->chunk_addr((uint32_t)d->chunk);
      for (uint32_t s = 0; s < kSegsPerBlock; ++s)
        if ((d->packed >> s) & 1u) {
          memcpy(side + at, old + d->off[s], d->len[s]);
          d->off[s] = (uint32_t)at;
          at = al(at + d->len[s]);
        }
      Tracker t = b->tracker;
      for (auto& f : t.fences()) d->arena->add_reuse_fence((uint32_t)d->chunk, f);
      d->arena->free_when_unpinned((uint32_t)d->chunk);
    }
    d->arena = arena;
    d->chunk = nch;
    d->used = (uint32_t)at;
  }
  uint8_t* side = (uint8_t*)d->arena->chunk_addr((uint32_t)d->chunk);
  uint64_t at = al(d->used);
  uint64_t saved = 0;
  for (uint32_t s = 0; s < kSegsPerBlock; ++s) {
    if (!((ok >> s) & 1u)) continue;
    memcpy(side + at, enc + (uint64_t)s * kSegBytes, len[s]);
    d->off[s] = (uint32_t)at;
    d->len[s] = len[s];
    at = al(at + len[s]);
    saved += kSegBytes - len[s];
  }
  d->used = (uint32_t)at;
  d->packed |= ok;
  y->seg = d;
  b->seg_pack_queued = false;
  Tools::get().inc(Counter::SegPacked, (uint64_t)__builtin_popcount(ok));
  Tools::get().inc(Counter::PackedBytesSaved, saved);
  return false;
}

void Runtime::pack_enqueue(Block* b) {
  if (!config().pack_host_copies || b->pack_queued || b->pack_skip) return;
  Range* r = b->range;
  if (r->type != RangeType::MANAGED || (r->flags & RANGE_COMPRESS_BF16) || r->dead.load(std::memory_order_relaxed))
    return;
  // Evidence that the data is read-mostly: an HBM copy dropped without a
  // copy-out - once for a READ_MOSTLY block (the advice alone is no proof: the
  // transparent mode's allocator sets it on every tensor for read duplication),
  // pack_auto_clean_evictions times for any other.
  const int64_t auto_n = config().pack_auto_clean_evictions;
  const uint64_t dup_n = (uint64_t)std::max<int64_t>(1, config().pack_read_dup_clean_evictions);
  if (!(b->policy.read_dup && b->clean_evictions >= dup_n) && !(auto_n > 0 && b->clean_evictions >= (uint64_t)auto_n))
    return;
  if (!pack_candidate(b)) return;
  b->pack_queued = true;
  {
    std::lock_guard<std::mutex> g(pack_m_);
    if (pack_stop_) {
      b->pack_queued = false;
      return;
    }
    pack_q_.push_back(PackJob{r->id, b->index, 0});
    if (pack_threads_.empty()) {
      const int n = (int)std::max<int64_t>(1, config().pack_threads);
      for (int i = 0; i < n; ++i) pack_threads_.emplace_back([this] { pack_worker(); });
    }
  }
  pack_cv_.notify_one();
}

void Runtime::pack_worker() {
  std::vector<uint16_t> raw(kBlockSize / 2);
  std::vector<uint8_t> enc(kBlockSize);
  for (;;) {
    PackJob job;
    {
      std::unique_lock<std::mutex> g(pack_m_);
      pack_cv_.wait(g, [this] { return pack_stop_ || !pack_q_.empty(); });
      if (pack_stop_) return;
      job = pack_q_.front();
      pack_q_.pop_front();
      ++pack_busy_;
    }
    // a block deferred behind readers: give them a moment
    if (job.tries) std::this_thread::sleep_for(std::chrono::milliseconds(std::min<uint32_t>(job.tries, 20)));
    const bool again = job.seg ? pack_segments(job.range, job.block, raw.data(), enc.data())
                               : pack_block(job.range, job.block, raw.data(), enc.data());
    if (again && job.tries >= 200) {  // still busy after ~4 s: leave it to its next clean eviction
      std::shared_lock<OrderedRWLock> vg(vs_.lock);
      if (Range* r = vs_.by_id_locked(job.range); r && job.block < r->nblocks) {
        Block* b = r->block(job.block);
        std::lock_guard<OrderedMutex> g(b->lock);
        (job.seg ? b->seg_pack_queued : b->pack_queued) = false;
      }
    }
    {
      std::lock_guard<std::mutex> g(pack_m_);
      if (again && job.tries < 200 && !pack_stop_)
        pack_q_.push_back(PackJob{job.range, job.block, job.tries + 1, job.seg});
      --pack_busy_;
    }
    if (again) pack_cv_.notify_one();
    pack_idle_cv_.notify_all();
  }
}

// One block through phases 1-3 (see the file comment). True: deferred (queued
// readers / copies still pending) - retry later.
bool Runtime::pack_block(uint64_t range_id, uint64_t bi, uint16_t* raw, uint8_t* enc) {
  ChunkArena* arena = nullptr;
  int64_t chunk = -1;
  uint32_t nv = 0;
  {  // 1) snapshot
    std::shared_lock<OrderedRWLock> vg(vs_.lock);
    Range* r = vs_.by_id_locked(range_id);
    if (!r || bi >= r->nblocks) return false;
    {
      std::lock_guard<std::mutex> g(dev_tables_m_);
      if (dev_tables_.count(range_id)) return false;  // kernels may read the host copy through the table
    }
    Block* b = r->block(bi);
    std::lock_guard<OrderedMutex> g(b->lock);
    Residency* x = pack_candidate(b);
    if (!x || r->dead.load() || b->user_pins) {
      b->pack_queued = false;
      return false;
    }
    // A lease of the host copy itself (a CPU or zero-copy remote lease pins its
    // chunk) defers the packing; leases of the block's GPU copy do not read it
    // (a hot block is leased again within a step: dropping the job here left
    // it raw until its next clean eviction, which races the same way).
    if (x->arena->pinned((uint32_t)x->chunk)) return true;
    if (b->unpublished || !b->tracker.query()) return true;  // copies into the block still in flight
    nv = b->npages << (kPageShift - 1);
    arena = x->arena;
    chunk = x->chunk;
    memcpy(raw, (const void*)arena->chunk_addr((uint32_t)chunk), (size_t)nv * 2);
  }
  // 2) encode, unlocked
  const uint64_t raw_bytes = (uint64_t)nv * 2;
  const uint64_t cap = raw_bytes * (uint64_t)std::max<int64_t>(0, 100 - config().pack_min_saving_pct) / 100;
  const uint64_t e = ans_encode(raw, nv, enc, cap);
  // 3) install
  std::shared_lock<OrderedRWLock> vg(vs_.lock);
  Range* r = vs_.by_id_locked(range_id);
  if (!r || bi >= r->nblocks) return false;
  Block* b = r->block(bi);
  std::lock_guard<OrderedMutex> g(b->lock);
  Residency* y = nullptr;
  for (auto& x : b->res)
    if (x.arena == arena && x.chunk == chunk) y = &x;
  if (!y || y->fmt != 0 || !(y->resident == b->valid_pages()) || r->dead.load() || b->user_pins) {
    b->pack_queued = false;
    return false;
  }
  if (arena->pinned((uint32_t)chunk)) return true;
  if (b->unpublished || !b->tracker.query()) return true;
  if (!e) {
    b->pack_queued = false;
    b->pack_skip = true;
    Tools::get().inc(Counter::PackSkips);
    return false;
  }
  Tracker readers = arena->reuse_fence((uint32_t)chunk);
  if (!readers.query()) return true;  // a queued copy still reads the raw pages
  uint8_t* base = (uint8_t*)arena->chunk_addr((uint32_t)chunk);
  y->fmt = 2;  // the CPU view stops mapping this copy
  cpu_map_block(b);
  if (memcmp(base, raw, raw_bytes) != 0) {  // written through the CPU view meanwhile
    y->fmt = 0;
    cpu_map_block(b);
    b->pack_queued = false;
    return false;
  }
  memcpy(base, enc, e);
  y->enc_bytes = (uint32_t)e;
  b->pack_queued = false;
  Tools::get().inc(Counter::PackedBlocks);
  Tools::get().inc(Counter::PackedBytesSaved, raw_bytes - e);
  update_device_table(b);
  return false;
}

bool Runtime::pack_wait(uint64_t timeout_ms) {
  std::unique_lock<std::mutex> g(pack_m_);
  return pack_idle_cv_.wait_for(g, std::chrono::milliseconds(timeout_ms),
                                [this] { return pack_q_.empty() && pack_busy_ == 0; });
}

Runtime::PackStats Runtime::pack_stats() {
  PackStats s;
  {
    std::lock_guard<std::mutex> g(pack_m_);
    s.queued = pack_q_.size();
    s.busy = pack_busy_;
    s.threads = pack_threads_.size();
  }
  std::shared_lock<OrderedRWLock> vg(vs_.lock);
  for (auto& kv : vs_.ranges)
    for (auto& bp : kv.second->blocks) {
      Block* b = bp.get();
      std::lock_guard<OrderedMutex> g(b->lock);
      for (auto& x : b->res) {
        if (x.fmt == 2) {
          s.packed_blocks++;
          s.packed_bytes += x.enc_bytes;
          s.raw_bytes += (uint64_t)b->npages << kPageShift;
        } else if (x.fmt == 3 && x.seg) {
          s.seg_blocks++;
          const uint32_t np = (uint32_t)__builtin_popcount(x.seg->packed);
          s.seg_packed += np;
          s.seg_raw += kSegsPerBlock - np;
          s.packed_bytes += x.seg->packed_bytes();
          s.raw_bytes += (uint64_t)np * kSegBytes;
        }
      }
    }
  return s;
}

void Runtime::stop_packer() {
  {
    std::lock_guard<std::mutex> g(pack_m_);
    pack_stop_ = true;
    pack_q_.clear();
  }
  pack_cv_.notify_all();
  for (auto& t : pack_threads_) t.join();
  pack_threads_.clear();
}

}  // namespace ogkm
