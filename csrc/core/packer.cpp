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
  if (!(b->policy.read_dup && b->clean_evictions >= 1) && !(auto_n > 0 && b->clean_evictions >= (uint64_t)auto_n))
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
    const bool again = pack_block(job.range, job.block, raw.data(), enc.data());
    if (again && job.tries >= 200) {  // still busy after ~4 s: leave it to its next clean eviction
      std::shared_lock<OrderedRWLock> vg(vs_.lock);
      if (Range* r = vs_.by_id_locked(job.range); r && job.block < r->nblocks) {
        Block* b = r->block(job.block);
        std::lock_guard<OrderedMutex> g(b->lock);
        b->pack_queued = false;
      }
    }
    {
      std::lock_guard<std::mutex> g(pack_m_);
      if (again && job.tries < 200 && !pack_stop_) pack_q_.push_back(PackJob{job.range, job.block, job.tries + 1});
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
      for (auto& x : b->res)
        if (x.fmt == 2) {
          s.packed_blocks++;
          s.packed_bytes += x.enc_bytes;
          s.raw_bytes += (uint64_t)b->npages << kPageShift;
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
