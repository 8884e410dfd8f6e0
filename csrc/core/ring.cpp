// SQ/CQ ring implementation.
#include "ogkm/ring.hpp"

#include <algorithm>
#include <thread>

#include "ogkm/codec.hpp"
#include "ogkm/config.hpp"
#include "ogkm/events.hpp"
#include "ogkm/runtime.hpp"

namespace ogkm {

const char* ring_kind_str(RingKind k) {
  static const char* n[] = {"cpu_to_gpu", "gpu_to_cpu", "gpu_internal", "gpu_to_gpu", "memops", "cxl"};
  return n[(int)k];
}

Ring::Ring(Backend* be, int dev, RingKind kind, uint32_t entries) : be_(be), dev_(dev), kind_(kind), entries_(entries) {
  // Migration rings get high priority (-1) so copies are not starved by compute.
  stream_ = be_->stream_create(dev, kind == RingKind::MEMOPS ? 0 : -1);
  void* p = nullptr;
  if (be_->host_alloc_coherent(64, &p) == Status::OK) {
    sem_ = (uint64_t*)p;
    *sem_ = 0;
  }
  if (!stream_ || !sem_) {
    err_ = Status::NO_MEMORY;
    RT_ERR("ring %s/%d init failed", ring_kind_str(kind), dev);
  }
  // PCIe / xGMI rings run their copies on a copy engine (SDMA) when there is one.
  dma_ = config().copy_engine == 3 && kind != RingKind::GPU_INTERNAL && kind != RingKind::MEMOPS &&
         !(kind == RingKind::GPU_TO_GPU && config().peer_copy_engine == 0) && be_->dma_supported(dev) &&
         err_ == Status::OK;
  if (dma_) worker_ = std::thread([this] { worker(); });
}

Ring::~Ring() {
  if (dma_) {
    {
      std::lock_guard<std::mutex> g(wm_);
      stop_ = true;
    }
    wcv_.notify_all();
    worker_.join();
  }
  if (stream_) {
    be_->stream_sync(stream_);
    last_fence_.reset();
    be_->stream_destroy(stream_);
  }
  for (void*& e : stage_ev_)
    if (e) be_->event_destroy(e);
  if (stage_) be_->hbm_free(dev_, stage_, stage_bytes_);
  if (sem_) be_->host_free_coherent(sem_);
}

void Ring::push_wait(const FenceRef& f) {
  if (!f || f->ring == this || f->done.load(std::memory_order_relaxed)) return;
  // A tracking-value fence of another ring must be submitted before anything
  // waits on it (never from inside a submission: two ring locks at once).
  if (f->ring && !f->event && f->seq > f->ring->submitted_seq()) f->ring->submit();
  // A stream ring turns this into a GPU-side wait on the DMA ring's value:
  // that value's work must be on the engines first (issued_seq).
  if (!dma_ && f->ring && !f->event) (void)f->ring->wait_issued(f->seq);
  Sqe w;
  w.op = SqeOp::WAIT_FENCE;
  w.wait = f;
  push(std::move(w));
}

uint64_t Ring::push(Sqe&& s) {
  std::unique_lock<OrderedMutex> g(m_);
  // SQ full (GPFIFO full): submit, then wait for the oldest in-flight entries.
  while (sq_.size() + inflight_.size() >= entries_) {
    if (!sq_.empty()) submit_locked();
    uint64_t oldest = inflight_.empty() ? 0 : inflight_.front().first;
    if (oldest) {
      g.unlock();
      wait_seq(oldest);
      g.lock();
      while (!inflight_.empty() && inflight_.front().first <= completed_seq()) inflight_.pop_front();
    }
  }
  uint64_t seq = next_seq_++;
  sq_.emplace_back(seq, std::move(s));
  return seq;
}

FenceRef Ring::submit() {
  std::lock_guard<OrderedMutex> g(m_);
  return submit_locked();
}

FenceRef Ring::submit_dma_locked() {
  Runtime* rt = Runtime::get();
  Batch b;
  uint64_t last = 0;
  for (auto& e : sq_) {
    Sqe& s = e.second;
    int32_t cqe_status = 0;
    if (s.op == SqeOp::COPY && rt && rt->inject().copy_drop.load() > 0 && rt->inject().copy_drop.fetch_sub(1) > 0) {
      // Simulated link error (uvm_volta_ce.c:137-138 analog): dropped + reported.
      Tools::get().inc(Counter::InjectedErrors);
      cqe_status = (int32_t)Status::INJECTED_ERROR;
      if (err_ == Status::OK) {
        err_ = Status::INJECTED_ERROR;
        err_desc_ = std::string(s.file) + ":" + std::to_string(s.line) + " " + s.desc;
      }
    } else if (err_ != Status::OK) {
      cqe_status = (int32_t)err_.load();
    } else {
      b.ops.push_back(std::move(s));
    }
    last = std::max(last, e.first);
    inflight_.emplace_back(e.first, Cqe{s.user_data, e.first, cqe_status});
  }
  sq_.clear();
  b.last = last;
  if (err_ == Status::OK) {
    Tools::get().inc(Counter::CopyKernelLaunches);  // one engine submission per batch
    {
      std::lock_guard<std::mutex> g(wm_);
      work_.push_back(std::move(b));
      queued_.fetch_add(1, std::memory_order_relaxed);
    }
    wcv_.notify_one();
  } else {
    // Robust-channel style: a failed ring never leaves CPU waiters hanging. The
    // (empty) batch still goes through the worker, so the tracking value is
    // published in submission order after the batches queued before it: a
    // direct store here would race the worker's stores of smaller values.
    {
      std::lock_guard<std::mutex> g(wm_);
      work_.push_back(std::move(b));
      queued_.fetch_add(1, std::memory_order_relaxed);
    }
    wcv_.notify_one();
    RT_ERR("ring %s/%d error %s at %s", ring_kind_str(kind_), dev_, status_str(err_), err_desc_.c_str());
    tools_event(ToolsEventType::RingError, Cause::User, Loc::gpu(dev_), Loc::gpu(dev_), dev_, 0, 0, 0);
  }
  submitted_ = last;
  batches_++;
  Tools::get().inc(Counter::RingSubmissions);
  auto f = std::make_shared<Fence>();
  f->be = be_;
  f->dev = dev_;
  f->ring = this;
  f->seq = last;
  last_fence_ = f;
  return f;
}

// A batch of copies only (the common streaming case): its engine copies,
// adjacent ones merged as run_batch does. False when it holds anything else
// (fence waits, kernels) or the ring splits peer copies over engines.
bool Ring::pure_copies(const Batch& b, std::vector<CopyDesc>* out) const {
  if (kind_ == RingKind::GPU_TO_GPU) return false;
  out->clear();
  for (const auto& s : b.ops) {
    if (s.op == SqeOp::NOP) continue;
    if (s.op != SqeOp::COPY) return false;
    if (!out->empty() && out->back().dst + out->back().bytes == s.dst && out->back().src + out->back().bytes == s.src)
      out->back().bytes += s.bytes;
    else
      out->push_back(CopyDesc{s.dst, s.src, s.bytes});
  }
  return true;
}

// Batches whose packed-block decodes still run on the stream (run_batch
// batch_ev_) are published, in order, once their event completed (all: wait
// for them). Worker thread only.
Status Ring::publish_deferred_locked(bool all) {
  Status st = Status::OK;
  while (!deferred_.empty()) {
    auto& d = deferred_.front();
    if (!all && !be_->event_query(d.ev)) break;
    set_phase(Phase::STREAM_DRAIN, d.last);
    Status s = be_->event_sync(d.ev);
    if (st == Status::OK) st = s;
    be_->event_destroy(d.ev);
    publish(d.last);
    deferred_.pop_front();
  }
  return st;
}

bool Ring::copies_hit_deferred(const std::vector<CopyDesc>& copies) const {
  for (const auto& d : deferred_)
    for (const CopyDesc& c : copies)
      for (const auto& r : d.dst)
        if (c.dst < r.first + r.second && r.first < c.dst + c.bytes) return true;
  return false;
}

// DMA ring worker: batches complete in submission order. A batch of plain
// copies is issued on one of two completion slots and the worker moves on:
// the next batch goes to the engines while this one is still copying, so
// small batches (a stable-VA fault's blocks, a planner-off unit) no longer
// leave the link idle for the worker's complete -> publish -> issue turn
// (ring_pipeline; the tracking value is still published in order, after the
// batch's copies completed).
void Ring::worker() {
  int pend = -1;  // slot of the issued, not yet completed batch
  uint64_t pend_last = 0;
  auto fail = [&](Status st, uint64_t last) {
    if (st != Status::OK && err_ == Status::OK) {
      err_ = st;
      RT_ERR("ring %s/%d batch up to seq %llu failed: %s (%s)", ring_kind_str(kind_), dev_,
             (unsigned long long)last, status_str(st), be_->last_error().c_str());
      if (st != Status::INJECTED_ERROR) set_fatal(st, "DMA ring batch failed");
    }
  };
  auto& deferred = deferred_;
  auto publish_deferred = [&](bool all) {
    Status st = publish_deferred_locked(all);
    if (st != Status::OK) fail(st, submitted_.load());
  };
  auto complete_pending = [&] {
    if (pend < 0) return;
    set_phase(Phase::COMPLETE, pend_last);
    const uint64_t t0 = now_ns();
    fail(be_->dma_complete(pend), pend_last);
    if (kind_ == RingKind::CPU_TO_GPU) Tools::get().inc(Counter::RingCopyNs, now_ns() - t0);
    publish_deferred(true);  // (tracking values are published in order)
    publish(pend_last);
    pend = -1;
  };
  std::vector<CopyDesc> copies;
  for (;;) {
    Batch b;
    {
      std::unique_lock<std::mutex> g(wm_);
      if (work_.empty() && (pend >= 0 || !deferred.empty())) {  // nothing to overlap with: finish what is in flight
        g.unlock();
        complete_pending();
        publish_deferred(true);
        g.lock();
      }
      if (work_.empty() && !stop_) {
        set_phase(Phase::IDLE, 0);
        const uint64_t t_idle = now_ns();
        wcv_.wait(g, [&] { return stop_ || !work_.empty(); });
        if (kind_ == RingKind::CPU_TO_GPU) Tools::get().inc(Counter::RingIdleNs, now_ns() - t_idle);
      }
      if (work_.empty()) return;  // stop_ with nothing left
      b = std::move(work_.front());
      work_.pop_front();
      queued_.fetch_sub(1, std::memory_order_relaxed);
      // Batches of packed-block decodes queued behind this one run as ONE batch
      // (up to ring_merge_packed_mb of packed bytes): their staging copies and
      // decodes then fill the staging halves instead of one launch per batch
      // (the transparent 70B step: ~5 blocks per launch, a latency-bound
      // decode each). Batches that wait on fences are never merged: a wait
      // behind this batch's own tracking value would never end.
      if (const uint64_t cap = (uint64_t)std::max<int64_t>(0, config().ring_merge_packed_mb) << 20) {
        uint64_t packed = packed_bytes(b);
        while (packed && packed < cap && !work_.empty()) {
          const uint64_t np = packed_bytes(work_.front());
          if (!np) break;
          Batch& n = work_.front();
          b.ops.insert(b.ops.end(), std::make_move_iterator(n.ops.begin()), std::make_move_iterator(n.ops.end()));
          b.last = n.last;
          packed += np;
          work_.pop_front();
          queued_.fetch_sub(1, std::memory_order_relaxed);
          Tools::get().inc(Counter::RingMergedBatches);
        }
      }
    }
    if (err_ == Status::OK && config().ring_pipeline && pure_copies(b, &copies)) {
      const int slot = pend == 0 ? 1 : 0;
      // a copy into a chunk a deferred packed-block decode still writes (the
      // chunk was handed out again): that decode first (see run_batch)
      if (!deferred_.empty() && copies_hit_deferred(copies)) {
        publish_deferred(true);
        Tools::get().inc(Counter::DecodeReuseWaits);
      }
      set_phase(Phase::ISSUE, b.last);
      const uint64_t t0 = now_ns();
      Status st = copies.empty() ? Status::OK : be_->dma_issue(dev_, copies.data(), copies.size(), (int)kind_, slot);
      mark_issued(b.last);  // on the engines (or failed: published below)
      if (kind_ == RingKind::CPU_TO_GPU) {
        Tools::get().inc(Counter::RingCopyNs, now_ns() - t0);
        Tools::get().inc(Counter::RingCopyCalls, copies.size());
      }
      complete_pending();  // the batch before (its copies are ahead of these on the engines)
      if (st != Status::OK) {
        fail(st, b.last);
        (void)be_->dma_complete(slot);
        publish(b.last);
        continue;
      }
      pend = slot;
      pend_last = b.last;
      continue;
    }
    complete_pending();
    publish_deferred(false);  // decodes of earlier batches that are done already
    set_phase(Phase::ISSUE, b.last);
    Status st = err_ == Status::OK ? run_batch(b) : err_.load();
    fail(st, b.last);
    if (batch_ev_ && st == Status::OK) {
      deferred.push_back(Deferred{batch_ev_, b.last, std::move(batch_dst_)});
      batch_ev_ = nullptr;
      batch_dst_.clear();
      continue;
    }
    if (batch_ev_) {
      (void)be_->event_sync(batch_ev_);
      be_->event_destroy(batch_ev_);
      batch_ev_ = nullptr;
    }
    batch_dst_.clear();
    // Publish even on error (robust channel): waiters then see err_.
    publish_deferred(true);
    publish(b.last);
  }
}

// Packed bytes a batch stages for DECODE_ANS; 0 for a batch with none or with a
// fence wait (never merged, Ring::worker).
uint64_t Ring::packed_bytes(const Batch& b) {
  uint64_t n = 0;
  for (const Sqe& s : b.ops) {
    if (s.op == SqeOp::WAIT_FENCE) return 0;
    if (s.op == SqeOp::DECODE_ANS || s.op == SqeOp::DECODE_SEGS || (s.op == SqeOp::DECODE_BF12 && config().bf12_stage))
      n += s.bytes;
  }
  return n;
}

std::vector<CopyDesc> split_over_engines(const std::vector<CopyDesc>& in, uint32_t mask, uint64_t min_piece,
                                         uint32_t* rot) {
  std::vector<uint32_t> engs;
  for (int b = 0; b < 32; ++b)
    if ((mask >> b) & 1) engs.push_back(1u << b);
  std::vector<CopyDesc> out;
  if (engs.empty()) {
    out = in;
    return out;
  }
  constexpr uint64_t kAlign = 64 << 10;
  for (const CopyDesc& c : in) {
    uint64_t k = min_piece ? c.bytes / min_piece : 1;
    if (k > engs.size()) k = engs.size();
    if (k < 2) {
      CopyDesc d = c;
      d.engine = engs[(*rot)++ % engs.size()];
      out.push_back(d);
      continue;
    }
    uint64_t piece = (c.bytes / k + kAlign - 1) / kAlign * kAlign;
    for (uint64_t off = 0; off < c.bytes; off += piece) {
      CopyDesc d{c.dst + off, c.src + off, std::min(piece, c.bytes - off)};
      d.engine = engs[(*rot)++ % engs.size()];
      out.push_back(d);
    }
  }
  return out;
}

Status Ring::run_batch(Batch& b) {
  // Copies go to the engine (synchronously, from this thread); kernel SQEs
  // (fused decode, memset, page gather / scatter) go to the side stream
  // asynchronously - consecutive decodes as ONE launch - so a decode overlaps
  // the engine copies after it. The stream is drained before an engine copy
  // that follows kernels (the copy may read their output) and at batch end.
  std::vector<CopyDesc> copies;
  std::vector<int> copy_dst;  // GPU_TO_GPU: the peer each copy writes
  std::vector<DecodeDesc> decodes;
  std::vector<DecodeDesc> staged;  // packed blocks whose bytes are on their way into stage_
  uint64_t stage_off = 0;
  Status st = Status::OK;
  bool kernels_pending = false;
  bool decodes_deferred = false;  // packed-block decodes in flight on the stream (see flush_staged)
  bool final_flush = false;
  auto drain = [&] {
    if (st == Status::OK && kernels_pending) {
      set_phase(Phase::STREAM_DRAIN, b.last);
      st = be_->stream_sync(stream_);
      set_phase(Phase::ISSUE, b.last);
    }
    kernels_pending = false;
  };
  auto flush_decodes = [&] {
    if (st == Status::OK && !decodes.empty()) {
      st = be_->decode_bf12(dev_, decodes.data(), decodes.size(), stream_);
      kernels_pending = true;
    }
    decodes.clear();
  };
  // A staging half whose copies are on the engines and whose decode is not
  // launched yet: the next half's copies are issued BEFORE the host waits for
  // these (the engines never idle while the host launches a decode), then its
  // decode goes out (complete_stage).
  struct PendStage {
    bool on = false;
    int slot = 0, half = 0;
    std::vector<DecodeDesc> staged;
  } ps;
  auto launch_decodes = [&](std::vector<DecodeDesc>& dec, int half) {
    // one launch per format present (ANS1 blocks: k_ans_blocks; BF12: k_bf12_decode)
    std::vector<DecodeDesc> ans, b12;
    for (const DecodeDesc& d : dec) (d.fmt == 1 ? b12 : ans).push_back(d);
    if (!ans.empty()) st = be_->decode_ans_blocks(dev_, ans.data(), ans.size(), stream_);
    if (st == Status::OK && !b12.empty()) st = be_->decode_bf12(dev_, b12.data(), b12.size(), stream_);
    Tools::get().inc(Counter::PackedDecodes, dec.size());
    for (const DecodeDesc& d : dec) batch_dst_.emplace_back(d.dst, 2ull * d.n_values);
    if (st != Status::OK) return;
    if (!stage_ev_[half]) stage_ev_[half] = be_->event_create(dev_);
    if (!config().ring_defer_decodes) {
      kernels_pending = true;  // drained before the next copies, as any kernel
    } else if (stage_ev_[half] && be_->event_record(stage_ev_[half], stream_) == Status::OK) {
      stage_used_[half] = true;
      decodes_deferred = true;
    } else {
      kernels_pending = true;  // no event: drain as for any kernel
    }
  };
  auto complete_stage = [&] {
    if (!ps.on) return;
    ps.on = false;
    if (st == Status::OK) {
      set_phase(Phase::ENGINE_WAIT, b.last);
      const uint64_t t0 = now_ns();
      st = be_->dma_complete(ps.slot);
      if (kind_ == RingKind::CPU_TO_GPU) Tools::get().inc(Counter::RingCopyNs, now_ns() - t0);
      set_phase(Phase::ISSUE, b.last);
    }
    if (st == Status::OK) launch_decodes(ps.staged, ps.half);
    ps.staged.clear();
  };
  // Engine copies: issued on `slot`; waited for unless `async` (a staging
  // half's copies: complete_stage waits).
  auto issue_copies = [&](int slot, bool async) {
    if (!copies.empty()) {
      drain();
      if (kind_ == RingKind::GPU_TO_GPU) {
        // xGMI peer copies, pushed by this (source) GPU: large copies split over
        // every SDMA engine of the (peer, source) pair, each piece on its own
        // engine - the per-link split the reference does with one CE channel per
        // peer (uvm_va_block.c:3390-3460, uvm_channel.c peer pools).
        std::vector<CopyDesc> split;
        const uint64_t min_piece = (uint64_t)std::max<int64_t>(1, config().peer_split_min_mb) << 20;
        for (size_t i = 0; i < copies.size();) {
          size_t j = i;
          while (j < copies.size() && copy_dst[j] == copy_dst[i]) ++j;
          std::vector<CopyDesc> run(copies.begin() + i, copies.begin() + j);
          uint32_t mask = copy_dst[i] >= 0 ? be_->copy_engine_mask(copy_dst[i], dev_) : 0;
          std::vector<CopyDesc> part = split_over_engines(run, mask, min_piece, &engine_rot_);
          split.insert(split.end(), part.begin(), part.end());
          i = j;
        }
        copies.swap(split);
      }
      // A copy into a chunk a still-running packed-block decode writes (the
      // chunk was freed and handed out again since - same-ring fences are not
      // waited for, the ring used to be in order) waits for that decode:
      // earlier batches' (deferred) or this batch's own.
      if (st == Status::OK && (!deferred_.empty() || decodes_deferred)) {
        auto hits = [&](const std::vector<std::pair<uint64_t, uint64_t>>& dst) {
          for (const CopyDesc& c : copies)
            for (const auto& d : dst)
              if (c.dst < d.first + d.second && d.first < c.dst + c.bytes) return true;
          return false;
        };
        const bool prior = copies_hit_deferred(copies);
        if (prior) st = publish_deferred_locked(true);
        if (st == Status::OK && decodes_deferred && hits(batch_dst_)) {
          set_phase(Phase::STREAM_DRAIN, b.last);
          st = be_->stream_sync(stream_);
          set_phase(Phase::ISSUE, b.last);
          Tools::get().inc(Counter::DecodeReuseWaits);
        }
        if (prior) Tools::get().inc(Counter::DecodeReuseWaits);
      }
      if (st == Status::OK) {
        const uint64_t t_copy = now_ns();
        snprintf(phase_what_, sizeof(phase_what_), "engine copy: %zu descriptors, first %llu B", copies.size(),
                 (unsigned long long)copies[0].bytes);
        set_phase(Phase::ENGINE_ISSUE, b.last);
        st = be_->dma_issue(dev_, copies.data(), copies.size(), (int)kind_, slot);
        // the batch's last copies are on the engines: GPU waits may be enqueued
        if (final_flush && st == Status::OK) mark_issued(b.last);
        if (!async) {
          set_phase(Phase::ENGINE_WAIT, b.last);
          if (st == Status::OK) st = be_->dma_complete(slot);
          set_phase(Phase::ISSUE, b.last);
        }
        if (kind_ == RingKind::CPU_TO_GPU) {
          Tools::get().inc(Counter::RingCopyNs, now_ns() - t_copy);
          Tools::get().inc(Counter::RingCopyCalls, copies.size());
        }
      }
    }
    copies.clear();
    copy_dst.clear();
  };
  auto flush_copies = [&] {
    complete_stage();  // a pending half's decode goes out first (order, chunk-reuse checks)
    issue_copies(0, false);
  };
  // Packed blocks: their staging copies go out with the batch's other engine
  // copies; once those landed ONE k_ans_blocks launch decodes them all - and
  // runs while the engines already fill the other half of the staging buffer
  // (a half is refilled only after the decode that read it, its event). The
  // decodes' outputs are consumed only through the batch's tracking value,
  // which the worker publishes once they completed (deferred publish): the
  // ring never drains its stream for them.
  bool half_ready = false;  // the current staging half's previous decode is done
  auto flush_staged = [&] {
    if (staged.empty()) return;
    if (config().ring_stage_overlap) {
      // this half's copies go out now; the previous half's (if any) are waited
      // for and its decode launched while these run
      // (other copies flushed with these that write a chunk the pending half
      // decodes into - handed out again within this batch - wait for it)
      if (ps.on) {
        bool hit = false;
        for (const CopyDesc& c : copies)
          for (const DecodeDesc& d : ps.staged)
            hit |= c.dst < d.dst + 2ull * d.n_values && d.dst < c.dst + c.bytes;
        if (hit) complete_stage();
      }
      const int slot = ps.on ? (ps.slot ^ 1) : 0;
      issue_copies(slot, true);
      complete_stage();
      if (st == Status::OK) {
        ps.on = true;
        ps.slot = slot;
        ps.half = stage_half_;
        ps.staged.swap(staged);
      }
    } else {
      flush_copies();
      if (st == Status::OK) launch_decodes(staged, stage_half_);
    }
    staged.clear();
    stage_off = 0;
    stage_half_ ^= 1;
    half_ready = false;
  };
  // A staged decode queued before an engine copy into the same chunk (the
  // chunk's block was evicted and the chunk handed to another block between
  // two submissions that the worker merged into this batch - copy_pages skips
  // same-ring fences, the ring being in order) must land first: staged
  // decodes are launched only after their half's copies completed, so a copy
  // issued with those would be overwritten (or raced) by the older decode.
  auto staged_hit = [&](uint64_t dst, uint64_t bytes) {
    for (const DecodeDesc& d : staged)
      if (dst < d.dst + 2ull * d.n_values && d.dst < dst + bytes) return true;
    if (ps.on)
      for (const DecodeDesc& d : ps.staged)
        if (dst < d.dst + 2ull * d.n_values && d.dst < dst + bytes) return true;
    return false;
  };
  for (auto& s : b.ops) {
    if (st != Status::OK) break;
    switch (s.op) {
      case SqeOp::COPY:
        flush_decodes();
        if (staged_hit(s.dst, s.bytes)) {
          // launch them (the copy then waits for them: kernels_pending /
          // decodes_deferred + batch_dst_ in issue_copies)
          flush_staged();
          flush_copies();
          Tools::get().inc(Counter::DecodeReuseWaits);
        }
        if (!copies.empty() && copies.back().dst + copies.back().bytes == s.dst &&
            copies.back().src + copies.back().bytes == s.src && copy_dst.back() == s.dst_dev) {
          copies.back().bytes += s.bytes;
        } else {
          copies.push_back(CopyDesc{s.dst, s.src, s.bytes});
          copy_dst.push_back(s.dst_dev);
        }
        break;
      case SqeOp::DECODE_BF12:
        if (!config().bf12_stage || (!stage_ && config().ans_stage_mb <= 0)) {
          // fused copy + decode: the kernel reads the host copy itself
          flush_staged();
          flush_copies();
          decodes.push_back(DecodeDesc{s.src, s.dst, s.n_values});
          break;
        }
        [[fallthrough]];
      case SqeOp::DECODE_SEGS:
      case SqeOp::DECODE_ANS: {
        const uint32_t fmt = s.op == SqeOp::DECODE_BF12 ? 1 : 0;
        const bool segs = s.op == SqeOp::DECODE_SEGS;
        flush_decodes();
        const uint64_t need = (s.bytes + 255) & ~255ull;
        if (!stage_ && st == Status::OK && config().ans_stage_mb > 0) {  // (0: decode from the host copy)
          stage_bytes_ = std::max<uint64_t>((uint64_t)config().ans_stage_mb << 20, 4 * kBlockSize);  // two halves
          if (be_->hbm_alloc_kind(dev_, stage_bytes_, &stage_, (int)config().ans_stage_mem) != Status::OK) {
            stage_ = nullptr;
            stage_bytes_ = 0;
          }
        }
        if (!stage_) {  // no staging memory: the decode kernel reads the host copy itself
          flush_staged();
          flush_copies();
          if (st == Status::OK) {
            std::vector<DecodeDesc> dd;
            if (segs) {
              for (size_t i = 0; i + 1 < s.idx.size(); i += 2)
                dd.push_back(DecodeDesc{s.src + s.idx[i + 1], s.dst + (uint64_t)(s.idx[i] & 31u) * (64u << 10),
                                        kAnsSegValues});
            } else {
              dd.push_back(DecodeDesc{s.src, s.dst, s.n_values});
            }
            st = fmt ? be_->decode_bf12(dev_, dd.data(), dd.size(), stream_)
                     : be_->decode_ans_blocks(dev_, dd.data(), dd.size(), stream_);
            kernels_pending = true;
            Tools::get().inc(Counter::PackedDecodes, dd.size());
          }
          break;
        }
        const uint64_t half = stage_bytes_ / 2;
        const size_t ndesc = segs ? s.idx.size() / 2 : 1;
        if (stage_off + need > half || staged.size() + ndesc > 256) flush_staged();
        if (!half_ready) {  // the decode that read this half last must be done before the engines refill it
          if (stage_used_[stage_half_] && st == Status::OK) {
            set_phase(Phase::STREAM_DRAIN, b.last);
            st = be_->event_sync(stage_ev_[stage_half_]);
            set_phase(Phase::ISSUE, b.last);
          }
          stage_used_[stage_half_] = false;
          half_ready = true;
        }
        const uint64_t at = (uint64_t)stage_ + stage_half_ * half + stage_off;
        if (segs) {
          for (size_t i = 0; i + 1 < s.idx.size(); i += 2)
            staged.push_back(DecodeDesc{at + s.idx[i + 1], s.dst + (uint64_t)(s.idx[i] & 31u) * (64u << 10),
                                        kAnsSegValues, 0});
        } else {
          staged.push_back(DecodeDesc{at, s.dst, s.n_values, fmt});
        }
        stage_off += need;
        // Packed segments of one block are back to back in its sidecar and land
        // back to back here: one engine copy for all of them.
        if (!copies.empty() && copy_dst.back() == -1 && copies.back().src + copies.back().bytes == s.src &&
            copies.back().dst + copies.back().bytes == at) {
          copies.back().bytes += need;
          break;
        }
        CopyDesc d{at, s.src, need};
        // Packed blocks are ~1.3 MB copies that never coalesce: spread them over
        // several full-rate engines so one engine's per-copy setup overlaps
        // another's transfer (config ans_stage_engines; 0 = the ring's engine).
        if (const uint32_t m = (uint32_t)config().ans_stage_engines & be_->copy_engine_mask(dev_, -1)) {
          const int nb = __builtin_popcount(m);
          int want = (int)(engine_rot_++ % (uint32_t)nb);
          for (int bit = 0; bit < 32; ++bit)
            if (((m >> bit) & 1) && want-- == 0) {
              d.engine = 1u << bit;
              break;
            }
        }
        copies.push_back(d);
        copy_dst.push_back(-1);
        break;
      }
      case SqeOp::WAIT_FENCE:
        // Dependencies are waited for where the work is issued: here, on the
        // host, before the engine / stream is handed anything after the wait.
        flush_decodes();
        flush_staged();
        flush_copies();
        if (st == Status::OK && s.wait && !s.wait->done.load(std::memory_order_acquire)) {
          // Our own deferred tracking values go out before we block on another
          // ring: that ring may be waiting for one of them (no cycle).
          if (!deferred_.empty()) st = publish_deferred_locked(true);
          const uint64_t t_wait = now_ns();
          snprintf(phase_what_, sizeof(phase_what_), "%s %s/%d seq %llu (%s:%d %s)",
                   s.wait->event ? "event" : "ring", s.wait->ring ? ring_kind_str(s.wait->ring->kind()) : "-",
                   s.wait->dev, (unsigned long long)s.wait->seq, s.file, s.line, s.desc.c_str());
          set_phase(Phase::FENCE_WAIT, b.last);
          st = s.wait->wait();
          set_phase(Phase::ISSUE, b.last);
          if (kind_ == RingKind::CPU_TO_GPU) Tools::get().inc(Counter::RingFenceWaitNs, now_ns() - t_wait);
        }
        break;
      case SqeOp::NOP:
        break;
      default: {
        flush_decodes();
        flush_staged();
        flush_copies();
        if (st != Status::OK) break;
        snprintf(phase_what_, sizeof(phase_what_), "kernel op %d (%s:%d %s)", (int)s.op, s.file, s.line,
                 s.desc.c_str());
        if (s.op == SqeOp::MEMSET) {
          st = be_->memset32(dev_, s.dst, s.pattern, s.bytes, stream_);
        } else if (s.op == SqeOp::PAGE_COPY) {
          st = be_->page_copy(dev_, s.dst, s.src, s.idx.data(), (uint32_t)s.idx.size(), stream_);
        } else {
          PageListDesc d{s.op == SqeOp::GATHER ? s.src : s.dst, s.op == SqeOp::GATHER ? s.dst : s.src, s.idx.data(),
                         (uint32_t)s.idx.size(), s.page_bytes};
          st = s.op == SqeOp::GATHER ? be_->gather_pages(dev_, d, stream_) : be_->scatter_pages(dev_, d, stream_);
        }
        kernels_pending = true;
        break;
      }
    }
  }
  flush_decodes();
  flush_staged();
  complete_stage();
  if (!kernels_pending) final_flush = true;  // (with kernels queued, the drain below comes first)
  flush_copies();
  drain();
  if (decodes_deferred && st == Status::OK && !kernels_pending) {
    // every copy and decode of the batch is issued: the worker publishes its
    // tracking value when this event completes (in order, Ring::worker)
    void* ev = be_->event_create(dev_);
    if (ev && be_->event_record(ev, stream_) == Status::OK) {
      batch_ev_ = ev;
      mark_issued(b.last);
    } else {
      if (ev) be_->event_destroy(ev);
      set_phase(Phase::STREAM_DRAIN, b.last);
      st = be_->stream_sync(stream_);
      set_phase(Phase::ISSUE, b.last);
    }
  }
  return st;
}

FenceRef Ring::submit_locked() {
  if (sq_.empty()) {
    if (last_fence_) return last_fence_;
    auto f = std::make_shared<Fence>();
    f->done.store(true);
    return f;
  }
  if (dma_) return submit_dma_locked();
  // Hoist the fence waits of every run of copy-like SQEs (COPY / DECODE /
  // WAIT_FENCE / NOP) to the front of the run, so the run becomes ONE
  // copy-kernel launch instead of one launch per wait (each launch boundary is
  // tens of microseconds of idle link). Waiting earlier is conservative: it
  // can only delay a copy that did not need to wait. No wait can depend on a
  // copy of this submission (its fence does not exist until the end).
  auto copy_like = [](SqeOp op) {
    return op == SqeOp::COPY || op == SqeOp::DECODE_BF12 || op == SqeOp::DECODE_ANS || op == SqeOp::DECODE_SEGS ||
           op == SqeOp::WAIT_FENCE || op == SqeOp::NOP;
  };
  for (auto it = sq_.begin(); it != sq_.end();) {
    if (!copy_like(it->second.op)) {
      ++it;
      continue;
    }
    auto end = it;
    while (end != sq_.end() && copy_like(end->second.op)) ++end;
    std::stable_partition(it, end, [](const std::pair<uint64_t, Sqe>& e) { return e.second.op == SqeOp::WAIT_FENCE; });
    it = end;
  }
  Runtime* rt = Runtime::get();
  Status st = err_;
  uint64_t last = 0;
  std::vector<CopyDesc> batch;
  std::vector<DecodeDesc> dbatch;
  std::vector<DecodeDesc> abatch;  // DECODE_ANS: decoded straight from the host copies
  int engine = kind_ == RingKind::GPU_INTERNAL ? 2
               : (kind_ == RingKind::GPU_TO_GPU && config().peer_copy_engine == 0) ? 4
                                                                                  : (int)config().copy_engine;
  auto flush = [&]() {
    if (st == Status::OK && !batch.empty()) {
      st = be_->copy_batch(dev_, batch.data(), batch.size(), stream_, engine);
      Tools::get().inc(Counter::CopyKernelLaunches);
    }
    if (st == Status::OK && !dbatch.empty()) {
      st = be_->decode_bf12(dev_, dbatch.data(), dbatch.size(), stream_);
      Tools::get().inc(Counter::CopyKernelLaunches);
    }
    if (st == Status::OK && !abatch.empty()) {
      st = be_->decode_ans_blocks(dev_, abatch.data(), abatch.size(), stream_);
      Tools::get().inc(Counter::CopyKernelLaunches);
      Tools::get().inc(Counter::PackedDecodes, abatch.size());
    }
    batch.clear();
    dbatch.clear();
    abatch.clear();
  };
  std::vector<std::pair<uint64_t, Cqe>> done;
  for (auto& e : sq_) {
    Sqe& s = e.second;
    int32_t cqe_status = 0;
    if (st == Status::OK) {
      switch (s.op) {
        case SqeOp::COPY:
          if (rt && rt->inject().copy_drop.load() > 0 && rt->inject().copy_drop.fetch_sub(1) > 0) {
            // Simulated link error: the copy is dropped and reported
            // (NVLink error injection analog, uvm_volta_ce.c:137-138).
            Tools::get().inc(Counter::InjectedErrors);
            cqe_status = (int32_t)Status::INJECTED_ERROR;
            err_ = Status::INJECTED_ERROR;
            err_desc_ = std::string(s.file) + ":" + std::to_string(s.line) + " " + s.desc;
            st = Status::INJECTED_ERROR;
            break;
          }
          if (!dbatch.empty() || !abatch.empty()) flush();
          // Coalesce physically adjacent copies (consecutive 2 MB blocks of one
          // extent) into a single descriptor.
          if (!batch.empty() && batch.back().dst + batch.back().bytes == s.dst &&
              batch.back().src + batch.back().bytes == s.src)
            batch.back().bytes += s.bytes;
          else
            batch.push_back(CopyDesc{s.dst, s.src, s.bytes});
          break;
        case SqeOp::DECODE_BF12:
          if (!batch.empty() || !abatch.empty()) flush();
          dbatch.push_back(DecodeDesc{s.src, s.dst, s.n_values});
          break;
        case SqeOp::DECODE_ANS:
          if (!batch.empty() || !dbatch.empty()) flush();
          abatch.push_back(DecodeDesc{s.src, s.dst, s.n_values});
          break;
        case SqeOp::DECODE_SEGS:
          if (!batch.empty() || !dbatch.empty()) flush();
          for (size_t i = 0; i + 1 < s.idx.size(); i += 2)
            abatch.push_back(DecodeDesc{s.src + s.idx[i + 1], s.dst + (uint64_t)(s.idx[i] & 31u) * (64u << 10),
                                        kAnsSegValues});
          break;
        case SqeOp::GATHER:
        case SqeOp::SCATTER: {
          flush();
          PageListDesc d{s.op == SqeOp::GATHER ? s.src : s.dst, s.op == SqeOp::GATHER ? s.dst : s.src, s.idx.data(),
                         (uint32_t)s.idx.size(), s.page_bytes};
          if (st == Status::OK) st = s.op == SqeOp::GATHER ? be_->gather_pages(dev_, d, stream_)
                                                          : be_->scatter_pages(dev_, d, stream_);
          break;
        }
        case SqeOp::MEMSET:
          flush();
          if (st == Status::OK) st = be_->memset32(dev_, s.dst, s.pattern, s.bytes, stream_);
          break;
        case SqeOp::PAGE_COPY:
          flush();
          if (st == Status::OK) st = be_->page_copy(dev_, s.dst, s.src, s.idx.data(), (uint32_t)s.idx.size(), stream_);
          break;
        case SqeOp::WAIT_FENCE:
          flush();
          if (st == Status::OK && s.wait && !s.wait->done.load()) {
            if (s.wait->event) st = be_->stream_wait_event(stream_, s.wait->event);
            else if (s.wait->ring && s.wait->ring != this)
              // tracking-value fence (its ring was submitted when the wait was pushed)
              st = be_->wait_value(stream_, s.wait->ring->semaphore(), s.wait->seq);
            else st = s.wait->wait();
          }
          break;
        case SqeOp::NOP:
          break;
      }
      if (st != Status::OK && cqe_status == 0) {
        cqe_status = (int32_t)st;
        if (err_ == Status::OK) {
          err_ = st;
          err_desc_ = std::string(s.file) + ":" + std::to_string(s.line) + " " + s.desc;
        }
      }
    } else {
      cqe_status = (int32_t)st;
    }
    last = std::max(last, e.first);
    done.emplace_back(e.first, Cqe{s.user_data, e.first, cqe_status});
  }
  flush();
  sq_.clear();
  std::sort(done.begin(), done.end(), [](const auto& a, const auto& b) { return a.first < b.first; });
  if (st == Status::OK) st = be_->signal(dev_, sem_, last, stream_);
  if (st != Status::OK) {
    if (err_ == Status::OK) err_ = st;
    // Robust-channel style: mark the ring failed; CPU waiters must not hang.
    // Signal kernels of earlier batches may still be queued on the stream:
    // drain it first so none of them stores a smaller value afterwards.
    (void)be_->stream_sync(stream_);
    publish(last);
    RT_ERR("ring %s/%d error %s at %s", ring_kind_str(kind_), dev_, status_str(err_), err_desc_.c_str());
    if (err_ != Status::INJECTED_ERROR) set_fatal(err_, "ring submission failed");
    tools_event(ToolsEventType::RingError, Cause::User, Loc::gpu(dev_), Loc::gpu(dev_), dev_, 0, 0, 0);
  }
  for (auto& d : done) inflight_.push_back(d);
  submitted_ = last;
  batches_++;
  Tools::get().inc(Counter::RingSubmissions);
  last_fence_ = fence_record(be_, dev_, stream_, this, last);
  return last_fence_;
}

// Monotonic release store of the tracking value (a waiter on seq s must never
// see the value drop below s once it was published).
void Ring::publish(uint64_t seq) {
  mark_issued(seq);
  if (!sem_) return;
  uint64_t cur = __atomic_load_n(sem_, __ATOMIC_RELAXED);
  while (cur < seq && !__atomic_compare_exchange_n(sem_, &cur, seq, true, __ATOMIC_RELEASE, __ATOMIC_RELAXED)) {
  }
}

uint64_t Ring::completed_seq() { return sem_ ? __atomic_load_n(sem_, __ATOMIC_ACQUIRE) : 0; }

Status Ring::wait_seq(uint64_t seq) {
  if (seq > submitted_) submit();
  uint64_t spins = 0;
  while (completed_seq() < seq) {
    if (++spins > 64) std::this_thread::yield();
    if (spins > (1ull << 34)) return Status::TIMEOUT;
  }
  return check_errors();
}

Status Ring::wait_issued(uint64_t seq) {
  if (!dma_ || !config().ring_wait_issued) return Status::OK;
  if (seq > submitted_) submit();
  uint64_t spins = 0;
  while (issued_.load(std::memory_order_acquire) < seq) {
    if (err_ != Status::OK) return err_;
    if (++spins > 64) std::this_thread::yield();
    if (spins > (1ull << 34)) return Status::TIMEOUT;
  }
  return Status::OK;
}

Status Ring::check_errors() {
  if (err_ != Status::OK) return err_;
  Status st = Status::OK;
  Runtime* rt = Runtime::get();
  bool injected = false;
  if (rt && rt->inject().async_copy_error.load() > 0 && rt->inject().async_copy_error.fetch_sub(1) > 0) {
    Tools::get().inc(Counter::InjectedErrors);
    st = Status::INJECTED_ERROR;
    injected = true;
  } else if (!dma_ && stream_) {
    st = be_->stream_check(stream_);
  }
  if (st == Status::OK) return Status::OK;
  Status expected = Status::OK;
  if (err_.compare_exchange_strong(expected, st)) {
    RT_ERR("ring %s/%d: work failed after submission: %s (%s)", ring_kind_str(kind_), dev_, status_str(st),
           injected ? "injected" : be_->last_error().c_str());
    tools_event(ToolsEventType::RingError, Cause::User, Loc::gpu(dev_), Loc::gpu(dev_), dev_, 0, 0, 0);
    if (!injected) set_fatal(st, "ring work failed after submission");
  }
  return err_;
}

size_t Ring::reap(Cqe* out, size_t max) {
  std::lock_guard<OrderedMutex> g(m_);
  uint64_t c = completed_seq();
  // Completed entries are checked before they are retired: a failure after
  // submission is attributed to the CQEs that complete with it.
  Status post = (!inflight_.empty() && inflight_.front().first <= c) ? check_errors() : Status::OK;
  size_t n = 0;
  while (!inflight_.empty() && inflight_.front().first <= c && n < max) {
    out[n] = inflight_.front().second;
    if (post != Status::OK && out[n].status == 0) out[n].status = (int32_t)post;
    ++n;
    inflight_.pop_front();
  }
  Tools::get().inc(Counter::RingCompletions, n);
  return n;
}

void Ring::clear_error_for_test() {
  std::lock_guard<OrderedMutex> g(m_);
  err_ = Status::OK;
  err_desc_.clear();
}

std::string Ring::debug_state() {
  static const char* ph[] = {"idle", "issue", "complete", "fence_wait", "stream_drain", "engine_issue", "engine_wait"};
  char buf[512];
  const int p = phase_.load(std::memory_order_acquire);
  const uint64_t since = phase_ns_.load(std::memory_order_relaxed);
  const double age_ms = since ? (now_ns() - since) / 1e6 : 0.0;
  size_t sq = 0, infl = 0;
  bool locked = m_.try_lock();
  if (locked) {
    sq = sq_.size();
    infl = inflight_.size();
    m_.unlock();
  }
  snprintf(buf, sizeof(buf),
           "ring %s/%d%s pushed=%llu submitted=%llu issued=%llu completed=%llu sq=%s inflight=%s worker_queue=%llu "
           "phase=%s for %.1f ms (batch up to %llu)%s%s err=%s",
           ring_kind_str(kind_), dev_, dma_ ? " dma" : " stream", (unsigned long long)pushed_seq(),
           (unsigned long long)submitted_.load(), (unsigned long long)issued_seq(), (unsigned long long)completed_seq(),
           locked ? std::to_string(sq).c_str() : "?(locked)", locked ? std::to_string(infl).c_str() : "?",
           (unsigned long long)queued_.load(), dma_ ? ph[p < 7 ? p : 0] : "-", dma_ ? age_ms : 0.0,
           (unsigned long long)phase_seq_.load(), p >= (int)Phase::FENCE_WAIT ? ": " : "", p >= (int)Phase::FENCE_WAIT ? phase_what_ : "", status_str(err_.load()));
  return buf;
}

std::string Ring::last_error_desc() {
  std::lock_guard<OrderedMutex> g(m_);
  return err_desc_;
}

}  // namespace ogkm
