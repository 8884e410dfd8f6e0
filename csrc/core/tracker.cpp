// Fences and trackers.
#include "ogkm/tracker.hpp"

#include <algorithm>

#include "ogkm/config.hpp"
#include "ogkm/ring.hpp"

namespace ogkm {

Fence::~Fence() {
  if (be && event) be->event_destroy(event);
}

bool Fence::query() {
  if (done.load(std::memory_order_acquire)) return true;
  bool d = true;
  if (ring && ring->completed_seq() < seq) d = false;
  if (d && be && event) d = be->event_query(event);
  if (d) done.store(true, std::memory_order_release);
  return d;
}

Status Fence::wait() {
  if (done.load(std::memory_order_acquire)) return Status::OK;
  Status s = Status::OK;
  uint64_t t0 = now_ns();
  if (be && event) s = be->event_sync(event);
  uint64_t t1 = now_ns();
  if (s == Status::OK && ring) s = ring->wait_seq(seq);
  uint64_t t2 = now_ns();
  if (t2 - t0 > 1000000000ull)
    RT_WARN("slow fence wait: event_sync %.1f ms, ring wait %.1f ms (ring %s/%d seq %llu completed %llu submitted %llu)",
            (t1 - t0) / 1e6, (t2 - t1) / 1e6, ring ? ring_kind_str(ring->kind()) : "-", ring ? ring->dev() : -1,
            (unsigned long long)seq, (unsigned long long)(ring ? ring->completed_seq() : 0),
            (unsigned long long)(ring ? ring->submitted_seq() : 0));
  if (s == Status::OK) done.store(true, std::memory_order_release);
  return s;
}

FenceRef fence_record(Backend* be, int dev, void* stream, Ring* ring, uint64_t seq) {
  auto f = std::make_shared<Fence>();
  f->be = be;
  f->dev = dev;
  f->ring = ring;
  f->seq = seq;
  f->stream = stream;
  f->event = be->event_create(dev);
  if (!f->event || be->event_record(f->event, stream) != Status::OK) {
    // Could not record: degrade to a ring-only fence (or completed).
    if (f->event) be->event_destroy(f->event);
    f->event = nullptr;
    if (!ring) f->done.store(true);
  }
  return f;
}

FenceRef ring_fence(Ring* ring, uint64_t seq) {
  auto f = std::make_shared<Fence>();
  f->ring = ring;
  f->seq = seq;
  f->dev = ring->dev();
  return f;
}

void Tracker::add(const FenceRef& f) {
  if (!f || f->done.load(std::memory_order_relaxed)) return;
  for (auto& x : fences_)
    if (x == f) return;
  // Keep only the newest fence per ring: ring fences complete in order (DMA
  // ring fences carry no event; stream ring fences always carry one).
  if (f->ring) {
    for (auto& x : fences_)
      if (x->ring == f->ring && (x->event != nullptr) == (f->event != nullptr)) {
        if (x->seq <= f->seq) x = f;
        return;
      }
  }
  fences_.push_back(f);
  if (fences_.size() > 16) prune();
}

void Tracker::merge(const Tracker& o) {
  for (auto& f : o.fences_) add(f);
}

void Tracker::prune() {
  fences_.erase(std::remove_if(fences_.begin(), fences_.end(), [](const FenceRef& f) { return f->query(); }),
                fences_.end());
}

bool Tracker::query() {
  prune();
  return fences_.empty();
}

Status Tracker::wait() {
  Status st = Status::OK;
  for (auto& f : fences_) {
    Status s = f->wait();
    if (s != Status::OK && st == Status::OK) st = s;
  }
  if (st == Status::OK) fences_.clear();
  return st;
}

Status Tracker::gpu_wait(Backend* be, void* stream) const {
  bool ring_wait = false;  // a GPU-side wait on a ring's tracking value was queued
  for (auto& f : fences_) {
    if (f->done.load(std::memory_order_relaxed)) continue;
    // An event recorded on this very stream is already ordered before
    // anything enqueued on it now: no barrier packet (a lease of a unit whose
    // previous readers ran on the consumer's own stream - every resident unit
    // of a decode step).
    // Never for the null stream: nullptr names a different stream on each
    // device, so a fence on GPU0's null stream says nothing about GPU1's.
    if (f->event && stream && f->stream == stream) continue;
    // Already retired (the flag is only set by whoever polled last): no packet.
    if (f->ring && !f->event && f->ring->completed_seq() >= f->seq) {
      f->done.store(true, std::memory_order_release);
      continue;
    }
    Status s;
    uint64_t t0 = now_ns();
    bool had_event = f->event != nullptr;
    bool ev_done = had_event && be->event_query(f->event);
    if (ev_done && (!f->ring || f->ring->completed_seq() >= f->seq)) {
      f->done.store(true, std::memory_order_release);
      continue;
    }
    if (f->event) s = be->stream_wait_event(stream, f->event);
    else if (f->ring) {
      // Tracking-value fence: make sure the ring work is submitted, then let
      // the stream wait for the ring's semaphore GPU-side.
      if (f->seq > f->ring->submitted_seq()) f->ring->submit();
      // ... and issued to the engines, so no copy of it can queue behind work
      // enqueued after this wait (Ring::issued_seq)
      s = f->ring->wait_issued(f->seq);
      if (s == Status::OK) s = be->wait_value(stream, f->ring->semaphore(), f->seq);
      ring_wait = true;
    }
    else s = f->wait();
    uint64_t dt = now_ns() - t0;
    if (dt > 20000000ull)  // a GPU-side dependency should cost microseconds of host time
      RT_WARN("slow gpu_wait: %.1f ms event=%d event_done=%d ring=%s seq=%llu completed=%llu submitted=%llu",
              dt / 1e6, (int)had_event, (int)ev_done, f->ring ? ring_kind_str(f->ring->kind()) : "-",
              (unsigned long long)f->seq, (unsigned long long)(f->ring ? f->ring->completed_seq() : 0),
              (unsigned long long)(f->ring ? f->ring->submitted_seq() : 0));
    if (s != Status::OK) return s;
  }
  if (ring_wait && config().gpu_wait_acquire) return be->acquire_caches(stream);
  return Status::OK;
}

}  // namespace ogkm
