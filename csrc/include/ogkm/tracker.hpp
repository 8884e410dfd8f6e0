// Completion tracking (analog of uvm_tracker.h:82-201 and the GPU tracking
// semaphores of uvm_gpu_semaphore.c).
//
// A Fence is one completion point: a backend event recorded on some stream,
// optionally tagged with the (ring, seq) it retires. A Tracker is a small set of
// fences with add / merge / query / wait / prune, exactly the operations the
// reference's uvm_tracker_t exposes. Waiting can happen on the CPU
// (event_sync) or be turned into a GPU-side dependency (stream_wait_event) so
// the compute stream never blocks the host.
#pragma once

#include <memory>
#include <mutex>
#include <vector>

#include "ogkm/backend.hpp"
#include "ogkm/common.hpp"

namespace ogkm {

class Ring;

struct Fence {
  Backend* be = nullptr;
  void* event = nullptr;   // owned; returned to the backend on destruction
  Ring* ring = nullptr;    // ring whose work this fence retires (may be null)
  uint64_t seq = 0;        // ring tracking value
  int dev = -1;
  void* stream = nullptr;  // stream the event was recorded on (fence_record)
  std::atomic<bool> done{false};
  ~Fence();
  bool query();
  Status wait();
};
using FenceRef = std::shared_ptr<Fence>;

// Records an event on `stream` and wraps it in a fence.
FenceRef fence_record(Backend* be, int dev, void* stream, Ring* ring = nullptr, uint64_t seq = 0);
// A fence on ring work by tracking value alone (no event): valid as soon as the
// SQE is pushed, before the ring is submitted - waiting on it submits the ring;
// GPU-side waits use the ring's tracking semaphore.
FenceRef ring_fence(Ring* ring, uint64_t seq);

class Tracker {
 public:
  void add(const FenceRef& f);
  void merge(const Tracker& o);
  bool query();                 // true when all fences completed (prunes completed)
  Status wait();                // CPU wait for all
  Status gpu_wait(Backend* be, void* stream) const;  // stream waits on every pending fence
  void prune();
  void clear() { fences_.clear(); }
  bool empty() const { return fences_.empty(); }
  size_t size() const { return fences_.size(); }
  const std::vector<FenceRef>& fences() const { return fences_; }

 private:
  std::vector<FenceRef> fences_;
};

}  // namespace ogkm
