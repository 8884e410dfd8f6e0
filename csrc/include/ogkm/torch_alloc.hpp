// PyTorch pluggable allocator and the transparent managed mode's op holds
// (csrc/core/torch_allocator.cpp; Python side open-gpu-kernel-modules_amd/
// allocator.py and managed.py).
#pragma once

#include <cstdint>
#include <utility>
#include <vector>

#include "ogkm/common.hpp"

namespace ogkm {

// One managed storage an aten op touches, described by the geometry of its
// views (storage offset, sizes, strides): the op holds only the pages of that
// extent, and a write invalidates the other copies of only the pages written.
struct TorchOperand {
  uint64_t ptr = 0;      // storage base (the managed allocation's stable VA)
  bool write = false;
  uint64_t lo = 0, hi = 0;  // byte extent of every view of this storage in the op; hi == 0: the whole allocation
  // byte intervals written; empty with `write`: the whole extent
  std::vector<std::pair<uint64_t, uint64_t>> written;
};

// Cached extents / empty slabs back to the HBM arena (before an arena re-init).
void torch_alloc_trim(int device);
void torch_alloc_stats(int device, uint64_t* allocated, uint64_t* peak, uint64_t* nallocs, uint64_t* stream_waits,
                       uint64_t* lazy_fences = nullptr, uint64_t* extent_hits = nullptr);
void* torch_alloc(size_t size, int device, void* stream);
void torch_free(void* p, int device, void* stream);
Status torch_park(void* p, int device, void* stream);
Status torch_unpark(void* p, int device, void* stream);
void torch_managed_stats(int device, uint64_t* active, uint64_t* parked, uint64_t* parks, uint64_t* unparks);
void torch_park_all(int device, void* stream);
Status torch_op_begin(const std::vector<TorchOperand>& ops, int device, void* stream, std::vector<uint64_t>* held,
                      std::vector<uint64_t>* persistent);
// hints: (storage, op-clock time of its next use) from the recorded op trace;
// now: the current op clock (0: no trace yet - no hints).
Status torch_op_end(const std::vector<uint64_t>& held, const std::vector<uint64_t>& outs, int device, void* stream,
                    const std::vector<std::pair<uint64_t, uint64_t>>& hints = {}, uint64_t now = 0);
Status torch_set_read_mostly(void* p, int device, bool on);
Status torch_advise(void* p, int device, int advice, int loc_kind, int loc_id, int proc);
bool torch_is_managed(void* p, int device);
// (storage, op-clock time it is needed at; 0 = unknown): prefetches evict only
// data needed later than that.
size_t torch_prefetch(const std::vector<std::pair<uint64_t, uint64_t>>& ptrs, int device);
void torch_prefetch_wait(int device);  // every queued (asynchronous) prefetch placed
uint64_t torch_managed_size(void* p, int device);
uint64_t torch_managed_range_id(void* p, int device);  // 0: not a managed tensor
uint64_t torch_resident_bytes(void* p, int device);  // bytes of the tensor resident in HBM
// Last allocation failure on `device` (empty: none): the message a caller
// surfaces instead of aborting.
const char* torch_last_error(int device);

}  // namespace ogkm
