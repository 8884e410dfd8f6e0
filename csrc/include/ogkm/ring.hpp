// io_uring-style submission/completion ring per (GPU, channel kind).
//
// Analog of the UVM channel / pushbuffer / GPFIFO machinery
// (uvm_channel.c:934 begin_push, :1484-1580 end_push + doorbell, uvm_push.c,
// uvm_pushbuffer.c) re-designed for MI355X:
//   * producers append SQEs (copy / gather / scatter / memset / fence-wait)
//     to a fixed-size submission queue (channel_num_gpfifo_entries, default 1024);
//   * submit() drains the SQ onto the ring's side hipStream, coalescing
//     consecutive copies into ONE copy-kernel launch (a batch of descriptors),
//     then issues a system-scope release of the ring's tracking value into
//     host-coherent memory (the tracking semaphore) and records a fence;
//   * completions are reaped as CQEs {user_data, seq, status}; every SQE keeps
//     its push description (file:line + text, uvm_push.c:169) so a ring error
//     can name the work that failed (uvm_channel.c:2080-2112);
//   * errors are sticky per ring and propagate to the runtime's fatal status.
//
// DMA rings (copy_engine 3: CPU_TO_GPU, GPU_TO_CPU, GPU_TO_GPU, CXL when the
// backend has copy engines): submit() hands the batch to the ring's worker
// thread, which waits for the batch's fence dependencies, runs its copies on
// the ring's SDMA engine (Backend::dma_copy - no CU, no stream), its rare
// kernel SQEs (memset, fused decode, gather/scatter) on the side stream, and
// then publishes the tracking value with a release store. GPU consumers wait
// on that value GPU-side (hipStreamWaitValue64), so the fences of a DMA ring
// carry no event.
#pragma once

#include <atomic>
#include <condition_variable>
#include <deque>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "ogkm/backend.hpp"
#include "ogkm/common.hpp"
#include "ogkm/lock_order.hpp"
#include "ogkm/tracker.hpp"

namespace ogkm {

enum class RingKind : int {
  CPU_TO_GPU = 0,   // H2D (host / CXL -> HBM)
  GPU_TO_CPU = 1,   // D2H
  GPU_INTERNAL = 2, // D2D within one GPU (compaction, relocation)
  GPU_TO_GPU = 3,   // peer pushes over xGMI (issued by the source GPU)
  MEMOPS = 4,       // memset / zero-fill of new chunks
  CXL = 5,          // cxl_dma requests
  COUNT = 6
};
const char* ring_kind_str(RingKind k);

// DECODE_BF12: fused copy + decode of an encoded block (dst = raw bf16, bytes = 2 * values).
// DECODE_ANS: an ANS1-packed block (src, `bytes` packed bytes) -> n_values bf16
// at dst: DMA rings land the packed bytes in an HBM staging buffer by SDMA and
// decode them there (k_ans_blocks, many blocks per launch); stream rings
// decode straight from the host copy.
// PAGE_COPY: scattered pages of one block, page idx[i] of src -> page idx[i] of
// dst (one LDS-staged kernel instead of one copy per run).
// DECODE_SEGS: packed segments of a segmented host copy (Residency fmt 3): the
// `bytes` at src (the sidecar span holding them, ONE staging copy) hold
// single-segment ANS1 chunks; idx = pairs (segment s | length << 5, offset of
// its chunk from src) and segment s decodes to dst + s * 64 KB.
enum class SqeOp : uint8_t {
  COPY = 0, GATHER, SCATTER, MEMSET, WAIT_FENCE, NOP, DECODE_BF12, PAGE_COPY, DECODE_ANS, DECODE_SEGS
};

struct Sqe {
  SqeOp op = SqeOp::NOP;
  uint64_t user_data = 0;
  uint64_t dst = 0, src = 0, bytes = 0;
  int32_t dst_dev = -1;            // COPY on a GPU_TO_GPU ring: the peer GPU written (engine-mask lookup)
  uint32_t pattern = 0;            // MEMSET
  uint32_t page_bytes = 0;         // GATHER / SCATTER
  uint32_t n_values = 0;           // DECODE_ANS
  std::vector<uint32_t> idx;       // GATHER / SCATTER page indices
  FenceRef wait;                   // WAIT_FENCE
  const char* file = "";
  int line = 0;
  std::string desc;
};

struct Cqe {
  uint64_t user_data;
  uint64_t seq;
  int32_t status;
};

// Split copies over the SDMA engines in `mask` (bit per engine): a copy of at
// least 2 * min_piece bytes becomes min(#engines, bytes / min_piece) pieces
// (64 KB aligned), each on the next engine in rotation (`rot`, carried across
// calls, so small copies spread over the engines too). mask 0: unchanged.
std::vector<CopyDesc> split_over_engines(const std::vector<CopyDesc>& in, uint32_t mask, uint64_t min_piece,
                                         uint32_t* rot);

class Ring {
 public:
  Ring(Backend* be, int dev, RingKind kind, uint32_t entries);
  ~Ring();
  // Append an SQE. Returns its sequence number (tracking value).
  uint64_t push(Sqe&& s);
  // Append a WAIT_FENCE on `f` (skipped for this ring's own / completed fences).
  void push_wait(const FenceRef& f);
  // Submit everything pushed so far; returns the fence of the last batch
  // (an already-completed fence if nothing was pending).
  FenceRef submit();
  // Highest sequence number known complete (read from host-coherent memory).
  uint64_t completed_seq();
  uint64_t submitted_seq() const { return submitted_; }
  uint64_t pushed_seq() const { return next_seq_ - 1; }
  Status wait_seq(uint64_t seq);
  // DMA rings: highest tracking value whose work has been handed to the copy
  // engines / streams (every batch up to it issued; it may still be running).
  // A GPU-side wait on a DMA ring's value is enqueued only once that value is
  // issued (wait_issued): otherwise a queue waiting on it could sit ahead of
  // HIP's own engine copies (torch / gloo D2H on a stream behind the wait) and
  // the worker's later copies would queue behind those - a cycle through the
  // shared SDMA engine (the round-4 2-rank peer-shard hang, gpurun_out/r5).
  uint64_t issued_seq() const { return dma_ ? issued_.load(std::memory_order_acquire) : submitted_.load(); }
  Status wait_issued(uint64_t seq);
  size_t reap(Cqe* out, size_t max);
  // Post-completion error check (uvm_channel.c:2047-2112 channel error
  // detection): a copy or kernel that failed AFTER submission - a faulting
  // kernel, an ECC / link error - marks the ring failed; the CQEs retired
  // since carry the status and fence waits return it.
  Status check_errors();
  Status error() const { return err_; }
  void clear_error_for_test();
  void* stream() const { return stream_; }
  int dev() const { return dev_; }
  RingKind kind() const { return kind_; }
  uint64_t batches() const { return batches_; }
  std::string last_error_desc();
  bool is_dma() const { return dma_; }
  uint64_t* semaphore() const { return sem_; }
  // Hang diagnostics (Runtime::debug_dump): sequence numbers, queued worker
  // batches and what the DMA worker is doing right now, and for how long.
  // Lock-free or try-lock only: safe to call while another thread is stuck.
  std::string debug_state();
  enum class Phase : int { IDLE = 0, ISSUE, COMPLETE, FENCE_WAIT, STREAM_DRAIN, ENGINE_ISSUE, ENGINE_WAIT };

 private:
  struct Batch {
    std::vector<Sqe> ops;   // in submission order (WAIT_FENCE included)
    uint64_t last = 0;      // tracking value published when the batch is done
  };
  FenceRef submit_locked();
  FenceRef submit_dma_locked();
  void worker();
  bool pure_copies(const Batch& b, std::vector<CopyDesc>* out) const;
  static uint64_t packed_bytes(const Batch& b);
  Status run_batch(Batch& b);
  void publish(uint64_t seq);
  Backend* be_;
  int dev_;
  RingKind kind_;
  uint32_t entries_;
  void* stream_ = nullptr;
  uint64_t* sem_ = nullptr;  // host-coherent tracking semaphore
  OrderedMutex m_{LockOrder::RING};
  std::deque<std::pair<uint64_t, Sqe>> sq_;   // pushed, not yet submitted
  std::deque<std::pair<uint64_t, Cqe>> inflight_;  // submitted, not yet reaped
  std::atomic<uint64_t> next_seq_{1};  // read lock-free by pushed_seq()
  std::atomic<uint64_t> submitted_{0};  // read lock-free by wait_seq
  uint64_t batches_ = 0;
  uint32_t engine_rot_ = 0;  // GPU_TO_GPU: engine rotation across split pieces (worker thread only)
  FenceRef last_fence_;
  std::atomic<Status> err_{Status::OK};
  std::string err_desc_;
  // DMA mode
  bool dma_ = false;
  void* stage_ = nullptr;          // HBM staging of packed blocks (DECODE_ANS, worker thread only): two halves
  uint64_t stage_bytes_ = 0;
  uint32_t stage_half_ = 0;        // the half being filled
  void* stage_ev_[2] = {nullptr, nullptr};  // the last decode that read each half
  bool stage_used_[2] = {false, false};
  void* batch_ev_ = nullptr;       // run_batch -> worker: the batch's decodes complete with this event
  std::vector<std::pair<uint64_t, uint64_t>> batch_dst_;  // this batch's decode destinations (addr, bytes)
  struct Deferred {
    void* ev;
    uint64_t last;
    std::vector<std::pair<uint64_t, uint64_t>> dst;  // HBM the decodes write
  };
  std::deque<Deferred> deferred_;  // published once its event completes
  Status publish_deferred_locked(bool all);
  bool copies_hit_deferred(const std::vector<CopyDesc>& copies) const;
  std::thread worker_;
  std::mutex wm_;
  std::condition_variable wcv_;
  std::deque<Batch> work_;
  bool stop_ = false;
  std::atomic<int> phase_{0};             // Phase of the worker
  std::atomic<uint64_t> phase_ns_{0};     // when it entered it
  std::atomic<uint64_t> phase_seq_{0};    // the batch (last seq) it works on
  std::atomic<uint64_t> queued_{0};       // batches handed to the worker, not yet taken
  std::atomic<uint64_t> issued_{0};       // see issued_seq()
  void mark_issued(uint64_t seq) {
    uint64_t cur = issued_.load(std::memory_order_relaxed);
    while (cur < seq && !issued_.compare_exchange_weak(cur, seq, std::memory_order_release)) {
    }
  }
  char phase_what_[128] = {0};            // the fence / kernel it waits for (worker writes; the dump reads racily)
  void set_phase(Phase p, uint64_t seq) {
    phase_ns_.store(now_ns(), std::memory_order_relaxed);
    phase_seq_.store(seq, std::memory_order_relaxed);
    phase_.store((int)p, std::memory_order_release);
  }
};

}  // namespace ogkm
