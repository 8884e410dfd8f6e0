// Observability: the internal perf-event bus (uvm_perf_events.h:52-78,
// uvm_perf_events.c:56-94) and the user-visible tools event queues + counters
// (uvm_tools.c:448-509, event types uvm_types.h:362-392, counters
// uvm_types.h:283-313).
//
// EventQueue keeps the reference's control-block protocol (put_ahead /
// put_behind / get_ahead / get_behind + per-type dropped counters) in one
// mmap'ed region so a reader (Python, or another process via /dev/shm) can
// consume entries without a syscall.
#pragma once

#include <atomic>
#include <cstdint>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "ogkm/common.hpp"
#include "ogkm/lock_order.hpp"

namespace ogkm {

// ------------------------------------------------------------- perf event bus
enum class PerfEvent : int {
  BLOCK_DESTROY = 0,
  BLOCK_SHRINK,
  BLOCK_MUNMAP,
  RANGE_DESTROY,
  RANGE_SHRINK,
  MODULE_UNLOAD,
  FAULT,
  MIGRATION,
  REVOCATION,
  COUNT
};

struct PerfEventData {
  PerfEvent type;
  uint64_t range_id = 0;
  uint64_t block_index = 0;
  Loc src{}, dst{};
  int processor = 0;
  uint64_t bytes = 0;
  int cause = 0;
  uint32_t first_page = 0, npages = 0;
  bool is_write = false;
  bool moved = false;      // MIGRATION: other copies were revoked (not a read duplicate)
  void* block = nullptr;   // in-process subscribers: the Block (its lock is held by the notifier)
};

class PerfEventBus {
 public:
  using Cb = std::function<void(const PerfEventData&)>;
  int subscribe(PerfEvent e, Cb cb);
  void unsubscribe(int token);
  void notify(const PerfEventData& d);

 private:
  struct Sub { int token; PerfEvent e; Cb cb; };
  std::mutex m_;  // writers
  std::shared_ptr<const std::vector<Sub>> subs_;  // snapshot read by notify()
  int next_ = 1;
};

// ------------------------------------------------------------- tools events
enum class ToolsEventType : uint8_t {
  CpuFault = 1,
  Migration = 2,
  GpuFault = 3,
  GpuFaultReplay = 4,
  FaultBufferOverflow = 5,
  FatalFault = 6,
  ReadDuplicate = 7,
  ReadDuplicateInvalidate = 8,
  PageSizeChange = 9,
  ThrashingDetected = 10,
  ThrottlingStart = 11,
  ThrottlingEnd = 12,
  MapRemote = 13,
  Eviction = 14,
  // framework additions
  Prefetch = 15,
  AccessCounter = 16,
  CxlDma = 17,
  RingError = 18,
  Checkpoint = 19,
  NumTypes = 20
};

// Migration / eviction causes (UvmEventMigrationCause analog).
enum class Cause : uint8_t { User = 0, Coherence, Prefetch, Eviction, AccessCounters, ApiMigrate, Thrashing, Cxl };

struct ToolsEvent {  // 64 bytes, POD
  uint8_t type;
  uint8_t cause;
  uint8_t src_slot;
  uint8_t dst_slot;
  uint32_t processor;
  uint64_t address;     // range-relative or absolute address
  uint64_t bytes;
  uint64_t ts_begin_ns;
  uint64_t ts_end_ns;
  uint64_t range_id;
  uint64_t seq;
  uint64_t aux;
};
static_assert(sizeof(ToolsEvent) == 64, "tools event is 64 bytes");

struct ToolsQueueCtrl {  // lives at the head of the mmap'ed queue region
  std::atomic<uint32_t> put_ahead;
  std::atomic<uint32_t> put_behind;
  std::atomic<uint32_t> get_ahead;
  std::atomic<uint32_t> get_behind;
  uint32_t entries;      // power of two
  uint32_t enabled_mask; // bit per ToolsEventType
  std::atomic<uint64_t> dropped[(int)ToolsEventType::NumTypes];
};

class EventQueue {
 public:
  EventQueue(uint32_t entries, uint32_t enabled_mask, const std::string& shm_name = "");
  ~EventQueue();
  // Producer side; returns false if the queue is full (counted as dropped).
  bool push(const ToolsEvent& e);
  // Consumer side; copies up to max entries out, advancing get.
  size_t pop(ToolsEvent* out, size_t max);
  ToolsQueueCtrl* ctrl() { return ctrl_; }
  uint32_t enabled_mask() const { return ctrl_->enabled_mask; }
  void set_enabled_mask(uint32_t m) { ctrl_->enabled_mask = m; }
  void* region() { return base_; }
  size_t region_bytes() const { return bytes_; }
  const std::string& shm_name() const { return shm_name_; }

 private:
  void* base_ = nullptr;
  size_t bytes_ = 0;
  ToolsQueueCtrl* ctrl_ = nullptr;
  ToolsEvent* ring_ = nullptr;
  std::mutex produce_m_;
  std::string shm_name_;
};

enum class Counter : int {
  BytesXferHtD = 0,
  BytesXferDtH,
  BytesXferDtD,     // peer / intra-GPU
  BytesXferHtC,     // host -> cxl
  BytesXferCtH,
  BytesXferCtD,     // cxl -> gpu
  BytesXferDtC,
  CpuPageFaultCount,
  GpuPageFaultCount,
  PrefetchBytesXferHtD,
  PrefetchBytesXferDtH,
  Evictions,
  EvictedBytes,
  ThrashingDetected,
  ThrottleEvents,
  PinEvents,
  MapRemote,
  AccessCounterNotifications,
  AccessCounterMigrations,
  ReadDuplications,
  Revocations,
  RingSubmissions,
  RingCompletions,
  CopyKernelLaunches,
  FaultBatches,
  FaultsCoalesced,
  CxlDmaRequests,
  CxlDmaBytes,
  AllocRetries,
  InjectedErrors,
  DecodedBytes,     // raw bytes produced by the fused BF12 copy+decode
  EncodedBytes,     // raw bytes stored BF12-packed in host / CXL tiers
  TableShootdowns,  // device residency-table entries cleared before their chunk was released
  FaultReplays,     // replay tokens issued after serviced device-fault batches
  FaultRecordsConsumed,  // device fault-buffer records consumed from GET
  PageListCopies,   // fragmented block copies issued as one page-list kernel
  VmmRemaps,        // stable-VA block remaps (unmap / map of a 2 MB VMM handle)
  VmmErrors,        // failed stable-VA unmaps / maps / translation flushes
  TlbFlushes,       // GPU translation flushes after stable-VA remaps
  FaultsCancelled,  // channels whose device faults were cancelled (precise cancel)
  TlbFlushesElided, // stable-VA maps that needed no flush (a flush since the VA's last unmap covered it)
  WriteInvalidations,  // blocks whose other copies were revoked for a page-granular write (invalidate_others)
  RemoteFallbacks,     // remote (zero-copy) decisions served by a local copy (acquire allow_remote=false)
  VmmMapNs,            // host time in stable-VA maps (map + access)
  VmmUnmapNs,          // host time in stable-VA unmaps
  TlbFlushNs,          // host time in translation flushes
  PlaceStableNs,       // host time in stable-VA placement (place_stable, incl. the above and evictions)
  StableWaitNs,        // host time waiting for kernels still using a stable VA before its remap / unmap
  RingFenceWaitNs,     // H2D DMA ring workers: host time waiting for a copy's dependencies (reuse fences)
  RingCopyNs,          // H2D DMA ring workers: time in engine copies (issue + completion)
  RingIdleNs,          // H2D DMA ring workers: time with no batch to run
  RingCopyCalls,       // H2D DMA ring workers: engine copy calls (merged runs)
  DemotionFallbacks,   // evictions demoted past a full node (node-wide budget spent) to the next tier / node
  LedgerRefusals,      // host / CXL segments the node-wide ledger refused (budget shared by all ranks)
  LeaseFastPaths,      // acquires served by the resident-extent fast path (Runtime::fast_lease)
  PackedBlocks,        // host / CXL copies packed to ANS1 (Runtime::pack_block)
  PackedBytesSaved,    // bytes those packings saved
  PackSkips,           // blocks found incompressible (left raw)
  PackExpansions,      // packed copies expanded back to raw pages (a write / CPU access)
  PackedDecodes,       // packed blocks decoded into HBM by the H2D ring (DECODE_ANS)
  PressureReliefs,     // reservations that found nothing evictable until soft pins let go
  DecodeReuseWaits,    // H2D copies that waited for a running packed-block decode into the same chunk
  RingMergedBatches,   // packed-decode batches the H2D ring ran merged into the batch before (Ring::worker)
  VictimSearchNs,      // host time in next-use victim searches (ChunkArena::next_victims_locked)
  VictimRisenSeen,     // re-hinted chunks those searches re-ranked (summed over calls)
  SegPacked,           // 64 KB segments of written blocks' host copies packed (fmt 3, Runtime::pack_segments)
  SegExpansions,       // packed segments decoded back to raw pages (a write-back touched them)
  SegDecodes,          // packed segments decoded into HBM by the H2D ring
  NumCounters
};
const char* counter_name(Counter c);

class Tools {
 public:
  static Tools& get();
  void record(const ToolsEvent& e);  // fan out to all queues that enable e.type
  void inc(Counter c, uint64_t v = 1) { counters_[(int)c].fetch_add(v, std::memory_order_relaxed); }
  uint64_t counter(Counter c) const { return counters_[(int)c].load(std::memory_order_relaxed); }
  void reset_counters();
  int create_queue(uint32_t entries, uint32_t enabled_mask, const std::string& shm_name = "");
  EventQueue* queue(int id);
  void destroy_queue(int id);
  bool any_queue() const { return nqueues_.load(std::memory_order_relaxed) > 0; }
  PerfEventBus& bus() { return bus_; }

 private:
  std::atomic<uint64_t> counters_[(int)Counter::NumCounters] = {};
  OrderedMutex m_{LockOrder::TOOLS};
  std::vector<std::unique_ptr<EventQueue>> queues_;
  std::atomic<int> nqueues_{0};
  PerfEventBus bus_;
};

// Convenience: record a migration-like event if any queue is listening.
void tools_event(ToolsEventType t, Cause c, Loc src, Loc dst, int proc, uint64_t addr, uint64_t bytes,
                 uint64_t range_id, uint64_t t0 = 0, uint64_t t1 = 0, uint64_t aux = 0);

}  // namespace ogkm
