// Virtual-address data model: VaSpace -> Range -> 2 MB Block.
//
//  * VaSpace  (uvm_va_space.h:186): per-runtime container of ranges, keyed by the
//    CPU view address in an ordered map (range tree, uvm_range_tree.c:98-156).
//  * Range    (uvm_va_range.h:107-113): MANAGED, EXTERNAL, CXL or DEVICE_P2P.
//    A managed range owns a CPU view (mmap reservation whose 2 MB windows are
//    mapped onto host/CXL arena pages on demand) and, in stable-VA mode, a
//    device VA reservation whose blocks are VMM-mapped onto HBM chunks.
//  * Block    (uvm_va_block.h:101-523): residency per memory location as 4 KB
//    page masks plus the backing chunk, CPU mapping state, policy, perf state,
//    lease pins and a tracker of outstanding copies.
//  * Policy   (uvm_va_policy.h:57-82): read duplication, preferred location
//    (incl. NUMA node -> CXL tier), accessed_by.
#pragma once

#include <atomic>
#include <deque>
#include <map>
#include <memory>
#include <string>
#include <unordered_map>
#include <vector>

#include "ogkm/arena.hpp"
#include "ogkm/common.hpp"
#include "ogkm/lock_order.hpp"
#include "ogkm/tracker.hpp"

namespace ogkm {

class Range;
class VaSpace;
class RangeGroup;

struct Policy {
  bool read_dup = false;
  bool has_preferred = false;
  Loc preferred{};
  ProcMask accessed_by = 0;
};

// Thrashing detection state (uvm_perf_thrashing.c:37-82 analog, block granularity).
struct ThrashState {
  uint64_t last_migration_ns = 0;
  uint64_t window_start_ns = 0;
  uint32_t events_in_window = 0;
  uint32_t throttles = 0;
  uint32_t resets = 0;
  uint64_t epoch_start_ns = 0;
  uint64_t pinned_until_ns = 0;
  int last_dst_slot = -1;
  bool detected = false;
  // THROTTLE (uvm_perf_thrashing.c:1535-1762 hints): the processor pulling the
  // block back and forth naps - its faults on the block map remotely or wait -
  // until throttle_until_ns.
  uint64_t throttle_until_ns = 0;
  int throttle_slot = -1;
  bool throttling = false;  // ThrottlingStart emitted, ThrottlingEnd pending
};

// Software access counters (uvm_gpu_access_counters.c analog): remote accesses
// per accessing processor to this 2 MB region.
struct AccessCounterState {
  uint32_t remote_hits[kMaxGpus + 1] = {0};
  // Hot for this processor: its next residency decision migrates the block to
  // it instead of mapping remotely (uvm_gpu_access_counters.c:1617,1704).
  bool promote[kMaxGpus + 1] = {false};
};

// Segmented packed host copy (Residency::fmt 3): the block's 2 MB cut into
// 32 segments of 64 KB (16 pages). Segments that are not being written rest
// packed - each its own ANS1 chunk, laid out back to back in a sidecar chunk of
// the same arena - while written segments stay raw at their natural offsets in
// the residency's own chunk. A write-back of a few pages expands (decodes)
// only the segments it touches; a refill moves the packed segments' bytes
// (ONE staging copy: they are contiguous) plus the raw segments' pages. The
// reference tracks residency per 4 KB page inside each 2 MB block
// (uvm_va_block.h:104-112) and moves per-page runs through staging
// (uvm_va_block.c:3673-3760); this keeps its packed form per 64 KB.
constexpr uint32_t kSegPages = 16;
constexpr uint32_t kSegsPerBlock = kPagesPerBlock / kSegPages;  // 32
constexpr uint32_t kSegBytes = kSegPages << kPageShift;        // 64 KB
struct SegDir {
  ChunkArena* arena = nullptr;
  int64_t chunk = -1;           // the sidecar chunk holding the packed segments
  uint32_t packed = 0;          // bit s: segment s rests packed (its raw pages are stale)
  uint32_t used = 0;            // sidecar bytes in use (256-B aligned appends)
  uint32_t off[kSegsPerBlock] = {0};
  uint32_t len[kSegsPerBlock] = {0};
  uint32_t packed_bytes() const {
    uint32_t n = 0;
    for (uint32_t s = 0; s < kSegsPerBlock; ++s)
      if ((packed >> s) & 1u) n += len[s];
    return n;
  }
};
// Pages of segment s / the segments a page mask touches.
inline PageMask seg_pages(uint32_t s) { return PageMask::range(s * kSegPages, kSegPages); }
inline uint32_t segs_of(const PageMask& m) {
  uint32_t r = 0;
  for (uint32_t s = 0; s < kSegsPerBlock; ++s)
    if (m.count_range(s * kSegPages, kSegPages)) r |= 1u << s;
  return r;
}
// Segments every page of which is in m.
inline uint32_t segs_full(const PageMask& m) {
  uint32_t r = 0;
  for (uint32_t s = 0; s < kSegsPerBlock; ++s)
    if (m.count_range(s * kSegPages, kSegPages) == kSegPages) r |= 1u << s;
  return r;
}

struct Residency {
  int slot = -1;             // Loc::slot()
  Loc loc{};
  PageMask resident;
  ChunkArena* arena = nullptr;
  int64_t chunk = -1;
  // chunk content: 0 raw pages, 1 BF12-encoded block (RANGE_COMPRESS_BF16),
  // 2 ANS1-packed block (a packed host / CXL copy of any managed block,
  // Runtime::pack_block; lossless, whole block, never written in place -
  // expanded back to raw pages before any write or CPU mapping).
  // 3: segmented packed host copy (SegDir above): raw segments in `chunk`,
  // packed ones in `seg->chunk`.
  uint8_t fmt = 0;
  uint32_t enc_bytes = 0;    // encoded size when fmt 1 / 2
  std::shared_ptr<SegDir> seg;  // fmt 3
};

class Block {
 public:
  Block(Range* r, uint64_t index, uint32_t npages) : range(r), index(index), npages(npages) {}
  Range* range;
  uint64_t index;      // block number inside the range
  uint32_t npages;     // < 512 for a partial last block
  OrderedMutex lock{LockOrder::VA_BLOCK};
  Policy policy;

  // One entry per location holding a chunk. A deque: appending never moves
  // existing entries, so Residency* stay valid while copies are queued.
  std::deque<Residency> res;
  PageMask cpu_ro, cpu_rw;     // CPU view protection state
  ChunkArena* cpu_arena = nullptr;  // host/CXL chunk currently mapped in the CPU window
  int64_t cpu_chunk = -1;
  // HBM chunk VMM-mapped at the stable device VA (-1 = none). Written under
  // Runtime::stable_m_ (a remap of another block may tear a stale mapping down).
  std::atomic<int64_t> stable_chunk{-1};
  // Work that may still access the stable VA through its current mapping (the
  // block's tracker - copies and lease-release fences - when it was evicted):
  // the mapping is torn down only once it completed (a kernel queued before the
  // release would otherwise fault on an unmapped VA). Guarded by Runtime::stable_m_.
  Tracker stable_users;
  // Value of Runtime::tlb_started_ when the stable VA was last unmapped (~0:
  // unknown - a fresh block): a translation of the VA can linger in a GPU TLB
  // until a flush that started after that unmap has completed, so a remap
  // needs a flush only then (Runtime::stable_map_block). Guarded by stable_m_.
  uint64_t va_unmap_seq = ~0ull;
  // Value of Runtime::tlb_started_ when the stable VA was last remapped in a
  // way that needs a translation flush (~0: none needed): a lease of the block
  // from ANY thread must see a flush started after that complete before its
  // kernels use the VA (another thread's remap may still await its flush).
  // Guarded by the block lock.
  uint64_t map_seq = ~0ull;
  // The stable VA still maps a chunk the block left (its users were running at
  // the eviction): listed in Runtime::stale_maps_ until the mapping goes.
  std::atomic<bool> stale_mapping{false};
  bool in_stale_list = false;  // listed in Runtime::stale_maps_ (guarded by stable_m_)
  uint32_t lease_pins = 0;
  // Packed host copies (Runtime::pack_block): queued for the pack workers /
  // found incompressible (cleared when the block is written) / GPU copies
  // evicted without a copy-out (read-mostly detection).
  bool pack_queued = false;
  bool pack_skip = false;
  // Segments written by the latest write-back into the host copy (fmt 0 / 3):
  // the others are candidates for segment packing; seg_gen counts such writes
  // (a segment pack in flight that sees it move starts over).
  uint32_t seg_written = 0;
  uint64_t seg_gen = 0;
  bool seg_pack_queued = false;
  uint32_t clean_evictions = 0;
  uint32_t gpu_evictions = 0;  // times an HBM copy of this block was evicted (refault detection)
  uint64_t gpu_evicted_at = 0; // the HBM arena's eviction count when it last was (refault distance)
  uint32_t user_pins = 0;      // range-group / explicit pins (non-migratable)
  uint64_t last_access_ns = 0;
  uint32_t faults_by_proc[kMaxGpus + 1] = {0};
  ThrashState thrash;
  AccessCounterState counters;
  Tracker tracker;             // outstanding copies touching this block
  // Copies queued into this block whose fence is not yet in `tracker` (between
  // make_resident and finish_ctx). While non-zero the new residency bits must
  // not be trusted by another thread (CPU mapping, leases).
  uint32_t unpublished = 0;

  Residency* find(const Loc& l);
  Residency* find_slot(int slot);
  Residency& get_or_add(const Loc& l);
  void drop(const Loc& l);
  PageMask resident_anywhere() const;
  LocMask resident_locs(const PageMask& pages) const;  // locations holding any of `pages`
  uint64_t block_offset() const { return index << kBlockShift; }
  PageMask valid_pages() const { return PageMask::range(0, npages); }
};

enum class RangeType : int { MANAGED = 0, EXTERNAL = 1, CXL = 2, DEVICE_P2P = 3 };
const char* range_type_str(RangeType t);

enum RangeFlags : uint32_t {
  RANGE_STABLE_VA = 1u << 0,   // device VA fixed for the lifetime (VMM mapped)
  RANGE_NO_CPU_VIEW = 1u << 1, // skip the CPU view reservation
  // Contents are bf16 and read-only on GPUs: host / CXL copies are stored
  // BF12-packed (lossless) and decoded by the H2D copy kernel. Implies no CPU view.
  RANGE_COMPRESS_BF16 = 1u << 2,
  // Never-populated pages need no zero-fill (torch allocations: the caller
  // writes before it reads, as with any caching allocator). Saves a memset per
  // fresh block - and keeps fresh-block fills kernel-free on the copy engines.
  RANGE_NO_ZERO_FILL = 1u << 3,
};

class Range {
 public:
  // want_view != 0: the CPU window must sit exactly there (in-place restore); cpu_view stays null otherwise.
  Range(VaSpace* vs, uint64_t id, RangeType t, uint64_t size, uint32_t flags, std::string name,
        uint64_t want_view = 0);
  ~Range();
  VaSpace* vs;
  uint64_t id;
  RangeType type;
  uint64_t size;        // requested bytes
  uint64_t nblocks;
  uint32_t flags;
  std::string name;
  uint8_t* cpu_view = nullptr;  // CPU VA (reserved PROT_NONE, 2 MB aligned)
  uint64_t cpu_view_bytes = 0;
  void* dev_va = nullptr;       // stable VA reservation
  int stable_dev = -1;
  // EXTERNAL / DEVICE_P2P: foreign memory registered into the VA space
  uint64_t ext_ptr = 0;
  int ext_dev = -1;
  bool ext_owned = false;       // allocated by the runtime (DEVICE_P2P)
  RangeGroup* group = nullptr;
  std::vector<std::unique_ptr<Block>> blocks;
  std::atomic<int64_t> views{0};  // live tensor views / leases
  // Op-clock time of the range's next use (0 = unknown), from a recorded
  // access trace (the transparent mode, torch_allocator.cpp): its HBM chunks
  // then carry it and eviction picks the data used furthest in the future.
  std::atomic<uint64_t> next_use{0};
  // Contents are dead (a freed torch allocation waiting for reuse or for its
  // stream fence): evicting its blocks copies nothing out.
  std::atomic<bool> dead{false};
  // Spread class the runtime gave the range's hints (SpreadPolicy): -1 none,
  // 0 keep, 1 stream. HBM extents of the two classes are laid out from
  // opposite ends of the arena (PlacementSide) so the stream class's turnover
  // does not fragment the keep class's chunks.
  std::atomic<int> spread_cls{-1};
  // Bumped by every write through the runtime and every revocation of a copy's
  // pages: a lease kept across uses (UnitStream hold mode) is re-validated
  // against it instead of re-walking the blocks.
  std::atomic<uint64_t> mod_gen{0};
  bool destroyed = false;
  OrderedMutex place_lock{LockOrder::RANGE_PLACE};  // GPU extent placement

  uint64_t addr() const { return (uint64_t)cpu_view; }
  Block* block(uint64_t i) { return i < blocks.size() ? blocks[i].get() : nullptr; }
};

class RangeGroup {
 public:
  explicit RangeGroup(uint64_t id) : id(id) {}
  uint64_t id;
  bool migratable = true;   // false = residency frozen (UVM non-migratable range group)
  std::vector<Range*> ranges;
};

class VaSpace {
 public:
  VaSpace() = default;
  OrderedRWLock lock{LockOrder::VA_SPACE};
  std::map<uint64_t, Range*> tree;  // cpu_view start -> range
  std::map<uint64_t, Range*> dev_tree;  // stable device VA start -> range (RANGE_STABLE_VA)
  std::unordered_map<uint64_t, std::unique_ptr<Range>> ranges;
  std::unordered_map<uint64_t, std::unique_ptr<RangeGroup>> groups;
  uint64_t next_range_id = 1;
  uint64_t next_group_id = 1;
  ProcMask registered_gpus = 0;
  uint64_t peers_enabled = 0;  // bit (a*kMaxGpus+b) compressed into a set below
  std::vector<std::pair<int, int>> peer_pairs;

  Range* find_locked(uint64_t addr);  // caller holds lock (shared or exclusive)
  Range* by_id_locked(uint64_t id);
};

}  // namespace ogkm
