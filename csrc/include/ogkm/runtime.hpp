// The runtime: devices, tiers, rings, the VA space, and every operation of the
// public API (cudaMallocManaged / cudaMemAdvise / cudaMemPrefetchAsync-shaped,
// in our own namespace), plus fault service, eviction, leases, CXL, checkpoint,
// injection and stats. One Runtime per process (analog of the per-fd VA space
// created by UVM_INITIALIZE, uvm.c:950, plus uvm_global.c state).
#pragma once

#include <atomic>
#include <condition_variable>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <tuple>
#include <unordered_map>
#include <vector>

#include "ogkm/arena.hpp"
#include "ogkm/backend.hpp"
#include "ogkm/common.hpp"
#include "ogkm/config.hpp"
#include "ogkm/cxl.hpp"
#include "ogkm/events.hpp"
#include "ogkm/fault_abi.hpp"
#include "ogkm/ring.hpp"
#include "ogkm/spread.hpp"
#include "ogkm/tracker.hpp"
#include "ogkm/va_space.hpp"

namespace ogkm {

enum class Advice : int {
  SET_READ_MOSTLY = 1,
  UNSET_READ_MOSTLY = 2,
  SET_PREFERRED_LOCATION = 3,
  UNSET_PREFERRED_LOCATION = 4,
  SET_ACCESSED_BY = 5,
  UNSET_ACCESSED_BY = 6,
};

enum class Access : int { READ = 1, WRITE = 2, ATOMIC = 3, PREFETCH = 4 };

// One software fault: a processor is about to access [offset, offset+bytes) of a range.
struct FaultEntry {
  uint64_t range_id = 0;
  uint64_t offset = 0;
  uint64_t bytes = 0;
  int proc = 0;             // GPU id or kCpuProc
  uint16_t channel = 0;     // user channel of the faulting kernel (0 = none)
  Access access = Access::READ;
  uint64_t ts_ns = 0;
  // filled by preprocessing
  uint64_t block = 0;
  uint32_t first_page = 0, npages = 0;
  bool duplicate = false;
  Status status = Status::OK;  // set by service_faults: this entry's group outcome (precise cancel)
};

// Device fault buffer: GET/PUT ring of DeviceFaultRecord (ogkm/fault_abi.hpp)
// in host-coherent memory, appended to by kernels (k_managed_gather,
// k_fault_gate) and drained by the fault-service thread.
struct DeviceFaultBuffer {
  FaultBufHeader* hdr = nullptr;
  DeviceFaultRecord* recs = nullptr;
  uint32_t entries = 0;       // power of two
  uint64_t overflows = 0;     // records producers dropped on a full ring (host total)
  uint32_t overflow_seen = 0; // last value of hdr->overflow accounted for
};

// Per-range device residency table (2 entries per block: hbm address, remote
// address; 0 = absent). Lives in host-coherent memory so kernels can consult
// it and record misses without a host round trip.
struct DeviceResidencyTable {
  uint64_t* entries = nullptr;
  uint64_t nblocks = 0;
  int dev = 0;
};

struct Lease {
  uint64_t id = 0;
  Range* range = nullptr;
  uint64_t offset = 0, bytes = 0;
  int proc = 0;
  bool remote = false;   // pointer targets host/CXL/peer memory (zero-copy)
  uint64_t dptr = 0;     // device pointer of range byte `offset`
  std::vector<std::pair<ChunkArena*, uint32_t>> pinned_chunks;
  std::vector<Block*> blocks;
  Tracker ready;         // consumer must wait on this before use
};

// Init-time check that a stable-VA remap followed by a translation flush is
// seen by kernels on this GPU (Runtime::vmm_self_test): a canary VA is
// remapped between two chunks of known contents and read through the shader
// path after every flush (and once before it, to record whether the stack
// leaves stale translations at all). A failed check refuses stable-VA ranges
// - the transparent managed mode - instead of risking silent stale reads
// (the reference invalidates explicitly, uvm_hal.h:797-799, in batches,
// uvm_tlb_batch.c:27-116).
struct VmmSelfTest {
  bool ran = false, ok = true;
  uint32_t rounds = 0, flushed_ok = 0, unflushed_stale = 0;
  std::string detail;
};

struct Device {
  int id = 0;
  VmmSelfTest vmm_test;
  int numa = 0;
  // Managed by this process (config local_devices). One process per GPU keeps
  // every other GPU non-local: no rings, fault buffer or arena are created on
  // it (no contexts on the neighbours' GPUs).
  bool local = true;
  std::unique_ptr<HbmArena> hbm;
  std::atomic<HbmArena*> hbm_live{nullptr};  // published `hbm` for lock-free readers (arena_for)
  std::unique_ptr<Ring> rings[(int)RingKind::COUNT];
  DeviceFaultBuffer fault_buf;
  // RAS counters at init (the baseline) and the last check: an uncorrectable
  // error past the baseline makes the runtime FATAL (uvm_gpu.c:1328-1354).
  SpreadPolicy spread;  // keep / stream classes of cyclically hinted data (ogkm/spread.hpp)
  Backend::Health health0, health;
  bool health_ok = false;           // the platform reports RAS counters
  std::string health_reason;        // why they are unreadable (empty when readable)
  uint64_t health_checked_ns = 0;
  std::mutex health_m;
};

struct Injection {
  std::atomic<int64_t> alloc_fail_after{-1};   // HBM chunk allocations that succeed before failing
  std::atomic<int64_t> evict_fail{0};          // next N evictions fail
  std::atomic<int64_t> copy_drop{0};           // next N ring copies are dropped (link error)
  std::atomic<uint64_t> peer_link_down{0};     // bit g: peer link of GPU g down
  std::atomic<int64_t> populate_error{0};      // next N populates fail
  std::atomic<int64_t> host_alloc_error{0};    // next N host chunk allocs fail
  std::atomic<int64_t> async_copy_error{0};     // next N ring completions report a post-submission failure
  std::atomic<int64_t> ecc_ue{0}, ecc_ce{0}, link_ue{0};  // fake backend RAS counters
  // Fake backend translation model: 0 coherent (a remap is visible at once),
  // 1 stale until tlb_flush (what gfx950 VMM does), 2 stale and tlb_flush
  // ineffective (a box where the flush does not work).
  std::atomic<int> tlb_mode{0};
};

struct ResidencyInfo {   // UVM_TEST_VA_RESIDENCY_INFO analog (uvm_test_ioctl.h:626-674)
  std::vector<Loc> resident_on;
  std::vector<int64_t> chunk;       // per resident_on entry
  std::vector<uint32_t> pages;      // resident page count per entry
  std::vector<uint32_t> enc_bytes;  // encoded size per entry (0 = raw; fmt 3: the bytes a full refill moves)
  std::vector<uint32_t> seg_packed; // fmt 3: packed 64 KB segments per entry (0 otherwise)
  std::vector<int> mapped_on;       // processors with a mapping (CPU view / stable VA / leases)
  bool read_dup = false;
  bool pinned = false;
  bool thrashing = false;
  int64_t stable_chunk = -1;        // HBM chunk the stable VA maps (may be stale after an eviction)
  Policy policy;
};

class Runtime {
 public:
  static Runtime* get();                          // nullptr before init
  static Runtime* init(const std::string& backend, int fake_devices, uint64_t fake_hbm_bytes);
  static void shutdown();
  ~Runtime();

  Backend* be() { return be_.get(); }
  int ndev() const { return (int)devs_.size(); }
  Device& dev(int i) { return *devs_[i]; }
  bool is_local(int d) const { return d >= 0 && d < (int)devs_.size() && devs_[d]->local; }
  std::vector<int> local_devices() const;
  VaSpace& vs() { return vs_; }
  Injection& inject() { return inject_; }
  CxlTopology& cxl_topology() { return cxl_topo_; }
  CxlRegistry& cxl() { return *cxl_; }
  int host_node() const { return host_node_; }
  Loc cpu_loc() const { return Loc::host(host_node_); }
  Loc proc_loc(int proc) const { return proc == kCpuProc ? cpu_loc() : Loc::gpu(proc); }

  // ---- tiers
  Status init_device(int d, uint64_t budget_bytes);   // (re)create the HBM arena of d
  // Run the stable-VA translation self-test on d's (VMM) arena; see VmmSelfTest.
  Status vmm_self_test(int d);
  HostArena* host_arena(Tier t, int node);            // created on first use
  ChunkArena* arena_for(const Loc& l);
  // d's HBM arena if one exists; never creates the default one (arena_for does)
  ChunkArena* hbm_arena_if_any(int d) { return is_local(d) ? devs_[d]->hbm_live.load(std::memory_order_acquire) : nullptr; }
  // nullptr for a non-local device
  Ring* ring(int dev, RingKind k) { return is_local(dev) ? devs_[dev]->rings[(int)k].get() : nullptr; }

  // ---- allocation / ranges (UvmMemMap + mmap analog)
  Status malloc_managed(uint64_t size, uint32_t flags, const std::string& name, Range** out, int stable_dev = 0);
  // In-place re-creation (checkpoint restore): range id `id`, CPU window at
  // `cpu_addr`, stable device VA at `dev_va` (each 0 = none). BUSY when the id
  // or an address is taken - the caller may fall back to a relocating restore.
  Status malloc_managed_at(uint64_t size, uint32_t flags, const std::string& name, uint64_t id, uint64_t cpu_addr,
                           uint64_t dev_va, int stable_dev, Range** out);
  Status map_external(uint64_t ptr, uint64_t size, int dev, const std::string& name, Range** out);
  Status alloc_device_p2p(uint64_t size, int dev, const std::string& name, Range** out);
  Status free_range(Range* r);
  Range* find_range(uint64_t addr);
  Range* range_by_id(uint64_t id);

  // ---- policy (uvm_policy.c)
  Status mem_advise(Range* r, uint64_t off, uint64_t len, Advice a, Loc loc, int proc);
  Status create_range_group(uint64_t* id);
  Status set_range_group(Range* r, uint64_t group_id);
  Status set_group_migratable(uint64_t group_id, bool migratable);

  // ---- migration (uvm_migrate.c / uvm_va_block.c make_resident)
  Status prefetch(Range* r, uint64_t off, uint64_t len, Loc dst, Tracker* out, Cause cause = Cause::ApiMigrate);
  Status migrate_sync(Range* r, uint64_t off, uint64_t len, Loc dst);
  Status evict_range(Range* r, Loc from);  // push blocks resident at `from` down a tier

  // ---- software faults / leases
  Status service_faults(std::vector<FaultEntry>& faults, Tracker* out);
  // allow_remote = false: a zero-copy (remote) decision - thrashing pin,
  // accessed_by - is overridden by a local copy (callers that need the data at a
  // fixed device address, e.g. the stable VA of a managed torch tensor).
  Status acquire(Range* r, uint64_t off, uint64_t len, int proc, Access access, Lease** out,
                 bool allow_remote = true);
  // consumer's last use recorded on `stream` (or `use`: a fence the caller
  // recorded on it after its last use, shared with its own bookkeeping)
  Status release(Lease* l, void* stream, const FenceRef& use = nullptr);
  // acquire() fast path: a GPU read of a range span resident in one contiguous
  // extent of that GPU's arena - pin + touch + readiness only (false: take the
  // full path).
  bool fast_lease(Range* r, uint64_t off, uint64_t len, int proc, Lease* L);
  // True (and the blocks' chunks LRU-touched as prefetched) when the span is
  // resident on `gpu` in one contiguous extent with nothing pending.
  bool resident_extent(Range* r, uint64_t off, uint64_t len, int gpu);
  // Page-granular write fault: revoke the other copies of these byte intervals
  // of r (resident on gpu) so only written pages are dirty.
  Status invalidate_others(Range* r, const std::vector<std::pair<uint64_t, uint64_t>>& bytes, int gpu);
  // Next-use (Belady) eviction hints: the op-clock time of r's next use, and the
  // current op clock of a device's HBM arena (see ChunkArena::set_next_use).
  void hint_next_use(Range* r, uint64_t when);
  // The same for a range leased whole: its HBM chunks are the lease's pinned
  // chunks (no block walk).
  void hint_next_use(Lease* l, uint64_t when);
  void set_op_clock(int dev, uint64_t now);
  void reset_op_clock(int dev);
  // The spread class flag (0 / kEvictFirst) the runtime gives a hint of r that
  // carries none (config perf_spread_enable; SpreadPolicy).
  uint64_t classify_hint(Range* r, uint64_t when);
  SpreadPolicy::Stats spread_stats(int dev);
  int spread_class(int dev, uint64_t range_id) { return is_local(dev) ? devs_[dev]->spread.range_class(range_id) : -1; }
  // Mark r's contents dead (free: no copy-out, off-GPU copies dropped) or live.
  void set_dead(Range* r, bool dead);
  Lease* lease_by_id(uint64_t id);
  Status cpu_fault(uint64_t addr, bool write);        // SIGSEGV path
  // Several CPU faults (addr, write) serviced as one batch; out[i] per fault.
  void cpu_fault_batch(const std::vector<std::pair<uint64_t, bool>>& faults, std::vector<Status>* out);
  Status cpu_fault_finish(Range* r, uint64_t addr, bool write);
  size_t poll_device_faults(int dev);                  // service device-recorded faults
  // Consume up to `max` published records from GET (no servicing).
  size_t drain_fault_records(int dev, std::vector<DeviceFaultRecord>* out, size_t max);
  Status device_table(Range* r, DeviceResidencyTable** out);
  // Streams whose kernels resolve addresses through device residency tables
  // (k_managed_gather, table-indirect fetches). Before an HBM chunk listed in a
  // table is released, its entry is cleared and an event is recorded on every
  // such stream of the device into the chunk's reuse fence: a kernel that read
  // the old entry finishes before the chunk is overwritten (the TLB-shootdown
  // + membar step of unmapping, uvm_va_block.c unmap + tlb_invalidate).
  void register_table_stream(int dev, void* stream, bool on);
  void refresh_device_tables();  // publish entries whose copies have landed since

  // ---- data movement helpers
  Status write(Range* r, uint64_t off, const void* src, uint64_t bytes, int src_dev);
  Status write_compressed(Range* r, uint64_t off, const void* src, uint64_t bytes, int src_dev);
  Status read(Range* r, uint64_t off, void* dst, uint64_t bytes, int dst_dev);
  Status fill(Range* r, uint64_t off, uint64_t bytes, uint32_t pattern);

  // ---- introspection
  Status residency_info(Range* r, uint64_t off, ResidencyInfo* out);
  // Bytes of [off, off + len) resident at `loc` (page granular; one block lock at a time).
  uint64_t resident_bytes(Range* r, Loc loc, uint64_t off = 0, uint64_t len = ~0ull);
  Status sync_all();
  // Hang diagnostics: every local ring's sequence numbers and worker phase,
  // the outstanding leases (oldest first), the fatal status. Try-locks only, so
  // it can run from a watchdog / signal thread while another thread is stuck
  // inside the runtime (the push description dump of uvm_channel.c:2090-2100).
  std::string debug_dump(size_t max_leases = 24);

  // ---- CXL (fork capability)
  Status cxl_dma(uint64_t handle, uint64_t gpu_ptr, int dev, uint64_t cxl_off, uint64_t size, int dir, bool async,
                 uint64_t* transfer_id);
  Status cxl_dma_wait(uint64_t transfer_id);

  // ---- checkpoint (residency map, §5.4) + suspend/resume (uvm_global.c:272-415)
  Status quiesce();
  Status resume();
  Status checkpoint_save(const std::string& path, bool with_data);
  // in_place: ranges come back under their recorded ids and VAs (CPU window and
  // stable device VA) - pointers taken before the save stay valid (FBSR restores
  // VRAM in place, fbsr.c:37-104; suspend/resume keeps VA spaces, uvm_global.c:272-415).
  Status checkpoint_load(const std::string& path, bool with_data, std::vector<uint64_t>* new_range_ids,
                         bool in_place = false);

  // ---- user channels (uvm_user_channel.c / the channel+TSG attribution of
  // uvm_gpu_replayable_faults.c): a stream registered as a channel gets the
  // device faults of kernels it runs attributed to it (the producers encode
  // dev | channel << 16 in the record's proc field). A fault that cannot be
  // serviced (freed range, address past its end) is fatal for its channel only:
  // the channel is marked errored (the precise-cancel target), the runtime and
  // other channels carry on.
  struct Channel {
    uint16_t id = 0;
    int dev = 0;
    void* stream = nullptr;
    std::string name;
    uint64_t faults = 0, remote_accesses = 0, fatal_faults = 0, cancelled_faults = 0;
    Status error = Status::OK;
  };
  uint16_t register_channel(int dev, void* stream, const std::string& name);
  void unregister_channel(uint16_t id);
  uint32_t fault_client(int dev, void* stream);  // the proc value a producer on `stream` records
  std::vector<Channel> channels();

  // ---- GPU health (ECC / xGMI link errors, rate-limited sysfs reads)
  // OK, or FATAL once an uncorrectable error appeared since init. `force`
  // skips the rate limit (min_interval_ms).
  Status check_health(int dev, bool force = false);

  // ---- peers
  Status enable_peer(int a, int b);

  // ---- fault service threads (ISR top half + bottom half analog,
  // uvm_gpu_isr.c:86-119,218-280,598-700): one host thread per GPU polls the
  // device fault buffer's put index and services batches (faults + access
  // counter notifications) without any caller involvement.
  Status start_fault_service(uint32_t poll_us);
  void stop_fault_service();
  uint64_t fault_service_batches() const { return fs_batches_.load(); }

  // ---- memory pressure: holders of soft pins (UnitStream hold mode) register a
  // handler that lets go of them; a GPU reservation that finds nothing
  // evictable runs the device's handlers once and retries.
  using PressureFn = std::function<bool()>;  // true: something was released
  uint64_t add_pressure_handler(int dev, PressureFn f);
  void remove_pressure_handler(uint64_t id);
  bool relieve_pressure(const Loc& l);

  // ---- packed host copies (packer.cpp): read-mostly blocks keep a lossless
  // ANS1-packed host / CXL copy; the H2D ring moves and decodes the packed bytes.
  Status expand_packed(Block* b, Residency* r);  // back to raw pages (block lock held)
  void pack_enqueue(Block* b);                   // a packing candidate (block lock held)
  // Segmented packed copies (fmt 3, SegDir): decode packed segments `segs`
  // into the raw chunk (`overwrite`: segments whose every page is about to be
  // written - no decode, only the bit), and free the sidecar once nothing
  // rests packed (block lock held).
  Status expand_segments(Block* b, Residency* r, uint32_t segs, uint32_t overwrite = 0);
  // A write of `pages` into host copy r (`full`: the pages written entirely):
  // the written segments are noted (and a fmt 3 copy expands them); the
  // untouched ones become segment-packing candidates (block lock held).
  Status note_host_write(Block* b, Residency* r, const PageMask& pages, const PageMask& full);
  void seg_pack_enqueue(Block* b);
  void free_sidecar(Block* b, Residency* r);     // fmt 3 -> drop the sidecar (after its readers)
  bool pack_wait(uint64_t timeout_ms);           // true once nothing is queued or being packed
  struct PackStats {
    uint64_t queued = 0, busy = 0, threads = 0, packed_blocks = 0, packed_bytes = 0, raw_bytes = 0;
    uint64_t seg_blocks = 0, seg_packed = 0, seg_raw = 0;  // fmt 3 copies, their packed / raw segments
  };
  PackStats pack_stats();
  void stop_packer();

  // ---- perf modules
  void set_prefetch_enabled(bool on);
  // internal helpers used by engine files
  ThrashState& thrash_of(Block* b) { return b->thrash; }

  std::mutex leases_m_;
  std::unordered_map<uint64_t, std::unique_ptr<Lease>> leases_;
  uint64_t next_lease_ = 1;

  // Engine internals (migrate.cpp)
  struct Ctx;  // per-operation migration context
  Status make_resident(Ctx& c, Block* b, const PageMask& pages, Loc dst, bool read_dup, Cause cause);
  Status populate(Ctx& c, Block* b, Loc dst, int64_t chunk_hint, Residency** out);
  Status evict_chunk(ChunkArena* a, uint32_t chunk);
  Status evict_batch(ChunkArena* a, const std::vector<uint32_t>& victims);
  Status evict_one(Ctx& c, ChunkArena* a, uint32_t chunk, bool* detached);
  void seal_evictions(Ctx& c, ChunkArena* a, const std::vector<uint32_t>& victims);
  // GPU residency of a stable-VA range: any HBM chunk per block (the VA is
  // mapped block by block), victims evicted in batches, one translation flush.
  Status place_stable(Range* r, uint64_t off, uint64_t len, int gpu, const std::vector<bool>& read_dup, Lease* L,
                      Tracker* out, Cause cause);
  Status ensure_capacity(ChunkArena* a, uint32_t n, Reservation* r, bool pin = false);
  // owner / pin are applied atomically with the allocation (see ChunkArena::alloc).
  Status alloc_chunks(ChunkArena* a, uint32_t n, int64_t hint, uint32_t* first, Block* owner = nullptr,
                      bool pin = false);
  Loc demotion_target(const Loc& from);
  std::vector<Loc> fallback_targets(const Loc& full);  // when `full` refuses evicted data (node budget spent)
  void cpu_map_block(Block* b);  // refresh CPU view protections
  void stable_map_block(Block* b);
  // stable_m_ held: tear down b's stable-VA mapping after its users finished.
  void stable_unmap_locked(Block* b);
  std::mutex stable_m_;  // stable-VA mappings (Block::stable_chunk / stable_users)
  // Flush GPU translations of devices whose stable VAs were remapped since the
  // last flush (before any consumer of the new mapping can run).
  void flush_translations();
  std::string describe_device_address(uint64_t va);  // for GPU memory-fault reports
  std::atomic<uint32_t> tlb_dirty_{0};  // bit d: device d has remapped stable VAs
  // Translation-flush sequence per device: started (numbered at their start)
  // and the highest completed. A VA unmapped when tlb_started_ was S is
  // covered once tlb_done_ > S (a flush begun after the unmap finished).
  std::atomic<uint64_t> tlb_started_[kMaxGpus] = {};
  std::atomic<uint64_t> tlb_done_[kMaxGpus] = {};
  // The calling thread's remaps that still need a covering flush (per device
  // bit): another thread clearing tlb_dirty_ does not release them (its flush
  // may still be running).
  static uint32_t& thread_tlb_need();
  // Blocks with a stale stable-VA mapping (Block::stale_mapping), guarded by
  // stable_m_: torn down before each translation flush once their users are
  // done, so that flush covers the unmap and the block's next remap needs none.
  std::vector<Block*> stale_maps_;
  void reap_stale_maps_locked();
  Status finish_ctx(Ctx& c, Tracker* out);
  void drop_copy(Ctx& c, Block* b, const Loc& l);  // release a residency (block lock held)
  void touch_residency(Block* b, Residency* r, bool prefetched = false);  // LRU bump (preferred / prefetch aware)
  Tracker published_tracker(Block* b);  // tracker once all queued copies into b published their fences
  Status gpu_extent_resident(Range* r, uint64_t off, uint64_t len, int gpu, const std::vector<bool>& read_dup,
                             Lease* L, Tracker* out, Cause cause);
  Status place_extent(Range* r, uint64_t off, uint64_t len, int gpu, const std::vector<bool>& read_dup, Lease* L,
                      Tracker* out, Cause cause, bool* conflict);
  Status queue_copy(Ctx& c, Block* b, Residency* from, Residency* to, const PageMask& pages);
  void update_device_table(Block* b);
  void shootdown(Block* b, Residency* r);  // block lock held; before r's GPU chunk is released

  std::atomic<bool> quiesced_{false};
  std::atomic<uint64_t> cxl_transfers_{0};

 private:
  Runtime() = default;
  std::unique_ptr<Backend> be_;
  std::vector<std::unique_ptr<Device>> devs_;
  std::vector<std::unique_ptr<HostArena>> host_arenas_;  // index = tier*kMaxNodes + node
  std::mutex host_arenas_m_;
  VaSpace vs_;
  Injection inject_;
  CxlTopology cxl_topo_;
  std::unique_ptr<CxlRegistry> cxl_;
  int host_node_ = 0;
  std::unordered_map<uint64_t, std::unique_ptr<DeviceResidencyTable>> dev_tables_;
  std::mutex dev_tables_m_;
  std::vector<void*> table_streams_[kMaxGpus];  // guarded by dev_tables_m_
  std::vector<std::pair<uint64_t, uint64_t>> table_pending_;  // (range, block) entries awaiting copies
  std::mutex poll_m_;  // fault-buffer consumers drain one at a time
  std::unordered_map<uint64_t, std::pair<Ring*, uint64_t>> cxl_pending_;
  std::mutex cxl_m_;
  std::vector<std::thread> fs_threads_;
  std::atomic<bool> fs_stop_{false};
  std::atomic<uint64_t> fs_batches_{0};
  std::mutex fs_m_;
  OrderedMutex pm_{LockOrder::GLOBAL_PM};
  std::vector<int> perf_subs_;  // perf-module subscriptions on the tools bus
  std::mutex channels_m_;
  std::vector<Channel> channels_;  // slot id - 1 (id 0 = no channel); unregistered slots keep id 0
  std::mutex pressure_m_;
  std::vector<std::tuple<uint64_t, int, PressureFn>> pressure_;
  uint64_t pressure_next_ = 1;
  // packer (packer.cpp)
  struct PackJob {
    uint64_t range = 0, block = 0;
    uint32_t tries = 0;
    bool seg = false;  // segment packing (pack_segments) instead of a whole-block pack
  };
  void pack_worker();
  bool pack_block(uint64_t range_id, uint64_t bi, uint16_t* raw, uint8_t* enc);
  bool pack_segments(uint64_t range_id, uint64_t bi, uint16_t* raw, uint8_t* enc);
  std::mutex pack_m_;
  std::condition_variable pack_cv_, pack_idle_cv_;
  std::deque<PackJob> pack_q_;
  std::vector<std::thread> pack_threads_;
  uint32_t pack_busy_ = 0;
  bool pack_stop_ = false;
};

// Scoped profiler range around a runtime operation (no-op on the fake backend).
// level 1: per operation (acquire, place, eviction batch); level 2 also per
// block / phase (trace_ranges >= 2, for host-time profiles).
struct TraceRange {
  Backend* be;
  explicit TraceRange(Backend* b, const char* name, int level = 1)
      : be(config().trace_ranges >= level ? b : nullptr) {
    if (be) be->range_push(name);
  }
  ~TraceRange() {
    if (be) be->range_pop();
  }
  TraceRange(const TraceRange&) = delete;
  TraceRange& operator=(const TraceRange&) = delete;
};

// Per-operation migration context: rings used, blocks touched, chunks read by
// queued copies (their reuse fences) and chunks to free once those copies land.
struct Runtime::Ctx {
  Cause cause = Cause::User;
  struct Touch { Ring* ring; Block* block; };
  struct ChunkUse { Ring* ring; ChunkArena* arena; uint32_t chunk; bool free_after; };
  std::vector<Touch> touched;
  std::vector<ChunkUse> chunk_uses;
  std::vector<Ring*> rings;
  std::vector<Block*> cpu_refresh;    // CPU views to refresh after submission
  ChunkArena* need_arena = nullptr;   // set on MORE_PROCESSING_REQUIRED
  uint32_t need_n = 0;
  // GPU-side waits already queued. The fences are held: a raw pointer would
  // let a freed fence's address come back as a new, unsignalled fence that
  // this context then believes it already waited for.
  std::vector<std::pair<Ring*, FenceRef>> waited;
  bool defer_flush = false;           // finish_ctx leaves the translation flush to the caller
  // Migration invalidations are applied only once the copies that replace the
  // data were submitted successfully; a failed submission invalidates the
  // destination instead, so a link/copy error never loses the source.
  struct Inval { Block* b; Loc dst; PageMask pages; };
  std::vector<Inval> invals;
  void use_ring(Ring* r) {
    for (Ring* x : rings)
      if (x == r) return;
    rings.push_back(r);
  }
  // True the first time (ring, fence) is seen: one WAIT_FENCE per pair per operation.
  bool first_wait(Ring* r, const FenceRef& f) {
    for (auto& w : waited)
      if (w.first == r && w.second == f) return false;
    waited.emplace_back(r, f);
    return true;
  }
};

// Select where a fault from `proc` on block `b` should be serviced
// (uvm_va_block_select_residency, uvm_va_block.c:11560-11762).
struct ResidencyDecision {
  Loc dst;
  bool read_dup = false;
  bool map_remote = false;  // keep data where it is, access it remotely
};
ResidencyDecision select_residency(Runtime* rt, Block* b, int proc, Access access, const PageMask& pages);

// Bitmap-tree prefetch hint (uvm_perf_prefetch.c:102-250).
PageMask prefetch_hint(const PageMask& resident_on_dst, const PageMask& faulted, uint32_t npages, uint32_t threshold_pct);

// Thrashing hint (uvm_perf_thrashing.c:1615).
enum class ThrashHint { NONE = 0, THROTTLE = 1, PIN = 2 };
ThrashHint thrash_on_migration(Block* b, int dst_slot, uint64_t now);
// Hint for a fault by processor slot `slot` on b at `now` (block lock held):
// PIN while pinned, THROTTLE while `slot` naps; emits ThrottlingEnd once a nap
// has expired.
ThrashHint thrash_hint(Block* b, int slot, uint64_t now);
// The perf modules (thrashing, prefetch) as PerfEventBus subscribers
// (uvm_perf_events.c:56-94 registration); returns the subscription tokens.
std::vector<int> perf_modules_register(PerfEventBus& bus);
bool thrash_pinned(Block* b, uint64_t now);

// CPU faults on managed CPU views (csrc/core/cpu_fault.cpp): an
// async-signal-safe SIGSEGV handler posts the fault to a service thread.
void install_cpu_fault_handler();
void start_cpu_fault_service();
void stop_cpu_fault_service();
void cpu_views_add(uint64_t start, uint64_t bytes);
void cpu_views_remove(uint64_t start);
void cpu_fault_stats(uint64_t* serviced, uint64_t* passed_on);

}  // namespace ogkm
