// Perf event bus + tools event queues + counters.
#include "ogkm/events.hpp"

#include <fcntl.h>
#include <sys/mman.h>
#include <unistd.h>

#include <algorithm>

namespace ogkm {

// ------------------------------------------------------------- perf bus
// Copy-on-write subscriber list: notify() (hot: every migration and fault
// group) reads a snapshot without copying callbacks or holding the mutex.
int PerfEventBus::subscribe(PerfEvent e, Cb cb) {
  std::lock_guard<std::mutex> g(m_);
  int t = next_++;
  auto v = std::make_shared<std::vector<Sub>>(subs_ ? *subs_ : std::vector<Sub>{});
  v->push_back({t, e, std::move(cb)});
  std::atomic_store(&subs_, std::shared_ptr<const std::vector<Sub>>(std::move(v)));
  return t;
}

void PerfEventBus::unsubscribe(int token) {
  std::lock_guard<std::mutex> g(m_);
  if (!subs_) return;
  auto v = std::make_shared<std::vector<Sub>>(*subs_);
  v->erase(std::remove_if(v->begin(), v->end(), [&](const Sub& s) { return s.token == token; }), v->end());
  std::atomic_store(&subs_, std::shared_ptr<const std::vector<Sub>>(std::move(v)));
}

void PerfEventBus::notify(const PerfEventData& d) {
  std::shared_ptr<const std::vector<Sub>> v = std::atomic_load(&subs_);
  if (!v) return;
  for (const Sub& s : *v)
    if (s.e == d.type) s.cb(d);
}

// ------------------------------------------------------------- event queue
EventQueue::EventQueue(uint32_t entries, uint32_t enabled_mask, const std::string& shm_name) {
  uint32_t n = 1;
  while (n < entries) n <<= 1;
  bytes_ = align_up(sizeof(ToolsQueueCtrl), 64) + (size_t)n * sizeof(ToolsEvent);
  int fd = -1;
  if (!shm_name.empty()) {
    fd = shm_open(shm_name.c_str(), O_CREAT | O_RDWR, 0600);
    if (fd >= 0 && ftruncate(fd, bytes_) != 0) {
      close(fd);
      fd = -1;
    }
    if (fd >= 0) shm_name_ = shm_name;
  }
  base_ = mmap(nullptr, bytes_, PROT_READ | PROT_WRITE, fd >= 0 ? MAP_SHARED : (MAP_PRIVATE | MAP_ANONYMOUS), fd, 0);
  if (fd >= 0) close(fd);
  if (base_ == MAP_FAILED) {
    base_ = nullptr;
    RT_ERR("tools queue mmap failed");
    return;
  }
  memset(base_, 0, bytes_);
  ctrl_ = new (base_) ToolsQueueCtrl();
  ctrl_->entries = n;
  ctrl_->enabled_mask = enabled_mask;
  ring_ = reinterpret_cast<ToolsEvent*>((char*)base_ + align_up(sizeof(ToolsQueueCtrl), 64));
}

EventQueue::~EventQueue() {
  if (base_) munmap(base_, bytes_);
  if (!shm_name_.empty()) shm_unlink(shm_name_.c_str());
}

bool EventQueue::push(const ToolsEvent& e) {
  if (!ctrl_) return false;
  std::lock_guard<std::mutex> g(produce_m_);
  uint32_t put = ctrl_->put_ahead.load(std::memory_order_relaxed);
  uint32_t get = ctrl_->get_behind.load(std::memory_order_acquire);
  if (put - get >= ctrl_->entries) {
    ctrl_->dropped[e.type < (int)ToolsEventType::NumTypes ? e.type : 0].fetch_add(1, std::memory_order_relaxed);
    return false;
  }
  ctrl_->put_ahead.store(put + 1, std::memory_order_relaxed);
  ring_[put & (ctrl_->entries - 1)] = e;
  ctrl_->put_behind.store(put + 1, std::memory_order_release);
  return true;
}

size_t EventQueue::pop(ToolsEvent* out, size_t max) {
  if (!ctrl_) return 0;
  uint32_t get = ctrl_->get_ahead.load(std::memory_order_relaxed);
  uint32_t put = ctrl_->put_behind.load(std::memory_order_acquire);
  size_t n = 0;
  while (get != put && n < max) {
    out[n++] = ring_[get & (ctrl_->entries - 1)];
    ++get;
  }
  ctrl_->get_ahead.store(get, std::memory_order_relaxed);
  ctrl_->get_behind.store(get, std::memory_order_release);
  return n;
}

// ------------------------------------------------------------- tools
const char* counter_name(Counter c) {
  static const char* n[] = {"bytes_xfer_htd",
                            "bytes_xfer_dth",
                            "bytes_xfer_dtd",
                            "bytes_xfer_htc",
                            "bytes_xfer_cth",
                            "bytes_xfer_ctd",
                            "bytes_xfer_dtc",
                            "cpu_page_faults",
                            "gpu_page_faults",
                            "prefetch_bytes_htd",
                            "prefetch_bytes_dth",
                            "evictions",
                            "evicted_bytes",
                            "thrashing_detected",
                            "throttle_events",
                            "pin_events",
                            "map_remote",
                            "access_counter_notifications",
                            "access_counter_migrations",
                            "read_duplications",
                            "revocations",
                            "ring_submissions",
                            "ring_completions",
                            "copy_kernel_launches",
                            "fault_batches",
                            "faults_coalesced",
                            "cxl_dma_requests",
                            "cxl_dma_bytes",
                            "alloc_retries",
                            "injected_errors",
                            "decoded_bytes",
                            "encoded_bytes",
                            "table_shootdowns",
                            "fault_replays",
                            "fault_records_consumed",
                            "page_list_copies",
                            "vmm_remaps",
                            "vmm_errors",
                            "tlb_flushes",
                            "faults_cancelled",
                            "tlb_flushes_elided",
                            "write_invalidations",
                            "remote_fallbacks",
                            "vmm_map_ns",
                            "vmm_unmap_ns",
                            "tlb_flush_ns",
                            "place_stable_ns",
                            "stable_wait_ns",
                            "ring_fence_wait_ns",
                            "ring_copy_ns",
                            "ring_idle_ns",
                            "ring_copy_calls",
                            "demotion_fallbacks",
                            "ledger_refusals",
                            "lease_fast_paths",
                            "packed_blocks",
                            "packed_bytes_saved",
                            "pack_skips",
                            "pack_expansions",
                            "packed_decodes",
                            "pressure_reliefs",
                            "decode_reuse_waits",
                            "ring_merged_batches",
                            "victim_search_ns",
                            "victim_risen_seen",
                            "seg_packed",
                            "seg_expansions",
                            "seg_decodes"};
  static_assert(sizeof(n) / sizeof(n[0]) == (size_t)Counter::NumCounters, "counter names");
  return n[(int)c];
}

Tools& Tools::get() {
  static Tools* t = new Tools();
  return *t;
}

void Tools::record(const ToolsEvent& e) {
  if (!any_queue()) return;
  std::lock_guard<OrderedMutex> g(m_);
  for (auto& q : queues_)
    if (q && (q->enabled_mask() & (1u << e.type))) q->push(e);
}

void Tools::reset_counters() {
  for (auto& c : counters_) c.store(0);
}

int Tools::create_queue(uint32_t entries, uint32_t enabled_mask, const std::string& shm_name) {
  std::lock_guard<OrderedMutex> g(m_);
  queues_.push_back(std::make_unique<EventQueue>(entries, enabled_mask, shm_name));
  nqueues_.fetch_add(1);
  return (int)queues_.size() - 1;
}

EventQueue* Tools::queue(int id) {
  std::lock_guard<OrderedMutex> g(m_);
  return id >= 0 && id < (int)queues_.size() ? queues_[id].get() : nullptr;
}

void Tools::destroy_queue(int id) {
  std::lock_guard<OrderedMutex> g(m_);
  if (id >= 0 && id < (int)queues_.size() && queues_[id]) {
    queues_[id].reset();
    nqueues_.fetch_sub(1);
  }
}

void tools_event(ToolsEventType t, Cause c, Loc src, Loc dst, int proc, uint64_t addr, uint64_t bytes,
                 uint64_t range_id, uint64_t t0, uint64_t t1, uint64_t aux) {
  Tools& tl = Tools::get();
  if (!tl.any_queue()) return;
  static std::atomic<uint64_t> seq{0};
  ToolsEvent e{};
  e.type = (uint8_t)t;
  e.cause = (uint8_t)c;
  e.src_slot = (uint8_t)src.slot();
  e.dst_slot = (uint8_t)dst.slot();
  e.processor = (uint32_t)proc;
  e.address = addr;
  e.bytes = bytes;
  e.ts_begin_ns = t0 ? t0 : now_ns();
  e.ts_end_ns = t1 ? t1 : e.ts_begin_ns;
  e.range_id = range_id;
  e.seq = seq.fetch_add(1);
  e.aux = aux;
  tl.record(e);
}

}  // namespace ogkm
