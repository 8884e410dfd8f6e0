// FakeBackend: CPU-only devices for the test-suite and the CPU-only config.
// HBM is host memory, streams are in-order worker threads, copies are memcpy.
// This generalises the reference's fake CE HAL (uvm_page_tree_test.c:65-100),
// which executes CE memcopy/memset methods on CPU addresses.
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <atomic>
#include <condition_variable>
#include <deque>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <map>
#include <mutex>
#include <chrono>
#include <thread>

#include "ogkm/backend.hpp"
#include "ogkm/config.hpp"
#include "ogkm/codec.hpp"
#include "ogkm/runtime.hpp"

namespace ogkm {

namespace {

// Events may be destroyed while a stream still holds a queued record/wait on
// them (like hipEventDestroy on a pending event): they are reference counted
// by the owner plus every queued operation.
struct FakeEvent {
  std::atomic<bool> done{true};
  std::atomic<int> refs{1};
  void ref() { refs.fetch_add(1, std::memory_order_relaxed); }
  void unref() {
    if (refs.fetch_sub(1, std::memory_order_acq_rel) == 1) delete this;
  }
};

class FakeStream {
 public:
  FakeStream() : th_([this] { run(); }) {}
  ~FakeStream() {
    {
      std::lock_guard<std::mutex> g(m_);
      stop_ = true;
    }
    cv_.notify_all();
    th_.join();
  }
  void enqueue(std::function<void()> f) {
    {
      std::lock_guard<std::mutex> g(m_);
      q_.push_back(std::move(f));
      ++pending_;
    }
    cv_.notify_all();
  }
  void sync() {
    std::unique_lock<std::mutex> g(m_);
    idle_cv_.wait(g, [&] { return pending_ == 0; });
  }

 private:
  void run() {
    for (;;) {
      std::function<void()> f;
      {
        std::unique_lock<std::mutex> g(m_);
        cv_.wait(g, [&] { return stop_ || !q_.empty(); });
        if (q_.empty()) return;
        f = std::move(q_.front());
        q_.pop_front();
      }
      f();
      {
        std::lock_guard<std::mutex> g(m_);
        --pending_;
      }
      idle_cv_.notify_all();
    }
  }
  std::mutex m_;
  std::condition_variable cv_, idle_cv_;
  std::deque<std::function<void()>> q_;
  size_t pending_ = 0;
  bool stop_ = false;
  std::thread th_;
};

class FakeBackend : public Backend {
 public:
  FakeBackend(int ndev, size_t hbm) : ndev_(ndev), hbm_(hbm), used_(ndev, 0) {}
  const char* name() const override { return "fake"; }
  bool is_fake() const override { return true; }
  int device_count() override { return ndev_; }
  // Like a two-socket node: GPUs 0..n/2-1 on node 0, the rest on node 1 (with
  // fake_numa_nodes = 2), so per-rank host-tier placement is testable on a CPU.
  int device_numa_node(int d) override {
    int64_t nodes = config().fake_numa_nodes;
    if (nodes <= 1 || ndev_ <= 0 || d < 0) return 0;
    return (int)((int64_t)d * nodes / ndev_);
  }
  Status device_mem_info(int dev, size_t* f, size_t* t) override {
    if (dev < 0 || dev >= ndev_) return Status::INVALID_ARGUMENT;
    *t = hbm_;
    *f = hbm_ - used_[dev];
    return Status::OK;
  }
  Status set_device(int) override { return Status::OK; }

  // Fake HBM is a shared memfd mapping, so an allocation can be exported as a
  // file descriptor (the dma-buf stand-in) and opened by another process.
  Status hbm_alloc(int dev, size_t bytes, void** p) override {
    if (dev < 0 || dev >= ndev_) return Status::INVALID_ARGUMENT;
    std::lock_guard<std::mutex> g(m_);
    if (used_[dev] + bytes > hbm_) return Status::NO_MEMORY;
    int fd = memfd_create("ogkm-fake-hbm", MFD_CLOEXEC);
    if (fd < 0) return Status::NO_MEMORY;
    if (ftruncate(fd, bytes) != 0) {
      close(fd);
      return Status::NO_MEMORY;
    }
    void* m = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_SHARED | MAP_NORESERVE, fd, 0);
    if (m == MAP_FAILED) {
      close(fd);
      return Status::NO_MEMORY;
    }
    used_[dev] += bytes;
    allocs_[(uint64_t)m] = FakeAlloc{fd, bytes, dev};
    *p = m;
    return Status::OK;
  }
  void hbm_free(int dev, void* p, size_t bytes) override {
    std::lock_guard<std::mutex> g(m_);
    if (p) {
      munmap(p, bytes);
      auto it = allocs_.find((uint64_t)p);
      if (it != allocs_.end()) {
        close(it->second.fd);
        allocs_.erase(it);
      }
    }
    if (dev >= 0 && dev < ndev_) used_[dev] -= bytes;
  }

  // Fake RAS counters: tests raise them through Injection (ecc_ue / ecc_ce / link_ue).
  Status device_health(int dev, Health* out) override {
    if (dev < 0 || dev >= ndev_) return Status::INVALID_ARGUMENT;
    Runtime* rt = Runtime::get();
    *out = Health{};
    out->source = "fake";
    out->ue = rt ? rt->inject().ecc_ue.load() : 0;
    out->ce = rt ? rt->inject().ecc_ce.load() : 0;
    out->link_ue = rt ? rt->inject().link_ue.load() : 0;
    out->link_ce = 0;
    return Status::OK;
  }
  bool vmm_supported(int) override { return true; }
  Status vmm_create(int dev, size_t bytes, uint64_t* h) override {
    if (used_[dev] + bytes > hbm_) return Status::NO_MEMORY;
    int fd = memfd_create("ogkm-fake-vmm", MFD_CLOEXEC);
    if (fd < 0 || ftruncate(fd, bytes) != 0) {
      if (fd >= 0) close(fd);
      return Status::NO_MEMORY;
    }
    used_[dev] += bytes;
    std::lock_guard<std::mutex> g(m_);
    handles_[(uint64_t)fd] = {dev, bytes};
    *h = (uint64_t)fd;
    return Status::OK;
  }
  void vmm_release(uint64_t h) override {
    std::lock_guard<std::mutex> g(m_);
    auto it = handles_.find(h);
    if (it == handles_.end()) return;
    used_[it->second.first] -= it->second.second;
    close((int)h);
    handles_.erase(it);
  }
  Status va_reserve(size_t bytes, void** va, void* want) override {
    void* m = mmap(want, bytes, PROT_NONE, MAP_PRIVATE | MAP_ANONYMOUS | MAP_NORESERVE | (want ? MAP_FIXED_NOREPLACE : 0),
                   -1, 0);
    if (m == MAP_FAILED) return want ? Status::BUSY : Status::NO_MEMORY;
    if (want && m != want) {
      munmap(m, bytes);
      return Status::BUSY;
    }
    *va = m;
    return Status::OK;
  }
  void va_free(void* va, size_t bytes) override {
    {
      std::lock_guard<std::mutex> g(tlb_m_);
      for (auto it = live_.lower_bound((uint64_t)va); it != live_.end() && it->first < (uint64_t)va + bytes;)
        it = live_.erase(it);
      for (auto it = pending_.lower_bound((uint64_t)va); it != pending_.end() && it->first < (uint64_t)va + bytes;)
        it = pending_.erase(it);
    }
    munmap(va, bytes);
  }
  // Translation model (Injection::tlb_mode): with mode >= 1 a VA whose old
  // mapping may be cached keeps serving it after an unmap / remap until
  // tlb_flush applies the new state (mode 2: the flush does nothing) - the
  // behaviour of gfx950 VMM remaps (tools/probe_vmm_tlb.hip), on the CPU.
  int tlb_mode() {
    Runtime* rt = Runtime::get();
    return rt ? rt->inject().tlb_mode.load() : 0;
  }
  static Status apply_map(void* va, size_t bytes, uint64_t h) {
    void* m = h ? mmap(va, bytes, PROT_READ | PROT_WRITE, MAP_SHARED | MAP_FIXED, (int)h, 0)
                : mmap(va, bytes, PROT_NONE, MAP_PRIVATE | MAP_ANONYMOUS | MAP_FIXED | MAP_NORESERVE, -1, 0);
    return m == MAP_FAILED ? Status::IO_ERROR : Status::OK;
  }
  Status set_translation(void* va, size_t bytes, uint64_t h) {
    {
      std::lock_guard<std::mutex> g(race_m_);
      if (h)
        vmaps_[(uint64_t)va] = {bytes, h};
      else
        vmaps_.erase((uint64_t)va);
    }
    std::lock_guard<std::mutex> g(tlb_m_);
    auto lv = live_.find((uint64_t)va);
    const bool cached = lv != live_.end() && lv->second.second != 0;  // a translation may be cached
    if (tlb_mode() >= 1 && cached) {
      pending_[(uint64_t)va] = {bytes, h};
      return Status::OK;
    }
    pending_.erase((uint64_t)va);
    live_[(uint64_t)va] = {bytes, h};
    return apply_map(va, bytes, h);
  }
  Status vmm_map(void* va, size_t bytes, uint64_t h, int) override { return set_translation(va, bytes, h); }
  Status vmm_unmap(void* va, size_t bytes) override { return set_translation(va, bytes, 0); }
  Status tlb_flush(int) override {
    if (tlb_mode() >= 2) return Status::OK;  // a flush that does not work
    std::lock_guard<std::mutex> g(tlb_m_);
    Status st = Status::OK;
    for (auto& kv : pending_) {
      live_[kv.first] = kv.second;
      if (apply_map((void*)kv.first, kv.second.first, kv.second.second) != Status::OK) st = Status::IO_ERROR;
    }
    pending_.clear();
    return st;
  }
  // Race detector for tests (fake_race_check): the VMM handle behind an
  // address, and the handles an in-flight engine copy reads / writes.
  uint64_t handle_of(uint64_t a) {
    auto it = vmaps_.upper_bound(a);
    if (it == vmaps_.begin()) return 0;
    --it;
    return a < it->first + it->second.first ? it->second.second : 0;
  }
  void race_begin(const CopyDesc* d, size_t n, int64_t delta) {
    if (!config().fake_race_check) return;
    std::lock_guard<std::mutex> g(race_m_);
    for (size_t i = 0; i < n; ++i) {
      for (uint64_t o = 0; o < d[i].bytes; o += kBlockSize) {
        uint64_t hw = handle_of(d[i].dst + o), hr = handle_of(d[i].src + o);
        if (hw) busy_w_[hw] += delta;
        if (hr) busy_r_[hr] += delta;
        if ((hw && busy_k_[hw] > 0) || (hr && busy_kw_[hr] > 0)) {
          races_++;
          fprintf(stderr, "[fake RACE] engine copy %#llx <- %#llx (%s) while a kernel uses handle %llu\n",
                  (unsigned long long)d[i].dst, (unsigned long long)d[i].src, delta > 0 ? "start" : "end",
                  (unsigned long long)(hw && busy_k_[hw] > 0 ? hw : hr));
        }
      }
    }
  }
  void race_kernel(uint64_t ptr, uint64_t bytes, bool write, int64_t delta) {
    if (!config().fake_race_check) return;
    std::lock_guard<std::mutex> g(race_m_);
    for (uint64_t o = 0; o < bytes; o += kBlockSize)
      if (uint64_t h = handle_of(ptr + o)) {
        busy_k_[h] += delta;
        if (write) busy_kw_[h] += delta;
      }
  }
  void race_touch(uint64_t ptr, bool write) {
    if (!config().fake_race_check) return;
    std::lock_guard<std::mutex> g(race_m_);
    uint64_t h = handle_of(ptr);
    if (!h) return;
    if (busy_w_[h] > 0 || (write && busy_r_[h] > 0)) {
      races_++;
      fprintf(stderr, "[fake RACE] kernel %s VA %#llx (handle %llu) while an engine copy %s it\n",
              write ? "writes" : "reads", (unsigned long long)ptr, (unsigned long long)h,
              busy_w_[h] > 0 ? "writes" : "reads");
    }
  }
  std::mutex race_m_;
  std::mutex tlb_m_;
  std::map<uint64_t, std::pair<size_t, uint64_t>> live_;     // va -> (bytes, handle) the "GPU" sees (0 = none)
  std::map<uint64_t, std::pair<size_t, uint64_t>> pending_;  // va -> mapping applied at the next tlb_flush
  std::map<uint64_t, std::pair<uint64_t, uint64_t>> vmaps_;  // va -> (bytes, handle)
  std::map<uint64_t, int64_t> busy_w_, busy_r_, busy_k_, busy_kw_;
  std::atomic<uint64_t> races_{0};

  Status host_register(void*, size_t) override { return Status::OK; }
  void host_unregister(void*) override {}
  Status host_alloc_coherent(size_t bytes, void** p) override {
    void* m = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    if (m == MAP_FAILED) return Status::NO_MEMORY;
    std::lock_guard<std::mutex> g(m_);
    coherent_[m] = bytes;
    *p = m;
    return Status::OK;
  }
  void host_free_coherent(void* p) override {
    std::lock_guard<std::mutex> g(m_);
    auto it = coherent_.find(p);
    if (it != coherent_.end()) {
      munmap(p, it->second);
      coherent_.erase(it);
    }
  }

  void* stream_create(int, int) override { return new FakeStream(); }
  void stream_destroy(void* s) override { delete (FakeStream*)s; }
  Status stream_sync(void* s) override {
    if (s) ((FakeStream*)s)->sync();
    return Status::OK;
  }
  void* event_create(int) override { return new FakeEvent(); }
  void event_destroy(void* e) override { ((FakeEvent*)e)->unref(); }
  Status event_record(void* e, void* s) override {
    auto* ev = (FakeEvent*)e;
    if (!s) {
      ev->done.store(true);
      return Status::OK;
    }
    ev->done.store(false);
    ev->ref();
    ((FakeStream*)s)->enqueue([ev] {
      ev->done.store(true, std::memory_order_release);
      ev->unref();
    });
    return Status::OK;
  }
  bool event_query(void* e) override { return ((FakeEvent*)e)->done.load(std::memory_order_acquire); }
  Status event_sync(void* e) override {
    auto* ev = (FakeEvent*)e;
    while (!ev->done.load(std::memory_order_acquire)) std::this_thread::yield();
    return Status::OK;
  }
  Status stream_wait_event(void* s, void* e) override {
    auto* ev = (FakeEvent*)e;
    if (!s) return event_sync(e);
    ev->ref();
    ((FakeStream*)s)->enqueue([ev] {
      while (!ev->done.load(std::memory_order_acquire)) std::this_thread::yield();
      ev->unref();
    });
    return Status::OK;
  }

  void run(void* s, std::function<void()> f) {
    if (s) ((FakeStream*)s)->enqueue(std::move(f));
    else f();
  }
  Status copy_batch(int dev, const CopyDesc* d, size_t n, void* s, int engine) override {
    if (engine == 4)  // k_peer_push stand-in: counted per source device
      for (size_t i = 0; i < n; ++i) __atomic_fetch_add(&push_bytes_[dev & 31], d[i].bytes, __ATOMIC_RELAXED);
    std::vector<CopyDesc> v(d, d + n);
    run(s, [v] {
      for (auto& c : v) memmove((void*)c.dst, (const void*)c.src, c.bytes);
    });
    return Status::OK;
  }
  // The fake "SDMA engine": the ring worker's own thread does the copy.
  bool dma_supported(int) override { return true; }
  // Synthetic SDMA topology: engine 0 host->GPU, engine 1 GPU->host, and two
  // xGMI engines per peer pair that differ between destinations (engines 2..7).
  uint32_t copy_engine_mask(int dst_dev, int src_dev) override {
    if (src_dev < 0) return dst_dev >= 0 && dst_dev < ndev_ ? 0x1u : 0;
    if (src_dev >= ndev_) return 0;
    if (dst_dev < 0) return 0x2u;
    if (dst_dev == src_dev || dst_dev >= ndev_) return 0;
    return (1u << (2 + dst_dev % 6)) | (1u << (2 + (dst_dev + 3) % 6));
  }
  void engine_bytes(int dev, uint64_t out[32]) override {
    for (int i = 0; i < 32; ++i)
      out[i] = i < 31 ? __atomic_load_n(&eng_bytes_[dev & 31][i], __ATOMIC_RELAXED)
                      : __atomic_load_n(&push_bytes_[dev & 31], __ATOMIC_RELAXED);  // slot 31: k_peer_push bytes
  }
  Status dma_copy(int dev, const CopyDesc* d, size_t n, int channel) override {
    for (size_t i = 0; i < n; ++i) {
      const uint32_t e = d[i].engine ? d[i].engine : (1u << (channel % 2));
      __atomic_fetch_add(&eng_bytes_[dev & 31][__builtin_ctz(e) % 31], d[i].bytes, __ATOMIC_RELAXED);
    }
    race_begin(d, n, 1);
    if (int64_t us = config().fake_dma_delay_us) std::this_thread::sleep_for(std::chrono::microseconds(us));
    for (size_t i = 0; i < n; ++i) memmove((void*)d[i].dst, (const void*)d[i].src, d[i].bytes);
    race_begin(d, n, -1);
    return Status::OK;
  }
  Status decode_bf12(int, const DecodeDesc* d, size_t n, void* s, uint32_t) override {
    std::vector<DecodeDesc> v(d, d + n);
    run(s, [v] {
      for (auto& x : v) bf12_decode((const uint8_t*)x.src, (uint16_t*)x.dst, x.n_values);
    });
    return Status::OK;
  }
  Status decode_ans_blocks(int, const DecodeDesc* d, size_t n, void* s) override {
    std::vector<DecodeDesc> v(d, d + n);
    const int64_t delay = config().fake_kernel_delay_us;  // a slow decode: exposes ordering races in tests
    run(s, [v, delay] {
      if (delay) std::this_thread::sleep_for(std::chrono::microseconds(delay));
      for (auto& x : v)
        if (!ans_decode((const uint8_t*)x.src, (uint16_t*)x.dst, x.n_values)) memset((void*)x.dst, 0, 2ull * x.n_values);
    });
    return Status::OK;
  }
  Status unpack_bf12_stream(int, uint64_t src, uint64_t dst, uint32_t, uint32_t, uint64_t n, void* s,
                            uint32_t, uint64_t dst_stride, uint32_t row_shift) override {
    run(s, [src, dst, n, dst_stride, row_shift] {
      bf12_unpack((const uint8_t*)src, (uint16_t*)dst, n, dst_stride, row_shift);
    });
    return Status::OK;
  }
  Status dgemm(int, const DGemmArgs& a, int mode, void* s) override {
    run(s, [a, mode] {
      dgemm_cpu(a, mode != DGEMM_W_RAW);
      if (a.fix_cnt || a.direct) dgemm_reduce_cpu(a.fix);  // the in-kernel epilogue's result
    });
    return Status::OK;
  }
  Status dgemm_reduce(int, const DGemmReduceArgs& a, void* s) override {
    run(s, [a] { dgemm_reduce_cpu(a); });
    return Status::OK;
  }
  Status rmsnorm(int, const ResidNormArgs& a, void* s) override {
    run(s, [a] { rmsnorm_cpu(a); });
    return Status::OK;
  }
  Status rope_kv(int, const RopeKvArgs& a, void* s) override {
    run(s, [a] { rope_kv_cpu(a); });
    return Status::OK;
  }
  Status attn_decode(int, const AttnArgs& a, void* s) override {
    run(s, [a] { attn_decode_cpu(a); });
    return Status::OK;
  }
  Status gather_pages(int, const PageListDesc& d, void* s) override {
    std::vector<uint32_t> idx(d.idx, d.idx + d.npages);
    PageListDesc dd = d;
    run(s, [dd, idx] {
      for (uint32_t i = 0; i < dd.npages; ++i)
        memcpy((char*)dd.contig + (uint64_t)i * dd.page_bytes, (char*)dd.base + (uint64_t)idx[i] * dd.page_bytes,
               dd.page_bytes);
    });
    return Status::OK;
  }
  Status page_copy(int, uint64_t dst_base, uint64_t src_base, const uint32_t* idx, uint32_t npages,
                   void* s) override {
    std::vector<uint32_t> v(idx, idx + npages);
    run(s, [dst_base, src_base, v] {
      for (uint32_t p : v) memcpy((char*)dst_base + ((uint64_t)p << 12), (char*)src_base + ((uint64_t)p << 12), 4096);
    });
    return Status::OK;
  }
  Status scatter_pages(int, const PageListDesc& d, void* s) override {
    std::vector<uint32_t> idx(d.idx, d.idx + d.npages);
    PageListDesc dd = d;
    run(s, [dd, idx] {
      for (uint32_t i = 0; i < dd.npages; ++i)
        memcpy((char*)dd.base + (uint64_t)idx[i] * dd.page_bytes, (char*)dd.contig + (uint64_t)i * dd.page_bytes,
               dd.page_bytes);
    });
    return Status::OK;
  }
  Status memset32(int, uint64_t dst, uint32_t pat, size_t bytes, void* s) override {
    run(s, [dst, pat, bytes] {
      uint32_t* p = (uint32_t*)dst;
      for (size_t i = 0; i < bytes / 4; ++i) p[i] = pat;
    });
    return Status::OK;
  }
  Status signal(int, uint64_t* addr, uint64_t v, void* s) override {
    run(s, [addr, v] { __atomic_store_n(addr, v, __ATOMIC_RELEASE); });
    return Status::OK;
  }
  Status debug_touch(void* s, uint64_t ptr, uint64_t bytes, uint32_t delay_us, bool write) override {
    run(s, [this, ptr, bytes, delay_us, write] {
      if (delay_us) std::this_thread::sleep_for(std::chrono::microseconds(delay_us));
      for (uint64_t o = 0; o < bytes; o += kBlockSize) race_touch(ptr + o, write);
      race_kernel(ptr, bytes, write, 1);
      uint32_t sum = 0;
      for (uint64_t o = 0; o < bytes; o += 4096) {
        volatile uint32_t* w = (volatile uint32_t*)(ptr + o);
        if (write) *w = *w + 1;
        else sum += *w;
      }
      (void)sum;
      race_kernel(ptr, bytes, write, -1);
    });
    return Status::OK;
  }
  Status wait_value(void* s, uint64_t* addr, uint64_t v) override {
    auto f = [addr, v] {
      while (__atomic_load_n(addr, __ATOMIC_ACQUIRE) < v) std::this_thread::yield();
    };
    run(s, f);
    return Status::OK;
  }

  LinkType link_type(int a, int b) override { return a == b ? LinkType::SELF : LinkType::XGMI; }
  bool can_access_peer(int a, int b) override { return a != b && a < ndev_ && b < ndev_; }
  Status enable_peer(int a, int b) override { return can_access_peer(a, b) ? Status::OK : Status::NOT_SUPPORTED; }

  Status export_dmabuf(void* p, size_t bytes, int* fd, uint64_t* off) override {
    std::lock_guard<std::mutex> g(m_);
    const FakeAlloc* a = containing((uint64_t)p, bytes, off);
    if (!a) return Status::INVALID_ARGUMENT;
    *fd = fcntl(a->fd, F_DUPFD_CLOEXEC, 0);
    return *fd < 0 ? Status::IO_ERROR : Status::OK;
  }
  Status import_dmabuf(int, int fd, void** ptr, size_t* bytes) override {
    struct stat stt;
    if (fstat(fd, &stt) != 0 || stt.st_size <= 0) return Status::INVALID_ARGUMENT;
    void* p = mmap(nullptr, (size_t)stt.st_size, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    if (p == MAP_FAILED) return Status::IO_ERROR;
    std::lock_guard<std::mutex> g(m_);
    imports_[p] = (size_t)stt.st_size;
    *ptr = p;
    *bytes = (size_t)stt.st_size;
    return Status::OK;
  }
  Status unimport_dmabuf(void* ptr) override {
    std::lock_guard<std::mutex> g(m_);
    auto it = imports_.find(ptr);
    if (it == imports_.end()) return Status::INVALID_ARGUMENT;
    munmap(ptr, it->second);
    imports_.erase(it);
    return Status::OK;
  }
  // Handle = "fake:<pid>:<fd>:<offset>:<alloc bytes>"; another process opens the
  // allocation's memfd through /proc/<pid>/fd (hipIpcGetMemHandle analog).
  Status ipc_handle(void* p, std::string* h) override {
    std::lock_guard<std::mutex> g(m_);
    uint64_t off = 0;
    const FakeAlloc* a = containing((uint64_t)p, 1, &off);
    if (!a) return Status::INVALID_ARGUMENT;
    char b[96];
    snprintf(b, sizeof b, "fake:%d:%d:%llu:%llu", (int)getpid(), a->fd, (unsigned long long)off,
             (unsigned long long)a->bytes);
    *h = b;
    return Status::OK;
  }
  Status ipc_open(const std::string& h, void** p) override {
    int pid = 0, fd = -1;
    unsigned long long off = 0, bytes = 0;
    if (sscanf(h.c_str(), "fake:%d:%d:%llu:%llu", &pid, &fd, &off, &bytes) != 4 || off >= bytes)
      return Status::INVALID_ARGUMENT;
    char path[64];
    snprintf(path, sizeof path, "/proc/%d/fd/%d", pid, fd);
    int lfd = open(path, O_RDWR | O_CLOEXEC);
    if (lfd < 0) return Status::NOT_FOUND;
    void* m = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_SHARED, lfd, 0);
    close(lfd);
    if (m == MAP_FAILED) return Status::NO_MEMORY;
    std::lock_guard<std::mutex> g(m_);
    opened_[(uint64_t)m + off] = {(uint64_t)m, (size_t)bytes};
    *p = (char*)m + off;
    return Status::OK;
  }
  void ipc_close(void* p) override {
    std::lock_guard<std::mutex> g(m_);
    auto it = opened_.find((uint64_t)p);
    if (it == opened_.end()) return;
    munmap((void*)it->second.first, it->second.second);
    opened_.erase(it);
  }

 private:
  struct FakeAlloc {
    int fd;
    size_t bytes;
    int dev;
  };
  const FakeAlloc* containing(uint64_t p, size_t bytes, uint64_t* off) const {
    auto it = allocs_.upper_bound(p);
    if (it == allocs_.begin()) return nullptr;
    --it;
    if (p + bytes > it->first + it->second.bytes) return nullptr;
    *off = p - it->first;
    return &it->second;
  }
  int ndev_;
  size_t hbm_;
  std::vector<size_t> used_;
  std::mutex m_;
  std::map<uint64_t, std::pair<int, size_t>> handles_;
  std::map<void*, size_t> coherent_;
  std::map<uint64_t, FakeAlloc> allocs_;                        // base -> memfd
  std::map<uint64_t, std::pair<uint64_t, size_t>> opened_;      // ipc ptr -> (map base, bytes)
  std::map<void*, size_t> imports_;                             // imported dma-buf mappings
  uint64_t eng_bytes_[32][31] = {};                             // per device, per synthetic SDMA engine
  uint64_t push_bytes_[32] = {};                                // k_peer_push stand-in bytes per source device
};

}  // namespace

std::unique_ptr<Backend> make_fake_backend(int ndev, size_t hbm) {
  return std::unique_ptr<Backend>(new FakeBackend(ndev, hbm));
}

std::unique_ptr<Backend> make_backend(const std::string& want) {
  if (want != "fake") {
    auto b = make_hip_backend();
    if (b) return b;
    if (want == "hip") return nullptr;
  }
  const char* nd = getenv("RT_FAKE_DEVICES");
  const char* hb = getenv("RT_FAKE_HBM_MB");
  return make_fake_backend(nd ? atoi(nd) : 2, (size_t)(hb ? atoll(hb) : 256) << 20);
}

}  // namespace ogkm
