// Runtime: init/shutdown, tiers, ranges, policy, data helpers, introspection,
// CPU/stable-VA mapping maintenance, CXL DMA, quiesce/resume and the
// residency-map checkpoint format.
#include "ogkm/runtime.hpp"
#include "ogkm/unit_stream.hpp"
#include "ogkm/ledger.hpp"
#include "ogkm/codec.hpp"
#include "ogkm/torch_alloc.hpp"

#include <sys/mman.h>
#include <unistd.h>

#include <algorithm>
#include <cstring>
#include <fstream>
#include <mutex>
#include <shared_mutex>

namespace ogkm {

static std::atomic<Runtime*> g_rt{nullptr};
static std::mutex g_rt_m;

Runtime* Runtime::get() { return g_rt.load(std::memory_order_acquire); }

Runtime* Runtime::init(const std::string& backend, int fake_devices, uint64_t fake_hbm_bytes) {
  std::lock_guard<std::mutex> g(g_rt_m);
  if (Runtime* r = g_rt.load()) return r;
  auto* rt = new Runtime();
  if (backend == "fake") rt->be_ = make_fake_backend(fake_devices > 0 ? fake_devices : 2, fake_hbm_bytes);
  else rt->be_ = make_backend(backend);
  if (!rt->be_) {
    delete rt;
    return nullptr;
  }
  Config& cfg = config();
  int nd = rt->be_->device_count();
  const uint64_t mask = (uint64_t)cfg.local_devices;
  auto local = [&](int d) { return mask == 0 || ((mask >> d) & 1); };
  // Host tier = the NUMA node of this process's (first) GPU: a rank on socket 1
  // rests its streamed data in socket-1 DRAM.
  int first_local = -1;
  for (int d = 0; d < nd && first_local < 0; ++d)
    if (local(d)) first_local = d;
  rt->host_node_ = cfg.host_node >= 0 ? (int)cfg.host_node
                                       : (first_local >= 0 ? rt->be_->device_numa_node(first_local) : 0);
  rt->cxl_topo_.discover((int)cfg.cxl_emulate_node, "/sys", (uint64_t)cfg.cxl_emulate_mask);
  rt->cxl_ = std::make_unique<CxlRegistry>(rt->be_.get());
  rt->cxl_->init(system_ram_bytes() / 100 * (uint64_t)cfg.cxl_pin_budget_pct, (uint32_t)cfg.cxl_max_buffers,
                 (uint64_t)cfg.cxl_max_buffer_gb << 30);
  for (int d = 0; d < nd; ++d) {
    auto dev = std::make_unique<Device>();
    dev->id = d;
    dev->numa = rt->be_->device_numa_node(d);
    dev->local = local(d);
    if (!dev->local) {
      rt->devs_.push_back(std::move(dev));
      continue;
    }
    for (int k = 0; k < (int)RingKind::COUNT; ++k)
      dev->rings[k] = std::make_unique<Ring>(rt->be_.get(), d, (RingKind)k, (uint32_t)cfg.channel_num_gpfifo_entries);
    void* p = nullptr;
    uint32_t entries = 64;  // power of two >= 16 fault batches
    while (entries < (uint32_t)cfg.perf_fault_batch_count * 16) entries <<= 1;
    if (rt->be_->host_alloc_coherent(sizeof(FaultBufHeader) + (size_t)entries * sizeof(DeviceFaultRecord), &p) ==
        Status::OK) {
      dev->fault_buf.hdr = (FaultBufHeader*)p;
      dev->fault_buf.recs = (DeviceFaultRecord*)((char*)p + sizeof(FaultBufHeader));
      dev->fault_buf.entries = entries;
    }
    dev->health_ok = rt->be_->device_health(d, &dev->health0) == Status::OK;
    dev->health = dev->health0;
    if (!dev->health_ok && !rt->be_->is_fake()) {
      // Not silently "healthy": the condition is reported (stats, device_health()).
      dev->health_reason = rt->be_->last_error();
      RT_WARN("GPU %d: no readable RAS / ECC counters (%s): uncorrectable errors cannot be detected", d,
              dev->health_reason.c_str());
    }
    rt->devs_.push_back(std::move(dev));
  }
  rt->perf_subs_ = perf_modules_register(Tools::get().bus());
  g_rt.store(rt, std::memory_order_release);
  install_cpu_fault_handler();
  start_cpu_fault_service();
  RT_INFO("runtime up: backend=%s devices=%d local=0x%llx host_node=%d cxl_nodes=%zu", rt->be_->name(), nd,
          (unsigned long long)mask, rt->host_node_, rt->cxl_topo_.info().numa_nodes.size());
  return rt;
}

std::vector<int> Runtime::local_devices() const {
  std::vector<int> v;
  for (auto& d : devs_)
    if (d->local) v.push_back(d->id);
  return v;
}

void Runtime::shutdown() {
  std::lock_guard<std::mutex> g(g_rt_m);
  Runtime* rt = g_rt.exchange(nullptr);
  if (rt) UnitStream::detach_all(rt);  // (streams still alive in Python hold leases of rt)
  delete rt;
}

void torch_alloc_reset();

Runtime::~Runtime() {
  stop_packer();
  torch_alloc_reset();
  for (int t : perf_subs_) Tools::get().bus().unsubscribe(t);
  stop_cpu_fault_service();
  stop_fault_service();
  for (auto& d : devs_)
    for (auto& r : d->rings)
      if (r) r->submit();
  sync_all();
  {
    std::lock_guard<std::mutex> g(leases_m_);
    leases_.clear();
  }
  // Ranges reference arenas: free them first.
  std::vector<Range*> rs;
  for (auto& kv : vs_.ranges) rs.push_back(kv.second.get());
  for (Range* r : rs) {
    r->views.store(0);
    free_range(r);
  }
  for (auto& t : dev_tables_)
    if (t.second->entries) be_->host_free_coherent(t.second->entries);
  cxl_.reset();
  for (auto& d : devs_) {
    for (auto& r : d->rings) r.reset();
    if (d->fault_buf.hdr) be_->host_free_coherent(d->fault_buf.hdr);
    d->hbm_live.store(nullptr);
    d->hbm.reset();
  }
  host_arenas_.clear();  // (each arena returns its ledger reservations)
  NodeLedger::get().detach();
}

// ------------------------------------------------------------------ tiers
Status Runtime::init_device(int d, uint64_t budget) {
  if (!is_local(d)) return Status::INVALID_ARGUMENT;
  // Freed torch memory the pluggable allocator still caches goes back first -
  // only when an arena exists and is not empty. (An unguarded trim used to go
  // through arena_for, which creates the default half-of-HBM arena on first
  // touch: every init built and destroyed a ~140 GB VMM arena, and the GPU
  // dgemm test sequence hung in a driver fence wait; gpurun_out/r6 sessions
  // s-u. torch_alloc_trim now never creates an arena.)
  if (devs_[d]->hbm && devs_[d]->hbm->outstanding_bytes()) torch_alloc_trim(d);
  std::unique_lock<OrderedRWLock> vg(vs_.lock);
  if (devs_[d]->hbm && devs_[d]->hbm->outstanding_bytes()) return Status::BUSY;
  devs_[d]->hbm_live.store(nullptr);
  devs_[d]->hbm.reset();
  if (budget == 0) {
    size_t f = 0, t = 0;
    if (be_->device_mem_info(d, &f, &t) != Status::OK) return Status::IO_ERROR;
    budget = config().hbm_budget_mb ? (uint64_t)config().hbm_budget_mb << 20 : f / 2;
  }
  devs_[d]->hbm = std::make_unique<HbmArena>(be_.get(), d, budget, (int)config().hbm_provider);
  devs_[d]->hbm_live.store(devs_[d]->hbm.get(), std::memory_order_release);
  if (devs_[d]->hbm->init_status() == Status::OK && devs_[d]->hbm->vmm()) (void)vmm_self_test(d);
  return devs_[d]->hbm->init_status();
}

Status Runtime::vmm_self_test(int d) {
  if (!is_local(d)) return Status::INVALID_ARGUMENT;
  HbmArena* ha = devs_[d]->hbm_live.load();
  VmmSelfTest& T = devs_[d]->vmm_test;
  T = VmmSelfTest{};
  if (!ha || !ha->vmm() || ha->nchunks() < 2) return Status::NOT_SUPPORTED;
  T.ran = true;
  uint32_t ch[2] = {0, 0};
  void* va = nullptr;
  uint32_t* out = nullptr;
  void* stream = nullptr;
  bool mapped = false;
  Status st = Status::OK;
  const uint32_t pat[2] = {0xA5C30F01u, 0x5A3CF102u};
  auto fail = [&](const char* what) {
    T.ok = false;
    T.detail = std::string(what) + ": " + be_->last_error();
  };
  int nch = 0;
  for (; nch < 2 && st == Status::OK; ++nch)
    if ((st = ha->alloc(1, nullptr, -1, &ch[nch], true)) != Status::OK) break;
  if (st != Status::OK) {
    fail("no free chunks");
  } else if ((st = be_->va_reserve(kBlockSize, &va)) != Status::OK) {
    fail("va_reserve");
  } else if ((st = be_->stable_va_prepare(va, kBlockSize, d)) != Status::OK) {  // the ranges' remap path
    fail("stable_va_prepare");
    be_->va_free(va, kBlockSize);
    va = nullptr;
  } else if ((st = be_->host_alloc_coherent(4096, (void**)&out)) != Status::OK) {
    fail("host_alloc_coherent");
  } else if (!(stream = be_->stream_create(d, 0))) {
    fail("stream_create");
  } else {
    for (int i = 0; i < 2 && st == Status::OK; ++i)
      st = be_->memset32(d, ha->chunk_addr(ch[i]), pat[i], kBlockSize, stream);
    if (st == Status::OK) st = be_->stream_sync(stream);
    if (st != Status::OK) fail("fill");
    // Read one page of the canary VA through a CU copy (the shader path that
    // kernels use) and return the number of words holding `want`.
    auto probe = [&](uint32_t want) -> int {
      memset(out, 0, 4096);
      CopyDesc cd{(uint64_t)out, (uint64_t)va + kBlockSize / 2, 4096, 0};
      if (be_->copy_batch(d, &cd, 1, stream, 0) != Status::OK || be_->stream_sync(stream) != Status::OK) return -1;
      int n = 0;
      for (int k = 0; k < 1024; ++k) n += out[k] == want;
      return n;
    };
    const uint32_t rounds = 6;
    for (uint32_t r = 0; r < rounds && T.ok; ++r) {
      const int h = r & 1;
      if (mapped && be_->vmm_unmap(va, kBlockSize) != Status::OK) {
        fail("vmm_unmap");
        break;
      }
      if (be_->vmm_map(va, kBlockSize, ha->handle(ch[h]), d) != Status::OK) {
        fail("vmm_map");
        break;
      }
      mapped = true;
      if (r > 0 && probe(pat[h]) != 1024) T.unflushed_stale++;  // before the flush: informational
      if (be_->tlb_flush(d) != Status::OK) {
        fail("tlb_flush");
        break;
      }
      T.rounds++;
      int n = probe(pat[h]);
      if (n == 1024) {
        T.flushed_ok++;
      } else {
        T.ok = false;
        T.detail = "after a remap and a translation flush a kernel read " + std::to_string(n < 0 ? 0 : n) +
                   "/1024 words of the new chunk (stale translation)";
      }
    }
  }
  if (mapped) be_->vmm_unmap(va, kBlockSize);
  (void)be_->tlb_flush(d);
  if (stream) be_->stream_destroy(stream);
  if (out) be_->host_free_coherent(out);
  if (va) {
    be_->stable_va_release(va, kBlockSize);
    be_->va_free(va, kBlockSize);
  }
  for (int i = 0; i < nch; ++i) ha->free(ch[i], 1);
  if (!T.ok)
    RT_ERR("gpu %d: stable-VA translation self-test FAILED (%s): stable-VA managed ranges (the transparent "
           "managed mode) are refused on this GPU",
           d, T.detail.c_str());
  return T.ok ? Status::OK : Status::NOT_SUPPORTED;
}

HostArena* Runtime::host_arena(Tier t, int node) {
  if (node < 0 || node >= kMaxNodes) return nullptr;
  std::lock_guard<std::mutex> g(host_arenas_m_);
  size_t idx = (size_t)(t == Tier::CXL ? 1 : 0) * kMaxNodes + node;
  if (host_arenas_.size() <= idx) host_arenas_.resize(2 * kMaxNodes);
  if (!host_arenas_[idx]) {
    // This process's view of the node: at most the node's budget (its memory,
    // not the machine's); the node-wide ledger splits it between processes.
    uint64_t cap = config().host_budget_mb ? (uint64_t)config().host_budget_mb << 20 : node_budget_bytes(node);
    (void)NodeLedger::get().attach();
    auto a = std::make_unique<HostArena>(be_.get(), t, node, cap);
    if (a->init_status() != Status::OK) return nullptr;
    host_arenas_[idx] = std::move(a);
  }
  return host_arenas_[idx].get();
}

ChunkArena* Runtime::arena_for(const Loc& l) {
  if (l.is_gpu()) {
    if (!is_local(l.id)) return nullptr;
    Device& d = *devs_[l.id];
    if (HbmArena* a = d.hbm_live.load(std::memory_order_acquire)) return a;
    // First touch of a GPU: create its arena with the default budget (once).
    size_t f = 0, t = 0;
    if (be_->device_mem_info(l.id, &f, &t) != Status::OK) return nullptr;
    uint64_t budget = config().hbm_budget_mb ? (uint64_t)config().hbm_budget_mb << 20 : f / 2;
    static std::mutex m;
    std::lock_guard<std::mutex> g(m);
    if (!d.hbm) {
      d.hbm = std::make_unique<HbmArena>(be_.get(), l.id, budget, (int)config().hbm_provider);
      d.hbm_live.store(d.hbm.get(), std::memory_order_release);
      if (d.hbm->init_status() == Status::OK && d.hbm->vmm()) (void)vmm_self_test(l.id);
    }
    return d.hbm.get();
  }
  if (l.tier == Tier::CXL && !cxl_topo_.is_cxl_node(l.id)) return nullptr;
  return host_arena(l.tier, l.id);
}

// ------------------------------------------------------------------ ranges
Status Runtime::malloc_managed(uint64_t size, uint32_t flags, const std::string& name, Range** out, int stable_dev) {
  if (global_status() != Status::OK) return global_status();
  if (size == 0) return Status::INVALID_ARGUMENT;
  if (flags & RANGE_COMPRESS_BF16) {
    if ((size & (kPageSize - 1)) || (flags & RANGE_STABLE_VA)) return Status::INVALID_ARGUMENT;
    flags |= RANGE_NO_CPU_VIEW;  // the host copy is encoded: no direct CPU mapping
  }
  std::unique_lock<OrderedRWLock> vg(vs_.lock);
  uint64_t id = vs_.next_range_id++;
  auto r = std::make_unique<Range>(&vs_, id, RangeType::MANAGED, size, flags, name);
  if (!(flags & RANGE_NO_CPU_VIEW) && !r->cpu_view) return Status::NO_MEMORY;
  if (flags & RANGE_STABLE_VA) {
    if (!is_local(stable_dev)) return Status::INVALID_ARGUMENT;
    vg.unlock();
    ChunkArena* a = arena_for(Loc::gpu(stable_dev));
    vg.lock();
    if (!a || !static_cast<HbmArena*>(a)->vmm()) return Status::NOT_SUPPORTED;  // needs hbm_provider=1
    if (!devs_[stable_dev]->vmm_test.ok) return Status::NOT_SUPPORTED;  // remaps are not seen reliably here
    void* va = nullptr;
    Status st = be_->va_reserve(r->cpu_view_bytes, &va);
    if (st != Status::OK) return st;
    if ((st = be_->stable_va_prepare(va, r->cpu_view_bytes, stable_dev)) != Status::OK) {
      be_->va_free(va, r->cpu_view_bytes);
      return st;
    }
    r->dev_va = va;
    r->stable_dev = stable_dev;
    vs_.dev_tree[(uint64_t)va] = r.get();
  }
  if (r->cpu_view) {
    vs_.tree[r->addr()] = r.get();
    cpu_views_add(r->addr(), r->cpu_view_bytes);  // the SIGSEGV handler's lock-free index
  }
  *out = r.get();
  vs_.ranges[id] = std::move(r);
  return Status::OK;
}

Status Runtime::malloc_managed_at(uint64_t size, uint32_t flags, const std::string& name, uint64_t id,
                                  uint64_t cpu_addr, uint64_t dev_va, int stable_dev, Range** out) {
  if (global_status() != Status::OK) return global_status();
  if (size == 0 || id == 0) return Status::INVALID_ARGUMENT;
  if (!cpu_addr) flags |= RANGE_NO_CPU_VIEW;
  if (!dev_va) flags &= ~RANGE_STABLE_VA;
  std::unique_lock<OrderedRWLock> vg(vs_.lock);
  if (vs_.ranges.count(id)) return Status::BUSY;
  auto r = std::make_unique<Range>(&vs_, id, RangeType::MANAGED, size, flags, name, cpu_addr);
  if (cpu_addr && (uint64_t)r->cpu_view != cpu_addr) return Status::BUSY;  // the window is taken
  if (flags & RANGE_STABLE_VA) {
    if (!is_local(stable_dev)) return Status::INVALID_ARGUMENT;
    vg.unlock();
    ChunkArena* a = arena_for(Loc::gpu(stable_dev));
    vg.lock();
    if (!a || !static_cast<HbmArena*>(a)->vmm() || !devs_[stable_dev]->vmm_test.ok) return Status::NOT_SUPPORTED;
    void* va = nullptr;
    Status st = be_->va_reserve(r->cpu_view_bytes, &va, (void*)dev_va);
    if (st != Status::OK) return st;
    if ((st = be_->stable_va_prepare(va, r->cpu_view_bytes, stable_dev)) != Status::OK) {
      be_->va_free(va, r->cpu_view_bytes);
      return st;
    }
    r->dev_va = va;
    r->stable_dev = stable_dev;
    vs_.dev_tree[(uint64_t)va] = r.get();
  }
  if (vs_.ranges.count(id)) return Status::BUSY;  // raced with another restore while unlocked
  if (r->cpu_view) {
    vs_.tree[r->addr()] = r.get();
    cpu_views_add(r->addr(), r->cpu_view_bytes);
  }
  vs_.next_range_id = std::max<uint64_t>(vs_.next_range_id, id + 1);
  *out = r.get();
  vs_.ranges[id] = std::move(r);
  return Status::OK;
}

Status Runtime::map_external(uint64_t ptr, uint64_t size, int dev, const std::string& name, Range** out) {
  if (!ptr || !size || !is_local(dev)) return Status::INVALID_ARGUMENT;
  std::unique_lock<OrderedRWLock> vg(vs_.lock);
  uint64_t id = vs_.next_range_id++;
  auto r = std::make_unique<Range>(&vs_, id, RangeType::EXTERNAL, size, RANGE_NO_CPU_VIEW, name);
  r->ext_ptr = ptr;
  r->ext_dev = dev;
  *out = r.get();
  vs_.ranges[id] = std::move(r);
  return Status::OK;
}

Status Runtime::alloc_device_p2p(uint64_t size, int dev, const std::string& name, Range** out) {
  if (!size || !is_local(dev)) return Status::INVALID_ARGUMENT;
  void* p = nullptr;
  Status st = be_->hbm_alloc(dev, align_up(size, kBlockSize), &p);
  if (st != Status::OK) return st;
  std::unique_lock<OrderedRWLock> vg(vs_.lock);
  uint64_t id = vs_.next_range_id++;
  auto r = std::make_unique<Range>(&vs_, id, RangeType::DEVICE_P2P, size, RANGE_NO_CPU_VIEW, name);
  r->ext_ptr = (uint64_t)p;
  r->ext_dev = dev;
  r->ext_owned = true;
  *out = r.get();
  vs_.ranges[id] = std::move(r);
  return Status::OK;
}

Status Runtime::free_range(Range* r) {
  if (!r) return Status::INVALID_ARGUMENT;
  if (r->views.load() > 0) return Status::BUSY;
  std::unique_lock<OrderedRWLock> vg(vs_.lock);
  auto it = vs_.ranges.find(r->id);
  if (it == vs_.ranges.end()) return Status::NOT_FOUND;
  for (auto& bp : r->blocks) {
    Block* b = bp.get();
    std::lock_guard<OrderedMutex> g(b->lock);
    b->tracker.wait();
    if (r->dev_va) {
      std::lock_guard<std::mutex> sg(stable_m_);
      if (b->stable_chunk.load() >= 0) stable_unmap_locked(b);  // after the kernels still reading through the mapping
      if (b->in_stale_list) {  // the block is about to go: no dangling stale_maps_ entry
        stale_maps_.erase(std::remove(stale_maps_.begin(), stale_maps_.end(), b), stale_maps_.end());
        b->in_stale_list = false;
      }
    }
    for (auto& x : b->res) {
      if (x.chunk >= 0) x.arena->free((uint32_t)x.chunk, 1);
      if (x.seg && x.seg->chunk >= 0) x.seg->arena->free((uint32_t)x.seg->chunk, 1);
    }
    b->res.clear();
    Tools::get().bus().notify(PerfEventData{PerfEvent::BLOCK_DESTROY, r->id, b->index});
  }
  if (r->dev_va) {
    vs_.dev_tree.erase((uint64_t)r->dev_va);
    be_->stable_va_release(r->dev_va, r->cpu_view_bytes);
    be_->va_free(r->dev_va, r->cpu_view_bytes);
  }
  if (r->ext_owned && r->ext_ptr) be_->hbm_free(r->ext_dev, (void*)r->ext_ptr, align_up(r->size, kBlockSize));
  if (r->group) {
    auto& v = r->group->ranges;
    v.erase(std::remove(v.begin(), v.end(), r), v.end());
  }
  if (r->cpu_view) {
    cpu_views_remove(r->addr());
    vs_.tree.erase(r->addr());
  }
  {
    std::lock_guard<std::mutex> g(dev_tables_m_);
    auto t = dev_tables_.find(r->id);
    if (t != dev_tables_.end()) {
      be_->host_free_coherent(t->second->entries);
      dev_tables_.erase(t);
    }
  }
  Tools::get().bus().notify(PerfEventData{PerfEvent::RANGE_DESTROY, r->id});
  vs_.ranges.erase(it);
  return Status::OK;
}

Range* Runtime::find_range(uint64_t addr) {
  std::shared_lock<OrderedRWLock> vg(vs_.lock);
  if (Range* r = vs_.find_locked(addr)) return r;
  // a stable device VA (RANGE_STABLE_VA ranges have one, often without a CPU view)
  auto it = vs_.dev_tree.upper_bound(addr);
  if (it == vs_.dev_tree.begin()) return nullptr;
  --it;
  return addr < it->first + it->second->cpu_view_bytes ? it->second : nullptr;
}

Range* Runtime::range_by_id(uint64_t id) {
  std::shared_lock<OrderedRWLock> vg(vs_.lock);
  return vs_.by_id_locked(id);
}

// ------------------------------------------------------------------ policy
Status Runtime::mem_advise(Range* r, uint64_t off, uint64_t len, Advice a, Loc loc, int proc) {
  if (!r || len == 0 || off + len > r->size) return Status::INVALID_ARGUMENT;
  if (r->type != RangeType::MANAGED) return Status::NOT_SUPPORTED;
  if (a == Advice::SET_PREFERRED_LOCATION && !arena_for(loc)) return Status::INVALID_ARGUMENT;
  if ((a == Advice::SET_ACCESSED_BY || a == Advice::UNSET_ACCESSED_BY) &&
      !(proc == kCpuProc || is_local(proc)))
    return Status::INVALID_ARGUMENT;
  std::shared_lock<OrderedRWLock> vg(vs_.lock);
  uint64_t b0 = off >> kBlockShift, b1 = (off + len - 1) >> kBlockShift;
  for (uint64_t bi = b0; bi <= b1; ++bi) {
    Block* b = r->block(bi);
    Ctx c;
    {
      std::lock_guard<OrderedMutex> g(b->lock);
      Policy& p = b->policy;
      switch (a) {
        case Advice::SET_READ_MOSTLY:
          p.read_dup = true;
          pack_enqueue(b);  // (packed once a GPU copy was dropped clean)
          break;
        case Advice::UNSET_READ_MOSTLY: {
          p.read_dup = false;
          // Collapse duplicates: keep the preferred copy, else a host copy, else the first.
          PageMask seen;
          std::vector<Residency*> order;
          if (p.has_preferred)
            if (Residency* x = b->find(p.preferred)) order.push_back(x);
          for (auto& x : b->res)
            if (!x.loc.is_gpu() && std::find(order.begin(), order.end(), &x) == order.end()) order.push_back(&x);
          for (auto& x : b->res)
            if (std::find(order.begin(), order.end(), &x) == order.end()) order.push_back(&x);
          std::vector<Loc> empty;
          for (Residency* x : order) {
            PageMask dup = x->resident & seen;
            seen |= x->resident;
            if (!dup.empty()) {
              x->resident = x->resident.andnot(dup);
              b->range->mod_gen.fetch_add(1, std::memory_order_acq_rel);
              Tools::get().inc(Counter::Revocations);
              if (x->resident.empty()) empty.push_back(x->loc);
            }
          }
          for (auto& l : empty) drop_copy(c, b, l);
          c.cpu_refresh.push_back(b);
          break;
        }
        case Advice::SET_PREFERRED_LOCATION:
          p.has_preferred = true;
          p.preferred = loc;
          break;
        case Advice::UNSET_PREFERRED_LOCATION: p.has_preferred = false; break;
        case Advice::SET_ACCESSED_BY: p.accessed_by |= 1ull << (proc == kCpuProc ? kCpuProc : proc); break;
        case Advice::UNSET_ACCESSED_BY: p.accessed_by &= ~(1ull << (proc == kCpuProc ? kCpuProc : proc)); break;
      }
    }
    finish_ctx(c, nullptr);
  }
  return Status::OK;
}

Status Runtime::create_range_group(uint64_t* id) {
  std::unique_lock<OrderedRWLock> vg(vs_.lock);
  uint64_t g = vs_.next_group_id++;
  vs_.groups[g] = std::make_unique<RangeGroup>(g);
  *id = g;
  return Status::OK;
}

Status Runtime::set_range_group(Range* r, uint64_t gid) {
  std::unique_lock<OrderedRWLock> vg(vs_.lock);
  if (r->group) {
    auto& v = r->group->ranges;
    v.erase(std::remove(v.begin(), v.end(), r), v.end());
    r->group = nullptr;
  }
  if (gid == 0) return Status::OK;
  auto it = vs_.groups.find(gid);
  if (it == vs_.groups.end()) return Status::NOT_FOUND;
  r->group = it->second.get();
  r->group->ranges.push_back(r);
  return Status::OK;
}

Status Runtime::set_group_migratable(uint64_t gid, bool m) {
  std::unique_lock<OrderedRWLock> vg(vs_.lock);
  auto it = vs_.groups.find(gid);
  if (it == vs_.groups.end()) return Status::NOT_FOUND;
  it->second->migratable = m;
  return Status::OK;
}

// ------------------------------------------------------------------ CPU view / stable VA / device tables
void Runtime::cpu_map_block(Block* b) {
  Range* r = b->range;
  if (!r->cpu_view) return;
  uint8_t* win = r->cpu_view + b->block_offset();
  // (a packed copy holds no raw pages: never mapped - a CPU access faults and
  // expands it; a segmented one maps its raw segments' pages only)
  Residency* h = nullptr;
  if (Residency* x = b->find(cpu_loc()); x && (x->fmt == 0 || x->fmt == 3)) h = x;
  if (!h)
    for (auto& x : b->res)
      if (!x.loc.is_gpu() && x.chunk >= 0 && (x.fmt == 0 || x.fmt == 3)) {
        h = &x;
        break;
      }
  if (!h) {
    if (b->cpu_arena) {
      mmap(win, kBlockSize, PROT_NONE, MAP_PRIVATE | MAP_ANONYMOUS | MAP_FIXED | MAP_NORESERVE, -1, 0);
      b->cpu_arena = nullptr;
      b->cpu_chunk = -1;
    }
    b->cpu_ro.zero();
    b->cpu_rw.zero();
    return;
  }
  HostArena* ha = static_cast<HostArena*>(h->arena);
  if (b->cpu_arena != h->arena || b->cpu_chunk != h->chunk) {
    void* m = mmap(win, kBlockSize, PROT_NONE, MAP_SHARED | MAP_FIXED, ha->fd(), (off_t)ha->file_offset((uint32_t)h->chunk));
    if (m == MAP_FAILED) {
      RT_ERR("CPU view remap failed for range %llu block %llu", (unsigned long long)r->id,
             (unsigned long long)b->index);
      return;
    }
    b->cpu_arena = h->arena;
    b->cpu_chunk = h->chunk;
    b->cpu_ro.zero();
    b->cpu_rw.zero();
  }
  bool pending = b->unpublished > 0 || !b->tracker.query();
  PageMask others;
  for (auto& x : b->res)
    if (&x != h) others |= x.resident;
  PageMask rw, ro;
  PageMask usable = h->resident;
  if (h->fmt == 3 && h->seg)
    for (uint32_t sg = 0; sg < kSegsPerBlock; ++sg)
      if ((h->seg->packed >> sg) & 1u) usable = usable.andnot(seg_pages(sg));
  if (!pending) {
    rw = usable.andnot(others) & b->valid_pages();
    ro = (usable & others) & b->valid_pages();
  }
  if (rw == b->cpu_rw && ro == b->cpu_ro) return;
  // Apply protections run by run.
  uint32_t p = 0;
  while (p < kPagesPerBlock) {
    int prot = rw.test(p) ? (PROT_READ | PROT_WRITE) : (ro.test(p) ? PROT_READ : PROT_NONE);
    uint32_t e = p + 1;
    while (e < kPagesPerBlock) {
      int pe = rw.test(e) ? (PROT_READ | PROT_WRITE) : (ro.test(e) ? PROT_READ : PROT_NONE);
      if (pe != prot) break;
      ++e;
    }
    mprotect(win + ((uint64_t)p << kPageShift), (uint64_t)(e - p) << kPageShift, prot);
    p = e;
  }
  b->cpu_rw = rw;
  b->cpu_ro = ro;
}

void Runtime::stable_unmap_locked(Block* b) {
  const int64_t c = b->stable_chunk.load();
  if (c < 0) return;
  Range* r = b->range;
  const uint64_t t_w = now_ns();
  if (b->stable_users.wait() != Status::OK)
    RT_ERR("stable VA users of range %llu block %llu failed", (unsigned long long)r->id, (unsigned long long)b->index);
  Tools::get().inc(Counter::StableWaitNs, now_ns() - t_w);
  b->stable_users.clear();
  Tools::get().inc(Counter::VmmRemaps);
  const uint64_t t_unmap = now_ns();
  const Status ust = be_->vmm_unmap((char*)r->dev_va + b->block_offset(), kBlockSize);
  Tools::get().inc(Counter::VmmUnmapNs, now_ns() - t_unmap);
  if (ust != Status::OK) {
    Tools::get().inc(Counter::VmmErrors);
    RT_ERR("stable VA unmap of range %llu block %llu failed: %s", (unsigned long long)r->id,
           (unsigned long long)b->index, be_->last_error().c_str());
  }
  b->stable_chunk.store(-1);
  b->va_unmap_seq = tlb_started_[r->stable_dev].load();
  b->stale_mapping = false;  // its stale_maps_ entry is dropped by the next reap
}

void Runtime::reap_stale_maps_locked() {
  size_t w = 0;
  for (Block* b : stale_maps_) {
    if (b->stale_mapping && (config().stable_lazy_unmap || !b->stable_users.query())) {
      stale_maps_[w++] = b;  // users still running (or lazy mode): keep
      continue;
    }
    if (b->stale_mapping) stable_unmap_locked(b);  // else remapped / unmapped meanwhile: drop the entry
    b->in_stale_list = false;
  }
  stale_maps_.resize(w);
}

uint32_t& Runtime::thread_tlb_need() {
  static thread_local uint32_t need = 0;
  return need;
}

// Point block b's stable VA at its HBM chunk (block lock held). A mapping is
// torn down only after the work that may use it finished
// (Block::stable_users); an evicted block keeps its now-stale mapping until it
// comes back - to the same chunk (nothing to do: the hint in place_stable
// prefers it) or to another one. A handle may then be mapped at several VAs at
// once (the arena view, its block's VA, stale VAs of earlier owners), which
// HIP's VMM layer handles (tools/probe_vmm_multimap.hip).
void Runtime::stable_map_block(Block* b) {
  Range* r = b->range;
  if (!r->dev_va) return;
  TraceRange tr(be_.get(), "ogkm:stable_map", 2);
  Residency* g = b->find(Loc::gpu(r->stable_dev));
  const int64_t want = (g && g->chunk >= 0) ? g->chunk : -1;
  if (want == b->stable_chunk.load() && !b->stale_mapping) return;
  if (want >= 0 && b->stable_chunk.load() >= 0 && want != b->stable_chunk.load()) {
    // Remap from a stale mapping: its users (kernels queued before the
    // eviction) must finish before the VA moves. Wait for them without
    // stable_m_ - other blocks' remaps, the reaper and translation flushes go
    // on meanwhile; b itself is held by its block lock (the reaper may still
    // unmap it, which only makes the unmap below a no-op).
    Tracker users;
    {
      std::lock_guard<std::mutex> sg(stable_m_);
      users = b->stable_users;
    }
    const uint64_t t_w = now_ns();
    if (users.wait() != Status::OK)
      RT_ERR("stable VA users of range %llu block %llu failed", (unsigned long long)r->id, (unsigned long long)b->index);
    Tools::get().inc(Counter::StableWaitNs, now_ns() - t_w);
  }
  std::lock_guard<std::mutex> sg(stable_m_);
  if (want == b->stable_chunk.load()) {  // back on the chunk it still maps: valid again
    b->stale_mapping = false;
    return;
  }
  if (want < 0) {
    // Evicted: kernels enqueued before the last lease release may still read
    // the VA. Unmap at once only when they are done (and not in lazy mode);
    // otherwise the stale mapping stays - a stray access then reads whatever
    // the chunk holds instead of faulting - and the reaper tears it down
    // before a later flush once they are.
    b->stable_users.merge(b->tracker);
    if (config().stable_lazy_unmap || !b->stable_users.query()) {
      if (b->stable_chunk.load() >= 0 && !b->stale_mapping) {
        b->stale_mapping = true;
        if (!b->in_stale_list) {
          b->in_stale_list = true;
          stale_maps_.push_back(b);
        }
      }
      return;
    }
    stable_unmap_locked(b);
    return;
  }
  HbmArena* ha = static_cast<HbmArena*>(g->arena);
  stable_unmap_locked(b);  // b's own previous mapping (stale, another chunk)
  char* va = (char*)r->dev_va + b->block_offset();
  Tools::get().inc(Counter::VmmRemaps);
  const uint64_t t_map = now_ns();
  const Status mst = be_->vmm_map(va, kBlockSize, ha->handle((uint32_t)want), r->stable_dev);
  Tools::get().inc(Counter::VmmMapNs, now_ns() - t_map);
  if (mst == Status::OK) {
    b->stable_chunk.store(want);
    // A translation of this VA can still sit in the GPU's TLB only if no
    // flush begun after its last unmap has completed; otherwise (the common
    // case of a block evicted a while ago) the new mapping needs no flush.
    if (b->va_unmap_seq == ~0ull || tlb_done_[r->stable_dev].load() <= b->va_unmap_seq) {
      thread_tlb_need() |= 1u << r->stable_dev;
      tlb_dirty_.fetch_or(1u << r->stable_dev);
      b->map_seq = tlb_started_[r->stable_dev].load();
    } else {
      Tools::get().inc(Counter::TlbFlushesElided);
      b->map_seq = ~0ull;
    }
  } else {
    Tools::get().inc(Counter::VmmErrors);
    RT_ERR("stable VA map of range %llu block %llu to chunk %lld failed: %s", (unsigned long long)r->id,
           (unsigned long long)b->index, (long long)want, be_->last_error().c_str());
  }
}

// Everything the runtime knows about a device address - for GPU memory-fault
// reports (the analog of the reference's fatal-fault reporting with the
// faulting VA, uvm_gpu_replayable_faults.c:2495-2875). Called from a ROCr
// thread: it only try-locks, so it never waits for a lock a stuck thread holds.
std::string Runtime::describe_device_address(uint64_t va) {
  char buf[512];
  std::string out;
  if (!vs_.lock.try_lock_shared()) return "(VA space busy)";
  auto it = vs_.dev_tree.upper_bound(va);
  if (it != vs_.dev_tree.begin()) {
    --it;
    Range* r = it->second;
    if (va >= it->first && va < it->first + r->cpu_view_bytes) {
      Block* b = r->block((va - it->first) >> kBlockShift);
      snprintf(buf, sizeof buf, "stable VA of range %llu '%s' (%llu B) block %llu: stable_chunk %lld", (unsigned long long)r->id,
               r->name.c_str(), (unsigned long long)r->size, (unsigned long long)b->index,
               (long long)b->stable_chunk.load());
      out = buf;
      if (b->lock.try_lock()) {
        for (auto& x : b->res) {
          snprintf(buf, sizeof buf, "; resident %s chunk %lld pages %u", x.loc.str().c_str(), (long long)x.chunk,
                   x.resident.count());
          out += buf;
        }
        snprintf(buf, sizeof buf, "; lease_pins %u tracker %zu stable_users %zu", (unsigned)b->lease_pins,
                 b->tracker.size(), b->stable_users.size());
        out += buf;
        b->lock.unlock();
      }
    }
  }
  for (auto& d : devs_) {
    HbmArena* ha = d->hbm_live.load();
    if (!ha || va < ha->base() || va >= ha->base() + ((uint64_t)ha->nchunks() << kBlockShift)) continue;
    snprintf(buf, sizeof buf, "%sarena view of gpu %d chunk %lld", out.empty() ? "" : "; ", d->id,
             (long long)ha->chunk_of(va));
    out += buf;
  }
  vs_.lock.unlock_shared();
  return out.empty() ? "(not a runtime address)" : out;
}

void Runtime::flush_translations() {
  {
    // stale mappings whose users finished go now, so this flush covers them
    std::lock_guard<std::mutex> sg(stable_m_);
    if (!stale_maps_.empty()) reap_stale_maps_locked();
  }
  uint32_t m = tlb_dirty_.exchange(0) | thread_tlb_need();
  thread_tlb_need() = 0;
  for (int d = 0; m; ++d, m >>= 1) {
    if (!(m & 1)) continue;
    const uint64_t k = tlb_started_[d].fetch_add(1) + 1;  // covers every unmap before this point
    const uint64_t t_fl = now_ns();
    Status fst = be_->tlb_flush(d);
    for (int64_t r = 1; fst == Status::OK && r < config().tlb_flush_repeat; ++r) fst = be_->tlb_flush(d);
    Tools::get().inc(Counter::TlbFlushNs, now_ns() - t_fl);
    if (fst != Status::OK) {
      Tools::get().inc(Counter::VmmErrors);
      RT_ERR("GPU %d translation flush after stable-VA remaps failed: %s", d, be_->last_error().c_str());
    } else {
      Tools::get().inc(Counter::TlbFlushes);
      uint64_t cur = tlb_done_[d].load();
      while (cur < k && !tlb_done_[d].compare_exchange_weak(cur, k)) {
      }
    }
  }
}

void Runtime::register_table_stream(int dev, void* stream, bool on) {
  if (dev < 0 || dev >= kMaxGpus) return;
  std::lock_guard<std::mutex> g(dev_tables_m_);
  auto& v = table_streams_[dev];
  auto it = std::find(v.begin(), v.end(), stream);
  if (on && it == v.end()) v.push_back(stream);
  if (!on && it != v.end()) v.erase(it);
}

void Runtime::shootdown(Block* b, Residency* r) {
  if (!r || !r->loc.is_gpu() || r->chunk < 0) return;
  std::lock_guard<std::mutex> g(dev_tables_m_);
  auto it = dev_tables_.find(b->range->id);
  if (it == dev_tables_.end() || it->second->dev != r->loc.id) return;
  uint64_t* e = &it->second->entries[2 * b->index];
  uint64_t addr = r->arena->chunk_addr((uint32_t)r->chunk);
  if (__atomic_load_n(e, __ATOMIC_RELAXED) != addr) return;
  __atomic_store_n(e, 0, __ATOMIC_RELEASE);
  // Kernels already queued on a table stream may have read the old entry.
  for (void* s : table_streams_[r->loc.id])
    if (FenceRef f = fence_record(be_.get(), r->loc.id, s)) r->arena->add_reuse_fence((uint32_t)r->chunk, f);
  Tools::get().inc(Counter::TableShootdowns);
}

void Runtime::update_device_table(Block* b) {
  std::lock_guard<std::mutex> g(dev_tables_m_);
  auto it = dev_tables_.find(b->range->id);
  if (it == dev_tables_.end()) return;
  DeviceResidencyTable* t = it->second.get();
  uint64_t hbm = 0, rem = 0;
  PageMask valid = b->valid_pages();
  for (auto& x : b->res) {
    if ((x.resident & valid) == valid) {
      if (x.loc == Loc::gpu(t->dev)) hbm = x.arena->chunk_addr((uint32_t)x.chunk);
      else if (!x.loc.is_gpu() && !rem && x.fmt == 0) rem = x.arena->chunk_addr((uint32_t)x.chunk);
    }
  }
  bool pending = b->unpublished > 0 || !b->tracker.query();
  uint64_t old = __atomic_load_n(&t->entries[2 * b->index], __ATOMIC_RELAXED);
  uint64_t now = pending ? 0 : hbm;
  // Copies still in flight: the entry is published once they land
  // (refresh_device_tables, run by the fault-service poll and sync points).
  if (pending && (hbm || rem)) table_pending_.emplace_back(b->range->id, b->index);
  if ((old == 0) != (now == 0))
    // The GPU's view of the block switches between one 2 MB mapping and
    // per-page (remote / absent) access: the PageSizeChange event of uvm_tools.
    tools_event(ToolsEventType::PageSizeChange, Cause::User, Loc{}, Loc::gpu(t->dev), t->dev,
                b->range->addr() + b->block_offset(), now ? kBlockSize : kPageSize, b->range->id);
  __atomic_store_n(&t->entries[2 * b->index], now, __ATOMIC_RELEASE);
  __atomic_store_n(&t->entries[2 * b->index + 1], pending ? 0 : rem, __ATOMIC_RELEASE);
}

void Runtime::refresh_device_tables() {
  std::vector<std::pair<uint64_t, uint64_t>> todo;
  {
    std::lock_guard<std::mutex> g(dev_tables_m_);
    if (table_pending_.empty()) return;
    todo.swap(table_pending_);
  }
  std::sort(todo.begin(), todo.end());
  todo.erase(std::unique(todo.begin(), todo.end()), todo.end());
  std::shared_lock<OrderedRWLock> vg(vs_.lock);
  for (auto& [rid, bi] : todo) {
    Range* r = vs_.by_id_locked(rid);
    if (!r || bi >= r->nblocks) continue;
    Block* b = r->block(bi);
    std::lock_guard<OrderedMutex> g(b->lock);
    update_device_table(b);  // re-queues itself while still pending
  }
}

Status Runtime::device_table(Range* r, DeviceResidencyTable** out) {
  {
    std::lock_guard<std::mutex> g(dev_tables_m_);
    auto it = dev_tables_.find(r->id);
    if (it != dev_tables_.end()) {
      *out = it->second.get();
      return Status::OK;
    }
    auto t = std::make_unique<DeviceResidencyTable>();
    void* p = nullptr;
    Status st = be_->host_alloc_coherent(std::max<uint64_t>(16, r->nblocks * 16), &p);
    if (st != Status::OK) return st;
    t->entries = (uint64_t*)p;
    t->nblocks = r->nblocks;
    std::vector<int> loc = local_devices();
    t->dev = loc.empty() ? 0 : loc.front();  // the table describes this process's GPU
    *out = t.get();
    dev_tables_[r->id] = std::move(t);
  }
  std::shared_lock<OrderedRWLock> vg(vs_.lock);
  for (auto& bp : r->blocks) {
    std::lock_guard<OrderedMutex> g(bp->lock);
    update_device_table(bp.get());
  }
  return Status::OK;
}

// ------------------------------------------------------------------ data helpers
// Write whole blocks of a RANGE_COMPRESS_BF16 range: the host / CXL copy is
// stored BF12-encoded (raw when a block does not compress). Encoding runs on a
// small thread pool; GPU sources are staged through pinned host chunks.
Status Runtime::write_compressed(Range* r, uint64_t off, const void* src, uint64_t bytes, int src_dev) {
  if ((off & (kBlockSize - 1)) || ((bytes & (kBlockSize - 1)) && off + bytes != r->size)) return Status::INVALID_ARGUMENT;
  uint64_t b0 = off >> kBlockShift, nb = (bytes + kBlockSize - 1) >> kBlockShift;
  std::shared_lock<OrderedRWLock> vg(vs_.lock);
  const uint64_t batch = 64;
  HostArena* stage = nullptr;
  uint32_t stage_first = 0;
  if (src_dev >= 0) {
    stage = host_arena(Tier::HOST, host_node_);
    if (!stage) return Status::NO_MEMORY;
    Status st = alloc_chunks(stage, (uint32_t)std::min<uint64_t>(batch, nb), -1, &stage_first, nullptr, true);
    if (st != Status::OK) return st;
  }
  Status result = Status::OK;
  unsigned nthreads = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  for (uint64_t s = 0; s < nb && result == Status::OK; s += batch) {
    uint64_t n = std::min(batch, nb - s);
    // 1) raw source pointers (staging GPU data to host first)
    std::vector<const uint8_t*> raw(n);
    if (src_dev >= 0) {
      Ring* rg = ring(src_dev, RingKind::GPU_TO_CPU);
      for (uint64_t k = 0; k < n; ++k) {
        uint64_t boff = (b0 + s + k) << kBlockShift;
        Sqe cp;
        cp.op = SqeOp::COPY;
        cp.dst = stage->chunk_addr(stage_first + (uint32_t)k);
        cp.src = (uint64_t)src + (boff - off);
        cp.bytes = std::min<uint64_t>(kBlockSize, r->size - boff);
        rg->push(std::move(cp));
        raw[k] = (const uint8_t*)stage->chunk_addr(stage_first + (uint32_t)k);
      }
      result = rg->submit()->wait();
      if (result != Status::OK) break;
    } else {
      for (uint64_t k = 0; k < n; ++k) raw[k] = (const uint8_t*)src + (((b0 + s + k) << kBlockShift) - off);
    }
    // 2) destination chunks (one block lock at a time)
    std::vector<Residency*> dst(n, nullptr);
    for (uint64_t k = 0; k < n && result == Status::OK; ++k) {
      Block* b = r->block(b0 + s + k);
      for (int attempt = 0; attempt < 8; ++attempt) {
        Ctx c;
        Status st;
        {
          std::lock_guard<OrderedMutex> g(b->lock);
          Loc d = b->policy.has_preferred && !b->policy.preferred.is_gpu() ? b->policy.preferred : cpu_loc();
          st = populate(c, b, d, -1, &dst[k]);
          if (st == Status::OK) {
            b->tracker.wait();
            Tracker rf = dst[k]->arena->reuse_fence((uint32_t)dst[k]->chunk);
            rf.wait();
          }
        }
        if (st != Status::MORE_PROCESSING_REQUIRED) {
          result = st;
          break;
        }
        Reservation rr;
        Status es = ensure_capacity(c.need_arena, c.need_n, &rr);
        if (es != Status::OK) {
          result = es;
          break;
        }
        c.need_arena->free((uint32_t)rr.first, rr.n);
      }
    }
    if (result != Status::OK) break;
    // 3) encode in parallel (no locks: the chunks carry no resident pages yet)
    std::vector<uint64_t> enc(n, 0);
    std::atomic<uint64_t> next{0};
    auto work = [&] {
      for (uint64_t k; (k = next.fetch_add(1)) < n;) {
        Block* b = r->block(b0 + s + k);
        uint8_t* out = (uint8_t*)dst[k]->arena->chunk_addr((uint32_t)dst[k]->chunk);
        uint32_t nv = b->npages << (kPageShift - 1);
        uint64_t nbytes = std::min<uint64_t>(kBlockSize, r->size - b->block_offset());
        if (nbytes == ((uint64_t)b->npages << kPageShift)) enc[k] = bf12_encode((const uint16_t*)raw[k], nv, out, kBlockSize);
        if (!enc[k]) {
          memcpy(out, raw[k], nbytes);
          if (nbytes < ((uint64_t)b->npages << kPageShift)) memset(out + nbytes, 0, ((uint64_t)b->npages << kPageShift) - nbytes);
        }
      }
    };
    std::vector<std::thread> pool;
    for (unsigned t = 1; t < std::min<uint64_t>(nthreads, n); ++t) pool.emplace_back(work);
    work();
    for (auto& t : pool) t.join();
    // 4) publish: this copy becomes the only valid one
    for (uint64_t k = 0; k < n; ++k) {
      Block* b = r->block(b0 + s + k);
      Ctx c;
      {
        std::lock_guard<OrderedMutex> g(b->lock);
        Residency* d = dst[k];
        d->fmt = enc[k] ? 1 : 0;
        d->enc_bytes = (uint32_t)enc[k];
        d->resident = b->valid_pages();
        if (enc[k]) Tools::get().inc(Counter::EncodedBytes, (uint64_t)b->npages << kPageShift);
        Loc keep = d->loc;
        std::vector<Loc> drop;
        for (auto& x : b->res)
          if (!(x.loc == keep)) drop.push_back(x.loc);
        for (auto& l : drop) {
          b->find(l)->resident.zero();
          drop_copy(c, b, l);
        }
        touch_residency(b, b->find(keep));
        c.cpu_refresh.push_back(b);
      }
      finish_ctx(c, nullptr);
    }
  }
  if (stage) stage->free(stage_first, (uint32_t)std::min<uint64_t>(batch, nb));
  return result;
}

Status Runtime::write(Range* r, uint64_t off, const void* src, uint64_t bytes, int src_dev) {
  if (!r || off + bytes > r->size || (src_dev >= 0 && !is_local(src_dev))) return Status::INVALID_ARGUMENT;
  if (quiesced_.load()) return Status::BUSY;  // checkpoint in progress
  if (r->type != RangeType::MANAGED) return Status::NOT_SUPPORTED;
  if (bytes == 0) return Status::OK;
  r->mod_gen.fetch_add(1, std::memory_order_acq_rel);
  if (r->flags & RANGE_COMPRESS_BF16) return write_compressed(r, off, src, bytes, src_dev);
  std::shared_lock<OrderedRWLock> vg(vs_.lock);
  uint64_t pos = off;
  while (pos < off + bytes) {
    uint64_t bi = pos >> kBlockShift;
    uint64_t end = std::min(off + bytes, (bi + 1) << kBlockShift);
    Block* b = r->block(bi);
    uint64_t lo = pos - (bi << kBlockShift), hi = end - (bi << kBlockShift);
    uint32_t p0 = (uint32_t)(lo >> kPageShift), p1 = (uint32_t)((hi + kPageSize - 1) >> kPageShift);
    PageMask pages = PageMask::range(p0, p1 - p0);
    // Fully-overwritten pages need no old data.
    PageMask full = pages;
    if (lo & (kPageSize - 1)) full.clear(p0);
    if ((hi & (kPageSize - 1)) && hi < ((uint64_t)b->npages << kPageShift)) full.clear(p1 - 1);
    Status st = Status::OK;
    for (int attempt = 0; attempt < 8; ++attempt) {
      Ctx c;
      c.cause = Cause::User;
      {
        std::lock_guard<OrderedMutex> g(b->lock);
        Loc dst;
        if (b->policy.has_preferred) dst = b->policy.preferred;
        else if (!b->res.empty()) dst = b->res.front().loc;
        else dst = src_dev >= 0 ? Loc::gpu(src_dev) : cpu_loc();
        Loc stage = dst;
        if (src_dev < 0 && dst.is_gpu()) stage = cpu_loc();  // pageable host source: stage on host
        Residency* to = nullptr;
        st = populate(c, b, stage, -1, &to);
        if (st == Status::OK) stage = to->loc;  // (a full node's data rests on the next one: populate)
        if (st == Status::OK && to->fmt == 2) st = expand_packed(b, to);  // raw pages land in it
        if (st == Status::OK && to->fmt == 3) st = note_host_write(b, to, pages, full);  // only their segments
        if (st == Status::OK) {
          // Old data only for partially covered pages.
          PageMask partial = pages.andnot(full);
          if (!partial.empty()) st = make_resident(c, b, partial, stage, false, Cause::User);
          to = b->find(stage);
        }
        if (st == Status::OK) {
          // Invalidate other copies of the written pages.
          std::vector<Loc> empty;
          for (auto& x : b->res)
            if (&x != to && x.resident.intersects(pages)) {
              x.resident = x.resident.andnot(pages);
              if (x.resident.empty()) empty.push_back(x.loc);
            }
          for (auto& l : empty) drop_copy(c, b, l);
          to = b->find(stage);
          to->resident |= pages;
          touch_residency(b, to);
          uint64_t dst_addr = to->arena->chunk_addr((uint32_t)to->chunk) + lo;
          const char* s = (const char*)src + (pos - off);
          if (src_dev < 0) {
            Tracker t = b->tracker;
            t.wait();
            Tracker rf = to->arena->reuse_fence((uint32_t)to->chunk);
            rf.wait();
            memcpy((void*)dst_addr, s, end - pos);
          } else {
            Loc sl = Loc::gpu(src_dev);
            Ring* rg = stage.is_gpu() ? (stage.id == src_dev ? ring(src_dev, RingKind::GPU_INTERNAL)
                                                            : ring(src_dev, RingKind::GPU_TO_GPU))
                                      : ring(src_dev, RingKind::GPU_TO_CPU);
            Tracker rf = to->arena->reuse_fence((uint32_t)to->chunk);
            rf.merge(b->tracker);
            for (auto& f : rf.fences()) rg->push_wait(f);
            Sqe cp;
            cp.op = SqeOp::COPY;
            cp.dst = dst_addr;
            cp.src = (uint64_t)s;
            cp.bytes = end - pos;
            cp.file = __FILE__;
            cp.line = __LINE__;
            rg->push(std::move(cp));
            FenceRef f = rg->submit();
            Tools::get().inc(stage.is_gpu() ? Counter::BytesXferDtD : Counter::BytesXferDtH, end - pos);
            (void)sl;
            st = f->wait();
          }
          c.cpu_refresh.push_back(b);
        }
        if (st == Status::OK && !(stage == dst)) st = make_resident(c, b, pages, dst, false, Cause::User);
      }
      if (st == Status::MORE_PROCESSING_REQUIRED) {
        finish_ctx(c, nullptr);
        Reservation rr;
        Status es = ensure_capacity(c.need_arena, c.need_n, &rr);
        if (es != Status::OK) return es;
        c.need_arena->free((uint32_t)rr.first, rr.n);
        continue;
      }
      Tracker t;
      Status fs = finish_ctx(c, &t);
      Status w = t.wait();
      if (st == Status::OK) st = fs;
      if (st == Status::OK) st = w;
      break;
    }
    if (st != Status::OK) return st;
    pos = end;
  }
  return Status::OK;
}

Status Runtime::read(Range* r, uint64_t off, void* dst, uint64_t bytes, int dst_dev) {
  if (!r || off + bytes > r->size || (dst_dev >= 0 && !is_local(dst_dev))) return Status::INVALID_ARGUMENT;
  if (r->type != RangeType::MANAGED) return Status::NOT_SUPPORTED;
  std::shared_lock<OrderedRWLock> vg(vs_.lock);
  uint64_t pos = off;
  while (pos < off + bytes) {
    uint64_t bi = pos >> kBlockShift;
    uint64_t end = std::min(off + bytes, (bi + 1) << kBlockShift);
    Block* b = r->block(bi);
    std::lock_guard<OrderedMutex> g(b->lock);
    b->tracker.wait();
    uint64_t lo = pos - (bi << kBlockShift);
    char* out = (char*)dst + (pos - off);
    // An encoded copy is decoded into a pinned scratch chunk and read from there.
    Residency decoded;
    Residency* encoded = nullptr;
    HostArena* scratch_arena = nullptr;
    for (auto& x : b->res)
      if (x.fmt && x.resident.intersects(PageMask::range((uint32_t)(lo >> kPageShift),
                                                         (uint32_t)((end - pos + kPageSize - 1) >> kPageShift))))
        encoded = &x;
    if (encoded) {
      scratch_arena = host_arena(Tier::HOST, host_node_);
      uint32_t tmp;
      Status st = scratch_arena ? alloc_chunks(scratch_arena, 1, -1, &tmp, nullptr, true) : Status::NO_MEMORY;
      if (st != Status::OK) return st;
      decoded = *encoded;
      decoded.arena = scratch_arena;
      decoded.chunk = tmp;
      decoded.fmt = 0;
      decoded.seg.reset();
      bool ok = true;
      if (encoded->fmt == 3) {  // raw segments as they are, packed ones decoded
        uint8_t* o = (uint8_t*)scratch_arena->chunk_addr(tmp);
        memcpy(o, (const void*)encoded->arena->chunk_addr((uint32_t)encoded->chunk), (size_t)b->npages << kPageShift);
        const SegDir& d = *encoded->seg;
        for (uint32_t sg = 0; sg < kSegsPerBlock && ok; ++sg)
          if ((d.packed >> sg) & 1u)
            ok = ans_decode((const uint8_t*)d.arena->chunk_addr((uint32_t)d.chunk) + d.off[sg],
                            (uint16_t*)(o + (uint64_t)sg * kSegBytes), kSegBytes / 2);
      } else {
        ok = block_decode(encoded->fmt, (const uint8_t*)encoded->arena->chunk_addr((uint32_t)encoded->chunk),
                          (uint16_t*)scratch_arena->chunk_addr(tmp), b->npages << (kPageShift - 1));
      }
      if (!ok) {
        scratch_arena->free(tmp, 1);
        return Status::IO_ERROR;
      }
    }
    struct ScratchGuard {
      HostArena* a;
      Residency* r;
      ~ScratchGuard() {
        if (a) a->free((uint32_t)r->chunk, 1);
      }
    } guard{scratch_arena, &decoded};
    // Walk page by page, coalescing by source.
    uint64_t cur = pos;
    while (cur < end) {
      uint32_t p = (uint32_t)((cur - (bi << kBlockShift)) >> kPageShift);
      uint64_t pend = std::min(end, (bi << kBlockShift) + ((uint64_t)(p + 1) << kPageShift));
      Residency* src = nullptr;
      for (auto& x : b->res)
        if (x.resident.test(p) && (!src || (!x.loc.is_gpu() && src->loc.is_gpu()))) src = &x;
      if (src && src == encoded) src = &decoded;
      char* o = out + (cur - pos);
      uint64_t n = pend - cur;
      uint64_t in_chunk = cur - (bi << kBlockShift);
      if (!src) {
        if (dst_dev < 0) memset(o, 0, n);
        else {
          Ring* rg = ring(dst_dev, RingKind::MEMOPS);
          Sqe s;
          s.op = SqeOp::MEMSET;
          s.dst = (uint64_t)o;
          s.bytes = n;
          rg->push(std::move(s));
          rg->submit()->wait();
        }
      } else if (dst_dev < 0 && !src->loc.is_gpu()) {
        memcpy(o, (const void*)(src->arena->chunk_addr((uint32_t)src->chunk) + in_chunk), n);
      } else {
        Ring* rg;
        int d = src->loc.is_gpu() ? src->loc.id : dst_dev;
        if (dst_dev < 0) {
          // GPU -> pageable host: bounce through a pinned host chunk.
          HostArena* ha = host_arena(Tier::HOST, host_node_);
          uint32_t tmp;
          Status st = ha ? alloc_chunks(ha, 1, -1, &tmp, nullptr, true) : Status::NO_MEMORY;
          if (st != Status::OK) return st;
          rg = ring(d, RingKind::GPU_TO_CPU);
          Sqe s;
          s.op = SqeOp::COPY;
          s.dst = ha->chunk_addr(tmp);
          s.src = src->arena->chunk_addr((uint32_t)src->chunk) + in_chunk;
          s.bytes = n;
          rg->push(std::move(s));
          st = rg->submit()->wait();
          memcpy(o, (const void*)ha->chunk_addr(tmp), n);
          ha->free(tmp, 1);
          if (st != Status::OK) return st;
        } else {
          rg = src->loc.is_gpu() ? (src->loc.id == dst_dev ? ring(d, RingKind::GPU_INTERNAL) : ring(d, RingKind::GPU_TO_GPU))
                                 : ring(dst_dev, RingKind::CPU_TO_GPU);
          Sqe s;
          s.op = SqeOp::COPY;
          s.dst = (uint64_t)o;
          s.src = src->arena->chunk_addr((uint32_t)src->chunk) + in_chunk;
          s.bytes = n;
          rg->push(std::move(s));
          Status st = rg->submit()->wait();
          if (st != Status::OK) return st;
        }
      }
      cur = pend;
    }
    (void)lo;
    pos = end;
  }
  return Status::OK;
}

Status Runtime::fill(Range* r, uint64_t off, uint64_t bytes, uint32_t pattern) {
  if (!r || off + bytes > r->size || (off & 3) || (bytes & 3)) return Status::INVALID_ARGUMENT;
  std::vector<uint32_t> buf(std::min<uint64_t>(bytes, kBlockSize) / 4, pattern);
  uint64_t pos = off;
  while (pos < off + bytes) {
    uint64_t n = std::min<uint64_t>(off + bytes - pos, kBlockSize - (pos & (kBlockSize - 1)));
    Status st = write(r, pos, buf.data(), n, -1);
    if (st != Status::OK) return st;
    pos += n;
  }
  return Status::OK;
}

// ------------------------------------------------------------------ introspection
uint64_t Runtime::resident_bytes(Range* r, Loc loc, uint64_t off, uint64_t len) {
  if (!r || r->type != RangeType::MANAGED || off >= r->size) return 0;
  const uint64_t end = len > r->size - off ? r->size : off + len;
  std::shared_lock<OrderedRWLock> vg(vs_.lock);
  uint64_t n = 0;
  for (uint64_t bi = off >> kBlockShift; bi <= (end - 1) >> kBlockShift; ++bi) {
    Block* b = r->block(bi);
    const uint64_t b0 = bi << kBlockShift;
    const uint64_t p0 = off > b0 ? (off - b0) >> kPageShift : 0;
    const uint64_t p1 = std::min<uint64_t>(kBlockSize, end - b0 + kPageSize - 1) >> kPageShift;
    std::lock_guard<OrderedMutex> g(b->lock);
    for (auto& x : b->res) {
      if (!(x.loc == loc)) continue;
      if (p0 == 0 && p1 == kPagesPerBlock) {
        n += (uint64_t)x.resident.count() << kPageShift;
      } else {
        for (uint64_t p = p0; p < p1; ++p) n += x.resident.test(p) ? kPageSize : 0;
      }
    }
  }
  return n;
}

Status Runtime::residency_info(Range* r, uint64_t off, ResidencyInfo* out) {
  if (!r || off >= r->size) return Status::INVALID_ARGUMENT;
  *out = ResidencyInfo{};
  if (r->type != RangeType::MANAGED) {
    out->resident_on.push_back(Loc::gpu(r->ext_dev));
    out->chunk.push_back(-1);
    out->pages.push_back((uint32_t)(std::min<uint64_t>(r->size, kBlockSize) >> kPageShift));
    out->mapped_on.push_back(r->ext_dev);
    return Status::OK;
  }
  std::shared_lock<OrderedRWLock> vg(vs_.lock);
  Block* b = r->block(off >> kBlockShift);
  std::lock_guard<OrderedMutex> g(b->lock);
  PageMask seen, dup;
  for (auto& x : b->res) {
    out->resident_on.push_back(x.loc);
    out->chunk.push_back(x.chunk);
    out->pages.push_back(x.resident.count());
    if (x.fmt == 3 && x.seg) {
      const uint32_t np = (uint32_t)__builtin_popcount(x.seg->packed);
      out->enc_bytes.push_back(x.seg->packed_bytes() + (kSegsPerBlock - np) * kSegBytes);
      out->seg_packed.push_back(np);
    } else {
      out->enc_bytes.push_back(x.fmt ? x.enc_bytes : 0);
      out->seg_packed.push_back(0);
    }
    dup |= seen & x.resident;
    seen |= x.resident;
  }
  out->read_dup = !dup.empty();
  if (!b->cpu_ro.empty() || !b->cpu_rw.empty()) out->mapped_on.push_back(kCpuProc);
  if (b->stable_chunk.load() >= 0) out->mapped_on.push_back(r->stable_dev);
  out->stable_chunk = b->stable_chunk.load();
  if (b->lease_pins)
    for (auto& x : b->res)
      if (x.loc.is_gpu()) out->mapped_on.push_back(x.loc.id);
  out->pinned = thrash_pinned(b, now_ns()) || b->user_pins > 0;
  out->thrashing = b->thrash.detected;
  out->policy = b->policy;
  return Status::OK;
}

uint16_t Runtime::register_channel(int dev, void* stream, const std::string& name) {
  if (!is_local(dev)) return 0;
  std::lock_guard<std::mutex> g(channels_m_);
  for (auto& c : channels_)
    if (c.id && c.dev == dev && c.stream == stream) return c.id;
  size_t slot = 0;
  while (slot < channels_.size() && channels_[slot].id) ++slot;
  // One cancel word per channel id (fault_abi.hpp): ids stay below
  // kFaultCancelSlots so no two channels share one. Past that a stream runs
  // unattributed (channel 0: its faults are serviced, never precisely cancelled).
  if (slot + 1 >= kFaultCancelSlots) {
    RT_WARN("register_channel: all %u channel ids in use; stream %p runs unattributed", kFaultCancelSlots - 1, stream);
    return 0;
  }
  if (slot == channels_.size()) channels_.emplace_back();
  Channel c;
  c.id = (uint16_t)(slot + 1);
  c.dev = dev;
  c.stream = stream;
  c.name = name;
  channels_[slot] = c;
  return c.id;
}

void Runtime::unregister_channel(uint16_t id) {
  std::lock_guard<std::mutex> g(channels_m_);
  if (id && id <= channels_.size()) channels_[id - 1] = Channel{};
}

uint32_t Runtime::fault_client(int dev, void* stream) {
  std::lock_guard<std::mutex> g(channels_m_);
  for (auto& c : channels_)
    if (c.id && c.dev == dev && c.stream == stream) return (uint32_t)dev | ((uint32_t)c.id << 16);
  return (uint32_t)dev;
}

std::vector<Runtime::Channel> Runtime::channels() {
  std::lock_guard<std::mutex> g(channels_m_);
  std::vector<Channel> v;
  for (auto& c : channels_)
    if (c.id) v.push_back(c);
  return v;
}

Status Runtime::check_health(int dev, bool force) {
  if (!is_local(dev)) return Status::INVALID_ARGUMENT;
  Device& d = *devs_[dev];
  std::lock_guard<std::mutex> g(d.health_m);
  uint64_t now = now_ns();
  if (!force && now - d.health_checked_ns < 20ull * 1000 * 1000) return global_status();
  d.health_checked_ns = now;
  Backend::Health h;
  if (be_->device_health(dev, &h) != Status::OK) {
    d.health_reason = be_->last_error();
    return global_status();
  }
  d.health_reason.clear();
  if (!d.health_ok) {  // counters appeared after init: take them as the baseline
    d.health0 = h;
    d.health_ok = true;
  }
  d.health = h;
  auto grew = [](int64_t now_v, int64_t base) { return now_v >= 0 && now_v > (base < 0 ? 0 : base); };
  const char* why = grew(h.ue, d.health0.ue) ? "uncorrectable ECC error"
                    : grew(h.link_ue, d.health0.link_ue) ? "uncorrectable xGMI link error" : nullptr;
  if (why && global_status() == Status::OK) {
    char msg[160];
    snprintf(msg, sizeof msg, "GPU %d: %s (ue %lld, link ue %lld since init)", dev, why,
             (long long)(h.ue - std::max<int64_t>(0, d.health0.ue)),
             (long long)(h.link_ue - std::max<int64_t>(0, d.health0.link_ue)));
    RT_ERR("%s", msg);
    tools_event(ToolsEventType::FatalFault, Cause::User, Loc::gpu(dev), Loc::gpu(dev), dev, 0, 0, 0);
    set_fatal(Status::FATAL, msg);
  }
  return global_status();
}

std::string Runtime::debug_dump(size_t max_leases) {
  std::string out;
  char buf[320];
  snprintf(buf, sizeof(buf), "[ogkm-dump] pid %d status %s%s%s\n", (int)getpid(), status_str(global_status()),
           global_status() == Status::OK ? "" : ": ", fatal_reason());
  out += buf;
  for (auto& d : devs_) {
    if (!d->local) continue;
    for (int k = 0; k < (int)RingKind::COUNT; ++k)
      if (d->rings[k]) out += "[ogkm-dump]   " + d->rings[k]->debug_state() + "\n";
  }
  if (leases_m_.try_lock()) {
    std::vector<const Lease*> ls;
    for (auto& kv : leases_) ls.push_back(kv.second.get());
    std::sort(ls.begin(), ls.end(), [](const Lease* a, const Lease* b) { return a->id < b->id; });
    snprintf(buf, sizeof(buf), "[ogkm-dump]   leases outstanding: %zu\n", ls.size());
    out += buf;
    for (size_t i = 0; i < ls.size() && i < max_leases; ++i) {
      const Lease* l = ls[i];
      snprintf(buf, sizeof(buf), "[ogkm-dump]     lease %llu range %llu '%s' [%llu, +%llu) proc %d %s chunks %zu ready_fences %zu\n",
               (unsigned long long)l->id, (unsigned long long)(l->range ? l->range->id : 0),
               l->range ? l->range->name.c_str() : "?", (unsigned long long)l->offset, (unsigned long long)l->bytes,
               l->proc, l->remote ? "remote" : "local", l->pinned_chunks.size(), l->ready.size());
      out += buf;
    }
    leases_m_.unlock();
  } else {
    out += "[ogkm-dump]   leases: (lease table locked by another thread)\n";
  }
  return out;
}

Status Runtime::sync_all() {
  Status st = Status::OK;
  for (auto& d : devs_)
    for (auto& r : d->rings) {
      if (!r) continue;
      FenceRef f = r->submit();
      Status s = f->wait();
      if (s != Status::OK && st == Status::OK) st = s;
    }
  refresh_device_tables();
  // Completed work is only trusted once the GPU reports no new uncorrectable
  // error (the post-push ECC check of uvm_gpu.c:1328-1354).
  for (auto& d : devs_)
    if (d->local && check_health(d->id) != Status::OK && st == Status::OK) st = global_status();
  return st;
}

Status Runtime::enable_peer(int a, int b) {
  if (!is_local(a) || b < 0 || b >= ndev() || a == b) return Status::INVALID_ARGUMENT;
  Status st = be_->enable_peer(a, b);
  if (st != Status::OK) return st;
  std::unique_lock<OrderedRWLock> vg(vs_.lock);
  for (auto& p : vs_.peer_pairs)
    if (p.first == a && p.second == b) return Status::OK;
  vs_.peer_pairs.emplace_back(a, b);
  return Status::OK;
}

void Runtime::set_prefetch_enabled(bool on) { config().perf_prefetch_enable = on ? 1 : 0; }

// ------------------------------------------------------------------ fault service threads
Status Runtime::start_fault_service(uint32_t poll_us) {
  std::lock_guard<std::mutex> g(fs_m_);
  if (!fs_threads_.empty()) return Status::OK;
  fs_stop_.store(false);
  for (int d = 0; d < ndev(); ++d) {
    if (!is_local(d)) continue;
    fs_threads_.emplace_back([this, d, poll_us] {
      DeviceFaultBuffer& fb = devs_[d]->fault_buf;
      while (!fs_stop_.load(std::memory_order_acquire)) {
        refresh_device_tables();
        // Top half: cheap check of the device-advanced PUT against GET.
        bool pending = fb.hdr && (__atomic_load_n(&fb.hdr->put, __ATOMIC_ACQUIRE) !=
                                      __atomic_load_n(&fb.hdr->get, __ATOMIC_RELAXED) ||
                                  __atomic_load_n(&fb.hdr->overflow, __ATOMIC_RELAXED) != fb.overflow_seen);
        if (!pending) {
          check_health(d);  // rate-limited: one sysfs scan per 20 ms at most
          std::this_thread::sleep_for(std::chrono::microseconds(poll_us ? poll_us : 50));
          continue;
        }
        // Bottom half: fetch + coalesce + service the batch.
        if (global_status() != Status::OK || quiesced_.load()) {
          std::this_thread::sleep_for(std::chrono::milliseconds(1));
          continue;
        }
        poll_device_faults(d);
        fs_batches_.fetch_add(1, std::memory_order_relaxed);
      }
    });
  }
  return Status::OK;
}

void Runtime::stop_fault_service() {
  std::lock_guard<std::mutex> g(fs_m_);
  fs_stop_.store(true);
  for (auto& t : fs_threads_) t.join();
  fs_threads_.clear();
}

// ------------------------------------------------------------------ CXL DMA
Status Runtime::cxl_dma(uint64_t handle, uint64_t gpu_ptr, int dev, uint64_t cxl_off, uint64_t size, int dir,
                        bool async, uint64_t* tid) {
  if (global_status() != Status::OK) return global_status();
  if (!is_local(dev) || !gpu_ptr || size == 0) return Status::INVALID_ARGUMENT;
  CxlBuffer buf;
  Status st = cxl_->lookup(handle, &buf);
  if (st != Status::OK) return st;
  if (cxl_off > buf.size || size > buf.size - cxl_off) return Status::INVALID_ARGUMENT;
  Ring* rg = ring(dev, RingKind::CXL);
  uint64_t piece = (uint64_t)config().cxl_max_dma_mb << 20;
  if (piece == 0) piece = size;
  uint64_t seq = 0;
  for (uint64_t o = 0; o < size; o += piece) {
    uint64_t n = std::min(piece, size - o);
    Sqe s;
    s.op = SqeOp::COPY;
    uint64_t cxl_addr = buf.base + cxl_off + o;
    if (dir & 1) {  // CXL -> GPU
      s.src = cxl_addr;
      s.dst = gpu_ptr + o;
    } else {
      s.src = gpu_ptr + o;
      s.dst = cxl_addr;
    }
    s.bytes = n;
    s.user_data = handle;
    s.file = __FILE__;
    s.line = __LINE__;
    s.desc = "cxl_dma";
    seq = rg->push(std::move(s));
  }
  rg->submit();
  Tools::get().inc(Counter::CxlDmaRequests);
  Tools::get().inc(Counter::CxlDmaBytes, size);
  tools_event(ToolsEventType::CxlDma, Cause::Cxl, (dir & 1) ? Loc::cxl(buf.numa_node) : Loc::gpu(dev),
              (dir & 1) ? Loc::gpu(dev) : Loc::cxl(buf.numa_node), dev, buf.base + cxl_off, size, 0);
  *tid = ((uint64_t)dev << 56) | seq;
  if (!async) return rg->wait_seq(seq);
  return rg->error();
}

Status Runtime::cxl_dma_wait(uint64_t tid) {
  int dev = (int)(tid >> 56);
  if (!is_local(dev)) return Status::INVALID_ARGUMENT;
  return ring(dev, RingKind::CXL)->wait_seq(tid & ((1ull << 56) - 1));
}

// ------------------------------------------------------------------ quiesce / checkpoint
Status Runtime::quiesce() {
  pm_.lock();
  quiesced_.store(true);
  Status st = sync_all();
  for (int d = 0; d < ndev(); ++d) poll_device_faults(d);
  std::shared_lock<OrderedRWLock> vg(vs_.lock);
  for (auto& kv : vs_.ranges)
    for (auto& bp : kv.second->blocks) {
      std::lock_guard<OrderedMutex> g(bp->lock);
      bp->tracker.wait();
      bp->tracker.clear();
    }
  return st;
}

Status Runtime::resume() {
  if (!quiesced_.load()) return Status::INVALID_ARGUMENT;
  quiesced_.store(false);
  pm_.unlock();
  return Status::OK;
}

namespace {
constexpr char kMagic[8] = {'O', 'G', 'K', 'M', 'R', 'M', 'A', 'P'};
// v2 adds each range's CPU window address, stable device VA and its GPU (in-place restore).
constexpr uint32_t kCkptVersion = 2;
template <class T> void wr(std::ostream& o, const T& v) { o.write((const char*)&v, sizeof v); }
template <class T> bool rd(std::istream& i, T* v) { return (bool)i.read((char*)v, sizeof *v); }
}  // namespace

// Residency-map checkpoint: one record per 2 MB block with
// per-location page masks, policy, and thrash pin state; optionally the data.
Status Runtime::checkpoint_save(const std::string& path, bool with_data) {
  bool was_quiesced = quiesced_.load();
  if (!was_quiesced) {
    Status qs = quiesce();
    if (qs != Status::OK) {  // in-flight work failed: the saved map would not match memory
      resume();
      return qs;
    }
  }
  std::ofstream o(path, std::ios::binary);
  if (!o) {
    if (!was_quiesced) resume();
    return Status::IO_ERROR;
  }
  o.write(kMagic, 8);
  wr(o, kCkptVersion);
  uint32_t flags = with_data ? 1 : 0;
  wr(o, flags);
  std::vector<Range*> rs;
  {
    std::shared_lock<OrderedRWLock> vg(vs_.lock);
    for (auto& kv : vs_.ranges)
      if (kv.second->type == RangeType::MANAGED) rs.push_back(kv.second.get());
  }
  std::sort(rs.begin(), rs.end(), [](Range* a, Range* b) { return a->id < b->id; });
  uint64_t n = rs.size();
  wr(o, n);
  std::vector<char> page(kBlockSize);
  for (Range* r : rs) {
    wr(o, r->id);
    wr(o, (uint32_t)r->type);
    wr(o, r->flags);
    wr(o, r->size);
    wr(o, r->nblocks);
    uint32_t nl = (uint32_t)r->name.size();
    wr(o, nl);
    o.write(r->name.data(), nl);
    uint64_t gid = r->group ? r->group->id : 0;
    uint8_t gm = r->group ? (uint8_t)r->group->migratable : 1;
    wr(o, gid);
    wr(o, gm);
    wr(o, (uint64_t)(r->cpu_view ? r->addr() : 0));
    wr(o, (uint64_t)r->dev_va);
    wr(o, (int32_t)r->stable_dev);
    {
    std::shared_lock<OrderedRWLock> vg(vs_.lock);
    for (auto& bp : r->blocks) {
      Block* b = bp.get();
      std::lock_guard<OrderedMutex> g(b->lock);
      wr(o, b->index);
      wr(o, b->npages);
      uint8_t rdup = b->policy.read_dup, hp = b->policy.has_preferred, pt = (uint8_t)b->policy.preferred.tier;
      int16_t pid = b->policy.preferred.id;
      wr(o, rdup);
      wr(o, hp);
      wr(o, pt);
      wr(o, pid);
      wr(o, b->policy.accessed_by);
      uint8_t pinned = thrash_pinned(b, now_ns());
      wr(o, pinned);
      uint32_t nres = (uint32_t)b->res.size();
      wr(o, nres);
      for (auto& x : b->res) {
        uint8_t t = (uint8_t)x.loc.tier;
        wr(o, t);
        wr(o, x.loc.id);
        o.write((const char*)x.resident.w, sizeof x.resident.w);
      }
    }
    }  // block table written; read() below takes the VA-space lock itself
    if (with_data) {
      for (auto& bp : r->blocks) {
        uint64_t bytes = (uint64_t)bp->npages << kPageShift;
        Status st = read(r, bp->block_offset(), page.data(), std::min(bytes, r->size - bp->block_offset()), -1);
        if (st != Status::OK) {
          if (!was_quiesced) resume();
          return st;
        }
        o.write(page.data(), std::min(bytes, r->size - bp->block_offset()));
      }
    }
  }
  tools_event(ToolsEventType::Checkpoint, Cause::User, Loc{}, Loc{}, kCpuProc, 0, n, 0);
  if (!was_quiesced) resume();
  return o ? Status::OK : Status::IO_ERROR;
}

Status Runtime::checkpoint_load(const std::string& path, bool with_data, std::vector<uint64_t>* new_ids,
                                bool in_place) {
  std::ifstream in(path, std::ios::binary);
  if (!in) return Status::NOT_FOUND;
  char magic[8];
  in.read(magic, 8);
  if (!in || memcmp(magic, kMagic, 8) != 0) return Status::INVALID_ARGUMENT;
  uint32_t ver = 0, flags = 0;
  rd(in, &ver);
  rd(in, &flags);
  if (ver != 1 && ver != kCkptVersion) return Status::NOT_SUPPORTED;
  if (in_place && ver < 2) return Status::NOT_SUPPORTED;  // v1 files carry no addresses
  bool has_data = flags & 1;
  uint64_t n = 0;
  rd(in, &n);
  std::vector<char> page(kBlockSize);
  // All or nothing: a failure part-way (an id or address taken, a short
  // file) frees every range this call created, so a caller falling back to a
  // relocating restore does not end up with duplicates of the first ones.
  std::vector<Range*> created;
  const size_t ids0 = new_ids ? new_ids->size() : 0;
  auto fail = [&](Status st) {
    for (Range* x : created) free_range(x);
    if (new_ids) new_ids->resize(ids0);
    return st;
  };
  for (uint64_t i = 0; i < n; ++i) {
    uint64_t id, size, nblocks, gid;
    uint32_t type, rflags, nl;
    uint8_t gm;
    if (!rd(in, &id) || !rd(in, &type) || !rd(in, &rflags) || !rd(in, &size) || !rd(in, &nblocks) ||
        !rd(in, &nl))
      return fail(Status::IO_ERROR);
    std::string name(nl, '\0');
    in.read(&name[0], nl);
    rd(in, &gid);
    rd(in, &gm);
    uint64_t cpu_addr = 0, dev_va = 0;
    int32_t sdev = -1;
    if (ver >= 2) {
      rd(in, &cpu_addr);
      rd(in, &dev_va);
      rd(in, &sdev);
    }
    Range* r = nullptr;
    Status st = in_place ? malloc_managed_at(size, rflags, name, id, cpu_addr, dev_va, sdev, &r)
                         : malloc_managed(size, rflags & ~RANGE_STABLE_VA, name, &r, 0);
    if (st != Status::OK) return fail(st);
    created.push_back(r);
    if (new_ids) new_ids->push_back(r->id);
    struct BlockRec {
      Policy pol;
      std::vector<std::pair<Loc, PageMask>> res;
    };
    std::vector<BlockRec> recs(nblocks);
    for (uint64_t k = 0; k < nblocks; ++k) {
      uint64_t idx;
      uint32_t np, nres;
      uint8_t rdup, hp, pt, pinned;
      int16_t pid;
      uint64_t ab;
      rd(in, &idx);
      rd(in, &np);
      rd(in, &rdup);
      rd(in, &hp);
      rd(in, &pt);
      rd(in, &pid);
      rd(in, &ab);
      rd(in, &pinned);
      rd(in, &nres);
      if (!in || idx >= nblocks) return fail(Status::IO_ERROR);
      recs[idx].pol.read_dup = rdup;
      recs[idx].pol.has_preferred = hp;
      recs[idx].pol.preferred = Loc{(Tier)pt, pid};
      recs[idx].pol.accessed_by = ab;
      for (uint32_t q = 0; q < nres; ++q) {
        uint8_t t;
        int16_t lid;
        PageMask m;
        rd(in, &t);
        rd(in, &lid);
        in.read((char*)m.w, sizeof m.w);
        recs[idx].res.emplace_back(Loc{(Tier)t, lid}, m);
      }
    }
    for (uint64_t k = 0; k < nblocks; ++k) {
      Block* b = r->block(k);
      std::lock_guard<OrderedMutex> g(b->lock);
      b->policy = recs[k].pol;
    }
    if (has_data) {
      for (uint64_t k = 0; k < nblocks; ++k) {
        uint64_t boff = k << kBlockShift;
        uint64_t bytes = std::min<uint64_t>(kBlockSize, size - boff);
        in.read(page.data(), bytes);
        if (!in) return fail(Status::IO_ERROR);
        if (!with_data) continue;
        // Restore data at the first recorded location, then re-create copies.
        const auto& rs = recs[k].res;
        if (rs.empty()) continue;
        Loc primary = rs.front().first;
        bool ok_loc = arena_for(primary) != nullptr;
        {
          std::lock_guard<OrderedMutex> g(r->block(k)->lock);
          Policy saved = r->block(k)->policy;
          r->block(k)->policy.has_preferred = ok_loc;
          if (ok_loc) r->block(k)->policy.preferred = primary;
          (void)saved;
        }
        // write() honours the (temporary) preferred location.
        st = write(r, boff, page.data(), bytes, -1);
        {
          std::lock_guard<OrderedMutex> g(r->block(k)->lock);
          r->block(k)->policy = recs[k].pol;
        }
        if (st != Status::OK) return fail(st);
        for (size_t q = 1; q < rs.size(); ++q) {
          if (!arena_for(rs[q].first)) continue;
          Tracker t;
          uint32_t first = rs[q].second.next_set(0);
          if (first >= kPagesPerBlock) continue;
          // Re-create the duplicate copy (read duplication) of the recorded pages.
          Ctx c;
          {
            std::shared_lock<OrderedRWLock> vg(vs_.lock);
            Block* b = r->block(k);
            std::lock_guard<OrderedMutex> g(b->lock);
            st = make_resident(c, b, rs[q].second, rs[q].first, true, Cause::User);
          }
          finish_ctx(c, &t);
          t.wait();
          if (st != Status::OK && st != Status::MORE_PROCESSING_REQUIRED) return fail(st);
        }
      }
    }
    if (gid) {
      uint64_t ng;
      create_range_group(&ng);
      set_range_group(r, ng);
      set_group_migratable(ng, gm);
    }
  }
  return Status::OK;
}

}  // namespace ogkm
