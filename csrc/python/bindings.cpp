// pybind11 bindings: the `_ogkm` extension module (loaded by
// open-gpu-kernel-modules_amd/_native.py). Thin: every call maps to one Runtime
// operation; Status codes become Python exceptions with the status name.
#include <pybind11/pybind11.h>
#include <pybind11/numpy.h>
#include <pybind11/stl.h>

#include <hip/hip_runtime.h>

#include <atomic>
#include <map>
#include <shared_mutex>
#include <cstring>

#include "ogkm/codec.hpp"
#include "ogkm/kernels.hpp"
#include "ogkm/lock_order.hpp"
#include "ogkm/runtime.hpp"
#include "ogkm/unit_stream.hpp"
#include "ogkm/ledger.hpp"
#include "ogkm/torch_alloc.hpp"

namespace py = pybind11;
using namespace ogkm;


namespace {

std::atomic<uint64_t> g_dgemm_fixups{0};

struct StatusError : std::runtime_error {
  using std::runtime_error::runtime_error;
};

void check(Status s, const char* what) {
  if (s != Status::OK) throw StatusError(std::string(what) + ": " + status_str(s));
}

Runtime* rt() {
  Runtime* r = Runtime::get();
  if (!r) throw StatusError("runtime not initialised: call ogkm.rt.init()");
  return r;
}

Ring* ring_of(int dev, int kind) {
  if (kind < 0 || kind >= (int)RingKind::COUNT) throw StatusError("bad ring kind");
  Ring* r = rt()->ring(dev, (RingKind)kind);
  if (!r) throw StatusError("gpu " + std::to_string(dev) + " is not managed by this process (local_devices)");
  return r;
}

Range* range(uint64_t id) {
  Range* r = rt()->range_by_id(id);
  if (!r) throw StatusError("unknown range id " + std::to_string(id));
  return r;
}

Loc make_loc(int tier, int id) {
  if (tier < 0 || tier > 2) throw StatusError("bad tier");
  return Loc{(Tier)tier, (int16_t)id};
}

py::dict loc_dict(const Loc& l) {
  py::dict d;
  d["tier"] = tier_str(l.tier);
  d["id"] = l.id;
  return d;
}

// ---- DLPack (ABI-compatible definitions; consumed by torch.from_dlpack)
struct DLDevice { int32_t device_type; int32_t device_id; };
struct DLDataType { uint8_t code; uint8_t bits; uint16_t lanes; };
struct DLTensor {
  void* data;
  DLDevice device;
  int32_t ndim;
  DLDataType dtype;
  int64_t* shape;
  int64_t* strides;
  uint64_t byte_offset;
};
struct DLManagedTensor {
  DLTensor dl_tensor;
  void* manager_ctx;
  void (*deleter)(DLManagedTensor*);
};
struct DLCtx {
  std::vector<int64_t> shape;
  uint64_t range_id = 0;
};

void dl_deleter(DLManagedTensor* t) {
  auto* c = (DLCtx*)t->manager_ctx;
  if (c->range_id)
    if (Runtime* r = Runtime::get())
      if (Range* rg = r->range_by_id(c->range_id)) rg->views.fetch_sub(1);
  delete c;
  delete t;
}

void capsule_destructor(PyObject* cap) {
  if (PyCapsule_IsValid(cap, "dltensor")) {
    auto* t = (DLManagedTensor*)PyCapsule_GetPointer(cap, "dltensor");
    if (t && t->deleter) t->deleter(t);
  }
}

py::object make_capsule(uint64_t ptr, std::vector<int64_t> shape, int code, int bits, int device_type, int device_id,
                        uint64_t range_id) {
  auto* t = new DLManagedTensor();
  auto* c = new DLCtx();
  c->shape = std::move(shape);
  // Tensor views do not pin the range (only leases do): a view is valid while
  // its lease / buffer is, like any pointer into a freed allocation.
  c->range_id = 0;
  (void)range_id;
  t->dl_tensor.data = (void*)ptr;
  t->dl_tensor.device = DLDevice{device_type, device_id};
  t->dl_tensor.ndim = (int32_t)c->shape.size();
  t->dl_tensor.dtype = DLDataType{(uint8_t)code, (uint8_t)bits, 1};
  t->dl_tensor.shape = c->shape.data();
  t->dl_tensor.strides = nullptr;
  t->dl_tensor.byte_offset = 0;
  t->manager_ctx = c;
  t->deleter = dl_deleter;
  return py::reinterpret_steal<py::object>(PyCapsule_New(t, "dltensor", capsule_destructor));
}

class PyTracker {
 public:
  Tracker t;
  void wait() {
    py::gil_scoped_release nogil;
    check(t.wait(), "tracker wait");
  }
  bool query() { return t.query(); }
  void gpu_wait(uint64_t stream) { check(t.gpu_wait(rt()->be(), (void*)stream), "tracker gpu_wait"); }
  size_t size() const { return t.size(); }
};

}  // namespace

PYBIND11_MODULE(_ogkm, m) {
  m.doc() = "ogkm: MI355X-native unified-memory + CXL tiering runtime (native core)";
  py::register_exception<StatusError>(m, "RuntimeStatusError");

  py::class_<PyTracker>(m, "Tracker")
      .def(py::init<>())
      .def("wait", &PyTracker::wait)
      .def("query", &PyTracker::query)
      .def("gpu_wait", &PyTracker::gpu_wait)
      .def("__len__", &PyTracker::size);

  // ---- lifecycle
  m.def("init", [](const std::string& backend, int fake_devices, uint64_t fake_hbm_mb) {
    Runtime* r = Runtime::init(backend, fake_devices, fake_hbm_mb << 20);
    if (!r) throw StatusError("no backend available for '" + backend + "'");
    return std::string(r->be()->name());
  }, py::arg("backend") = "auto", py::arg("fake_devices") = 2, py::arg("fake_hbm_mb") = 256);
  m.def("shutdown", [] {
    py::gil_scoped_release nogil;
    Runtime::shutdown();
  });
  m.def("is_initialized", [] { return Runtime::get() != nullptr; });
  m.def("backend_name", [] { return std::string(rt()->be()->name()); });
  m.def("device_count", [] { return rt()->ndev(); });
  m.def("local_devices", [] { return rt()->local_devices(); });
  m.def("host_node", [] { return rt()->host_node(); });
  m.def("device_numa_node", [](int d) { return rt()->dev(d).numa; });
  m.def("global_status", [] { return std::string(status_str(global_status())); });
  m.def("clear_fatal_for_test", [] { clear_fatal_for_test(); });
  // Sticky fatal error raised outside the core (e.g. a failed / timed-out RCCL
  // collective, parallel/comm.py): every later runtime entry point fails fast
  // (uvm_global_set_fatal_error_impl, uvm_global.c:420-438).
  m.def("set_fatal", [](const std::string& why) { set_fatal(Status::FATAL, why.c_str()); });
  m.def("fatal_reason", [] { return std::string(fatal_reason()); });
  m.def("init_device", [](int d, uint64_t budget) { check(rt()->init_device(d, budget), "init_device"); });
  m.def("debug_dump", [](size_t max_leases) {
    Runtime* rt = Runtime::get();
    return rt ? rt->debug_dump(max_leases) : std::string("[ogkm-dump] runtime not initialised\n");
  }, py::arg("max_leases") = 24, py::call_guard<py::gil_scoped_release>());
  m.def("sync_all", [] {
    py::gil_scoped_release nogil;
    check(rt()->sync_all(), "sync_all");
  });

  // ---- config
  m.def("configure", [](const std::string& name, int64_t v) {
    std::lock_guard<std::mutex> g(config_mutex());
    if (!config().set(name, v)) throw StatusError("unknown config knob " + name);
    if (name == "lock_check") lockcheck::set_enabled(v != 0);
  });
  m.def("get_config", [](const std::string& name) {
    int64_t v;
    if (!config().get(name, &v)) throw StatusError("unknown config knob " + name);
    return v;
  });
  m.def("config_names", [] { return config().names(); });
  m.def("config_reset", [] {
    std::lock_guard<std::mutex> g(config_mutex());
    config().reset();
    lockcheck::set_enabled(config().lock_check != 0);
  });
  m.def("config_doc", [](const std::string& n) { return config().doc(n); });
  m.def("set_log_level", [](int l) { set_log_level((LogLevel)l); });

  // ---- ranges
  m.def("malloc_managed", [](uint64_t size, uint32_t flags, const std::string& name, int stable_dev) {
    Range* r;
    check(rt()->malloc_managed(size, flags, name, &r, stable_dev), "malloc_managed");
    return r->id;
  }, py::arg("size"), py::arg("flags") = 0, py::arg("name") = "", py::arg("stable_dev") = 0);
  m.def("free", [](uint64_t id) {
    py::gil_scoped_release nogil;
    check(rt()->free_range(range(id)), "free");
  });
  m.def("map_external", [](uint64_t ptr, uint64_t size, int dev, const std::string& name) {
    Range* r;
    check(rt()->map_external(ptr, size, dev, name, &r), "map_external");
    return r->id;
  });
  m.def("alloc_device_p2p", [](uint64_t size, int dev, const std::string& name) {
    Range* r;
    check(rt()->alloc_device_p2p(size, dev, name, &r), "alloc_device_p2p");
    return r->id;
  });
  m.def("range_info", [](uint64_t id) {
    Range* r = range(id);
    py::dict d;
    d["id"] = r->id;
    d["size"] = r->size;
    d["addr"] = r->addr();
    d["nblocks"] = r->nblocks;
    d["type"] = range_type_str(r->type);
    d["name"] = r->name;
    d["dev_va"] = (uint64_t)r->dev_va;
    d["stable_dev"] = r->stable_dev;
    d["ext_ptr"] = r->ext_ptr;
    d["views"] = r->views.load();
    d["group"] = r->group ? r->group->id : 0;
    return d;
  });
  m.def("find_range", [](uint64_t addr) -> int64_t {
    Range* r = rt()->find_range(addr);
    return r ? (int64_t)r->id : -1;
  });
  m.def("range_ids", [] {
    std::vector<uint64_t> ids;
    std::shared_lock<OrderedRWLock> g(rt()->vs().lock);
    for (auto& kv : rt()->vs().ranges) ids.push_back(kv.first);
    return ids;
  });

  // ---- policy / migration
  m.def("mem_advise", [](uint64_t id, uint64_t off, uint64_t len, int advice, int tier, int loc, int proc) {
    check(rt()->mem_advise(range(id), off, len, (Advice)advice, make_loc(tier, loc), proc), "mem_advise");
  });
  // floor > 0 (next-use mode): the op-clock time the data is needed at; the
  // prefetch evicts only data needed later (VictimFloor), else it is refused
  // (NO_MEMORY) and the caller faults the data in at its use instead.
  m.def("prefetch", [](uint64_t id, uint64_t off, uint64_t len, int tier, int loc, uint64_t floor) {
    auto t = std::make_unique<PyTracker>();
    Status s;
    {
      py::gil_scoped_release nogil;
      VictimFloor vf(floor);
      s = rt()->prefetch(range(id), off, len, make_loc(tier, loc), &t->t, Cause::Prefetch);
    }
    check(s, "prefetch");
    return t;
  }, py::arg("id"), py::arg("off"), py::arg("len"), py::arg("tier"), py::arg("loc"), py::arg("floor") = 0);
  m.def("resident_bytes", [](uint64_t id, int tier, int loc, uint64_t off, uint64_t len) {
    Range* r = range(id);
    py::gil_scoped_release nogil;
    return rt()->resident_bytes(r, make_loc(tier, loc), off, len);
  }, py::arg("id"), py::arg("tier"), py::arg("loc"), py::arg("off") = 0, py::arg("len") = ~0ull);
  m.def("hint_next_use", [](uint64_t id, uint64_t when) { rt()->hint_next_use(range(id), when); });
  // Page-granular write invalidation (what the transparent mode's op holds do
  // for the byte intervals an op writes): the other copies of those pages go.
  m.def("invalidate_others", [](uint64_t id, const std::vector<std::pair<uint64_t, uint64_t>>& bytes, int gpu) {
    Range* r = range(id);
    py::gil_scoped_release nogil;
    check(rt()->invalidate_others(r, bytes, gpu), "invalidate_others");
  });
  m.def("node_ledger", [](int max_nodes) {
    NodeLedger& L = NodeLedger::get();
    py::dict d;
    d["attached"] = L.attached();
    d["path"] = L.path();
    d["refusals"] = L.refusals();
    py::list nodes;
    for (int n = 0; n < max_nodes && n < kMaxNodes; ++n) {
      auto v = L.view(n);
      py::dict e;
      e["node"] = n;
      e["capacity"] = v.capacity;
      e["reserved"] = v.reserved;
      e["mine"] = v.mine;
      nodes.append(e);
    }
    d["nodes"] = nodes;
    return d;
  }, py::arg("max_nodes") = 8);
  // Raw ledger operations (no runtime needed): the multi-process attach / reserve stress test.
  m.def("ledger_attach", [] { return NodeLedger::get().attach() == Status::OK; });
  m.def("ledger_reserve", [](int node, uint64_t bytes) { return NodeLedger::get().reserve(node, bytes); });
  m.def("ledger_release", [](int node, uint64_t bytes) { NodeLedger::get().release(node, bytes); });
  m.def("ledger_detach", [] { NodeLedger::get().detach(); });
  // Native per-unit fault / prefetch protocol of a cyclic consumer (TieredLlama, planner off).
  py::class_<UnitStream>(m, "UnitStream")
      .def(py::init([](int dev, const std::vector<uint64_t>& ids, uint64_t window, bool next_use, uint32_t max_ahead) {
             std::vector<Range*> rs;
             for (uint64_t id : ids) rs.push_back(range(id));
             return new UnitStream(rt(), dev, std::move(rs), window, next_use, max_ahead);
           }),
           py::arg("dev"), py::arg("ranges"), py::arg("window_bytes"), py::arg("next_use"), py::arg("max_ahead"))
      // on_stream: `stream` (0 = the null stream) waits GPU-side; False: the host waits
      .def("use", [](UnitStream& u, uint32_t pos, uint64_t stream, bool on_stream) {
             Lease* l = nullptr;
             Status s;
             {
               py::gil_scoped_release nogil;
               s = u.use(pos, (void*)stream, &l, on_stream);
             }
             check(s, "unit use");
             return py::make_tuple(l->id, l->dptr);
           }, py::arg("pos"), py::arg("stream"), py::arg("on_stream") = true)
      .def("release", [](UnitStream& u, uint64_t lid, uint64_t stream, bool on_stream) {
             Lease* l = rt()->lease_by_id(lid);
             if (!l) throw StatusError("unknown lease");
             py::gil_scoped_release nogil;
             check(u.release(l, (void*)stream, on_stream), "unit release");
           }, py::arg("lid"), py::arg("stream"), py::arg("on_stream") = true)
      .def("prefetch_window", [](UnitStream& u) {
             py::gil_scoped_release nogil;
             u.prefetch_window();
           })
      .def("stats", [](UnitStream& u) {
             const auto st = u.stats();
             py::dict d;
             d["prefetched"] = st.prefetched;
             d["refused"] = st.refused;
             d["demand"] = st.demand;
             d["prefetch_ms"] = st.prefetch_ns / 1e6;
             d["acquire_ms"] = st.acquire_ns / 1e6;
             d["ahead_wait_ms"] = st.ahead_wait_ns / 1e6;
             d["hint_ms"] = st.hint_ns / 1e6;
             d["wait_ms"] = st.wait_ns / 1e6;
             d["use_ms"] = st.use_ns / 1e6;
             d["held"] = st.held;
             d["hold_drops"] = st.hold_drops;
             d["quiet_passes"] = st.quiet_passes;
             d["loud_streaming"] = st.loud_streaming;
             d["loud_evictions"] = st.loud_evictions;
             d["pressure_calls"] = st.pressure_calls;
             return d;
           })
      .def("reset_stats", &UnitStream::reset_stats);
  // Packed host copies (packer.cpp).
  m.def("pack_wait", [](uint64_t timeout_ms) {
    py::gil_scoped_release nogil;
    return rt()->pack_wait(timeout_ms);
  }, py::arg("timeout_ms") = 60000);
  m.def("pack_stats", []() {
    Runtime::PackStats st;
    {
      py::gil_scoped_release nogil;
      st = rt()->pack_stats();
    }
    py::dict d;
    d["queued"] = st.queued;
    d["busy"] = st.busy;
    d["threads"] = st.threads;
    d["packed_blocks"] = st.packed_blocks;
    d["packed_bytes"] = st.packed_bytes;
    d["raw_bytes"] = st.raw_bytes;
    d["seg_blocks"] = st.seg_blocks;
    d["seg_packed"] = st.seg_packed;
    d["seg_raw"] = st.seg_raw;
    return d;
  });
  m.def("spread_class", [](int dev, uint64_t id) { return rt()->spread_class(dev, id); });
  m.def("spread_stats", [](int dev) {
    auto st = rt()->spread_stats(dev);
    py::dict d;
    d["ready"] = st.ready;
    d["ranges"] = st.ranges;
    d["cycle_bytes"] = st.cycle_bytes;
    d["keep_ranges"] = st.keep_ranges;
    d["keep_bytes"] = st.keep_bytes;
    d["passes"] = st.passes;
    d["keep_evictions"] = st.keep_evictions;
    d["adaptations"] = st.adaptations;
    d["keep_fraction"] = st.keep_fraction;
    d["window_reserve"] = st.window_reserve;
    d["last_pass_keep_evictions"] = st.last_pass_keep_evictions;
    return d;
  });
  m.def("set_op_clock", [](int dev, uint64_t now) { rt()->set_op_clock(dev, now); });
  m.def("reset_op_clock", [](int dev) { rt()->reset_op_clock(dev); });
  m.def("migrate", [](uint64_t id, uint64_t off, uint64_t len, int tier, int loc) {
    Range* r = range(id);
    py::gil_scoped_release nogil;
    check(rt()->migrate_sync(r, off, len, make_loc(tier, loc)), "migrate");
  });
  m.def("evict", [](uint64_t id, int tier, int loc) {
    Range* r = range(id);
    py::gil_scoped_release nogil;
    check(rt()->evict_range(r, make_loc(tier, loc)), "evict");
  });
  m.def("create_range_group", [] {
    uint64_t g;
    check(rt()->create_range_group(&g), "create_range_group");
    return g;
  });
  m.def("set_range_group", [](uint64_t id, uint64_t g) { check(rt()->set_range_group(range(id), g), "set_range_group"); });
  m.def("set_group_migratable", [](uint64_t g, bool mig) {
    check(rt()->set_group_migratable(g, mig), "set_group_migratable");
  });

  // ---- leases
  m.def("acquire", [](uint64_t id, uint64_t off, uint64_t len, int proc, int access, bool allow_remote) {
    Range* r = range(id);
    Lease* l = nullptr;
    Status s;
    {
      py::gil_scoped_release nogil;
      s = rt()->acquire(r, off, len, proc, (Access)access, &l, allow_remote);
    }
    check(s, "acquire");
    py::dict d;
    d["id"] = l->id;
    d["dptr"] = l->dptr;
    d["remote"] = l->remote;
    d["pending"] = l->ready.size();
    return d;
  }, py::arg("id"), py::arg("off"), py::arg("len"), py::arg("proc"), py::arg("access"),
     py::arg("allow_remote") = true);
  // on_stream: GPU-side dependency of `stream` (0 = the null stream) on the
  // lease's copies - the host never blocks. Otherwise the host waits.
  m.def("lease_wait", [](uint64_t lid, uint64_t stream, bool on_stream) {
    Lease* l = rt()->lease_by_id(lid);
    if (!l) throw StatusError("unknown lease");
    if (on_stream) check(l->ready.gpu_wait(rt()->be(), (void*)stream), "lease gpu_wait");
    else {
      py::gil_scoped_release nogil;
      check(l->ready.wait(), "lease wait");
    }
  }, py::arg("lease"), py::arg("stream"), py::arg("on_stream") = false);
  m.def("release", [](uint64_t lid, uint64_t stream) {
    Lease* l = rt()->lease_by_id(lid);
    if (!l) throw StatusError("unknown lease");
    check(rt()->release(l, (void*)stream), "release");
  });
  m.def("service_faults", [](std::vector<std::tuple<uint64_t, uint64_t, uint64_t, int, int>> fs) {
    std::vector<FaultEntry> faults;
    for (auto& f : fs) {
      FaultEntry e;
      e.range_id = std::get<0>(f);
      e.offset = std::get<1>(f);
      e.bytes = std::get<2>(f);
      e.proc = std::get<3>(f);
      e.access = (Access)std::get<4>(f);
      e.ts_ns = now_ns();
      faults.push_back(e);
    }
    py::gil_scoped_release nogil;
    Tracker t;
    Status s = rt()->service_faults(faults, &t);
    t.wait();
    check(s, "service_faults");
  });
  m.def("cpu_fault", [](uint64_t addr, bool write) { check(rt()->cpu_fault(addr, write), "cpu_fault"); });
  m.def("poll_device_faults", [](int dev) {
    py::gil_scoped_release nogil;
    return rt()->poll_device_faults(dev);
  });
  m.def("start_fault_service", [](uint32_t poll_us) { check(rt()->start_fault_service(poll_us), "start_fault_service"); },
        py::arg("poll_us") = 50);
  m.def("stop_fault_service", [] {
    py::gil_scoped_release nogil;
    rt()->stop_fault_service();
  });
  m.def("fault_service_batches", [] { return rt()->fault_service_batches(); });
  m.def("device_table", [](uint64_t id) {
    DeviceResidencyTable* t;
    check(rt()->device_table(range(id), &t), "device_table");
    return (uint64_t)t->entries;
  });
  m.def("managed_gather", [](uint64_t id, uint64_t rows_dptr, uint32_t nrows, uint32_t row_bytes, uint64_t out_dptr,
                             int dev, uint64_t stream) {
    Runtime* r = rt();
    if (r->be()->is_fake()) throw StatusError("managed_gather needs the HIP backend");
    Range* rg = range(id);
    DeviceResidencyTable* t;
    check(r->device_table(rg, &t), "device_table");
    DeviceFaultBuffer& fb = r->dev(dev).fault_buf;
    KFaultBuf kfb{fb.hdr, fb.recs, fb.entries};
    hipError_t e = launch_managed_gather(t->entries, rg->id, (const int64_t*)rows_dptr, nrows, row_bytes,
                                         (void*)out_dptr, kfb, r->fault_client(dev, (void*)stream),
                                         (hipStream_t)stream);
    if (e != hipSuccess) throw StatusError(std::string("managed_gather launch: ") + hipGetErrorString(e));
  });
  // Fault gate: a one-wave kernel that stalls the stream until blocks covering
  // [off, off+len) of the range are HBM-resident (records faults, waits for the
  // replay token). status_dptr: device uint32[2] {0 ok / 2 cancelled, replays}.
  m.def("fault_gate", [](uint64_t id, uint64_t off, uint64_t len, int dev, uint64_t stream, uint64_t status_dptr,
                         uint32_t timeout_ms, bool write) {
    Runtime* r = rt();
    if (r->be()->is_fake()) throw StatusError("fault_gate needs the HIP backend");
    Range* rg = range(id);
    if (len == 0 || off + len > rg->size || !status_dptr) throw StatusError("fault_gate: bad span");
    DeviceResidencyTable* t;
    check(r->device_table(rg, &t), "device_table");
    if (t->dev != dev) throw StatusError("fault_gate: the range's device table belongs to another GPU");
    DeviceFaultBuffer& fb = r->dev(dev).fault_buf;
    KFaultBuf kfb{fb.hdr, fb.recs, fb.entries};
    uint32_t b0 = (uint32_t)(off >> kBlockShift), b1 = (uint32_t)((off + len - 1) >> kBlockShift);
    hipError_t e = launch_fault_gate(t->entries, rg->id, b0, b1 - b0 + 1, kfb, r->fault_client(dev, (void*)stream),
                                     write ? 2 : 1,
                                     timeout_ms * 1000u, (uint32_t*)status_dptr, (hipStream_t)stream);
    if (e != hipSuccess) throw StatusError(std::string("fault_gate launch: ") + hipGetErrorString(e));
  }, py::arg("id"), py::arg("off"), py::arg("len"), py::arg("dev"), py::arg("stream"), py::arg("status_dptr"),
     py::arg("timeout_ms") = 5000, py::arg("write") = false);
  m.def("table_fetch", [](uint64_t id, uint64_t off, uint64_t len, uint64_t out_dptr, int dev, uint64_t stream) {
    Runtime* r = rt();
    if (r->be()->is_fake()) throw StatusError("table_fetch needs the HIP backend");
    Range* rg = range(id);
    if (len == 0 || off + len > rg->size || !out_dptr) throw StatusError("table_fetch: bad span");
    DeviceResidencyTable* t;
    check(r->device_table(rg, &t), "device_table");
    if (t->dev != dev) throw StatusError("table_fetch: the range's device table belongs to another GPU");
    hipError_t e = launch_table_fetch(t->entries, off, len, (void*)out_dptr, 64, (hipStream_t)stream);
    if (e != hipSuccess) throw StatusError(std::string("table_fetch launch: ") + hipGetErrorString(e));
  });
  m.def("register_table_stream", [](int dev, uint64_t stream, bool on) {
    rt()->register_table_stream(dev, (void*)stream, on);
  }, py::arg("dev"), py::arg("stream"), py::arg("on") = true);
  m.def("fault_stress", [](int dev, uint32_t waves, uint32_t per_lane, uint64_t gave_up_dptr, uint64_t stream) {
    Runtime* r = rt();
    if (r->be()->is_fake()) throw StatusError("fault_stress needs the HIP backend");
    DeviceFaultBuffer& fb = r->dev(dev).fault_buf;
    KFaultBuf kfb{fb.hdr, fb.recs, fb.entries};
    hipError_t e = launch_fault_stress(kfb, waves, per_lane, (uint32_t*)gave_up_dptr, (hipStream_t)stream);
    if (e != hipSuccess) throw StatusError(std::string("fault_stress launch: ") + hipGetErrorString(e));
  });
  m.def("register_channel", [](int dev, uint64_t stream, const std::string& name) {
    uint16_t id = rt()->register_channel(dev, (void*)stream, name);
    if (!id) throw StatusError("register_channel: not a local GPU or no channel slot left");
    return id;
  }, py::arg("dev"), py::arg("stream"), py::arg("name") = "");
  m.def("unregister_channel", [](uint16_t id) { rt()->unregister_channel(id); });
  m.def("fault_client", [](int dev, uint64_t stream) { return rt()->fault_client(dev, (void*)stream); });
  m.def("channels", [] {
    py::list out;
    for (auto& c : rt()->channels()) {
      py::dict d;
      d["id"] = c.id;
      d["dev"] = c.dev;
      d["stream"] = (uint64_t)c.stream;
      d["name"] = c.name;
      d["faults"] = c.faults;
      d["remote_accesses"] = c.remote_accesses;
      d["fatal_faults"] = c.fatal_faults;
      d["cancelled_faults"] = c.cancelled_faults;
      d["error"] = status_str(c.error);
      out.append(d);
    }
    return out;
  });
  // Host-side producer (the device protocol): fake backend / tests.
  m.def("inject_device_faults", [](int dev, const std::vector<std::tuple<uint64_t, uint32_t, uint32_t, uint32_t,
                                                                         uint32_t, uint32_t>>& recs) {
    DeviceFaultBuffer& fb = rt()->dev(dev).fault_buf;
    size_t ok = 0;
    for (auto& t : recs) {
      DeviceFaultRecord r{};
      r.range_id = std::get<0>(t);
      r.block = std::get<1>(t);
      r.page = (uint16_t)std::get<2>(t);
      r.access = (uint8_t)std::get<3>(t);
      r.kind = (uint8_t)std::get<4>(t);
      r.proc = std::get<5>(t);
      ok += fault_buf_produce(fb.hdr, fb.recs, fb.entries, r);
    }
    return ok;
  });
  m.def("drain_fault_records", [](int dev, size_t max) {
    std::vector<DeviceFaultRecord> v;
    {
      py::gil_scoped_release nogil;
      rt()->drain_fault_records(dev, &v, max);
    }
    py::list out;
    for (auto& r : v) out.append(py::make_tuple(r.range_id, r.block, r.page, r.access, r.kind, r.proc));
    return out;
  }, py::arg("dev"), py::arg("max") = (size_t)1 << 20);

  // ---- data
  m.def("write", [](uint64_t id, uint64_t off, uint64_t ptr, uint64_t bytes, int src_dev) {
    Range* r = range(id);
    py::gil_scoped_release nogil;
    check(rt()->write(r, off, (const void*)ptr, bytes, src_dev), "write");
  });
  m.def("read", [](uint64_t id, uint64_t off, uint64_t ptr, uint64_t bytes, int dst_dev) {
    Range* r = range(id);
    py::gil_scoped_release nogil;
    check(rt()->read(r, off, (void*)ptr, bytes, dst_dev), "read");
  });
  m.def("fill", [](uint64_t id, uint64_t off, uint64_t bytes, uint32_t pattern) {
    Range* r = range(id);
    py::gil_scoped_release nogil;
    check(rt()->fill(r, off, bytes, pattern), "fill");
  });
  m.def("dlpack", &make_capsule, py::arg("ptr"), py::arg("shape"), py::arg("code"), py::arg("bits"),
        py::arg("device_type"), py::arg("device_id"), py::arg("range_id") = 0);

  // ---- introspection
  m.def("residency_info", [](uint64_t id, uint64_t off) {
    ResidencyInfo ri;
    check(rt()->residency_info(range(id), off, &ri), "residency_info");
    py::dict d;
    py::list res;
    for (size_t i = 0; i < ri.resident_on.size(); ++i) {
      py::dict e = loc_dict(ri.resident_on[i]);
      e["pages"] = ri.pages[i];
      e["chunk"] = ri.chunk[i];
      if (i < ri.enc_bytes.size() && ri.enc_bytes[i]) e["encoded_bytes"] = ri.enc_bytes[i];
      if (i < ri.seg_packed.size() && ri.seg_packed[i]) e["packed_segments"] = ri.seg_packed[i];
      res.append(e);
    }
    d["resident_on"] = res;
    d["mapped_on"] = ri.mapped_on;
    d["read_dup"] = ri.read_dup;
    d["pinned"] = ri.pinned;
    d["thrashing"] = ri.thrashing;
    d["read_mostly"] = ri.policy.read_dup;
    d["preferred"] = ri.policy.has_preferred ? py::object(loc_dict(ri.policy.preferred)) : py::object(py::none());
    d["accessed_by"] = ri.policy.accessed_by;
    d["stable_chunk"] = ri.stable_chunk;
    return d;
  });
  m.def("stats", [] {
    Runtime* r = rt();
    py::dict d;
    for (int c = 0; c < (int)Counter::NumCounters; ++c) d[counter_name((Counter)c)] = Tools::get().counter((Counter)c);
    d["lock_violations"] = lockcheck::violations();
    uint64_t cf_serviced = 0, cf_passed = 0;
    cpu_fault_stats(&cf_serviced, &cf_passed);
    d["cpu_faults_serviced"] = cf_serviced;  // by the CPU-fault service thread
    d["cpu_faults_passed_on"] = cf_passed;   // not ours: chained to the previous handler
    py::list arenas;
    for (int g = 0; g < r->ndev(); ++g) {
      if (!r->dev(g).hbm) continue;
      auto s = r->dev(g).hbm->stats();
      py::dict a;
      a["name"] = r->dev(g).hbm->name();
      a["capacity"] = s.capacity;
      a["allocated"] = s.allocated;
      a["peak"] = s.peak;
      a["pinned"] = s.pinned;
      a["evictions"] = s.evictions;
      a["free_chunks"] = r->dev(g).hbm->free_chunks();
      a["largest_free_run"] = r->dev(g).hbm->largest_free_run();
      a["base"] = r->dev(g).hbm->base();
      uint64_t al, pk, na, sw;
      torch_alloc_stats(g, &al, &pk, &na, &sw);
      a["torch_allocated"] = al;
      a["torch_peak"] = pk;
      const VmmSelfTest& T = r->dev(g).vmm_test;
      py::dict vt;
      vt["ran"] = T.ran;
      vt["ok"] = T.ok;
      vt["rounds"] = T.rounds;
      vt["flushed_ok"] = T.flushed_ok;
      vt["unflushed_stale"] = T.unflushed_stale;
      vt["detail"] = T.detail;
      a["vmm_selftest"] = vt;
      arenas.append(a);
    }
    for (int t = 1; t <= 2; ++t)
      for (int n = 0; n < kMaxNodes; ++n) {
        // only arenas that exist
        ChunkArena* ha = nullptr;
        if (t == 2 && !r->cxl_topology().is_cxl_node(n)) continue;
        // host_arena() creates on demand; only report created ones via arena_for on HOST nodes in use
        (void)ha;
      }
    d["arenas"] = arenas;
    py::list rings;
    for (int g = 0; g < r->ndev(); ++g)
      for (int k = 0; k < (int)RingKind::COUNT; ++k) {
        Ring* rg = r->ring(g, (RingKind)k);
        if (!rg) continue;
        py::dict x;
        x["dev"] = g;
        x["kind"] = ring_kind_str((RingKind)k);
        x["pushed"] = rg->pushed_seq();
        x["submitted"] = rg->submitted_seq();
        x["completed"] = rg->completed_seq();
        x["batches"] = rg->batches();
        x["error"] = status_str(rg->error());
        rings.append(x);
      }
    d["rings"] = rings;
    d["global_status"] = status_str(global_status());
    return d;
  });
  m.def("device_health", [](int dev) {
    Status st = rt()->check_health(dev, true);
    Device& d = rt()->dev(dev);
    std::lock_guard<std::mutex> g(d.health_m);
    auto h2d = [](const Backend::Health& h) {
      py::dict x;
      x["ue"] = h.ue;
      x["ce"] = h.ce;
      x["link_ue"] = h.link_ue;
      x["link_ce"] = h.link_ce;
      x["source"] = h.source;
      return x;
    };
    py::dict out;
    out["reported"] = d.health_ok;
    out["unreadable_reason"] = d.health_reason;
    out["baseline"] = h2d(d.health0);
    out["now"] = h2d(d.health);
    out["status"] = status_str(st);
    return out;
  });
  m.def("vmm_self_test", [](int dev) {
    Status st = rt()->vmm_self_test(dev);
    return st == Status::OK;
  });
  m.def("inject_ras", [](int64_t ue, int64_t ce, int64_t link_ue) {
    rt()->inject().ecc_ue.store(ue);
    rt()->inject().ecc_ce.store(ce);
    rt()->inject().link_ue.store(link_ue);
  });
  m.def("reset_counters", [] { Tools::get().reset_counters(); });
  m.def("arena_stats", [](int tier, int id) {
    ChunkArena* a = rt()->arena_for(make_loc(tier, id));
    if (!a) throw StatusError("no such arena");
    auto s = a->stats();
    py::dict d;
    d["capacity"] = s.capacity;
    d["allocated"] = s.allocated;
    d["peak"] = s.peak;
    d["pinned"] = s.pinned;
    d["evictions"] = s.evictions;
    d["allocs"] = s.allocs;
    d["frees"] = s.frees;
    d["used_list"] = s.used_list;
    d["unused_list"] = s.unused_list;
    d["active"] = s.active;
    d["free_chunks"] = a->free_chunks();
    d["nchunks"] = a->nchunks();
    d["base"] = a->base();
    if (!a->loc().is_gpu()) {
      auto* h = static_cast<HostArena*>(a);
      d["numa_bound"] = h->numa_bound();
      d["thp_advised"] = h->thp_advised();
    }
    return d;
  });
  m.def("arena_check", [](int tier, int id) {
    ChunkArena* a = rt()->arena_for(make_loc(tier, id));
    if (!a) throw StatusError("no such arena");
    return a->check();
  });
  m.def("ring_reap", [](int dev, int kind) {
    Cqe buf[256];
    size_t n = ring_of(dev, kind)->reap(buf, 256);
    std::vector<std::tuple<uint64_t, uint64_t, int>> out;
    for (size_t i = 0; i < n; ++i) out.emplace_back(buf[i].user_data, buf[i].seq, buf[i].status);
    return out;
  });
  m.def("ring_error", [](int dev, int kind) {
    Ring* r = ring_of(dev, kind);
    return std::make_pair(std::string(status_str(r->error())), r->last_error_desc());
  });
  m.def("ring_clear_error", [](int dev, int kind) { ring_of(dev, kind)->clear_error_for_test(); });
  m.def("ring_copy", [](int dev, int kind, uint64_t dst, uint64_t src, uint64_t bytes, bool wait) {
    // Direct ring access (used by benchmarks and the CE-style tests).
    Ring* r = ring_of(dev, kind);
    Sqe s;
    s.op = SqeOp::COPY;
    s.dst = dst;
    s.src = src;
    s.bytes = bytes;
    uint64_t seq = r->push(std::move(s));
    FenceRef f = r->submit();
    if (wait) {
      py::gil_scoped_release nogil;
      check(f->wait(), "ring_copy");
    }
    return seq;
  });
  m.def("ring_memset", [](int dev, int kind, uint64_t dst, uint32_t pattern, uint64_t bytes) {
    Ring* r = ring_of(dev, kind);
    Sqe s;
    s.op = SqeOp::MEMSET;
    s.dst = dst;
    s.pattern = pattern;
    s.bytes = bytes;
    r->push(std::move(s));
    py::gil_scoped_release nogil;
    check(r->submit()->wait(), "ring_memset");
  });
  m.def("ring_gather", [](int dev, uint64_t base, uint64_t contig, std::vector<uint32_t> idx, uint32_t page_bytes,
                          bool scatter) {
    Ring* r = ring_of(dev, (int)RingKind::GPU_INTERNAL);
    Sqe s;
    s.op = scatter ? SqeOp::SCATTER : SqeOp::GATHER;
    s.src = scatter ? contig : base;
    s.dst = scatter ? base : contig;
    s.idx = std::move(idx);
    s.page_bytes = page_bytes;
    r->push(std::move(s));
    py::gil_scoped_release nogil;
    check(r->submit()->wait(), "ring_gather");
  });
  // One submission of raw ring ops, not waited for (ordering tests): tuples
  // (op, dst, src, bytes, n_values) with op 0 = COPY, 1 = DECODE_ANS (src:
  // ANS1 chunk of `bytes`, n_values bf16 out), 2 = WAIT_FENCE on an event
  // recorded now on stream `src`. Returns the submission's tracking value.
  m.def("debug_ring_submit", [](int dev, int kind, std::vector<std::tuple<int, uint64_t, uint64_t, uint64_t, uint32_t>> ops) {
    Ring* r = ring_of(dev, kind);
    for (auto& o : ops) {
      const int op = std::get<0>(o);
      if (op == 2) {
        r->push_wait(fence_record(rt()->be(), dev, (void*)std::get<2>(o)));
        continue;
      }
      Sqe s;
      s.op = op == 1 ? SqeOp::DECODE_ANS : SqeOp::COPY;
      s.dst = std::get<1>(o);
      s.src = std::get<2>(o);
      s.bytes = std::get<3>(o);
      s.n_values = std::get<4>(o);
      r->push(std::move(s));
    }
    return r->submit()->seq;
  });
  m.def("ring_stream", [](int dev, int kind) { return (uint64_t)ring_of(dev, kind)->stream(); });
  // Peer plane: SDMA engine masks per (dst, src) pair (-1 = host) and per-engine bytes.
  m.def("copy_engine_mask", [](int dst, int src) { return rt()->be()->copy_engine_mask(dst, src); });
  m.def("engine_bytes", [](int dev) {
    uint64_t v[32];
    rt()->be()->engine_bytes(dev, v);
    return std::vector<uint64_t>(v, v + 32);
  });
  m.def("split_over_engines", [](std::vector<std::tuple<uint64_t, uint64_t, uint64_t>> copies, uint32_t mask,
                                 uint64_t min_piece) {
    std::vector<CopyDesc> in;
    for (auto& c : copies) in.push_back(CopyDesc{std::get<0>(c), std::get<1>(c), std::get<2>(c)});
    uint32_t rot = 0;
    std::vector<std::tuple<uint64_t, uint64_t, uint64_t, uint32_t>> out;
    for (auto& d : split_over_engines(in, mask, min_piece, &rot)) out.emplace_back(d.dst, d.src, d.bytes, d.engine);
    return out;
  });
  // k_peer_push on `dev`'s stream (dst may be a peer's HBM or local), bounded grid.
  m.def("peer_push", [](int dev, uint64_t stream, uint64_t dst, uint64_t src, uint64_t bytes) {
    CopyDesc d{dst, src, bytes};
    check(rt()->be()->copy_batch(dev, &d, 1, (void*)stream, 4), "peer_push");
  });
  m.def("ring_wait_seq", [](int dev, int kind, uint64_t seq) {
    Ring* r = ring_of(dev, kind);
    py::gil_scoped_release nogil;
    return std::string(status_str(r->wait_seq(seq)));
  });
  m.def("debug_stream_create", [](int dev) { return (uint64_t)rt()->be()->stream_create(dev, 0); });
  m.def("debug_stream_destroy", [](uint64_t s) { rt()->be()->stream_destroy((void*)s); });
  m.def("debug_stream_sync", [](uint64_t s) {
    py::gil_scoped_release nogil;
    rt()->be()->stream_sync((void*)s);
  });
  m.def("debug_touch", [](uint64_t s, uint64_t ptr, uint64_t bytes, uint32_t delay_us, bool write) {
    check(rt()->be()->debug_touch((void*)s, ptr, bytes, delay_us, write), "debug_touch");
  }, py::arg("stream"), py::arg("ptr"), py::arg("bytes"), py::arg("delay_us"), py::arg("write") = true);
  m.def("ring_completed", [](int dev, int kind) { return ring_of(dev, kind)->completed_seq(); });

  // ---- tools
  m.def("tools_create_queue", [](uint32_t entries, uint32_t mask, const std::string& shm) {
    return Tools::get().create_queue(entries, mask, shm);
  }, py::arg("entries") = 4096, py::arg("mask") = 0xffffffffu, py::arg("shm") = "");
  m.def("tools_destroy_queue", [](int q) { Tools::get().destroy_queue(q); });
  m.def("tools_read", [](int q, size_t max) {
    EventQueue* eq = Tools::get().queue(q);
    if (!eq) throw StatusError("bad queue");
    std::vector<ToolsEvent> ev(max);
    size_t n = eq->pop(ev.data(), max);
    return py::bytes((const char*)ev.data(), n * sizeof(ToolsEvent));
  });
  m.def("tools_dropped", [](int q) {
    EventQueue* eq = Tools::get().queue(q);
    if (!eq) throw StatusError("bad queue");
    std::vector<uint64_t> d;
    for (int i = 0; i < (int)ToolsEventType::NumTypes; ++i) d.push_back(eq->ctrl()->dropped[i].load());
    return d;
  });
  m.def("counter_names", [] {
    std::vector<std::string> n;
    for (int c = 0; c < (int)Counter::NumCounters; ++c) n.push_back(counter_name((Counter)c));
    return n;
  });

  // ---- heuristics test hooks (UVM_TEST_SET_PAGE_PREFETCH_POLICY-style introspection)
  m.def("prefetch_hint", [](std::vector<uint32_t> resident, std::vector<uint32_t> faulted, uint32_t npages,
                            uint32_t threshold) {
    PageMask r, f;
    for (auto p : resident) r.set(p);
    for (auto p : faulted) f.set(p);
    PageMask h = prefetch_hint(r, f, npages, threshold);
    std::vector<uint32_t> out;
    for (uint32_t p = h.next_set(0); p < kPagesPerBlock; p = h.next_set(p + 1)) out.push_back(p);
    return out;
  });
  m.def("bf12_encode", [](py::bytes raw) {
    std::string s = raw;
    std::string out(kBlockSize + kBf12HeaderBytes, '\0');
    uint64_t n = bf12_encode((const uint16_t*)s.data(), (uint32_t)(s.size() / 2), (uint8_t*)out.data(), out.size());
    out.resize(n);
    return py::bytes(out);
  });
  m.def("bf12_decode", [](py::bytes enc, uint32_t n_values) {
    std::string s = enc;
    std::string out((size_t)n_values * 2, '\0');
    if (!bf12_decode((const uint8_t*)s.data(), (uint16_t*)out.data(), n_values)) throw StatusError("bf12_decode: bad block");
    return py::bytes(out);
  });
  // Self-describing BF12 streams of whole tensors (ops/bf12.py).
  m.def("bf12_pack_bound", [](uint64_t n, uint32_t chunk_values) { return bf12_pack_bound(n, chunk_values); });
  m.def("bf11_encode", [](py::bytes raw) {
    std::string s = raw;
    std::string out((size_t)kBlockSize + kBf11HeaderBytes, '\0');
    uint64_t n = bf11_encode((const uint16_t*)s.data(), (uint32_t)(s.size() / 2), (uint8_t*)out.data(), out.size());
    out.resize(n);
    return py::bytes(out);
  });
  // One ANS1 chunk of a bf16 buffer (the packed host copy's format); empty when
  // it would not fit in the raw size.
  m.def("ans_encode", [](py::bytes raw) {
    std::string s = raw;
    std::string out(s.size() + 4096, '\0');
    uint64_t n = ans_encode((const uint16_t*)s.data(), (uint32_t)(s.size() / 2), (uint8_t*)out.data(), s.size());
    out.resize(n);
    return py::bytes(out);
  });
  m.def("bf11_decode", [](py::bytes enc, uint32_t n_values) {
    std::string s = enc;
    std::string out((size_t)n_values * 2, '\0');
    if (!bf11_decode((const uint8_t*)s.data(), (uint16_t*)out.data(), n_values)) throw StatusError("bf11_decode: bad block");
    return py::bytes(out);
  });
  m.def("bf12_pack", [](uint64_t src, uint64_t n_values, uint64_t dst, uint64_t cap, uint32_t chunk_values,
                        unsigned threads, uint32_t fmt) {
    uint64_t total;
    {
      py::gil_scoped_release nogil;
      total = bf12_pack((const uint16_t*)src, n_values, chunk_values, (uint8_t*)dst, cap, threads, (PackFormat)fmt);
    }
    if (!total) throw StatusError("bf12_pack: bad arguments or buffer too small");
    return total;
  }, py::arg("src"), py::arg("n_values"), py::arg("dst"), py::arg("cap"), py::arg("chunk_values"),
     py::arg("threads"), py::arg("fmt") = 1);
  m.def("bf12_unpack_host", [](uint64_t src, uint64_t dst, uint64_t n_values) {
    bool ok;
    {
      py::gil_scoped_release nogil;
      ok = bf12_unpack((const uint8_t*)src, (uint16_t*)dst, n_values);
    }
    if (!ok) throw StatusError("bf12_unpack_host: corrupt stream");
  });
  // Unpack a stream resident on device `dev` into `dst` on `stream` (k_bf12_unpack).
  m.def("bf12_unpack", [](int dev, uint64_t src, uint64_t dst, uint32_t nchunks, uint32_t chunk_values,
                          uint64_t n_values, uint64_t stream, uint32_t workgroups, uint64_t dst_stride,
                          uint32_t row_shift) {
    check(rt()->be()->unpack_bf12_stream(dev, src, dst, nchunks, chunk_values, n_values, (void*)stream, workgroups,
                                         dst_stride, row_shift),
          "bf12_unpack");
  }, py::arg("dev"), py::arg("src"), py::arg("dst"), py::arg("nchunks"), py::arg("chunk_values"),
     py::arg("n_values"), py::arg("stream") = 0, py::arg("workgroups") = 0, py::arg("dst_stride") = 0, py::arg("row_shift") = 0);
  // Same for ANS streams (k_ans_unpack).
  m.def("ans_unpack", [](int dev, uint64_t src, uint64_t dst, uint32_t nchunks, uint32_t chunk_values,
                         uint64_t n_values, uint64_t stream, uint32_t workgroups, uint64_t dst_stride,
                          uint32_t row_shift) {
    check(rt()->be()->unpack_ans_stream(dev, src, dst, nchunks, chunk_values, n_values, (void*)stream, workgroups,
                                        dst_stride, row_shift),
          "ans_unpack");
  }, py::arg("dev"), py::arg("src"), py::arg("dst"), py::arg("nchunks"), py::arg("chunk_values"),
     py::arg("n_values"), py::arg("stream") = 0, py::arg("workgroups") = 0, py::arg("dst_stride") = 0, py::arg("row_shift") = 0);
  // Decode ANS1 chunks at device addresses (the ring's DECODE_ANS / DECODE_SEGS
  // kernels: single-segment chunks run one wave each, k_ans_segs).
  m.def("decode_ans_chunks", [](int dev, const std::vector<uint64_t>& src, const std::vector<uint64_t>& dst,
                                const std::vector<uint32_t>& n_values, uint64_t stream) {
    if (src.size() != dst.size() || src.size() != n_values.size()) throw StatusError("decode_ans_chunks: sizes");
    std::vector<DecodeDesc> d;
    for (size_t i = 0; i < src.size(); ++i) d.push_back(DecodeDesc{src[i], dst[i], n_values[i]});
    check(rt()->be()->decode_ans_blocks(dev, d.data(), d.size(), (void*)stream), "decode_ans_chunks");
  }, py::arg("dev"), py::arg("src"), py::arg("dst"), py::arg("n_values"), py::arg("stream") = 0);
  m.def("decode_errors", [](bool reset) {
    uint64_t e[4];
    rt()->be()->decode_errors(e, reset);
    py::dict d;
    d["count"] = e[0];
    d["stream"] = e[1];
    d["chunk"] = e[2];
    d["detail"] = e[3];
    return d;
  }, py::arg("reset") = false);
  // Decode GEMM + fused epilogue in one call: out = epi(X . W^T) (ops/dgemm.py).
  // (ksplit, klen) exactly as lib.dgemm plans it (lds: the LDS kernel's 4 waves per K split).
  m.def("dgemm_fixups", [] { return g_dgemm_fixups.load(); });  // GEMMs whose epilogue ran in the GEMM kernel
  m.def("dgemm_plan", [](uint32_t N, uint32_t K, uint32_t target_units, bool lds) {
    uint32_t ks, kl;
    dgemm_plan(N, K, lds ? std::max<uint32_t>(1, target_units / 4) : target_units, &ks, &kl);
    return py::make_tuple(ks, kl);
  }, py::arg("N"), py::arg("K"), py::arg("target_units"), py::arg("lds") = false);
  m.def("dgemm", [](int dev, uint64_t stream, uint64_t w, uint64_t w_off, int mode, uint32_t chunk_shift,
                    uint64_t x, uint32_t ldx, uint32_t M, uint32_t N, uint32_t K, uint64_t part, uint64_t part_bytes,
                    uint32_t epi, uint64_t resid, uint32_t ldr, uint64_t out, uint32_t ldo, uint32_t target_units, uint32_t unroll,
                    int lds_x, uint32_t wg_waves, uint32_t depth, bool reduce, bool x_frag, bool out_frag,
                    uint32_t out_cols, uint32_t out_col0, uint64_t fix_cnt, uint64_t fix_cnt_len, bool direct) {
    if (N % 16 || K % 32 || ldx % 8 || !M) throw StatusError("dgemm: N % 16, K % 32, ldx % 8 and M > 0 required");
    if (epi == DGEMM_EPI_SILU_MUL && (N % 32)) throw StatusError("dgemm: SILU_MUL needs N % 32 == 0");
    DGemmArgs a{};
    a.w = (const uint8_t*)w;
    a.w_off = w_off;
    a.x = (const uint16_t*)x;
    a.part = (float*)part;
    a.M = M; a.N = N; a.K = K; a.ldx = ldx;
    // Raw weights with LDS-shared activations: a workgroup of 4 waves per row
    // block, so the same wave count needs 4x fewer K splits (OGKM_DGEMM_LDS).
    a.lds_x = (mode == DGEMM_W_RAW && lds_x > 0) ? 1 : 0;
    dgemm_plan(N, K, a.lds_x ? std::max<uint32_t>(1, target_units / 4) : target_units, &a.ksplit, &a.klen);
    a.row_blocks = (N / 16 + 3) / 4;
    a.chunk_shift = chunk_shift;
    a.unroll = unroll;
    a.wg_waves = wg_waves;
    a.depth = depth;
    a.x_frag = x_frag ? 1 : 0;
    if (x_frag && K % 32) throw StatusError("dgemm: fragment-ordered x needs K % 32 == 0");
    if (reduce && out_frag && (out_cols % 32 || out_col0 % 4 ||
                               out_col0 + (epi == DGEMM_EPI_SILU_MUL ? N / 2 : N) > out_cols))
      throw StatusError("dgemm: fragment-ordered out needs out_cols % 32 == 0 and the columns inside it");
    if ((uint64_t)a.ksplit * M * N * 4 > part_bytes) throw StatusError("dgemm: partial workspace too small");
    if (mode < DGEMM_W_RAW || mode > DGEMM_W_PACKED_BF11) throw StatusError("dgemm: bad weight mode");
    DGemmReduceArgs r{};
    r.part = a.part;
    r.ksplit = a.ksplit; r.M = M; r.N = N; r.epi = epi;
    r.resid = (const uint16_t*)resid; r.ldr = ldr; r.ldo = ldo;
    r.out = (uint16_t*)out;
    r.out_frag = out_frag ? 1 : 0;
    r.out_cols = out_cols;
    r.out_col0 = out_col0;
    if (reduce && (fix_cnt || direct)) {  // epilogue in the GEMM kernel where it can run there
      a.fix = r;
      const uint64_t need = (uint64_t)((M + 63) / 64) * a.row_blocks;
      if (direct && a.ksplit == 1 && epi != DGEMM_EPI_SILU_MUL && dgemm_fixup_ok(a, mode))
        a.direct = 1;
      else if (fix_cnt && dgemm_fixup_ok(a, mode) && need <= fix_cnt_len)
        a.fix_cnt = (uint32_t*)fix_cnt;
    }
    check(rt()->be()->dgemm(dev, a, mode, (void*)stream), "dgemm");
    g_dgemm_fixups += (a.fix_cnt || a.direct) ? 1 : 0;
    if (!reduce || a.fix_cnt || a.direct) return a.ksplit;  // deferred: the consumer (rmsnorm / rope_kv) sums the splits
    check(rt()->be()->dgemm_reduce(dev, r, (void*)stream), "dgemm_reduce");
    return a.ksplit;
  }, py::arg("dev"), py::arg("stream"), py::arg("w"), py::arg("w_off"), py::arg("mode"), py::arg("chunk_shift"),
     py::arg("x"), py::arg("ldx"), py::arg("M"), py::arg("N"), py::arg("K"), py::arg("part"), py::arg("part_bytes"),
     py::arg("epi"), py::arg("resid"), py::arg("ldr"), py::arg("out"), py::arg("ldo"), py::arg("target_units") = 2048, py::arg("unroll") = 0,
     py::arg("lds_x") = 0, py::arg("wg_waves") = 4, py::arg("depth") = 0, py::arg("reduce") = true,
     py::arg("x_frag") = false, py::arg("out_frag") = false, py::arg("out_cols") = 0, py::arg("out_col0") = 0,
     py::arg("fix_cnt") = 0, py::arg("fix_cnt_len") = 0, py::arg("direct") = false);
  // Fused decode-step ops (ops/fused.py).
  m.def("rmsnorm", [](int dev, uint64_t stream, uint64_t x, uint64_t w, uint64_t y, uint32_t rows, uint32_t dim,
                      uint32_t ldx, uint32_t ldy, float eps, uint64_t part, uint32_t ksplit, bool y_frag,
                      uint64_t ssq, uint64_t ssq_bytes) {
    if (dim % 4 || dim < 4 || dim > 16384 || ldx % 4 || ldy % 4)
      throw StatusError("rmsnorm: dim % 4, 4 <= dim <= 16384, ld % 4");
    if (y_frag && dim % 32) throw StatusError("rmsnorm: fragment-ordered output needs dim % 32 == 0");
    if (ssq && (uint64_t)rows * ((dim + kNormCols - 1) / kNormCols) * 4 > ssq_bytes)
      throw StatusError("rmsnorm: ssq scratch too small");
    ResidNormArgs a{(const float*)part, ksplit, (uint16_t*)x, (const uint16_t*)w, (uint16_t*)y, rows, dim, ldx, ldy,
                    eps, y_frag ? 1u : 0u, (float*)ssq};
    check(rt()->be()->rmsnorm(dev, a, (void*)stream), "rmsnorm");
  }, py::arg("dev"), py::arg("stream"), py::arg("x"), py::arg("w"), py::arg("y"), py::arg("rows"), py::arg("dim"),
     py::arg("ldx"), py::arg("ldy"), py::arg("eps"), py::arg("part") = 0, py::arg("ksplit") = 0,
     py::arg("y_frag") = false, py::arg("ssq") = 0, py::arg("ssq_bytes") = 0);
  m.def("rope_kv", [](int dev, uint64_t stream, uint64_t qkv, uint32_t ldqkv, uint64_t cos, uint64_t sin,
                      uint64_t q_out, uint64_t cache, uint64_t tail, uint32_t B, uint32_t hq, uint32_t hkv,
                      uint32_t hd, uint32_t T, uint32_t pos, uint32_t tail_T, uint32_t tail_pos, uint64_t part,
                      uint32_t ksplit) {
    RopeKvArgs a{(const uint16_t*)qkv, ldqkv, (const float*)cos, (const float*)sin, (uint16_t*)q_out,
                 (uint16_t*)cache, (uint16_t*)tail, B, hq, hkv, hd, T, pos, tail_T, tail_pos,
                 (const float*)part, ksplit};
    check(rt()->be()->rope_kv(dev, a, (void*)stream), "rope_kv");
  }, py::arg("dev"), py::arg("stream"), py::arg("qkv"), py::arg("ldqkv"), py::arg("cos"), py::arg("sin"),
     py::arg("q_out"), py::arg("cache"), py::arg("tail"), py::arg("B"), py::arg("hq"), py::arg("hkv"), py::arg("hd"),
     py::arg("T"), py::arg("pos"), py::arg("tail_T"), py::arg("tail_pos"), py::arg("part") = 0,
     py::arg("ksplit") = 0);
  m.def("attn_decode", [](int dev, uint64_t stream, uint64_t q, uint64_t cache, uint64_t out, uint64_t part,
                          uint64_t part_bytes, uint32_t B, uint32_t hq, uint32_t hkv, uint32_t hd, uint32_t T,
                          uint32_t len, float scale, bool out_frag, uint32_t split_tokens) {
    AttnArgs a{};
    a.out_frag = out_frag ? 1 : 0;
    const bool ws = hd == 64 || hd == 128;
    a.split_tokens = ws && split_tokens ? split_tokens : kAttnSplitTokens;
    if (a.split_tokens != 64 && a.split_tokens != 256)
      throw StatusError("attn_decode: split_tokens must be 64 or 256");
    a.q = (const uint16_t*)q;
    a.cache = (const uint16_t*)cache;
    a.out = (uint16_t*)out;
    a.B = B; a.hq = hq; a.hkv = hkv; a.hd = hd; a.T = T; a.len = len; a.scale = scale;
    a.nsplit = (len + a.split_tokens - 1) / a.split_tokens;
    const uint64_t rows = (uint64_t)B * hq * a.nsplit;
    if (rows * (hd + 2) * 4 > part_bytes) throw StatusError("attn_decode: partial workspace too small");
    a.part_o = (float*)part;
    a.part_ml = (float*)part + rows * hd;
    check(rt()->be()->attn_decode(dev, a, (void*)stream), "attn_decode");
  }, py::arg("dev"), py::arg("stream"), py::arg("q"), py::arg("cache"), py::arg("out"), py::arg("part"),
     py::arg("part_bytes"), py::arg("B"), py::arg("hq"), py::arg("hkv"), py::arg("hd"), py::arg("T"), py::arg("len"),
     py::arg("scale"), py::arg("out_frag") = false, py::arg("split_tokens") = 0);
  m.def("fault_buffer_info", [](int dev) {
    DeviceFaultBuffer& fb = rt()->dev(dev).fault_buf;
    py::dict d;
    d["header"] = (uint64_t)fb.hdr;
    d["records"] = (uint64_t)fb.recs;
    d["entries"] = fb.entries;
    d["overflows"] = fb.overflows;
    d["put"] = fb.hdr ? __atomic_load_n(&fb.hdr->put, __ATOMIC_ACQUIRE) : 0;
    d["get"] = fb.hdr ? __atomic_load_n(&fb.hdr->get, __ATOMIC_ACQUIRE) : 0;
    d["replay"] = fb.hdr ? __atomic_load_n(&fb.hdr->replay, __ATOMIC_ACQUIRE) : 0;
    py::list cancel;
    for (uint32_t i = 0; i < kFaultCancelSlots; ++i)
      cancel.append(fb.hdr ? __atomic_load_n(&fb.hdr->cancel[i], __ATOMIC_ACQUIRE) : 0u);
    d["cancel"] = cancel;
    return d;
  });

  // ---- lock checker
  m.def("lock_violations", [] { return lockcheck::violations(); });
  m.def("reset_lock_violations", [] { lockcheck::reset_violations(); });
  m.def("set_lock_check", [](bool on) { lockcheck::set_enabled(on); });
  m.def("lock_check_self_test", [] {
    // Deliberately take VA_BLOCK then VA_SPACE (inverted) and report detection.
    uint64_t before = lockcheck::violations();
    OrderedMutex blk(LockOrder::VA_BLOCK);
    OrderedRWLock vs(LockOrder::VA_SPACE);
    blk.lock();
    vs.lock_shared();
    vs.unlock_shared();
    blk.unlock();
    // A trylock out of order is legal.
    blk.lock();
    OrderedMutex blk2(LockOrder::GLOBAL);
    bool got = blk2.try_lock();
    if (got) blk2.unlock();
    blk.unlock();
    return lockcheck::violations() - before;
  });

  // ---- tools: process memory access (UVM_TOOLS_READ/WRITE_PROCESS_MEMORY,
  // uvm_tools.c:2591,2601): read / write managed memory by virtual address
  // wherever its valid copy lives (no migration of the data for the tool).
  m.def("tools_read_process_memory", [](uint64_t addr, uint64_t nbytes) {
    Runtime* r = rt();
    Range* rg = r->find_range(addr);
    if (!rg || addr + nbytes > rg->addr() + rg->size) throw StatusError("read_process_memory: not managed memory");
    std::string buf(nbytes, '\0');
    {
      py::gil_scoped_release nogil;
      check(r->read(rg, addr - rg->addr(), buf.data(), nbytes, -1), "read_process_memory");
    }
    return py::bytes(buf);
  });
  m.def("tools_write_process_memory", [](uint64_t addr, py::bytes data) {
    Runtime* r = rt();
    std::string buf = data;
    Range* rg = r->find_range(addr);
    if (!rg || addr + buf.size() > rg->addr() + rg->size) throw StatusError("write_process_memory: not managed memory");
    py::gil_scoped_release nogil;
    check(r->write(rg, addr - rg->addr(), buf.data(), buf.size(), -1), "write_process_memory");
  });
  m.def("range_push", [](const std::string& name) { rt()->be()->range_push(name.c_str()); });
  m.def("range_pop", [] { rt()->be()->range_pop(); });
  m.def("mark", [](const std::string& name) { rt()->be()->mark(name.c_str()); });

  // ---- injection
  m.def("inject", [](const std::string& kind, int64_t v) {
    Injection& in = rt()->inject();
    if (kind == "alloc_fail_after") in.alloc_fail_after.store(v);
    else if (kind == "evict_fail") in.evict_fail.store(v);
    else if (kind == "copy_drop") in.copy_drop.store(v);
    else if (kind == "peer_link_down") in.peer_link_down.store((uint64_t)v);
    else if (kind == "populate_error") in.populate_error.store(v);
    else if (kind == "host_alloc_error") in.host_alloc_error.store(v);
    else if (kind == "async_copy_error") in.async_copy_error.store(v);
    else if (kind == "tlb_mode") in.tlb_mode.store((int)v);
    else throw StatusError("unknown injection " + kind);
  });

  // ---- CXL
  m.def("cxl_info", [] {
    const CxlInfo& i = rt()->cxl_topology().info();
    py::dict d;
    d["link_up"] = i.link_up;
    d["memory_expander"] = i.memory_expander;
    d["num_devices"] = i.num_devices;
    d["max_links"] = i.max_links;
    d["link_mask"] = i.link_mask;
    d["per_link_bw_mbps"] = i.per_link_bw_mbps;
    d["cxl_version"] = i.cxl_version;
    d["remote_type"] = i.remote_type;
    d["emulated"] = i.emulated;
    d["numa_nodes"] = i.numa_nodes;
    py::list devs;
    for (auto& x : i.devices) {
      py::dict e;
      e["name"] = x.name;
      e["numa_node"] = x.numa_node;
      e["bytes"] = x.bytes;
      e["version"] = x.version;
      e["link_up"] = x.link_up;
      devs.append(e);
    }
    d["devices"] = devs;
    d["registered_buffers"] = rt()->cxl().count();
    d["pinned_bytes"] = rt()->cxl().pins().pinned();
    d["pin_budget_bytes"] = rt()->cxl().pins().max_bytes();
    return d;
  });
  m.def("cxl_rediscover", [](int emulate_node, const std::string& root, uint64_t emulate_mask) {
    rt()->cxl_topology().discover(emulate_node, root, emulate_mask);
  }, py::arg("emulate_node") = -1, py::arg("root") = "/sys", py::arg("emulate_mask") = 0);
  m.def("cxl_nearest_node", [](int from) { return rt()->cxl_topology().nearest_node(from); });
  m.def("demotion_target", [](int tier, int id) {
    Loc l = rt()->demotion_target(make_loc(tier, id));
    return py::make_tuple((int)l.tier, l.id);
  });
  m.def("cxl_set_measured_bw", [](double mbps) { rt()->cxl_topology().mutable_info().per_link_bw_mbps = mbps; });
  m.def("cxl_register", [](uint64_t base, uint64_t size, int version) {
    uint64_t h;
    check(rt()->cxl().register_buffer(base, size, version, &h), "cxl_register");
    return h;
  });
  m.def("cxl_unregister", [](uint64_t h) { check(rt()->cxl().unregister_buffer(h), "cxl_unregister"); });
  m.def("cxl_buffer", [](uint64_t h) {
    CxlBuffer b;
    check(rt()->cxl().lookup(h, &b), "cxl_buffer");
    py::dict d;
    d["base"] = b.base;
    d["size"] = b.size;
    d["version"] = b.version;
    d["page_size"] = b.page_size;
    d["backing_page"] = b.backing_page;
    d["thp_bytes"] = b.thp_bytes;
    d["numa_node"] = b.numa_node;
    d["page_refs"] = b.page_refs;
    return d;
  });
  m.def("cxl_pages", [](uint64_t h, uint64_t off, uint64_t len) {
    std::vector<CxlExtent> ex;
    check(rt()->cxl().pages(h, off, len, &ex), "cxl_pages");
    std::vector<std::pair<uint64_t, uint64_t>> out;
    for (auto& e : ex) out.emplace_back(e.addr, e.bytes);
    return out;
  });
  m.def("cxl_put_pages", [](uint64_t h) { check(rt()->cxl().put_pages(h), "cxl_put_pages"); });
  m.def("cxl_dma", [](uint64_t h, uint64_t gpu_ptr, int dev, uint64_t off, uint64_t size, int dir, bool async) {
    uint64_t tid;
    Status s;
    {
      py::gil_scoped_release nogil;
      s = rt()->cxl_dma(h, gpu_ptr, dev, off, size, dir, async, &tid);
    }
    check(s, "cxl_dma");
    return tid;
  });
  m.def("cxl_dma_wait", [](uint64_t tid) {
    py::gil_scoped_release nogil;
    check(rt()->cxl_dma_wait(tid), "cxl_dma_wait");
  });

  // ---- checkpoint / PM
  m.def("quiesce", [] {
    py::gil_scoped_release nogil;
    check(rt()->quiesce(), "quiesce");
  });
  m.def("resume", [] { check(rt()->resume(), "resume"); });
  m.def("checkpoint_save", [](const std::string& path, bool with_data) {
    py::gil_scoped_release nogil;
    check(rt()->checkpoint_save(path, with_data), "checkpoint_save");
  });
  m.def("checkpoint_load", [](const std::string& path, bool with_data, bool in_place) {
    std::vector<uint64_t> ids;
    Status s;
    {
      py::gil_scoped_release nogil;
      s = rt()->checkpoint_load(path, with_data, &ids, in_place);
    }
    check(s, "checkpoint_load");
    return ids;
  }, py::arg("path"), py::arg("with_data") = true, py::arg("in_place") = false);

  // ---- peers / export
  m.def("enable_peer", [](int a, int b) { check(rt()->enable_peer(a, b), "enable_peer"); });
  m.def("link_type", [](int a, int b) { return (int)rt()->be()->link_type(a, b); });
  m.def("can_access_peer", [](int a, int b) { return rt()->be()->can_access_peer(a, b); });
  m.def("export_dmabuf", [](uint64_t ptr, uint64_t size) {
    int fd = -1;
    uint64_t off = 0;
    check(rt()->be()->export_dmabuf((void*)ptr, size, &fd, &off), "export_dmabuf");
    return std::make_pair(fd, off);
  });
  m.def("import_dmabuf", [](int dev, int fd) {
    void* p = nullptr;
    size_t n = 0;
    check(rt()->be()->import_dmabuf(dev, fd, &p, &n), "import_dmabuf");
    return std::make_pair((uint64_t)p, (uint64_t)n);
  });
  m.def("unimport_dmabuf", [](uint64_t ptr) { check(rt()->be()->unimport_dmabuf((void*)ptr), "unimport_dmabuf"); });
  m.def("ipc_handle", [](uint64_t ptr) {
    std::string h;
    check(rt()->be()->ipc_handle((void*)ptr, &h), "ipc_handle");
    return py::bytes(h);
  });
  m.def("ipc_open", [](py::bytes h) {
    void* p = nullptr;
    check(rt()->be()->ipc_open(std::string(h), &p), "ipc_open");
    return (uint64_t)p;
  });
  m.def("ipc_close", [](uint64_t p) { rt()->be()->ipc_close((void*)p); });

  // ---- pinned host helpers (tests / CXL emulation)
  m.def("alloc_coherent", [](uint64_t bytes) {
    void* p = nullptr;
    check(rt()->be()->host_alloc_coherent(bytes, &p), "alloc_coherent");
    return (uint64_t)p;
  });
  m.def("free_coherent", [](uint64_t p) { rt()->be()->host_free_coherent((void*)p); });

  // ---- torch pluggable allocator (in-process use / tests)
  m.def("torch_alloc", [](uint64_t size, int dev, uint64_t stream) {
    return (uint64_t)torch_alloc(size, dev, (void*)stream);
  }, py::arg("size"), py::arg("dev"), py::arg("stream") = 0);
  m.def("torch_free", [](uint64_t p, int dev, uint64_t stream) { torch_free((void*)p, dev, (void*)stream); },
        py::arg("ptr"), py::arg("dev"), py::arg("stream") = 0);
  m.def("torch_park", [](uint64_t p, int dev, uint64_t stream) {
    check(torch_park((void*)p, dev, (void*)stream), "torch_park");
  }, py::arg("ptr"), py::arg("dev"), py::arg("stream") = 0);
  m.def("torch_unpark", [](uint64_t p, int dev, uint64_t stream) {
    check(torch_unpark((void*)p, dev, (void*)stream), "torch_unpark");
  }, py::arg("ptr"), py::arg("dev"), py::arg("stream") = 0);
  m.def("torch_park_all", [](int dev, uint64_t stream) { torch_park_all(dev, (void*)stream); },
        py::arg("dev"), py::arg("stream") = 0);
  // operands: [(storage_ptr, write, lo, hi, written)] - lo/hi the byte extent
  // of the op's views (hi == 0: whole allocation), written None (the whole
  // extent) or a flat int64 array of [start, end) byte pairs.
  m.def("torch_op_begin", [](py::list operands, int dev, uint64_t stream) {
    std::vector<TorchOperand> ops;
    ops.reserve(operands.size());
    for (auto item : operands) {
      auto t = item.cast<py::tuple>();
      TorchOperand o;
      o.ptr = t[0].cast<uint64_t>();
      o.write = t[1].cast<bool>();
      if (t.size() >= 4) {  // (ptr, write) alone: the whole allocation
        o.lo = t[2].cast<uint64_t>();
        o.hi = t[3].cast<uint64_t>();
      }
      if (t.size() > 4 && !t[4].is_none()) {
        auto a = t[4].cast<py::array_t<int64_t, py::array::c_style | py::array::forcecast>>();
        auto r = a.unchecked<1>();
        if (r.shape(0) % 2) throw StatusError("torch_op_begin: written intervals must come in pairs");
        for (py::ssize_t i = 0; i + 1 < r.shape(0); i += 2) o.written.emplace_back((uint64_t)r(i), (uint64_t)r(i + 1));
      }
      ops.push_back(std::move(o));
    }
    std::vector<uint64_t> held, persistent;
    Status st;
    {
      py::gil_scoped_release nogil;
      st = torch_op_begin(ops, dev, (void*)stream, &held, &persistent);
    }
    check(st, "torch_op_begin");
    return py::make_tuple(held, persistent);
  });
  m.def("torch_op_end", [](const std::vector<uint64_t>& held, const std::vector<uint64_t>& outs, int dev,
                           uint64_t stream, const std::vector<std::pair<uint64_t, uint64_t>>& hints, uint64_t now) {
    Status st;
    {
      py::gil_scoped_release nogil;
      st = torch_op_end(held, outs, dev, (void*)stream, hints, now);
    }
    check(st, "torch_op_end");
  }, py::arg("held"), py::arg("outs"), py::arg("dev"), py::arg("stream"),
     py::arg("hints") = std::vector<std::pair<uint64_t, uint64_t>>{}, py::arg("now") = 0);
  m.def("torch_advise", [](uint64_t p, int dev, int advice, int loc_kind, int loc_id, int proc) {
    check(torch_advise((void*)p, dev, advice, loc_kind, loc_id, proc), "torch_advise");
  });
  m.def("torch_last_error", [](int dev) { return std::string(torch_last_error(dev)); });
  m.def("torch_set_read_mostly", [](uint64_t p, int dev, bool on) {
    check(torch_set_read_mostly((void*)p, dev, on), "torch_set_read_mostly");
  });
  m.def("torch_is_managed", [](uint64_t p, int dev) { return torch_is_managed((void*)p, dev); });
  m.def("torch_prefetch", [](const std::vector<std::pair<uint64_t, uint64_t>>& ptrs, int dev) {
    py::gil_scoped_release nogil;
    return torch_prefetch(ptrs, dev);
  });
  m.def("torch_managed_size", [](uint64_t p, int dev) { return torch_managed_size((void*)p, dev); });
  // (diagnostics) Every block residency's chunk: owned by that block in its
  // HBM arena, and held by no other residency. "" = consistent.
  m.def("check_ownership", [] {
    Runtime* r = rt();
    std::string out;
    std::map<std::pair<ChunkArena*, int64_t>, std::string> seen;
    std::shared_lock<OrderedRWLock> vg(r->vs().lock);
    for (auto& kv : r->vs().ranges) {
      Range* rg = kv.second.get();
      for (uint64_t bi = 0; bi < rg->nblocks; ++bi) {
        Block* b = rg->block(bi);
        std::lock_guard<OrderedMutex> g(b->lock);
        for (auto& x : b->res) {
          if (x.chunk < 0) continue;
          const std::string who = std::to_string(rg->id) + "[" + std::to_string(bi) + "]@" + x.loc.str() +
                                  (rg->dead.load() ? "(dead)" : "");
          auto key = std::make_pair(x.arena, x.chunk);
          auto it = seen.find(key);
          if (it != seen.end())
            out += "shared chunk " + std::to_string(x.chunk) + ": " + it->second + " and " + who + "; ";
          else
            seen.emplace(key, who);
          if (x.loc.is_gpu() && x.arena->owner((uint32_t)x.chunk) != b)
            out += "owner mismatch " + who + " chunk " + std::to_string(x.chunk) + "; ";
        }
      }
    }
    return out;
  });
  m.def("torch_managed_range_id", [](uint64_t p, int dev) { return torch_managed_range_id((void*)p, dev); });
  m.def("torch_prefetch_wait", [](int dev) {
    py::gil_scoped_release nogil;
    torch_prefetch_wait(dev);
  });
  m.def("torch_resident_bytes", [](uint64_t p, int dev) { return torch_resident_bytes((void*)p, dev); });
  m.def("torch_managed_stats", [](int dev) {
    uint64_t a, p, np, nu;
    torch_managed_stats(dev, &a, &p, &np, &nu);
    py::dict d;
    d["active_bytes"] = a;
    d["parked_bytes"] = p;
    d["parks"] = np;
    d["unparks"] = nu;
    return d;
  });
  m.def("torch_alloc_trim", [](int dev) {  // cached free memory back to the arena (torch.cuda.empty_cache)
    py::gil_scoped_release nogil;
    torch_alloc_trim(dev);
  });
  m.def("torch_alloc_stats", [](int dev) {
    uint64_t a, p, n, w, lf, eh;
    torch_alloc_stats(dev, &a, &p, &n, &w, &lf, &eh);
    return py::make_tuple(a, p, n, w, lf, eh);
  });
}
