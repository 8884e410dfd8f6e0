// HipBackend: MI355X (gfx950) implementation of the runtime HAL.
//
// * HBM: one hipMalloc slab per GPU (default) or 2 MB hipMemCreate handles
//   (VMM provider) mapped at an alias VA.
// * Host / CXL tiers: memfd pages registered with hipHostRegister (IOMMU-correct
//   device mapping, identity address) - never raw physical addresses (fixes the
//   reference's SKIP_IOMMU_MAPPING memdesc, p2p_cxl.c:167-217).
// * Copies (config copy_engine): SDMA engines driven by the ring's worker thread
//   (3, the default for PCIe / xGMI rings, below), hipMemcpyAsync on the ring's
//   side stream (1; the kernel trace shows it as the runtime's
//   __amd_rocclr_copyBuffer) or our hand-written copy kernels (0; engine 2 =
//   HBM<->HBM, always ours; engine 4 = k_peer_push). Measured under the 70B decode
//   (profiles/r1_copy_engine_interference.md): while our 16-WG copy kernel pulls
//   host memory over PCIe, the HBM-bound compute kernels on the other stream
//   run 3-7x slower (k_dgemm 42 -> 155 us, k_ans_unpack 114 -> 306 us); with
//   engine 1 they run at their unloaded speed and the step is link-bound.
// * Completion: k_signal system-scope release into host-coherent memory;
//   GPU-side waits with hipStreamWaitValue64 / hipStreamWaitEvent.
// * SDMA (copy_engine 3, the default for PCIe / xGMI rings): the ring's worker
//   thread drives the GPU's SDMA engines directly through ROCr
//   (hsa_amd_memory_async_copy_on_engine), one engine per ring kind, and waits
//   on the completion signal. No CU is used: measured beside a 2 GB HBM
//   streaming read (tools/probe_sdma.hip, profiles/r2_copy_engines.md) SDMA costs
//   the reader 1.06x, our 16-WG CU copy kernel 2.86x, at the same 56.8 GB/s.
#include <dirent.h>
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rocprofiler-sdk-roctx/roctx.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <amd_smi/amdsmi.h>

#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <map>
#include <unordered_map>
#include <mutex>
#include <string>

#include "ogkm/backend.hpp"
#include "ogkm/codec.hpp"
#include "ogkm/config.hpp"
#include "ogkm/kernels.hpp"
#include "ogkm/events.hpp"
#include "ogkm/ring.hpp"
#include "ogkm/runtime.hpp"

namespace ogkm {

namespace {

#define HIPCHK(expr)                                                                   \
  do {                                                                                 \
    hipError_t e_ = (expr);                                                            \
    if (e_ != hipSuccess) {                                                            \
      RT_ERR("%s failed: %s", #expr, hipGetErrorString(e_));                           \
      last_err_ = hipGetErrorString(e_);                                               \
      return Status::IO_ERROR;                                                         \
    }                                                                                  \
  } while (0)

class HipBackend : public Backend {
 public:
  explicit HipBackend(int n) : ndev_(n) {}
  const char* name() const override { return "hip"; }
  bool is_fake() const override { return false; }
  int device_count() override { return ndev_; }

  int device_numa_node(int dev) override {
    char bus[64] = {0};
    if (hipDeviceGetPCIBusId(bus, sizeof bus, dev) != hipSuccess) return 0;
    for (char* p = bus; *p; ++p) *p = (char)tolower(*p);
    std::string path = std::string("/sys/bus/pci/devices/") + bus + "/numa_node";
    FILE* f = fopen(path.c_str(), "r");
    if (!f) return 0;
    int n = 0;
    if (fscanf(f, "%d", &n) != 1) n = 0;
    fclose(f);
    return n < 0 ? 0 : n;
  }
  // GPU RAS counters. Two sources, the first that reads wins:
  //  1. amdgpu sysfs under the GPU's PCI device: ras/<block>_err_count (older
  //     kernels) or ras/aca_<block> (ACA-based RAS, what gfx950 boxes expose),
  //     each holding "ue: N" / "ce: N" (/ "de: N" deferred) lines;
  //  2. amd-smi (libamd_smi, dlopen'ed): total ECC counts plus the XGMI_WAFL
  //     block's counts.
  // Neither readable -> NOT_SUPPORTED with the reason in last_error(); the
  // runtime reports that as a condition instead of treating it as healthy.
  Status device_health(int dev, Health* out) override {
    char bus[64] = {0};
    if (hipDeviceGetPCIBusId(bus, sizeof bus, dev) != hipSuccess) return Status::INVALID_ARGUMENT;
    for (char* p = bus; *p; ++p) *p = (char)tolower(*p);
    std::string why;
    if (ras_sysfs(bus, out, &why) == Status::OK) return Status::OK;
    std::string why2;
    if (ras_amdsmi(bus, out, &why2) == Status::OK) return Status::OK;
    last_err_ = why + "; " + why2;
    return Status::NOT_SUPPORTED;
  }
  Status ras_sysfs(const char* bus, Health* out, std::string* why) {
    std::string dir = std::string("/sys/bus/pci/devices/") + bus + "/ras";
    DIR* d = opendir(dir.c_str());
    if (!d) {
      *why = "no " + dir;
      return Status::NOT_SUPPORTED;
    }
    *out = Health{};
    out->source = "sysfs:" + dir;
    int parsed = 0;
    while (dirent* e = readdir(d)) {
      std::string n = e->d_name;
      const bool legacy = n.size() > 10 && n.compare(n.size() - 10, 10, "_err_count") == 0;
      const bool aca = n.rfind("aca_", 0) == 0;
      if (!legacy && !aca) continue;
      FILE* f = fopen((dir + "/" + n).c_str(), "r");
      if (!f) continue;
      long long ue = -1, ce = -1, de = -1;
      char line[128];
      while (fgets(line, sizeof line, f)) {
        long long v;
        if (sscanf(line, "ue: %lld", &v) == 1) ue = v;
        else if (sscanf(line, "ce: %lld", &v) == 1) ce = v;
        else if (sscanf(line, "de: %lld", &v) == 1) de = v;
      }
      fclose(f);
      const std::string blk = aca ? n.substr(4) : n.substr(0, n.size() - 10);
      bool link = blk.rfind("xgmi", 0) == 0 || blk.find("wafl") != std::string::npos || blk.find("pcs") != std::string::npos;
      int64_t& U = link ? out->link_ue : out->ue;
      int64_t& C = link ? out->link_ce : out->ce;
      if (ue >= 0) U = (U < 0 ? 0 : U) + ue;
      if (ce >= 0 || de >= 0) C = (C < 0 ? 0 : C) + std::max(0ll, ce) + std::max(0ll, de);
      parsed += (ue >= 0 || ce >= 0);
    }
    closedir(d);
    if (!parsed) {  // the directory exists but no counter is readable (permissions, older kernel)
      *why = "no readable RAS counters under " + dir;
      return Status::NOT_SUPPORTED;
    }
    return Status::OK;
  }
  Status ras_amdsmi(const char* bus, Health* out, std::string* why) {
    using init_t = int (*)(uint64_t);
    using handle_t = int (*)(amdsmi_bdf_t, amdsmi_processor_handle*);
    using total_t = int (*)(amdsmi_processor_handle, amdsmi_error_count_t*);
    using block_t = int (*)(amdsmi_processor_handle, amdsmi_gpu_block_t, amdsmi_error_count_t*);
    static void* lib = dlopen("libamd_smi.so", RTLD_NOW | RTLD_LOCAL);
    if (!lib) {
      *why = "libamd_smi.so not loadable";
      return Status::NOT_SUPPORTED;
    }
    static auto init = (init_t)dlsym(lib, "amdsmi_init");
    static auto by_bdf = (handle_t)dlsym(lib, "amdsmi_get_processor_handle_from_bdf");
    static auto total = (total_t)dlsym(lib, "amdsmi_get_gpu_total_ecc_count");
    static auto block = (block_t)dlsym(lib, "amdsmi_get_gpu_ecc_count");
    static int init_rc = init ? init(AMDSMI_INIT_AMD_GPUS) : -1;
    if (!by_bdf || !total || init_rc != 0) {
      *why = "amd-smi init failed (" + std::to_string(init_rc) + ")";
      return Status::NOT_SUPPORTED;
    }
    unsigned dom = 0, b = 0, dv = 0, fn = 0;
    if (sscanf(bus, "%x:%x:%x.%x", &dom, &b, &dv, &fn) != 4) return Status::INVALID_ARGUMENT;
    amdsmi_bdf_t bdf{};
    bdf.domain_number = dom;
    bdf.bus_number = b;
    bdf.device_number = dv;
    bdf.function_number = fn;
    amdsmi_processor_handle h = nullptr;
    amdsmi_error_count_t ec{};
    if (by_bdf(bdf, &h) != 0 || total(h, &ec) != 0) {
      *why = std::string("amd-smi has no ECC counts for ") + bus;
      return Status::NOT_SUPPORTED;
    }
    *out = Health{};
    out->source = "amdsmi";
    out->ue = (int64_t)ec.uncorrectable_count;
    out->ce = (int64_t)(ec.correctable_count + ec.deferred_count);
    amdsmi_error_count_t xe{};
    if (block && block(h, AMDSMI_GPU_BLOCK_XGMI_WAFL, &xe) == 0) {
      out->link_ue = (int64_t)xe.uncorrectable_count;
      out->link_ce = (int64_t)xe.correctable_count;
      // the total includes the link block: keep the two classes disjoint
      out->ue = std::max<int64_t>(0, out->ue - out->link_ue);
      out->ce = std::max<int64_t>(0, out->ce - out->link_ce);
    }
    return Status::OK;
  }
  Status device_mem_info(int dev, size_t* f, size_t* t) override {
    HIPCHK(hipSetDevice(dev));
    HIPCHK(hipMemGetInfo(f, t));
    return Status::OK;
  }
  Status set_device(int dev) override {
    HIPCHK(hipSetDevice(dev));
    return Status::OK;
  }

  Status hbm_alloc(int dev, size_t bytes, void** p) override {
    HIPCHK(hipSetDevice(dev));
    hipError_t e = hipMalloc(p, bytes);
    if (e == hipErrorOutOfMemory || e == hipErrorMemoryAllocation) {
      (void)hipGetLastError();
      return Status::NO_MEMORY;
    }
    HIPCHK(e);
    return Status::OK;
  }
  Status hbm_alloc_kind(int dev, size_t bytes, void** p, int kind) override {
    if (kind <= 0) return hbm_alloc(dev, bytes, p);
    HIPCHK(hipSetDevice(dev));
    hipError_t e = hipExtMallocWithFlags(p, bytes, kind == 1 ? hipDeviceMallocFinegrained : hipDeviceMallocUncached);
    if (e == hipErrorOutOfMemory || e == hipErrorMemoryAllocation) {
      (void)hipGetLastError();
      return Status::NO_MEMORY;
    }
    HIPCHK(e);
    return Status::OK;
  }
  void hbm_free(int dev, void* p, size_t) override {
    if (!p) return;
    reg_gen_.fetch_add(1, std::memory_order_acq_rel);
    (void)hipSetDevice(dev);
    (void)hipFree(p);
  }

  bool vmm_supported(int dev) override {
    int v = 0;
    if (hipDeviceGetAttribute(&v, hipDeviceAttributeVirtualMemoryManagementSupported, dev) != hipSuccess) return false;
    return v != 0;
  }
  Status vmm_create(int dev, size_t bytes, uint64_t* h) override {
    hipMemAllocationProp prop = {};
    prop.type = hipMemAllocationTypePinned;
    prop.location.type = hipMemLocationTypeDevice;
    prop.location.id = dev;
    hipMemGenericAllocationHandle_t hh;
    hipError_t e = hipMemCreate(&hh, bytes, &prop, 0);
    if (e == hipErrorOutOfMemory) {
      (void)hipGetLastError();
      return Status::NO_MEMORY;
    }
    HIPCHK(e);
    *h = (uint64_t)(uintptr_t)hh;
    return Status::OK;
  }
  void vmm_release(uint64_t h) override {
    // Drop the ROCr handle retained for this chunk (rocr_handle) and its lookup
    // address before HIP frees it: a recreated arena may get the same numeric
    // handle back, and a stale cache entry would map the stable VA to the old
    // (leaked) physical chunk.
    hsa_amd_vmem_alloc_handle_t rh{0};
    {
      std::lock_guard<std::mutex> g(reg_m_);
      auto it = rocr_h_.find(h);
      if (it != rocr_h_.end()) {
        rh = it->second;
        rocr_h_.erase(it);
      }
      handle_home_.erase(h);
    }
    if (rh.handle) (void)hsa_amd_vmem_handle_release(rh);
    (void)hipMemRelease((hipMemGenericAllocationHandle_t)(uintptr_t)h);
  }
  Status va_reserve(size_t bytes, void** va, void* want) override {
    HIPCHK(hipMemAddressReserve(va, bytes, kBlockSize, want, 0));
    if (want && *va != want) {  // the address is only a hint to the driver
      (void)hipMemAddressFree(*va, bytes);
      return Status::BUSY;
    }
    return Status::OK;
  }
  void va_free(void* va, size_t bytes) override { (void)hipMemAddressFree(va, bytes); }
  Status vmm_map(void* va, size_t bytes, uint64_t h, int dev) override {
    if (rocr_va(va)) {  // a prepared stable VA: ROCr maps it (HIP keeps its placeholder view)
      hsa_amd_vmem_alloc_handle_t rh;
      if (!rocr_handle(h, &rh)) return Status::IO_ERROR;
      hsa_amd_memory_access_desc_t d{HSA_ACCESS_PERMISSION_RW, dma_[dev].gpu};
      if (hsa_amd_vmem_map(va, bytes, 0, rh, 0) != HSA_STATUS_SUCCESS) {
        last_err_ = "hsa_amd_vmem_map failed";
        return Status::IO_ERROR;
      }
      if (hsa_amd_vmem_set_access(va, bytes, &d, 1) != HSA_STATUS_SUCCESS) {
        (void)hsa_amd_vmem_unmap(va, bytes);
        last_err_ = "hsa_amd_vmem_set_access failed";
        return Status::IO_ERROR;
      }
      std::lock_guard<std::mutex> g(reg_m_);
      vmm_maps_[(uint64_t)va] = {bytes, dev};
      return Status::OK;
    }
    HIPCHK(hipMemMap(va, bytes, 0, (hipMemGenericAllocationHandle_t)(uintptr_t)h, 0));
    hipMemAccessDesc ad = {};
    ad.location.type = hipMemLocationTypeDevice;
    ad.location.id = dev;
    ad.flags = hipMemAccessFlagsProtReadWrite;
    HIPCHK(hipMemSetAccess(va, bytes, &ad, 1));
    std::lock_guard<std::mutex> g(reg_m_);
    vmm_maps_[(uint64_t)va] = {bytes, dev};
    handle_home_.insert_or_assign(h, (uint64_t)va);  // where ROCr can look the handle up (rocr_handle)
    return Status::OK;
  }
  Status vmm_unmap(void* va, size_t bytes) override {
    if (rocr_va(va)) {
      if (hsa_amd_vmem_unmap(va, bytes) != HSA_STATUS_SUCCESS) {
        last_err_ = "hsa_amd_vmem_unmap failed";
        return Status::IO_ERROR;
      }
    } else {
      HIPCHK(hipMemUnmap(va, bytes));
    }
    std::lock_guard<std::mutex> g(reg_m_);
    vmm_maps_.erase((uint64_t)va);
    return Status::OK;
  }
  // Stable VAs remapped through ROCr. HIP's VMM layer costs 14 us per 2 MB
  // unmap against ROCr's 2.3 (and 7.6 vs 5.3 per map + access;
  // tools/probe_vmm_rocr_path.hip), but HIP copies (torch's hipMemcpy on a
  // managed tensor) resolve only VAs HIP itself mapped - on a VA only ROCr
  // maps they crash. So HIP maps every block of the reservation once, to a
  // per-device placeholder handle, and ROCr unmaps them again: HIP's table
  // then always holds a mapping for the VA while ROCr's holds the real chunk
  // (or none), and copies through the VA reach whatever ROCr maps.
  Status stable_va_prepare(void* va, size_t bytes, int dev) override {
    if (!config().vmm_rocr_remap) return Status::OK;
    dma_init();
    if (dev < 0 || dev >= (int)dma_.size() || !dma_[dev].gpu.handle) return Status::OK;  // HIP path
    uint64_t ph = 0;
    {
      std::lock_guard<std::mutex> g(reg_m_);
      ph = placeholder_[dev];
    }
    if (!ph) {
      hipMemAllocationProp prop = {};
      prop.type = hipMemAllocationTypePinned;
      prop.location.type = hipMemLocationTypeDevice;
      prop.location.id = dev;
      hipMemGenericAllocationHandle_t hh;
      HIPCHK(hipMemCreate(&hh, kBlockSize, &prop, 0));
      std::lock_guard<std::mutex> g(reg_m_);
      if (!placeholder_[dev]) {
        placeholder_[dev] = (uint64_t)(uintptr_t)hh;
      } else {
        (void)hipMemRelease(hh);
      }
      ph = placeholder_[dev];
    }
    const size_t n = bytes / kBlockSize;
    size_t i = 0;
    for (; i < n; ++i)
      if (hipMemMap((char*)va + i * kBlockSize, kBlockSize, 0, (hipMemGenericAllocationHandle_t)(uintptr_t)ph, 0) !=
          hipSuccess)
        break;
    hipMemAccessDesc ad = {};
    ad.location.type = hipMemLocationTypeDevice;
    ad.location.id = dev;
    ad.flags = hipMemAccessFlagsProtReadWrite;
    if (i < n || hipMemSetAccess(va, bytes, &ad, 1) != hipSuccess) {
      (void)hipGetLastError();
      for (size_t k = 0; k < i; ++k) (void)hipMemUnmap((char*)va + k * kBlockSize, kBlockSize);
      last_err_ = "placeholder mapping of a stable VA failed";
      return Status::IO_ERROR;
    }
    {
      std::lock_guard<std::mutex> g(reg_m_);
      if (!placeholder_rh_[dev].handle &&
          hsa_amd_vmem_retain_alloc_handle(&placeholder_rh_[dev], va) != HSA_STATUS_SUCCESS)
        placeholder_rh_[dev].handle = 0;
    }
    bool ok = placeholder_rh_[dev].handle != 0;
    size_t u = 0;
    for (; ok && u < n; ++u) ok = hsa_amd_vmem_unmap((char*)va + u * kBlockSize, kBlockSize) == HSA_STATUS_SUCCESS;
    if (!ok) {  // back to HIP's own mappings, then undo them
      hsa_amd_memory_access_desc_t d{HSA_ACCESS_PERMISSION_RW, dma_[dev].gpu};
      for (size_t k = 0; k < u && placeholder_rh_[dev].handle; ++k) {
        (void)hsa_amd_vmem_map((char*)va + k * kBlockSize, kBlockSize, 0, placeholder_rh_[dev], 0);
        (void)hsa_amd_vmem_set_access((char*)va + k * kBlockSize, kBlockSize, &d, 1);
      }
      for (size_t k = 0; k < n; ++k) (void)hipMemUnmap((char*)va + k * kBlockSize, kBlockSize);
      last_err_ = "ROCr unmap of a placeholder mapping failed";
      return Status::IO_ERROR;
    }
    std::lock_guard<std::mutex> g(reg_m_);
    rocr_vas_[(uint64_t)va] = {bytes, dev};
    return Status::OK;
  }
  void stable_va_release(void* va, size_t bytes) override {
    int dev = -1;
    {
      std::lock_guard<std::mutex> g(reg_m_);
      auto it = rocr_vas_.find((uint64_t)va);
      if (it == rocr_vas_.end()) return;
      dev = it->second.second;
      rocr_vas_.erase(it);
    }
    // Restore HIP's view block by block (the placeholder), then let HIP unmap it.
    for (size_t k = 0; k < bytes / kBlockSize; ++k) {
      char* b = (char*)va + k * kBlockSize;
      bool mapped;
      {
        std::lock_guard<std::mutex> g(reg_m_);
        mapped = vmm_maps_.erase((uint64_t)b) != 0;
      }
      if (mapped) (void)hsa_amd_vmem_unmap(b, kBlockSize);
      (void)hsa_amd_vmem_map(b, kBlockSize, 0, placeholder_rh_[dev], 0);
      (void)hipMemUnmap(b, kBlockSize);
    }
    (void)hipGetLastError();
  }
  bool rocr_va(void* p) {
    const uint64_t a = (uint64_t)p;
    std::lock_guard<std::mutex> g(reg_m_);
    auto it = rocr_vas_.upper_bound(a);
    if (it == rocr_vas_.begin()) return false;
    --it;
    return a < it->first + it->second.first;
  }
  // ROCr's handle for a HIP VMM handle (looked up at an address where HIP mapped it; cached).
  bool rocr_handle(uint64_t h, hsa_amd_vmem_alloc_handle_t* out) {
    std::lock_guard<std::mutex> g(reg_m_);
    auto it = rocr_h_.find(h);
    if (it != rocr_h_.end()) {
      *out = it->second;
      return true;
    }
    auto home = handle_home_.find(h);
    hsa_amd_vmem_alloc_handle_t rh;
    if (home == handle_home_.end() || hsa_amd_vmem_retain_alloc_handle(&rh, (void*)home->second) != HSA_STATUS_SUCCESS) {
      last_err_ = "no ROCr handle for a VMM chunk (not mapped at its arena view)";
      return false;
    }
    rocr_h_[h] = rh;
    *out = rh;
    return true;
  }
  // Heavyweight translation flush provoked from user space: mapping a 4 KB SVM
  // page on the GPU and revoking it again runs the KFD SVM unmap path, which
  // flushes the process's GPU TLBs (VMM unmap / map on gfx950 here does not:
  // tools/probe_vmm_tlb.hip, 100/100 stale reads without, 99/100 right with).
  Status tlb_flush(int dev) override {
    dma_init();
    if (dev < 0 || dev >= (int)dma_.size() || !dma_[dev].gpu.handle) return Status::NOT_SUPPORTED;
    std::lock_guard<std::mutex> g(flush_m_);
    if (!flush_page_) {
      flush_page_ = aligned_alloc(4096, 4096);
      if (!flush_page_) return Status::NO_MEMORY;
      memset(flush_page_, 0, 4096);
    }
    hsa_amd_svm_attribute_pair_t on{HSA_AMD_SVM_ATTRIB_AGENT_ACCESSIBLE_IN_PLACE, dma_[dev].gpu.handle};
    hsa_amd_svm_attribute_pair_t off{HSA_AMD_SVM_ATTRIB_AGENT_NO_ACCESS, dma_[dev].gpu.handle};
    if (hsa_amd_svm_attributes_set(flush_page_, 4096, &on, 1) != HSA_STATUS_SUCCESS ||
        hsa_amd_svm_attributes_set(flush_page_, 4096, &off, 1) != HSA_STATUS_SUCCESS) {
      last_err_ = "hsa_amd_svm_attributes_set (TLB flush) failed";
      return Status::IO_ERROR;
    }
    return Status::OK;
  }
  // Device of the VMM mapping that contains `a` (-1 = none).
  int vmm_dev(uint64_t a) {
    std::lock_guard<std::mutex> g(reg_m_);
    auto it = vmm_maps_.upper_bound(a);
    if (it == vmm_maps_.begin()) return -1;
    --it;
    return a < it->first + it->second.first ? it->second.second : -1;
  }

  Status host_register(void* p, size_t bytes) override {
    HIPCHK(hipHostRegister(p, bytes, hipHostRegisterMapped | hipHostRegisterPortable));
    std::lock_guard<std::mutex> g(reg_m_);
    regs_[(uint64_t)p] = bytes;
    return Status::OK;
  }
  void host_unregister(void* p) override {
    reg_gen_.fetch_add(1, std::memory_order_acq_rel);
    (void)hipHostUnregister(p);
    std::lock_guard<std::mutex> g(reg_m_);
    regs_.erase((uint64_t)p);
  }
  // Bytes from `a` to the end of the host registration that contains it (0 = none).
  uint64_t reg_room(uint64_t a) {
    std::lock_guard<std::mutex> g(reg_m_);
    auto it = regs_.upper_bound(a);
    if (it == regs_.begin()) return 0;
    --it;
    return a < it->first + it->second ? it->first + it->second - a : 0;
  }
  Status host_alloc_coherent(size_t bytes, void** p) override {
    HIPCHK(hipHostMalloc(p, bytes, hipHostMallocCoherent | hipHostMallocMapped | hipHostMallocPortable));
    memset(*p, 0, bytes);
    return Status::OK;
  }
  void host_free_coherent(void* p) override {
    reg_gen_.fetch_add(1, std::memory_order_acq_rel);
    (void)hipHostFree(p);
  }

  void* stream_create(int dev, int prio) override {
    (void)hipSetDevice(dev);
    hipStream_t s = nullptr;
    if (hipStreamCreateWithPriority(&s, hipStreamNonBlocking, prio) != hipSuccess) return nullptr;
    return s;
  }
  void stream_destroy(void* s) override {
    if (s) (void)hipStreamDestroy((hipStream_t)s);
  }
  Status stream_sync(void* s) override {
    HIPCHK(hipStreamSynchronize((hipStream_t)s));
    return Status::OK;
  }
  void* event_create(int dev) override {
    std::lock_guard<std::mutex> g(ev_m_);
    if (dev >= 0 && dev < 64 && !free_events_[dev].empty()) {
      void* e = free_events_[dev].back();
      free_events_[dev].pop_back();
      return e;
    }
    int cur = 0;
    (void)hipGetDevice(&cur);
    if (dev >= 0) (void)hipSetDevice(dev);
    hipEvent_t e = nullptr;
    hipError_t r = hipEventCreateWithFlags(&e, hipEventDisableTiming);
    if (dev >= 0) (void)hipSetDevice(cur);
    if (r != hipSuccess) return nullptr;
    ev_dev_[e] = dev;
    return e;
  }
  void event_destroy(void* e) override {
    std::lock_guard<std::mutex> g(ev_m_);
    int dev = ev_dev_.count(e) ? ev_dev_[e] : -1;
    if (dev >= 0 && dev < 64 && free_events_[dev].size() < 4096) {
      free_events_[dev].push_back(e);
      return;
    }
    ev_dev_.erase(e);
    (void)hipEventDestroy((hipEvent_t)e);
  }
  Status event_record(void* e, void* s) override {
    HIPCHK(hipEventRecord((hipEvent_t)e, (hipStream_t)s));
    return Status::OK;
  }
  bool event_query(void* e) override { return hipEventQuery((hipEvent_t)e) == hipSuccess; }
  Status event_sync(void* e) override {
    HIPCHK(hipEventSynchronize((hipEvent_t)e));
    return Status::OK;
  }
  Status stream_wait_event(void* s, void* e) override {
    HIPCHK(hipStreamWaitEvent((hipStream_t)s, (hipEvent_t)e, 0));
    return Status::OK;
  }

  Status copy_batch(int dev, const CopyDesc* d, size_t n, void* s, int engine) override {
    if (n == 0) return Status::OK;
    if (engine == 1) {  // SDMA: split at host-registration boundaries (one hipMemcpy per allocation)
      for (size_t i = 0; i < n; ++i) {
        uint64_t dst = d[i].dst, src = d[i].src, left = d[i].bytes;
        while (left) {
          uint64_t len = left;
          uint64_t rs = reg_room(src), rd = reg_room(dst);
          if (rs && rs < len) len = rs;
          if (rd && rd < len) len = rd;
          HIPCHK(hipMemcpyAsync((void*)dst, (const void*)src, len, hipMemcpyDefault, (hipStream_t)s));
          dst += len;
          src += len;
          left -= len;
        }
      }
      return Status::OK;
    }
    uint32_t piece = (uint32_t)(config().copy_piece_kb * 1024);
    if (piece < 4096) piece = 4096;
    if (engine == 4) {  // k_peer_push: the source GPU writes the peer's HBM, bounded CU budget
      const uint32_t pw = config().peer_push_wgs > 0 ? (uint32_t)config().peer_push_wgs : 64;
      for (size_t base = 0; base < n; base += kInlineDescs) {
        size_t cnt = n - base < (size_t)kInlineDescs ? n - base : (size_t)kInlineDescs;
        KInlineDescs inl;
        uint64_t ps = 0;
        for (size_t i = 0; i < cnt; ++i) {
          inl.d[i] = KCopyDesc{d[base + i].dst, d[base + i].src, d[base + i].bytes};
          inl.piece_start[i] = ps;
          ps += (d[base + i].bytes + piece - 1) / piece;
        }
        inl.piece_start[cnt] = ps;
        HIPCHK(launch_peer_push(inl, (uint32_t)cnt, ps, piece, pw, (hipStream_t)s));
        launches_++;
      }
      return Status::OK;
    }
    uint32_t wgs = (uint32_t)config().copy_workgroups;
    if (wgs == 0) wgs = 64;
    for (size_t base = 0; base < n; base += kInlineDescs) {
      size_t cnt = n - base < (size_t)kInlineDescs ? n - base : (size_t)kInlineDescs;
      KInlineDescs inl;
      uint64_t ps = 0;
      bool hbm_only = engine == 2;
      for (size_t i = 0; i < cnt; ++i) {
        inl.d[i] = KCopyDesc{d[base + i].dst, d[base + i].src, d[base + i].bytes};
        inl.piece_start[i] = ps;
        ps += (d[base + i].bytes + piece - 1) / piece;
      }
      inl.piece_start[cnt] = ps;
      // HBM<->HBM copies are not PCIe bound: give them the whole chip.
      uint32_t g = hbm_only ? (wgs * 16 > 2048 ? 2048 : wgs * 16) : wgs;
      HIPCHK(launch_batch_copy(nullptr, nullptr, &inl, (uint32_t)cnt, ps, piece, g, (hipStream_t)s,
                                config().copy_nt_loads != 0));
      launches_++;
    }
    return Status::OK;
  }

  // ---- SDMA engines (copy_engine 3)
  bool dma_supported(int dev) override {
    dma_init();
    return dev >= 0 && dev < (int)dma_.size() && dma_[dev].ok;
  }

  Status dma_copy(int dev, const CopyDesc* d, size_t n, int channel) override {
    Status st = dma_issue(dev, d, n, channel, 0);
    if (st != Status::OK) return st;
    return dma_complete(0);
  }
  // Per worker thread: two completion signals (a batch in flight while the
  // next one is issued), each decremented by every copy of its batch.
  static hsa_signal_t* dma_sigs() {
    thread_local hsa_signal_t sig[2] = {{0}, {0}};
    return sig;
  }
  Status dma_complete(int slot) override {
    hsa_signal_t sig = dma_sigs()[slot & 1];
    if (sig.handle) dma_wait(sig);
    return Status::OK;
  }
  Status dma_issue(int dev, const CopyDesc* d, size_t n, int channel, int slot) override {
    if (!dma_supported(dev)) return Status::NOT_SUPPORTED;
    if (n == 0) return Status::OK;
    DmaDev& dd = dma_[dev];
    hsa_signal_t& sig = dma_sigs()[slot & 1];
    if (!sig.handle && hsa_signal_create(0, 0, nullptr, &sig) != HSA_STATUS_SUCCESS) {
      sig.handle = 0;
      last_err_ = "hsa_signal_create failed";
      return Status::NO_MEMORY;
    }
    dma_wait(sig);  // the slot's previous batch (normally completed already)
    struct Piece { void* dst; hsa_agent_t da; const void* src; hsa_agent_t sa; size_t len; uint32_t engine; };
    std::vector<Piece> pieces;
    pieces.reserve(n);
    for (size_t i = 0; i < n; ++i) {
      uint64_t dst = d[i].dst, src = d[i].src, left = d[i].bytes;
      while (left) {
        uint64_t len = left;
        uint64_t rs = reg_room(src), rd = reg_room(dst);
        if (rs && rs < len) len = rs;
        if (rd && rd < len) len = rd;
        Piece pc;
        if (!dma_resolve((void*)dst, dd, &pc.dst, &pc.da) || !dma_resolve((void*)src, dd, (void**)&pc.src, &pc.sa)) {
          last_err_ = "dma_copy: pointer unknown to ROCr";
          return Status::INVALID_ARGUMENT;
        }
        pc.len = len;
        pc.engine = d[i].engine;
        pieces.push_back(pc);
        dst += len;
        src += len;
        left -= len;
      }
    }
    hsa_signal_store_relaxed(sig, (hsa_signal_value_t)pieces.size());
    if (log_level() >= LogLevel::DEBUG)
      for (auto& pc : pieces)
        RT_DBG("dma_copy dev %d ch %d: %p (agent %llx) <- %p (agent %llx) %zu B [cpu agent %llx]", dev, channel,
               pc.dst, (unsigned long long)pc.da.handle, pc.src, (unsigned long long)pc.sa.handle, pc.len,
               (unsigned long long)dd.cpu.handle);
    for (auto& pc : pieces) {
      const bool h2d = pc.sa.handle == dd.cpu.handle, d2h = pc.da.handle == dd.cpu.handle;
      const uint32_t mask = h2d ? dd.h2d : (d2h ? dd.d2h : peer_mask(dd, pc.da));
      const uint32_t fast = h2d ? dd.h2d_fast : (d2h ? dd.d2h_fast : mask);
      uint32_t e = (pc.engine && (pc.engine & mask)) ? pc.engine : pick_engine(fast ? fast : mask, dma_channel(channel));
      hsa_amd_sdma_engine_id_t eng = (hsa_amd_sdma_engine_id_t)e;
      __atomic_fetch_add(&dd.eng_bytes[__builtin_ctz(e)], (uint64_t)pc.len, __ATOMIC_RELAXED);
      hsa_status_t st = hsa_amd_memory_async_copy_on_engine(pc.dst, pc.da, pc.src, pc.sa, pc.len, 0, nullptr, sig,
                                                            eng, true);
      if (st != HSA_STATUS_SUCCESS) {
        // Copies already issued still decrement the signal: drain them first.
        hsa_signal_subtract_relaxed(sig, (hsa_signal_value_t)(&pieces.back() - &pc + 1));
        dma_wait(sig);
        last_err_ = "hsa_amd_memory_async_copy_on_engine failed";
        return Status::IO_ERROR;
      }
    }
    dma_launches_ += pieces.size();
    return Status::OK;
  }

  Status decode_bf12(int, const DecodeDesc* d, size_t n, void* s, uint32_t workgroups) override {
    uint32_t wgs = workgroups ? workgroups : (uint32_t)config().decode_workgroups;
    if (wgs == 0) wgs = 256;
    for (size_t base = 0; base < n; base += kInlineDescs) {
      size_t cnt = n - base < (size_t)kInlineDescs ? n - base : (size_t)kInlineDescs;
      KBf12Descs inl;
      uint64_t items = 0;
      for (size_t i = 0; i < cnt; ++i) {
        inl.d[i] = KBf12Desc{d[base + i].src, d[base + i].dst, d[base + i].n_values, 0};
        inl.item_start[i] = items;
        items += (d[base + i].n_values + kBf12Tile - 1) / kBf12Tile;
      }
      inl.item_start[cnt] = items;
      HIPCHK(launch_bf12_decode(inl, (uint32_t)cnt, wgs, (hipStream_t)s));
      launches_++;
    }
    return Status::OK;
  }

  Status decode_ans_blocks(int, const DecodeDesc* d, size_t n, void* s) override {
    // Single-segment chunks (segmented host copies): one wave each (k_ans_segs).
    std::vector<DecodeDesc> blocks;
    KAnsSegs sg;
    uint32_t ns = 0;
    for (size_t i = 0; i < n; ++i) {
      if (d[i].n_values != kAnsSegValues) {
        blocks.push_back(d[i]);
        continue;
      }
      sg.src[ns] = d[i].src;
      sg.dst[ns] = d[i].dst;
      if (++ns == (uint32_t)kAnsInlineSegs) {
        HIPCHK(launch_ans_segs(sg, ns, (hipStream_t)s, decode_err()));
        launches_++;
        ns = 0;
      }
    }
    if (ns) {
      HIPCHK(launch_ans_segs(sg, ns, (hipStream_t)s, decode_err()));
      launches_++;
    }
    if (blocks.size() != n) {
      d = blocks.data();
      n = blocks.size();
    }
    for (size_t base = 0; base < n; base += kAnsInlineBlocks) {
      const size_t cnt = std::min<size_t>(n - base, kAnsInlineBlocks);
      KAnsBlocks b;
      uint32_t items = 0;
      for (size_t i = 0; i < cnt; ++i) {
        const DecodeDesc& x = d[base + i];
        b.src[i] = x.src;
        b.dst[i] = x.dst;
        b.n_values[i] = x.n_values;
        b.item_start[i] = items;
        const uint32_t segs = (x.n_values + kAnsSegValues - 1) / kAnsSegValues;
        items += (segs + 3) / 4;  // 4 segments (waves) per 256-thread item
      }
      b.item_start[cnt] = items;
      HIPCHK(launch_ans_blocks(b, (uint32_t)cnt, (hipStream_t)s, decode_err()));
      launches_++;
    }
    return Status::OK;
  }

  Status unpack_bf12_stream(int, uint64_t src, uint64_t dst, uint32_t nchunks, uint32_t chunk_values, uint64_t,
                            void* s, uint32_t workgroups, uint64_t dst_stride, uint32_t row_shift) override {
    HIPCHK(launch_bf12_unpack((const void*)src, (void*)dst, nchunks, chunk_values, workgroups, (hipStream_t)s,
                              dst_stride, row_shift));
    launches_++;
    return Status::OK;
  }

  Status unpack_ans_stream(int, uint64_t src, uint64_t dst, uint32_t nchunks, uint32_t chunk_values, uint64_t,
                           void* s, uint32_t workgroups, uint64_t dst_stride, uint32_t row_shift) override {
    HIPCHK(launch_ans_unpack((const void*)src, (void*)dst, nchunks, chunk_values, workgroups, (hipStream_t)s,
                             dst_stride, decode_err(), row_shift));
    launches_++;
    return Status::OK;
  }

  void decode_errors(uint64_t out[4], bool reset) override {
    uint64_t* e = decode_err();
    for (int i = 0; i < 4; ++i) out[i] = e ? __atomic_load_n(e + i, __ATOMIC_ACQUIRE) : 0;
    if (e && reset)
      for (int i = 0; i < 4; ++i) __atomic_store_n(e + i, 0ull, __ATOMIC_RELEASE);
  }

  Status dgemm(int, const DGemmArgs& a, int mode, void* s) override {
    HIPCHK(launch_dgemm(a, mode, (hipStream_t)s));
    launches_++;
    return Status::OK;
  }
  Status dgemm_reduce(int, const DGemmReduceArgs& a, void* s) override {
    HIPCHK(launch_dgemm_reduce(a, (hipStream_t)s));
    launches_++;
    return Status::OK;
  }
  Status rmsnorm(int, const ResidNormArgs& a, void* s) override {
    HIPCHK(launch_rmsnorm(a, (hipStream_t)s));
    return Status::OK;
  }
  Status rope_kv(int, const RopeKvArgs& a, void* s) override {
    HIPCHK(launch_rope_kv(a, (hipStream_t)s));
    return Status::OK;
  }
  Status attn_decode(int, const AttnArgs& a, void* s) override {
    HIPCHK(launch_attn_decode(a, (hipStream_t)s));
    return Status::OK;
  }

  Status page_list(int dev, const PageListDesc& d, void* s, bool scatter) {
    if (d.npages == 0) return Status::OK;
    reclaim();
    void* idx = nullptr;
    HIPCHK(hipHostMalloc(&idx, d.npages * sizeof(uint32_t), hipHostMallocMapped | hipHostMallocPortable));
    memcpy(idx, d.idx, d.npages * sizeof(uint32_t));
    uint32_t wgs = (uint32_t)config().copy_workgroups;
    HIPCHK(launch_gather_pages(scatter ? d.base : d.base, d.contig, (const uint32_t*)idx, d.npages, d.page_bytes,
                               scatter, wgs ? wgs : 64, (hipStream_t)s));
    defer_free(idx, s, dev);
    return Status::OK;
  }
  Status gather_pages(int dev, const PageListDesc& d, void* s) override { return page_list(dev, d, s, false); }
  void range_push(const char* name) override { roctxRangePushA(name); }
  void range_pop() override { roctxRangePop(); }
  void mark(const char* name) override { roctxMarkA(name); }
  Status stream_check(void* s) override {
    hipError_t e = hipStreamQuery((hipStream_t)s);
    if (e == hipSuccess || e == hipErrorNotReady) return Status::OK;
    last_err_ = std::string("stream: ") + hipGetErrorString(e);
    return Status::IO_ERROR;
  }
  Status page_copy(int, uint64_t dst_base, uint64_t src_base, const uint32_t* idx, uint32_t npages,
                   void* s) override {
    if (npages > 512) return Status::INVALID_ARGUMENT;
    KPageList pl;
    for (uint32_t i = 0; i < npages; ++i) pl.idx[i] = (uint16_t)idx[i];
    uint32_t wgs = (uint32_t)config().copy_workgroups;
    HIPCHK(launch_page_copy(dst_base, src_base, pl, npages, wgs ? wgs : 16, (hipStream_t)s));
    return Status::OK;
  }
  Status scatter_pages(int dev, const PageListDesc& d, void* s) override { return page_list(dev, d, s, true); }
  Status memset32(int, uint64_t dst, uint32_t pat, size_t bytes, void* s) override {
    HIPCHK(launch_memset32(dst, pat, bytes, (hipStream_t)s));
    return Status::OK;
  }
  Status signal(int, uint64_t* addr, uint64_t v, void* s) override {
    HIPCHK(launch_signal(addr, v, (hipStream_t)s));
    return Status::OK;
  }
  Status wait_value(void* s, uint64_t* addr, uint64_t v) override {
    HIPCHK(hipStreamWaitValue64((hipStream_t)s, addr, v, hipStreamWaitValueGte, ~0ull));
    return Status::OK;
  }
  Status acquire_caches(void* s) override {
    HIPCHK(launch_acquire((hipStream_t)s));
    return Status::OK;
  }

  LinkType link_type(int a, int b) override {
    if (a == b) return LinkType::SELF;
    uint32_t lt = 0, hops = 0;
    if (hipExtGetLinkTypeAndHopCount(a, b, &lt, &hops) != hipSuccess) return LinkType::NONE;
    if (lt == HSA_AMD_LINK_INFO_TYPE_XGMI) return LinkType::XGMI;
    if (lt == HSA_AMD_LINK_INFO_TYPE_PCIE) return LinkType::PCIE;
    return LinkType::NONE;
  }
  bool can_access_peer(int a, int b) override {
    int v = 0;
    if (hipDeviceCanAccessPeer(&v, a, b) != hipSuccess) return false;
    return v != 0;
  }
  Status enable_peer(int a, int b) override {
    HIPCHK(hipSetDevice(a));
    hipError_t e = hipDeviceEnablePeerAccess(b, 0);
    if (e == hipErrorPeerAccessAlreadyEnabled) {
      (void)hipGetLastError();
      return Status::OK;
    }
    HIPCHK(e);
    return Status::OK;
  }

  Status export_dmabuf(void* p, size_t bytes, int* fd, uint64_t* off) override {
    hsa_status_t s = hsa_amd_portable_export_dmabuf(p, bytes, fd, off);
    if (s != HSA_STATUS_SUCCESS) {
      last_err_ = "hsa_amd_portable_export_dmabuf failed";
      return Status::NOT_SUPPORTED;
    }
    return Status::OK;
  }
  Status import_dmabuf(int dev, int fd, void** ptr, size_t* bytes) override {
    dma_init();
    if (dev < 0 || dev >= (int)dma_.size() || !dma_[dev].ok) {
      last_err_ = "import_dmabuf: no HSA agent for the device";
      return Status::NOT_SUPPORTED;
    }
    hsa_agent_t ag = dma_[dev].gpu;
    size_t sz = 0;
    void* p = nullptr;
    hsa_status_t s = hsa_amd_interop_map_buffer(1, &ag, (hsa_handle_t)fd, 0, &sz, &p, nullptr, nullptr);
    if (s != HSA_STATUS_SUCCESS) {
      last_err_ = "hsa_amd_interop_map_buffer failed";
      return Status::IO_ERROR;
    }
    *ptr = p;
    *bytes = sz;
    return Status::OK;
  }
  Status unimport_dmabuf(void* ptr) override {
    return hsa_amd_interop_unmap_buffer(ptr) == HSA_STATUS_SUCCESS ? Status::OK : Status::IO_ERROR;
  }
  // Handle = hipIpcMemHandle_t of the containing allocation + 8-byte offset of
  // `p` inside it (arena chunks live inside one slab allocation).
  Status ipc_handle(void* p, std::string* h) override {
    hipIpcMemHandle_t hh;
    void* base = nullptr;
    size_t len = 0;
    HIPCHK(hipMemGetAddressRange(&base, &len, p));
    HIPCHK(hipIpcGetMemHandle(&hh, base));
    uint64_t off = (uint64_t)((char*)p - (char*)base);
    h->assign(reinterpret_cast<const char*>(&hh), sizeof hh);
    h->append(reinterpret_cast<const char*>(&off), sizeof off);
    return Status::OK;
  }
  Status ipc_open(const std::string& h, void** p) override {
    if (h.size() != sizeof(hipIpcMemHandle_t) + sizeof(uint64_t)) return Status::INVALID_ARGUMENT;
    hipIpcMemHandle_t hh;
    uint64_t off = 0;
    memcpy(&hh, h.data(), sizeof hh);
    memcpy(&off, h.data() + sizeof hh, sizeof off);
    void* base = nullptr;
    HIPCHK(hipIpcOpenMemHandle(&base, hh, hipIpcMemLazyEnablePeerAccess));
    *p = (char*)base + off;
    std::lock_guard<std::mutex> g(ev_m_);
    ipc_base_[*p] = base;
    return Status::OK;
  }
  void ipc_close(void* p) override {
    void* base = p;
    {
      std::lock_guard<std::mutex> g(ev_m_);
      auto it = ipc_base_.find(p);
      if (it != ipc_base_.end()) {
        base = it->second;
        ipc_base_.erase(it);
      }
    }
    (void)hipIpcCloseMemHandle(base);
  }
  std::string last_error() override { return last_err_; }

 private:
  void defer_free(void* p, void* s, int dev) {
    void* e = event_create(dev);
    if (e) (void)hipEventRecord((hipEvent_t)e, (hipStream_t)s);
    std::lock_guard<std::mutex> g(df_m_);
    deferred_.push_back({p, e});
  }
  void reclaim() {
    std::lock_guard<std::mutex> g(df_m_);
    while (!deferred_.empty()) {
      auto& f = deferred_.front();
      if (f.second && hipEventQuery((hipEvent_t)f.second) != hipSuccess) break;
      (void)hipHostFree(f.first);
      if (f.second) event_destroy(f.second);
      deferred_.pop_front();
    }
  }

  // ---- SDMA plumbing: HIP device -> ROCr agents and copy-engine masks.
  struct DmaDev {
    bool ok = false;
    hsa_agent_t gpu{0}, cpu{0};
    uint32_t h2d = 0, d2h = 0;        // engines able to copy host <-> this GPU
    uint32_t h2d_fast = 0, d2h_fast = 0;  // of those, the full-rate PCIe ones (preferred mask / config)
    uint32_t peer[kMaxGpus] = {};     // engines copying this GPU -> GPU e (hsa_amd_memory_copy_engine_status(e, this))
    uint64_t eng_bytes[32] = {};      // bytes per SDMA engine (atomic adds)
  };
  // Engines for a copy from dd's GPU into the HBM of the GPU owning agent `dst`.
  uint32_t peer_mask(const DmaDev& dd, hsa_agent_t dst) {
    for (size_t e = 0; e < dma_.size(); ++e)
      if (dma_[e].gpu.handle == dst.handle) return dd.peer[e] ? dd.peer[e] : dd.h2d | dd.d2h;
    return dd.h2d | dd.d2h;
  }
  static hsa_status_t dma_agent_cb(hsa_agent_t a, void* data) {
    auto* v = (std::vector<hsa_agent_t>*)data;
    v->push_back(a);
    return HSA_STATUS_SUCCESS;
  }
  // GPU memory faults (an illegal address, a page not mapped) reported by ROCr:
  // log the faulting VA with what the runtime knows about it (which range /
  // block / chunk), the attribution the reference prints for fatal faults.
  static hsa_status_t fault_event_cb(const hsa_amd_event_t* e, void*) {
    if (!e || e->event_type != HSA_AMD_GPU_MEMORY_FAULT_EVENT) return HSA_STATUS_SUCCESS;
    const uint64_t va = e->memory_fault.virtual_address;
    const uint32_t why = e->memory_fault.fault_reason_mask;
    Runtime* rt = Runtime::get();
    std::string what = rt ? rt->describe_device_address(va) : std::string("(no runtime)");
    fprintf(stderr, "[ogkm FAULT] GPU memory fault at VA %#llx reason %#x%s%s%s: %s\n", (unsigned long long)va, why,
            (why & HSA_AMD_MEMORY_FAULT_PAGE_NOT_PRESENT) ? " page-not-present" : "",
            (why & HSA_AMD_MEMORY_FAULT_READ_ONLY) ? " read-only" : "",
            (why & HSA_AMD_MEMORY_FAULT_IMPRECISE) ? " imprecise" : "", what.c_str());
    fflush(stderr);
    Tools::get().inc(Counter::VmmErrors);
    return HSA_STATUS_SUCCESS;
  }

  void dma_init() {
    std::call_once(dma_once_, [this] {
      dma_.assign(ndev_, DmaDev{});
      if (hsa_init() != HSA_STATUS_SUCCESS) return;  // agents are resolved for every engine choice
      (void)hsa_amd_register_system_event_handler(fault_event_cb, nullptr);
      std::vector<hsa_agent_t> agents;
      if (hsa_iterate_agents(dma_agent_cb, &agents) != HSA_STATUS_SUCCESS) return;
      hsa_agent_t cpu{0};
      std::vector<std::pair<uint64_t, hsa_agent_t>> gpus;  // (domain << 32 | bdf) -> agent
      for (auto a : agents) {
        hsa_device_type_t t;
        if (hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t) != HSA_STATUS_SUCCESS) continue;
        if (t == HSA_DEVICE_TYPE_CPU && !cpu.handle) cpu = a;
        if (t != HSA_DEVICE_TYPE_GPU) continue;
        uint32_t bdf = 0, dom = 0;
        hsa_agent_get_info(a, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_BDFID, &bdf);
        hsa_agent_get_info(a, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_DOMAIN, &dom);
        gpus.emplace_back(((uint64_t)dom << 32) | bdf, a);
      }
      for (int d = 0; d < ndev_; ++d) {
        char bus[64] = {0};
        unsigned dom = 0, b = 0, dv = 0, fn = 0;
        if (hipDeviceGetPCIBusId(bus, sizeof bus, d) != hipSuccess || sscanf(bus, "%x:%x:%x.%x", &dom, &b, &dv, &fn) != 4)
          continue;
        uint64_t key = ((uint64_t)dom << 32) | ((b << 8) | (dv << 3) | fn);
        for (auto& g : gpus)
          if (g.first == key) {
            DmaDev& dd = dma_[d];
            dd.gpu = g.second;
            dd.cpu = cpu;
            uint32_t m = 0;
            if (hsa_amd_memory_copy_engine_status(dd.gpu, cpu, &m) == HSA_STATUS_SUCCESS) dd.h2d = m;
            if (hsa_amd_memory_copy_engine_status(cpu, dd.gpu, &m) == HSA_STATUS_SUCCESS) dd.d2h = m;
            dd.ok = config().copy_engine == 3 && cpu.handle && dd.h2d && dd.d2h;
            // Not every engine runs PCIe copies at link rate: on MI355X engines
            // 0-3 move 56-57 GB/s each way to either socket's memory, engines
            // 4-15 (the xGMI ones) only 12.8 / 10 / 7 GB/s GPU->host
            // (profiles/r3_cxl_paths.md; ROCr's preferred masks, h2d 0x1 and d2h
            // 0x6 on the box, are subsets). Host / CXL rings use ROCr's preferred
            // engines plus 0-3, so H2D, D2H and CXL each get their own
            // full-rate engine; config sdma_pcie_mask overrides.
            uint32_t ph = 0, pd = 0;
            (void)hsa_amd_memory_get_preferred_copy_engine(dd.gpu, cpu, &ph);
            (void)hsa_amd_memory_get_preferred_copy_engine(cpu, dd.gpu, &pd);
            const uint32_t o = (uint32_t)config().sdma_pcie_mask;
            dd.h2d_fast = (o ? o : (ph | 0xFu)) & dd.h2d;
            dd.d2h_fast = (o ? o : (pd | 0xFu)) & dd.d2h;
            RT_INFO("GPU %d SDMA engines: h2d %#x (fast %#x) d2h %#x (fast %#x)", d, dd.h2d, dd.h2d_fast, dd.d2h,
                    dd.d2h_fast);
          }
      }
      // Per GPU pair (xGMI peers): the engines of the source that reach the
      // destination - not the host-direction masks (uvm_gpu.c:2332-2388).
      for (int a = 0; a < ndev_ && a < kMaxGpus; ++a)
        for (int b = 0; b < ndev_ && b < kMaxGpus; ++b) {
          if (a == b || !dma_[a].gpu.handle || !dma_[b].gpu.handle) continue;
          uint32_t m = 0;
          if (hsa_amd_memory_copy_engine_status(dma_[b].gpu, dma_[a].gpu, &m) == HSA_STATUS_SUCCESS) dma_[a].peer[b] = m;
        }
    });
  }
  uint32_t copy_engine_mask(int dst_dev, int src_dev) override {
    dma_init();
    if (src_dev < 0) return dst_dev >= 0 && dst_dev < (int)dma_.size() ? dma_[dst_dev].h2d : 0;
    if (src_dev >= (int)dma_.size()) return 0;
    if (dst_dev < 0) return dma_[src_dev].d2h;
    return dst_dev < kMaxGpus && dst_dev != src_dev ? dma_[src_dev].peer[dst_dev] : 0;
  }
  void engine_bytes(int dev, uint64_t out[32]) override {
    dma_init();
    for (int i = 0; i < 32; ++i)
      out[i] = dev >= 0 && dev < (int)dma_.size() ? __atomic_load_n(&dma_[dev].eng_bytes[i], __ATOMIC_RELAXED) : 0;
  }
  // Completion wait of a worker's SDMA batch: spin (HSA_WAIT_STATE_ACTIVE) for
  // at most config dma_spin_us - a small batch lands within it - then sleep in
  // the kernel (BLOCKED, interrupt signal) so a long batch does not burn a host
  // core per active ring (8 ranks x 4 DMA rings would compete with the codec
  // and fault-service threads).
  static void dma_wait(hsa_signal_t sig) {
    static const uint64_t freq = [] {
      uint64_t f = 0;
      if (hsa_system_get_info(HSA_SYSTEM_INFO_TIMESTAMP_FREQUENCY, &f) != HSA_STATUS_SUCCESS || !f) f = 100000000ull;
      return f;
    }();
    const uint64_t spin = (uint64_t)std::max<int64_t>(0, config().dma_spin_us) * freq / 1000000ull;
    if (spin && hsa_signal_wait_scacquire(sig, HSA_SIGNAL_CONDITION_EQ, 0, spin, HSA_WAIT_STATE_ACTIVE) == 0) return;
    while (hsa_signal_wait_scacquire(sig, HSA_SIGNAL_CONDITION_EQ, 0, UINT64_MAX, HSA_WAIT_STATE_BLOCKED) != 0) {
    }
  }
  // Ring kind -> engine slot: H2D, D2H and CXL rings get distinct engines of the
  // fast set (peer copies pick from the pair's own mask).
  static int dma_channel(int kind) {
    switch ((RingKind)kind) {
      case RingKind::CPU_TO_GPU: return 0;
      case RingKind::GPU_TO_CPU: return 1;
      case RingKind::CXL: return 2;
      default: return 3;
    }
  }
  // The ring kinds get distinct engines so H2D, D2H, CXL and peer traffic never
  // queue behind each other: channel k -> the k-th available engine of the mask.
  static uint32_t pick_engine(uint32_t mask, int channel) {
    int n = __builtin_popcount(mask);
    if (n == 0) return 1;
    int want = channel % n;
    for (int b = 0; b < 32; ++b)
      if ((mask >> b) & 1) {
        if (want-- == 0) return 1u << b;
      }
    return 1;
  }
  // Device-usable address and agent of `p` for an SDMA copy: HBM -> its GPU agent,
  // locked / pinned host (and CXL) memory -> the CPU agent at its agent address.
  // ROCr allocation lookups cached per worker thread: a ring worker resolves
  // two pointers per engine copy (~39k copies per transparent 70B step), each a
  // locked map lookup inside ROCr. Entries are dropped when any registration or
  // allocation goes away (reg_gen_).
  struct ResolveHit {
    uint64_t lo = 0, hi = 0, gen = ~0ull, agent = 0;
    int64_t delta = 0;
    const void* dd = nullptr;
  };
  bool dma_resolve(void* p, const DmaDev& dd, void** out, hsa_agent_t* agent) {
    thread_local ResolveHit cache[8];
    thread_local uint32_t next_slot = 0;
    const uint64_t a = (uint64_t)p, gen = reg_gen_.load(std::memory_order_acquire);
    for (auto& c : cache)
      if (c.gen == gen && c.dd == &dd && a >= c.lo && a < c.hi) {
        agent->handle = c.agent;
        *out = (void*)(a + c.delta);
        return true;
      }
    auto remember = [&](uint64_t lo, uint64_t bytes) {
      if (!bytes) return;
      ResolveHit& c = cache[next_slot++ % 8];
      c = ResolveHit{lo, lo + bytes, gen, agent->handle, (int64_t)((uint64_t)*out - a), &dd};
    };
    hsa_amd_pointer_info_t info;
    memset(&info, 0, sizeof info);
    info.size = sizeof info;
    if (hsa_amd_pointer_info(p, &info, nullptr, nullptr, nullptr) != HSA_STATUS_SUCCESS) return false;
    RT_DBG("dma_resolve %p: type %d agentBase %p hostBase %p size %zu", p, (int)info.type, info.agentBaseAddress,
           info.hostBaseAddress, info.sizeInBytes);
    switch (info.type) {
      case HSA_EXT_POINTER_TYPE_HSA:
      case HSA_EXT_POINTER_TYPE_HSA_VMEM:
      case HSA_EXT_POINTER_TYPE_IPC: {
        hsa_device_type_t t = HSA_DEVICE_TYPE_GPU;
        if (info.agentOwner.handle) hsa_agent_get_info(info.agentOwner, HSA_AGENT_INFO_DEVICE, &t);
        *agent = (t == HSA_DEVICE_TYPE_CPU || !info.agentOwner.handle) ? dd.cpu : info.agentOwner;
        *out = p;
        if (info.type != HSA_EXT_POINTER_TYPE_HSA_VMEM) remember((uint64_t)info.agentBaseAddress, info.sizeInBytes);
        return true;
      }
      case HSA_EXT_POINTER_TYPE_LOCKED:
        *agent = dd.cpu;
        *out = (char*)info.agentBaseAddress + ((char*)p - (char*)info.hostBaseAddress);
        remember((uint64_t)info.hostBaseAddress, info.sizeInBytes);
        return true;
      default:
        // Host memory registered through HIP's SVM path is not in ROCr's
        // allocation map: it is system memory mapped at the same address.
        if (reg_room((uint64_t)p)) {
          *agent = dd.cpu;
          *out = p;
          return true;
        }
        // HBM mapped through the VMM API at an alias VA (stable-VA arenas) is
        // not in that map either: the GPU VA is what the SDMA engine uses.
        if (int d = vmm_dev((uint64_t)p); d >= 0 && d < (int)dma_.size()) {
          *agent = dma_[d].gpu;
          *out = p;
          return true;
        }
        return false;
    }
  }

  // Host-coherent corrupt-chunk record shared by every decoder launch (lazy).
  uint64_t* decode_err() {
    std::call_once(dec_err_once_, [this] {
      void* p = nullptr;
      if (hipHostMalloc(&p, 64, hipHostMallocCoherent | hipHostMallocMapped | hipHostMallocPortable) == hipSuccess) {
        memset(p, 0, 64);
        dec_err_ = (uint64_t*)p;
      }
    });
    return dec_err_;
  }

  int ndev_;
  std::once_flag dma_once_;
  std::vector<DmaDev> dma_;
  std::atomic<uint64_t> dma_launches_{0};
  std::once_flag dec_err_once_;
  uint64_t* dec_err_ = nullptr;
  std::string last_err_;
  std::mutex ev_m_, df_m_, reg_m_;
  std::map<uint64_t, uint64_t> regs_;  // host registrations: base -> bytes
  std::map<uint64_t, std::pair<uint64_t, int>> vmm_maps_;  // VMM mappings: va -> (bytes, device)
  std::atomic<uint64_t> reg_gen_{0};  // bumped when memory dma_resolve may have cached goes away
  std::map<uint64_t, std::pair<uint64_t, int>> rocr_vas_;  // stable VAs remapped through ROCr: base -> (bytes, device)
  std::unordered_map<uint64_t, uint64_t> handle_home_;     // HIP VMM handle -> a VA HIP mapped it at
  std::unordered_map<uint64_t, hsa_amd_vmem_alloc_handle_t> rocr_h_;  // HIP VMM handle -> retained ROCr handle
  uint64_t placeholder_[kMaxGpus] = {};                    // per device: HIP's placeholder handle for stable VAs
  hsa_amd_vmem_alloc_handle_t placeholder_rh_[kMaxGpus] = {};
  std::mutex flush_m_;
  void* flush_page_ = nullptr;  // the SVM page toggled by tlb_flush (never freed: process lifetime)
  std::vector<void*> free_events_[64];
  std::map<void*, int> ev_dev_;
  std::map<void*, void*> ipc_base_;  // opened IPC pointer -> mapped allocation base
  std::deque<std::pair<void*, void*>> deferred_;
  uint64_t launches_ = 0;
};

}  // namespace

std::unique_ptr<Backend> make_hip_backend() {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) {
    (void)hipGetLastError();
    return nullptr;
  }
  return std::unique_ptr<Backend>(new HipBackend(n));
}

}  // namespace ogkm
