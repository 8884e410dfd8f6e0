// Can host (or CXL) memory be mapped at a managed range's stable device VA?
// The transparent mode keeps a managed torch tensor at one device VA; a remote
// (zero-copy) residency - accessed_by, a thrashing pin - needs that VA to map
// host pages instead of an HBM chunk (the reference maps sysmem into the GPU
// page tables, uvm_va_block.c:8414 block_map_gpu_to). Probes, each reported:
//  1. hipMemCreate on hipMemLocationTypeHostNuma / Host + hipMemMap into a
//     HIP-reserved VA + hipMemSetAccess(device): kernel read / write, CPU view,
//     GPU read bandwidth over the link;
//  2. the same handle mapped at a VA that first mapped an HBM chunk (a remap of
//     a stable VA from HBM to host), read by a kernel;
//  3. ROCr hsa_amd_vmem_handle_create on the CPU agent's memory pools;
//  4. /dev/udmabuf (memfd pages -> dma-buf -> ROCr import: the host arena's own
//     pages at a device VA);
//  5. is a hipMemCreate(Host) handle really host memory (device free-memory
//     delta, a cold read bigger than the 256 MB MALL), and can ROCr map it:
//     hsa_amd_vmem_retain_alloc_handle at a HIP mapping, then hsa_amd_vmem_map
//     at a second VA (the runtime's stable VAs are ROCr-mapped), kernel
//     read / write through it and the CPU view of the same pages.
//   hipcc --offload-arch=gfx950 -O2 tools/probe_vmm_host.hip -lhsa-runtime64 -o build/probe_vmm_host
#include <fcntl.h>
#include <setjmp.h>
#include <signal.h>
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <sys/ioctl.h>
#include <sys/mman.h>
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

constexpr size_t kSz = 2u << 20;

__global__ void k_fill(int* p, int v, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) p[i] = v;
}
__global__ void k_sum(const int4* p, size_t n, unsigned long long* out) {
  unsigned long long s = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    int4 v = p[i];
    s += (unsigned)v.x + (unsigned)v.y + (unsigned)v.z + (unsigned)v.w;
  }
  atomicAdd(out, s);
}

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static const char* hs(hipError_t e) { return hipGetErrorString(e); }

// Map `h` at `va` for device 0 (and optionally the host); returns false with a report.
static bool map_access(void* va, size_t sz, hipMemGenericAllocationHandle_t h, bool host_too, const char* what) {
  hipError_t e = hipMemMap(va, sz, 0, h, 0);
  if (e != hipSuccess) {
    std::printf("  %s: hipMemMap -> %s\n", what, hs(e));
    (void)hipGetLastError();
    return false;
  }
  hipMemAccessDesc ad[2] = {};
  ad[0].location.type = hipMemLocationTypeDevice;
  ad[0].location.id = 0;
  ad[0].flags = hipMemAccessFlagsProtReadWrite;
  ad[1].location.type = hipMemLocationTypeHost;
  ad[1].location.id = 0;
  ad[1].flags = hipMemAccessFlagsProtReadWrite;
  e = hipMemSetAccess(va, sz, ad, host_too ? 2 : 1);
  if (e != hipSuccess) {
    std::printf("  %s: hipMemSetAccess(%s) -> %s\n", what, host_too ? "device+host" : "device", hs(e));
    (void)hipGetLastError();
    if (host_too) {
      e = hipMemSetAccess(va, sz, ad, 1);
      std::printf("  %s: hipMemSetAccess(device) -> %s\n", what, hs(e));
      (void)hipGetLastError();
      return e == hipSuccess;
    }
    return false;
  }
  return true;
}

static void probe_host_handles() {
  for (int kind = 0; kind < 2; ++kind) {
    const char* name = kind == 0 ? "HostNuma(0)" : "Host";
    std::printf("[1] hipMemCreate on %s\n", name);
    hipMemAllocationProp prop = {};
    prop.type = hipMemAllocationTypePinned;
    prop.location.type = kind == 0 ? hipMemLocationTypeHostNuma : hipMemLocationTypeHost;
    prop.location.id = 0;
    size_t gran = 0;
    hipError_t e = hipMemGetAllocationGranularity(&gran, &prop, hipMemAllocationGranularityMinimum);
    std::printf("  granularity -> %s (%zu)\n", hs(e), gran);
    (void)hipGetLastError();
    const size_t sz = 32 * kSz;
    hipMemGenericAllocationHandle_t h;
    e = hipMemCreate(&h, sz, &prop, 0);
    std::printf("  hipMemCreate(64 MB) -> %s\n", hs(e));
    if (e != hipSuccess) {
      (void)hipGetLastError();
      continue;
    }
    void* va = nullptr;
    e = hipMemAddressReserve(&va, sz, kSz, nullptr, 0);
    if (e != hipSuccess || !map_access(va, sz, h, true, name)) {
      std::printf("  reserve -> %s\n", hs(e));
      (void)hipMemRelease(h);
      continue;
    }
    hipLaunchKernelGGL(k_fill, dim3(256), dim3(256), 0, 0, (int*)va, 7, sz / 4);
    e = hipDeviceSynchronize();
    std::printf("  kernel write -> %s\n", hs(e));
    int cpu = -1;
    if (e == hipSuccess) {
      // CPU view (if host access was granted the VA is CPU-readable)
      e = hipMemcpy(&cpu, (char*)va + 12345 * 4, 4, hipMemcpyDefault);
      std::printf("  hipMemcpy D->H of a word -> %s value %d\n", hs(e), cpu);
      unsigned long long* d_out;
      (void)hipMalloc(&d_out, 8);
      (void)hipMemset(d_out, 0, 8);
      const double t0 = now_us();
      for (int it = 0; it < 5; ++it) hipLaunchKernelGGL(k_sum, dim3(1024), dim3(256), 0, 0, (const int4*)va, sz / 16, d_out);
      e = hipDeviceSynchronize();
      const double t1 = now_us();
      unsigned long long s = 0;
      (void)hipMemcpy(&s, d_out, 8, hipMemcpyDeviceToHost);
      std::printf("  kernel read x5 -> %s, sum ok %d, %.1f GB/s over the link\n", hs(e),
                  (int)(s == 5ull * 7 * (sz / 4)), 5.0 * sz / (t1 - t0) / 1e3);
      (void)hipFree(d_out);
    }
    // [2] remap a VA from an HBM chunk to this host handle
    std::printf("[2] remap one 2 MB VA: HBM chunk -> %s handle\n", name);
    hipMemAllocationProp dp = {};
    dp.type = hipMemAllocationTypePinned;
    dp.location.type = hipMemLocationTypeDevice;
    dp.location.id = 0;
    hipMemGenericAllocationHandle_t dh;
    void* va2 = nullptr;
    if (hipMemCreate(&dh, kSz, &dp, 0) == hipSuccess && hipMemAddressReserve(&va2, kSz, kSz, nullptr, 0) == hipSuccess &&
        map_access(va2, kSz, dh, false, "hbm")) {
      hipLaunchKernelGGL(k_fill, dim3(64), dim3(256), 0, 0, (int*)va2, 3, kSz / 4);
      (void)hipDeviceSynchronize();
      (void)hipMemUnmap(va2, kSz);
      // a 2 MB sub-range of the host handle is not mappable alone: map a 2 MB host handle
      hipMemGenericAllocationHandle_t h2;
      if (hipMemCreate(&h2, kSz, &prop, 0) == hipSuccess && map_access(va2, kSz, h2, false, "host at stable VA")) {
        hipLaunchKernelGGL(k_fill, dim3(64), dim3(256), 0, 0, (int*)va2, 9, kSz / 4);
        e = hipDeviceSynchronize();
        int v = -1;
        (void)hipMemcpy(&v, (char*)va2 + 4096, 4, hipMemcpyDefault);
        std::printf("  kernel write + read back through the remapped VA -> %s value %d (want 9)\n", hs(e), v);
        (void)hipMemUnmap(va2, kSz);
        (void)hipMemRelease(h2);
      }
      (void)hipMemAddressFree(va2, kSz);
      (void)hipMemRelease(dh);
    }
    (void)hipMemUnmap(va, sz);
    (void)hipMemAddressFree(va, sz);
    (void)hipMemRelease(h);
  }
}

static hsa_agent_t g_cpu{0};
static hsa_status_t agent_cb(hsa_agent_t a, void*) {
  hsa_device_type_t t;
  hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t);
  if (t == HSA_DEVICE_TYPE_CPU && !g_cpu.handle) g_cpu = a;
  return HSA_STATUS_SUCCESS;
}
static hsa_status_t pool_cb(hsa_amd_memory_pool_t pool, void*) {
  bool alloc = false;
  hsa_amd_memory_pool_get_info(pool, HSA_AMD_MEMORY_POOL_INFO_RUNTIME_ALLOC_ALLOWED, &alloc);
  uint32_t flags = 0;
  hsa_amd_memory_pool_get_info(pool, HSA_AMD_MEMORY_POOL_INFO_GLOBAL_FLAGS, &flags);
  size_t gran = 0;
  hsa_amd_memory_pool_get_info(pool, HSA_AMD_MEMORY_POOL_INFO_RUNTIME_ALLOC_GRANULE, &gran);
  hsa_amd_vmem_alloc_handle_t h{0};
  hsa_status_t s = alloc ? hsa_amd_vmem_handle_create(pool, kSz, MEMORY_TYPE_PINNED, 0, &h) : HSA_STATUS_ERROR;
  std::printf("  cpu pool flags %#x alloc %d granule %zu: vmem_handle_create(PINNED) -> %d\n", flags, (int)alloc, gran,
              (int)s);
  if (s == HSA_STATUS_SUCCESS) (void)hsa_amd_vmem_handle_release(h);
  if (alloc) {
    s = hsa_amd_vmem_handle_create(pool, kSz, MEMORY_TYPE_NONE, 0, &h);
    std::printf("    vmem_handle_create(NONE) -> %d\n", (int)s);
    if (s == HSA_STATUS_SUCCESS) (void)hsa_amd_vmem_handle_release(h);
  }
  return HSA_STATUS_SUCCESS;
}

static void probe_rocr() {
  std::printf("[3] ROCr vmem handles on the CPU agent's pools\n");
  hsa_iterate_agents(agent_cb, nullptr);
  if (!g_cpu.handle) {
    std::printf("  no CPU agent\n");
    return;
  }
  hsa_amd_agent_iterate_memory_pools(g_cpu, pool_cb, nullptr);
}

static void probe_udmabuf() {
  std::printf("[4] /dev/udmabuf\n");
  int fd = open("/dev/udmabuf", O_RDWR);
  std::printf("  open -> %s\n", fd >= 0 ? "ok" : strerror(errno));
  if (fd >= 0) close(fd);
}

static sigjmp_buf g_jb;
static void on_segv(int) { siglongjmp(g_jb, 1); }
// a CPU load that may fault (the VA may have no CPU mapping): -1 then
static int cpu_load(volatile int* p) {
  struct sigaction sa = {}, old = {};
  sa.sa_handler = on_segv;
  sigaction(SIGSEGV, &sa, &old);
  int v = -1;
  if (!sigsetjmp(g_jb, 1)) v = *p;
  else std::printf("  (CPU load faulted)\n");
  sigaction(SIGSEGV, &old, nullptr);
  return v;
}

static hsa_agent_t g_gpu{0};
static hsa_status_t gpu_cb(hsa_agent_t a, void*) {
  hsa_device_type_t t;
  hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t);
  if (t == HSA_DEVICE_TYPE_GPU && !g_gpu.handle) g_gpu = a;
  return HSA_STATUS_SUCCESS;
}

static void probe_rocr_host_map() {
  std::printf("[5] hipMemCreate(Host): where it lives, and ROCr mapping of it\n");
  hsa_iterate_agents(gpu_cb, nullptr);
  hipMemAllocationProp prop = {};
  prop.type = hipMemAllocationTypePinned;
  prop.location.type = hipMemLocationTypeHost;
  prop.location.id = 0;
  const size_t sz = 512 * kSz;  // 1 GB: past the MALL
  size_t f0 = 0, f1 = 0, tot = 0;
  (void)hipMemGetInfo(&f0, &tot);
  hipMemGenericAllocationHandle_t h;
  hipError_t e = hipMemCreate(&h, sz, &prop, 0);
  (void)hipMemGetInfo(&f1, &tot);
  std::printf("  hipMemCreate(1 GB host) -> %s; device free %.0f -> %.0f MB\n", hs(e), f0 / 1e6, f1 / 1e6);
  if (e != hipSuccess) return;
  void* va = nullptr;
  if (hipMemAddressReserve(&va, sz, kSz, nullptr, 0) != hipSuccess || !map_access(va, sz, h, true, "host 1 GB")) return;
  hipLaunchKernelGGL(k_fill, dim3(1024), dim3(256), 0, 0, (int*)va, 5, sz / 4);
  e = hipDeviceSynchronize();
  std::printf("  kernel fill 1 GB -> %s\n", hs(e));
  // CPU view of the same pages (host access was granted at the HIP VA)
  volatile int* cp = (volatile int*)va;
  std::printf("  CPU load through the VA: %d (want 5)\n", cpu_load(cp + 777));
  unsigned long long* d_out;
  (void)hipMalloc(&d_out, 8);
  for (int it = 0; it < 3; ++it) {
    (void)hipMemset(d_out, 0, 8);
    (void)hipDeviceSynchronize();
    const double t0 = now_us();
    hipLaunchKernelGGL(k_sum, dim3(2048), dim3(256), 0, 0, (const int4*)va, sz / 16, d_out);
    e = hipDeviceSynchronize();
    const double t1 = now_us();
    unsigned long long s = 0;
    (void)hipMemcpy(&s, d_out, 8, hipMemcpyDeviceToHost);
    std::printf("  cold-ish read of 1 GB #%d -> %s, sum ok %d, %.1f GB/s\n", it, hs(e), (int)(s == 5ull * (sz / 4)),
                sz / (t1 - t0) / 1e3);
  }
  // ROCr: retain the handle at the HIP mapping, map it at a second VA
  hsa_amd_vmem_alloc_handle_t rh{0};
  hsa_status_t st = hsa_amd_vmem_retain_alloc_handle(&rh, va);
  std::printf("  hsa_amd_vmem_retain_alloc_handle -> %d\n", (int)st);
  if (st == HSA_STATUS_SUCCESS && g_gpu.handle) {
    void* va2 = nullptr;
    st = hsa_amd_vmem_address_reserve(&va2, kSz, 0, 0);
    std::printf("  hsa_amd_vmem_address_reserve -> %d\n", (int)st);
    if (st == HSA_STATUS_SUCCESS) {
      st = hsa_amd_vmem_map(va2, kSz, 0, rh, 0);
      std::printf("  hsa_amd_vmem_map(first 2 MB of the host handle) -> %d\n", (int)st);
      if (st == HSA_STATUS_SUCCESS) {
        hsa_amd_memory_access_desc_t d{HSA_ACCESS_PERMISSION_RW, g_gpu};
        st = hsa_amd_vmem_set_access(va2, kSz, &d, 1);
        std::printf("  hsa_amd_vmem_set_access(gpu) -> %d\n", (int)st);
        if (st == HSA_STATUS_SUCCESS) {
          (void)hipMemset(d_out, 0, 8);
          hipLaunchKernelGGL(k_sum, dim3(64), dim3(256), 0, 0, (const int4*)va2, kSz / 16, d_out);
          e = hipDeviceSynchronize();
          unsigned long long s = 0;
          (void)hipMemcpy(&s, d_out, 8, hipMemcpyDeviceToHost);
          std::printf("  kernel read through the ROCr mapping -> %s, sum ok %d\n", hs(e), (int)(s == 5ull * (kSz / 4)));
          hipLaunchKernelGGL(k_fill, dim3(64), dim3(256), 0, 0, (int*)va2, 11, kSz / 4);
          e = hipDeviceSynchronize();
          std::printf("  kernel write through the ROCr mapping -> %s; CPU sees %d (want 11)\n", hs(e), cpu_load(cp + 4099));
        }
        (void)hsa_amd_vmem_unmap(va2, kSz);
      }
      (void)hsa_amd_vmem_address_free(va2, kSz);
    }
    (void)hsa_amd_vmem_handle_release(rh);
  }
  (void)hipFree(d_out);
  (void)hipMemUnmap(va, sz);
  (void)hipMemAddressFree(va, sz);
  (void)hipMemRelease(h);
}

int main() {
  (void)hipFree(nullptr);
  probe_host_handles();
  probe_rocr();
  probe_udmabuf();
  probe_rocr_host_map();
  std::printf("done\n");
  return 0;
}
