// Can one VMM call map several arena chunks at once? The stable-VA placement
// of the transparent mode remaps one 2 MB chunk per call (~7 us map+access,
// ~2 us unmap: ~0.5 s of a 70B step). If a physical handle spanning several
// chunks can be mapped at a nonzero offset, a run of adjacent chunks placed for
// adjacent blocks maps in ONE call. Probes, each reported:
//  1. hipMemMap(va, 4 MB, offset = 4 MB, 32 MB handle): accepted? data right?
//  2. hsa_amd_vmem_map(va, 4 MB, in_offset = 6 MB, ROCr handle of the same
//     32 MB allocation): accepted? data right?
//  3. cost of map + set_access + unmap: 16 x 2 MB calls vs 1 x 32 MB call
//     (ROCr path).
//   hipcc --offload-arch=gfx950 -O2 tools/probe_vmm_offset.hip -lhsa-runtime64 -o build/probe_vmm_offset
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <chrono>
#include <cstdio>

constexpr size_t kSz = 2u << 20;
constexpr size_t kN = 16;  // chunks in the test handle

__global__ void k_fill_chunks(int* p) {  // word k of chunk c = c * 1000 + (k & 7)
  const size_t n = kN * kSz / 4;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    p[i] = (int)((i / (kSz / 4)) * 1000 + (i & 7));
}
__global__ void k_check(const int* p, size_t nchunks, int first, unsigned long long* bad) {
  const size_t n = nchunks * kSz / 4;
  unsigned long long b = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    if (p[i] != (int)((first + i / (kSz / 4)) * 1000 + (i & 7))) ++b;
  if (b) atomicAdd(bad, b);
}

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static hsa_agent_t g_gpu{0};
static hsa_status_t agent_cb(hsa_agent_t a, void*) {
  hsa_device_type_t t;
  hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t);
  if (t == HSA_DEVICE_TYPE_GPU && !g_gpu.handle) g_gpu = a;
  return HSA_STATUS_SUCCESS;
}

static unsigned long long check(const void* va, size_t nchunks, int first) {
  unsigned long long* d;
  (void)hipMalloc(&d, 8);
  (void)hipMemset(d, 0, 8);
  hipLaunchKernelGGL(k_check, dim3(256), dim3(256), 0, 0, (const int*)va, nchunks, first, d);
  hipError_t e = hipDeviceSynchronize();
  unsigned long long bad = ~0ull;
  if (e == hipSuccess) (void)hipMemcpy(&bad, d, 8, hipMemcpyDeviceToHost);
  else std::printf("  check kernel -> %s\n", hipGetErrorString(e));
  (void)hipFree(d);
  return bad;
}

int main() {
  (void)hipFree(nullptr);
  hsa_iterate_agents(agent_cb, nullptr);
  hipMemAllocationProp prop = {};
  prop.type = hipMemAllocationTypePinned;
  prop.location.type = hipMemLocationTypeDevice;
  prop.location.id = 0;
  hipMemGenericAllocationHandle_t h;
  if (hipMemCreate(&h, kN * kSz, &prop, 0) != hipSuccess) {
    std::printf("hipMemCreate(32 MB) failed\n");
    return 1;
  }
  hipMemAccessDesc ad = {};
  ad.location.type = hipMemLocationTypeDevice;
  ad.location.id = 0;
  ad.flags = hipMemAccessFlagsProtReadWrite;
  void* base = nullptr;
  (void)hipMemAddressReserve(&base, kN * kSz, kSz, nullptr, 0);
  if (hipMemMap(base, kN * kSz, 0, h, 0) != hipSuccess || hipMemSetAccess(base, kN * kSz, &ad, 1) != hipSuccess) {
    std::printf("arena view mapping failed\n");
    return 1;
  }
  hipLaunchKernelGGL(k_fill_chunks, dim3(256), dim3(256), 0, 0, (int*)base);
  (void)hipDeviceSynchronize();
  std::printf("[0] arena view: bad words %llu (want 0)\n", check(base, kN, 0));

  std::printf("[1] hipMemMap(4 MB at handle offset 4 MB)\n");
  void* v1 = nullptr;
  (void)hipMemAddressReserve(&v1, 4 * kSz, kSz, nullptr, 0);
  hipError_t e = hipMemMap(v1, 2 * kSz, 2 * kSz, h, 0);
  std::printf("  hipMemMap -> %s\n", hipGetErrorString(e));
  (void)hipGetLastError();
  if (e == hipSuccess) {
    e = hipMemSetAccess(v1, 2 * kSz, &ad, 1);
    std::printf("  hipMemSetAccess -> %s\n", hipGetErrorString(e));
    if (e == hipSuccess) std::printf("  bad words %llu (want 0: chunks 2,3)\n", check(v1, 2, 2));
    (void)hipMemUnmap(v1, 2 * kSz);
    (void)hipGetLastError();
  }

  std::printf("[2] hsa_amd_vmem_map(4 MB at in_offset 6 MB) of the ROCr handle\n");
  hsa_amd_vmem_alloc_handle_t rh{0};
  hsa_status_t hs = hsa_amd_vmem_retain_alloc_handle(&rh, base);
  std::printf("  retain_alloc_handle -> %d\n", (int)hs);
  void* v2 = nullptr;
  (void)hipMemAddressReserve(&v2, kN * kSz, kSz, nullptr, 0);
  hsa_amd_memory_access_desc_t d{HSA_ACCESS_PERMISSION_RW, g_gpu};
  bool offset_ok = false;
  if (hs == HSA_STATUS_SUCCESS) {
    hs = hsa_amd_vmem_map(v2, 2 * kSz, 3 * kSz, rh, 0);
    std::printf("  vmem_map -> %d\n", (int)hs);
    if (hs == HSA_STATUS_SUCCESS) {
      hs = hsa_amd_vmem_set_access(v2, 2 * kSz, &d, 1);
      std::printf("  vmem_set_access -> %d\n", (int)hs);
      if (hs == HSA_STATUS_SUCCESS) {
        unsigned long long bad = check(v2, 2, 3);
        std::printf("  bad words %llu (want 0: chunks 3,4)\n", bad);
        offset_ok = bad == 0;
      }
      (void)hsa_amd_vmem_unmap(v2, 2 * kSz);
    }
  }

  std::printf("[3] ROCr map + access + unmap cost\n");
  if (rh.handle) {
    // 16 separate 2 MB handles for the per-chunk case (what the arena uses now)
    hipMemGenericAllocationHandle_t hs16[kN];
    hsa_amd_vmem_alloc_handle_t r16[kN];
    void* tmp = nullptr;
    (void)hipMemAddressReserve(&tmp, kN * kSz, kSz, nullptr, 0);
    bool ok = true;
    for (size_t i = 0; i < kN && ok; ++i) {
      ok = hipMemCreate(&hs16[i], kSz, &prop, 0) == hipSuccess &&
           hipMemMap((char*)tmp + i * kSz, kSz, 0, hs16[i], 0) == hipSuccess &&
           hsa_amd_vmem_retain_alloc_handle(&r16[i], (char*)tmp + i * kSz) == HSA_STATUS_SUCCESS;
    }
    if (ok) {
      for (int rep = 0; rep < 3; ++rep) {
        double t0 = now_us();
        for (size_t i = 0; i < kN; ++i) {
          (void)hsa_amd_vmem_map((char*)v2 + i * kSz, kSz, 0, r16[i], 0);
          (void)hsa_amd_vmem_set_access((char*)v2 + i * kSz, kSz, &d, 1);
        }
        double t1 = now_us();
        for (size_t i = 0; i < kN; ++i) (void)hsa_amd_vmem_unmap((char*)v2 + i * kSz, kSz);
        double t2 = now_us();
        std::printf("  16 x 2 MB: map+access %.1f us/chunk, unmap %.1f us/chunk\n", (t1 - t0) / kN, (t2 - t1) / kN);
      }
    }
    if (offset_ok || true) {
      for (int rep = 0; rep < 3; ++rep) {
        double t0 = now_us();
        hsa_status_t a = hsa_amd_vmem_map(v2, kN * kSz, 0, rh, 0);
        hsa_status_t b = hsa_amd_vmem_set_access(v2, kN * kSz, &d, 1);
        double t1 = now_us();
        hsa_status_t c = hsa_amd_vmem_unmap(v2, kN * kSz);
        double t2 = now_us();
        std::printf("  1 x 32 MB (%d %d %d): map+access %.1f us, unmap %.1f us\n", (int)a, (int)b, (int)c, t1 - t0,
                    t2 - t1);
      }
    }
  }
  std::printf("done\n");
  return 0;
}
