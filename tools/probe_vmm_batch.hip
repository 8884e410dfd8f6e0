// Batched VMM remap cost probe: what does it cost to move a multi-block
// stable-VA tensor to other physical chunks, and which calls can be batched?
//   * per-block hipMemMap + hipMemSetAccess (what Runtime::stable_map_block does)
//   * per-block hipMemMap + ONE hipMemSetAccess over the whole tensor
//   * per-block hipMemUnmap vs ONE hipMemUnmap over the whole tensor
//   * the same through ROCr (hsa_amd_vmem_map / set_access / unmap)
//   * one translation flush (KFD SVM unmap of a 4 KB page) per batch
// and checks that a batch remap + one flush reads the NEW chunks everywhere.
//   hipcc --offload-arch=gfx950 -O2 tools/probe_vmm_batch.hip -lhsa-runtime64 -o /tmp/probe_vmm_batch
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                                      \
  do {                                                                                             \
    hipError_t e_ = (x);                                                                           \
    if (e_ != hipSuccess) {                                                                        \
      std::fprintf(stderr, "%s:%d %s -> %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));     \
      std::exit(1);                                                                                \
    }                                                                                              \
  } while (0)
#define HK(x)                                                                        \
  do {                                                                               \
    hsa_status_t s_ = (x);                                                           \
    if (s_ != HSA_STATUS_SUCCESS) {                                                  \
      std::fprintf(stderr, "%s:%d %s -> %d\n", __FILE__, __LINE__, #x, (int)s_);     \
      std::exit(1);                                                                  \
    }                                                                                \
  } while (0)

constexpr size_t kSz = 2u << 20;

__global__ void k_fill(int* p, int v, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) p[i] = v;
}
// One word per 64 KB of every block: out[i] = p[i * 16K words].
__global__ void k_sample(const int* p, int* out, size_t nsamples) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (i < nsamples) out[i] = p[i * (size_t)(64 << 10) / 4];
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
static char* g_svm = nullptr;
static void svm_flush() {
  if (!g_svm) {
    g_svm = (char*)aligned_alloc(4096, 4096);
    g_svm[0] = 1;
  }
  hsa_amd_svm_attribute_pair_t on{HSA_AMD_SVM_ATTRIB_AGENT_ACCESSIBLE_IN_PLACE, g_gpu.handle};
  hsa_amd_svm_attribute_pair_t off{HSA_AMD_SVM_ATTRIB_AGENT_NO_ACCESS, g_gpu.handle};
  HK(hsa_amd_svm_attributes_set(g_svm, 4096, &on, 1));
  HK(hsa_amd_svm_attributes_set(g_svm, 4096, &off, 1));
}

static hipMemAccessDesc rw_desc() {
  hipMemAccessDesc ad = {};
  ad.location.type = hipMemLocationTypeDevice;
  ad.location.id = 0;
  ad.flags = hipMemAccessFlagsProtReadWrite;
  return ad;
}

// Returns samples (of n blocks x 32 per block) that do not hold `want`.
static int check(void* va, int nblk, int want, int* out_d, std::vector<int>& host) {
  size_t ns = (size_t)nblk * 32;
  k_sample<<<(ns + 255) / 256, 256>>>((const int*)va, out_d, ns);
  CK(hipDeviceSynchronize());
  CK(hipMemcpy(host.data(), out_d, ns * sizeof(int), hipMemcpyDeviceToHost));
  int bad = 0;
  for (size_t i = 0; i < ns; ++i) bad += host[i] != want;
  return bad;
}

int main(int argc, char** argv) {
  const int nblk = argc > 1 ? std::atoi(argv[1]) : 256;  // 512 MB tensor
  const int trials = argc > 2 ? std::atoi(argv[2]) : 5;
  CK(hipSetDevice(0));
  HK(hsa_init());
  HK(hsa_iterate_agents(agent_cb, nullptr));
  int* out_d;
  CK(hipMalloc(&out_d, (size_t)nblk * 32 * sizeof(int)));
  std::vector<int> host((size_t)nblk * 32);

  hipMemAllocationProp prop = {};
  prop.type = hipMemAllocationTypePinned;
  prop.location.type = hipMemLocationTypeDevice;
  prop.location.id = 0;
  std::vector<hipMemGenericAllocationHandle_t> A(nblk), B(nblk);
  double t0 = now_us();
  for (int i = 0; i < nblk; ++i) CK(hipMemCreate(&A[i], kSz, &prop, 0));
  for (int i = 0; i < nblk; ++i) CK(hipMemCreate(&B[i], kSz, &prop, 0));
  std::printf("hipMemCreate: %.1f us per 2 MB handle\n", (now_us() - t0) / (2 * nblk));
  const size_t bytes = (size_t)nblk * kSz;
  void* va = nullptr;
  CK(hipMemAddressReserve(&va, bytes, kSz, nullptr, 0));
  // Alias mappings of every handle (the arena's own view), as in the runtime.
  void *aA = nullptr, *aB = nullptr;
  CK(hipMemAddressReserve(&aA, bytes, kSz, nullptr, 0));
  CK(hipMemAddressReserve(&aB, bytes, kSz, nullptr, 0));
  hipMemAccessDesc ad = rw_desc();
  for (int i = 0; i < nblk; ++i) {
    CK(hipMemMap((char*)aA + i * kSz, kSz, 0, A[i], 0));
    CK(hipMemMap((char*)aB + i * kSz, kSz, 0, B[i], 0));
  }
  CK(hipMemSetAccess(aA, bytes, &ad, 1));
  CK(hipMemSetAccess(aB, bytes, &ad, 1));
  k_fill<<<1024, 256>>>((int*)aA, 111, bytes / 4);
  k_fill<<<1024, 256>>>((int*)aB, 222, bytes / 4);
  CK(hipDeviceSynchronize());

  double map_pb = 0, set_pb = 0, set_once = 0, unmap_pb = 0, unmap_once = 0, flush = 0;
  int bad_batch = 0, bad_noflush = 0, unmap_once_ok = 1;
  for (int t = 0; t < trials; ++t) {
    // (1) per-block map + per-block set access -> A
    double a = now_us();
    for (int i = 0; i < nblk; ++i) CK(hipMemMap((char*)va + i * kSz, kSz, 0, A[i], 0));
    double b = now_us();
    for (int i = 0; i < nblk; ++i) CK(hipMemSetAccess((char*)va + i * kSz, kSz, &ad, 1));
    double c = now_us();
    map_pb += b - a;
    set_pb += c - b;
    if (check(va, nblk, 111, out_d, host)) std::printf("trial %d: A mapping reads wrong\n", t);
    // (2) per-block unmap
    a = now_us();
    for (int i = 0; i < nblk; ++i) CK(hipMemUnmap((char*)va + i * kSz, kSz));
    b = now_us();
    unmap_pb += b - a;
    // (3) per-block map + ONE set access -> B, no flush: stale?
    for (int i = 0; i < nblk; ++i) CK(hipMemMap((char*)va + i * kSz, kSz, 0, B[i], 0));
    a = now_us();
    CK(hipMemSetAccess(va, bytes, &ad, 1));
    b = now_us();
    set_once += b - a;
    bad_noflush += check(va, nblk, 222, out_d, host);
    // (4) one unmap over the whole tensor (several mappings)
    a = now_us();
    hipError_t e = hipMemUnmap(va, bytes);
    b = now_us();
    if (e != hipSuccess) {
      unmap_once_ok = 0;
      (void)hipGetLastError();
      for (int i = 0; i < nblk; ++i) CK(hipMemUnmap((char*)va + i * kSz, kSz));
    } else {
      unmap_once += b - a;
    }
    // (5) remap to A (batch set access) + ONE flush: must read A everywhere
    for (int i = 0; i < nblk; ++i) CK(hipMemMap((char*)va + i * kSz, kSz, 0, A[i], 0));
    CK(hipMemSetAccess(va, bytes, &ad, 1));
    a = now_us();
    svm_flush();
    b = now_us();
    flush += b - a;
    bad_batch += check(va, nblk, 111, out_d, host);
    for (int i = 0; i < nblk; ++i) CK(hipMemUnmap((char*)va + i * kSz, kSz));
  }
  const double n = (double)trials * nblk;
  std::printf("blocks %d (%.0f MB), trials %d\n", nblk, bytes / 1048576.0, trials);
  std::printf("per 2 MB block: hipMemMap %.1f us, hipMemSetAccess per block %.1f us, one SetAccess over tensor %.2f us/block\n",
              map_pb / n, set_pb / n, set_once / n);
  std::printf("per 2 MB block: hipMemUnmap per block %.1f us, one Unmap over tensor %s %.2f us/block\n", unmap_pb / n,
              unmap_once_ok ? "ok" : "UNSUPPORTED", unmap_once_ok ? unmap_once / n : 0.0);
  std::printf("translation flush: %.1f us per batch\n", flush / trials);
  std::printf("batched remap (map + one SetAccess): %.1f us/block -> %.1f GB/s of tensor remapped\n",
              (map_pb + set_once) / n, kSz / ((map_pb + set_once) / n) / 1e3);
  std::printf("stale samples after batch remap WITHOUT flush: %d / %d; WITH one flush: %d / %d\n", bad_noflush,
              trials * nblk * 32, bad_batch, trials * nblk * 32);

  // ROCr vmem directly.
  {
    std::vector<hsa_amd_vmem_alloc_handle_t> R(nblk);
    hsa_amd_memory_pool_t pool{0};
    auto pool_cb = [](hsa_amd_memory_pool_t p, void* d) -> hsa_status_t {
      hsa_amd_segment_t seg;
      uint32_t flags = 0;
      hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_SEGMENT, &seg);
      hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_GLOBAL_FLAGS, &flags);
      auto* out = (hsa_amd_memory_pool_t*)d;
      if (seg == HSA_AMD_SEGMENT_GLOBAL && (flags & HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_COARSE_GRAINED) && !out->handle)
        *out = p;
      return HSA_STATUS_SUCCESS;
    };
    HK(hsa_amd_agent_iterate_memory_pools(g_gpu, pool_cb, &pool));
    for (int i = 0; i < nblk; ++i) HK(hsa_amd_vmem_handle_create(pool, kSz, MEMORY_TYPE_NONE, 0, &R[i]));
    void* rv = nullptr;
    HK(hsa_amd_vmem_address_reserve(&rv, bytes, 0, 0));
    hsa_amd_memory_access_desc_t d{HSA_ACCESS_PERMISSION_RW, g_gpu};
    double m = 0, s = 0, u = 0;
    for (int t = 0; t < trials; ++t) {
      double a = now_us();
      for (int i = 0; i < nblk; ++i) HK(hsa_amd_vmem_map((char*)rv + i * kSz, kSz, 0, R[i], 0));
      double b = now_us();
      HK(hsa_amd_vmem_set_access(rv, bytes, &d, 1));
      double c = now_us();
      for (int i = 0; i < nblk; ++i) HK(hsa_amd_vmem_unmap((char*)rv + i * kSz, kSz));
      double e2 = now_us();
      m += b - a;
      s += c - b;
      u += e2 - c;
    }
    std::printf("ROCr per 2 MB block: vmem_map %.1f us, one set_access %.2f us/block, vmem_unmap %.1f us\n", m / n, s / n,
                u / n);
    HK(hsa_amd_vmem_address_free(rv, bytes));
    for (auto h : R) HK(hsa_amd_vmem_handle_release(h));
  }
  for (int i = 0; i < nblk; ++i) {
    CK(hipMemUnmap((char*)aA + i * kSz, kSz));
    CK(hipMemUnmap((char*)aB + i * kSz, kSz));
    CK(hipMemRelease(A[i]));
    CK(hipMemRelease(B[i]));
  }
  std::printf("done\n");
  return 0;
}
