// Stable-VA remaps through ROCr (hsa_amd_vmem_map / set_access / unmap) on a
// HIP-reserved VA, with the ROCr handles of chunks HIP created and mapped at an
// alias view (the arena's layout): cost per 2 MB block against hipMemMap /
// hipMemUnmap, idle and while H2D copies stream on another stream, and whether
// the HIP-side consumers still work on a VA that only ROCr maps: a kernel read,
// hipMemcpy D2H, hipMemcpyAsync (default kind) and hipMemcpyDtoD.
//   hipcc --offload-arch=gfx950 -O2 tools/probe_vmm_rocr_path.hip -lhsa-runtime64 -o /tmp/probe_vmm_rocr_path
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                                  \
  do {                                                                                         \
    hipError_t e_ = (x);                                                                       \
    if (e_ != hipSuccess) {                                                                    \
      std::fprintf(stderr, "%s:%d %s -> %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(1);                                                                            \
    }                                                                                          \
  } while (0)
#define HK(x)                                                                    \
  do {                                                                           \
    hsa_status_t s_ = (x);                                                       \
    if (s_ != HSA_STATUS_SUCCESS) {                                              \
      std::fprintf(stderr, "%s:%d %s -> %d\n", __FILE__, __LINE__, #x, (int)s_); \
      std::exit(1);                                                              \
    }                                                                            \
  } while (0)

constexpr size_t kSz = 2u << 20;

__global__ void k_fill(int* p, int v, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) p[i] = v;
}
// out[b] = first int of block b (+ a mismatch count over 32 probes of the block).
__global__ void k_check(const int* va, int nblk, int* out) {
  const int b = blockIdx.x;
  if (b >= nblk || threadIdx.x >= 32) return;
  const int* p = va + (size_t)b * (kSz / 4);
  const int v0 = p[0];
  const int v = p[threadIdx.x * 16384 + 7];
  if (threadIdx.x == 0) out[2 * b] = v0;
  if (v != v0) atomicAdd(&out[2 * b + 1], 1);
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

#define STEP(msg) std::fprintf(stderr, "step: %s\n", msg)

int main(int argc, char** argv) {
  // argv[1]: 1 = also exercise HIP copies on the ROCr-only-mapped VA (last: may crash)
  const bool copies = argc > 1 && argv[1][0] == '1';
  setvbuf(stdout, nullptr, _IONBF, 0);
  CK(hipSetDevice(0));
  HK(hsa_init());
  HK(hsa_iterate_agents(agent_cb, nullptr));
  const int n = 64, trials = 4;
  hipMemAllocationProp prop = {};
  prop.type = hipMemAllocationTypePinned;
  prop.location.type = hipMemLocationTypeDevice;
  prop.location.id = 0;
  hipMemAccessDesc ad = {};
  ad.location.type = hipMemLocationTypeDevice;
  ad.location.id = 0;
  ad.flags = hipMemAccessFlagsProtReadWrite;
  std::vector<hipMemGenericAllocationHandle_t> H(n);
  for (auto& h : H) CK(hipMemCreate(&h, kSz, &prop, 0));
  void* alias = nullptr;
  CK(hipMemAddressReserve(&alias, n * kSz, kSz, nullptr, 0));
  for (int i = 0; i < n; ++i) CK(hipMemMap((char*)alias + i * kSz, kSz, 0, H[i], 0));
  CK(hipMemSetAccess(alias, n * kSz, &ad, 1));
  for (int i = 0; i < n; ++i) k_fill<<<64, 256>>>((int*)((char*)alias + i * kSz), 1000 + i, kSz / 4);
  CK(hipDeviceSynchronize());
  STEP("retain");
  std::vector<hsa_amd_vmem_alloc_handle_t> R(n);
  for (int i = 0; i < n; ++i) HK(hsa_amd_vmem_retain_alloc_handle(&R[i], (char*)alias + i * kSz));
  void* va = nullptr;
  CK(hipMemAddressReserve(&va, n * kSz, kSz, nullptr, 0));
  int* out_d = nullptr;
  CK(hipMalloc(&out_d, 2 * n * sizeof(int)));
  std::vector<int> out(2 * n);
  hsa_amd_memory_access_desc_t d{HSA_ACCESS_PERMISSION_RW, g_gpu};

  // background load: 256 MB H2D copies on a second stream
  const size_t big = 256u << 20;
  void* hbuf = nullptr;
  void* dbuf = nullptr;
  CK(hipHostMalloc(&hbuf, big, hipHostMallocDefault));
  CK(hipMalloc(&dbuf, big));
  hipStream_t bg;
  CK(hipStreamCreateWithFlags(&bg, hipStreamNonBlocking));

  for (int loaded = 0; loaded < 2; ++loaded) {
    double hip_map = 0, hip_unmap = 0, r_map = 0, r_unmap = 0;
    int bad = 0, memcpy_bad = 0;
    for (int t = 0; t < trials; ++t) {
      if (loaded)
        for (int k = 0; k < 8; ++k) CK(hipMemcpyAsync(dbuf, hbuf, big, hipMemcpyHostToDevice, bg));
      // HIP path
      STEP("hip map");
      double a = now_us();
      for (int i = 0; i < n; ++i) {
        CK(hipMemMap((char*)va + i * kSz, kSz, 0, H[(i + t) % n], 0));
        CK(hipMemSetAccess((char*)va + i * kSz, kSz, &ad, 1));
      }
      hip_map += now_us() - a;
      a = now_us();
      for (int i = 0; i < n; ++i) CK(hipMemUnmap((char*)va + i * kSz, kSz));
      hip_unmap += now_us() - a;
      svm_flush();
      // ROCr path on the same HIP-reserved VA
      STEP("rocr map");
      a = now_us();
      for (int i = 0; i < n; ++i) {
        HK(hsa_amd_vmem_map((char*)va + i * kSz, kSz, 0, R[(i + t + 1) % n], 0));
        HK(hsa_amd_vmem_set_access((char*)va + i * kSz, kSz, &d, 1));
      }
      r_map += now_us() - a;
      svm_flush();
      STEP("kernel read");
      CK(hipMemset(out_d, 0, 2 * n * sizeof(int)));
      k_check<<<n, 64>>>((const int*)va, n, out_d);
      CK(hipDeviceSynchronize());
      CK(hipMemcpy(out.data(), out_d, 2 * n * sizeof(int), hipMemcpyDeviceToHost));
      for (int i = 0; i < n; ++i) bad += (out[2 * i] != 1000 + (i + t + 1) % n) + out[2 * i + 1];
      for (int i = 0; copies && i < n; i += 7) {
        int h1 = 0, h2 = 0, h3 = 0;
        STEP("hip copies");
        CK(hipMemcpy(&h1, (char*)va + i * kSz + 64, 4, hipMemcpyDeviceToHost));
        CK(hipMemcpyAsync(&h2, (char*)va + i * kSz + 128, 4, hipMemcpyDefault, 0));
        CK(hipMemcpyDtoD((hipDeviceptr_t)out_d, (hipDeviceptr_t)((char*)va + i * kSz + 256), 4));
        CK(hipStreamSynchronize(0));
        CK(hipMemcpy(&h3, out_d, 4, hipMemcpyDeviceToHost));
        const int want = 1000 + (i + t + 1) % n;
        memcpy_bad += (h1 != want) + (h2 != want) + (h3 != want);
      }
      STEP("rocr unmap");
      a = now_us();
      for (int i = 0; i < n; ++i) HK(hsa_amd_vmem_unmap((char*)va + i * kSz, kSz));
      r_unmap += now_us() - a;
      svm_flush();
      CK(hipStreamSynchronize(bg));
    }
    const double k = (double)trials * n;
    std::printf("%s: per 2 MB block  HIP map+access %.1f us unmap %.1f us | ROCr map+access %.1f us unmap %.1f us | "
                "kernel-read mismatches %d, hipMemcpy mismatches %d\n",
                loaded ? "streaming H2D" : "idle", hip_map / k, hip_unmap / k, r_map / k, r_unmap / k, bad, memcpy_bad);
  }
  for (auto h : R) HK(hsa_amd_vmem_handle_release(h));
  for (int i = 0; i < n; ++i) CK(hipMemUnmap((char*)alias + i * kSz, kSz));
  for (auto h : H) CK(hipMemRelease(h));
  CK(hipMemAddressFree(va, n * kSz));
  CK(hipMemAddressFree(alias, n * kSz));
  std::printf("done\n");
  return 0;
}
