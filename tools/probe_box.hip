// Box probe: measures the host<->HBM data plane the tiering runtime is built on.
//   * SDMA (hipMemcpyAsync) H2D / D2H bandwidth from pinned host memory
//   * CU copy-kernel bandwidth reading pinned host memory (zero-copy) at several grid sizes
//   * hipHostRegister cost, VMM (hipMemCreate/Map/SetAccess) cost per 2 MB chunk
// Build: hipcc --offload-arch=gfx950 -O3 tools/probe_box.hip -o build/probe_box
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <sys/mman.h>
#include <vector>

#define CK(x)                                                                                \
  do {                                                                                       \
    hipError_t e_ = (x);                                                                     \
    if (e_ != hipSuccess) {                                                                  \
      fprintf(stderr, "HIP error %s at %s:%d: %s\n", hipGetErrorString(e_), __FILE__, __LINE__, #x); \
      exit(1);                                                                               \
    }                                                                                        \
  } while (0)

using clk = std::chrono::steady_clock;
static double now_s() { return std::chrono::duration<double>(clk::now().time_since_epoch()).count(); }

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__global__ void __launch_bounds__(256) k_copy(const u32x4* __restrict__ src, u32x4* __restrict__ dst, size_t n16,
                                              int unroll_nt) {
  size_t tid = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  size_t stride = (size_t)gridDim.x * blockDim.x;
  size_t i = tid;
  for (; i + 3 * stride < n16; i += 4 * stride) {
    u32x4 a = __builtin_nontemporal_load(src + i);
    u32x4 b = __builtin_nontemporal_load(src + i + stride);
    u32x4 c = __builtin_nontemporal_load(src + i + 2 * stride);
    u32x4 d = __builtin_nontemporal_load(src + i + 3 * stride);
    dst[i] = a;
    dst[i + stride] = b;
    dst[i + 2 * stride] = c;
    dst[i + 3 * stride] = d;
  }
  for (; i < n16; i += stride) dst[i] = __builtin_nontemporal_load(src + i);
}

// Chunked copy: each workgroup owns contiguous 64 KB pieces (better DRAM/PCIe locality than grid-stride).
__global__ void __launch_bounds__(256) k_copy_chunked(const u32x4* __restrict__ src, u32x4* __restrict__ dst,
                                                      size_t n16, size_t chunk16) {
  size_t nchunks = (n16 + chunk16 - 1) / chunk16;
  for (size_t c = blockIdx.x; c < nchunks; c += gridDim.x) {
    size_t base = c * chunk16;
    size_t end = base + chunk16 < n16 ? base + chunk16 : n16;
    for (size_t i = base + threadIdx.x; i < end; i += 4 * 256) {
      u32x4 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (i + u * 256 < end) v[u] = __builtin_nontemporal_load(src + i + u * 256);
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (i + u * 256 < end) __builtin_nontemporal_store(v[u], dst + i + u * 256);
    }
  }
}

int main(int argc, char** argv) {
  size_t bytes = (argc > 1 ? atoll(argv[1]) : 4096) * (1ull << 20);
  int ndev = 0;
  CK(hipGetDeviceCount(&ndev));
  hipDeviceProp_t p;
  CK(hipGetDeviceProperties(&p, 0));
  size_t fr = 0, tot = 0;
  CK(hipMemGetInfo(&fr, &tot));
  printf("devices=%d name=%s arch=%s CUs=%d mem_free=%.1fGB total=%.1fGB\n", ndev, p.name, p.gcnArchName,
         p.multiProcessorCount, fr / 1e9, tot / 1e9);
  int attr = 0;
  hipDeviceGetAttribute(&attr, hipDeviceAttributeVirtualMemoryManagementSupported, 0);
  printf("vmm_supported=%d\n", attr);
  hipDeviceGetAttribute(&attr, hipDeviceAttributeCanUseStreamWaitValue, 0);
  printf("stream_wait_value=%d\n", attr);

  void *h = nullptr, *d = nullptr, *d2 = nullptr;
  double t0 = now_s();
  CK(hipHostMalloc(&h, bytes, hipHostMallocDefault));
  printf("hipHostMalloc %.1f GB: %.3f s\n", bytes / 1e9, now_s() - t0);
  memset(h, 1, bytes);
  CK(hipMalloc(&d, bytes));
  CK(hipMalloc(&d2, bytes));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));

  auto bw = [&](auto fn, const char* name, size_t nb, int reps) {
    fn();
    CK(hipStreamSynchronize(s));
    CK(hipEventRecord(e0, s));
    for (int r = 0; r < reps; ++r) fn();
    CK(hipEventRecord(e1, s));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    printf("%-44s %8.2f GB/s  (%.3f ms/iter)\n", name, nb * (double)reps / (ms * 1e-3) / 1e9, ms / reps);
  };
  for (size_t sz : {(size_t)2 << 20, (size_t)64 << 20, (size_t)1 << 30, bytes}) {
    if (sz > bytes) continue;
    char nm[128];
    snprintf(nm, sizeof nm, "sdma H2D %zu MB", sz >> 20);
    bw([&] { CK(hipMemcpyAsync(d, h, sz, hipMemcpyHostToDevice, s)); }, nm, sz, 5);
    snprintf(nm, sizeof nm, "sdma D2H %zu MB", sz >> 20);
    bw([&] { CK(hipMemcpyAsync(h, d, sz, hipMemcpyDeviceToHost, s)); }, nm, sz, 5);
  }
  // chunked 2MB memcpys (block migration granularity)
  {
    size_t sz = (size_t)1 << 30;
    bw([&] {
      for (size_t o = 0; o < sz; o += 2 << 20)
        CK(hipMemcpyAsync((char*)d + o, (char*)h + o, 2 << 20, hipMemcpyHostToDevice, s));
    }, "sdma H2D 1GB as 512x2MB", sz, 3);
  }
  // Kernel zero-copy reads from pinned host memory
  void* hd = nullptr;
  CK(hipHostGetDevicePointer(&hd, h, 0));
  size_t sz = (size_t)1 << 30;
  for (int grid : {16, 32, 64, 128, 256, 512, 1024, 2048}) {
    char nm[128];
    snprintf(nm, sizeof nm, "kernel H2D 1GB grid=%d", grid);
    bw([&] { k_copy<<<grid, 256, 0, s>>>((const u32x4*)hd, (u32x4*)d, sz / 16, 0); }, nm, sz, 5);
  }
  for (int grid : {32, 64, 128, 256, 512}) {
    char nm[128];
    snprintf(nm, sizeof nm, "kernel-chunked H2D 1GB grid=%d", grid);
    bw([&] { k_copy_chunked<<<grid, 256, 0, s>>>((const u32x4*)hd, (u32x4*)d, sz / 16, 4096); }, nm, sz, 5);
    snprintf(nm, sizeof nm, "kernel-chunked D2H 1GB grid=%d", grid);
    bw([&] { k_copy_chunked<<<grid, 256, 0, s>>>((const u32x4*)d, (u32x4*)hd, sz / 16, 4096); }, nm, sz, 5);
  }
  bw([&] { k_copy_chunked<<<2048, 256, 0, s>>>((const u32x4*)d2, (u32x4*)d, sz / 16, 4096); }, "kernel D2D 1GB", sz, 5);
  // concurrent H2D + D2H sdma on two streams
  {
    hipStream_t s2;
    CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    CK(hipDeviceSynchronize());
    double t = now_s();
    for (int r = 0; r < 3; ++r) {
      CK(hipMemcpyAsync(d, h, sz, hipMemcpyHostToDevice, s));
      CK(hipMemcpyAsync((char*)h + sz, d2, sz, hipMemcpyDeviceToHost, s2));
    }
    CK(hipDeviceSynchronize());
    printf("sdma bidirectional 1GB each way: %.2f GB/s total\n", 6.0 * sz / (now_s() - t) / 1e9);
  }
  // sdma + kernel concurrently for H2D (do they add?)
  {
    hipStream_t s2;
    CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    CK(hipDeviceSynchronize());
    double t = now_s();
    for (int r = 0; r < 3; ++r) {
      CK(hipMemcpyAsync(d, h, sz, hipMemcpyHostToDevice, s));
      k_copy_chunked<<<128, 256, 0, s2>>>((const u32x4*)((char*)hd + sz), (u32x4*)d2, sz / 16, 4096);
    }
    CK(hipDeviceSynchronize());
    printf("sdma H2D + kernel H2D concurrently: %.2f GB/s total\n", 6.0 * sz / (now_s() - t) / 1e9);
  }
  // hipHostRegister of mmap'd memory
  {
    size_t rb = bytes;
    void* m = mmap(nullptr, rb, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS | MAP_POPULATE, -1, 0);
    double t = now_s();
    CK(hipHostRegister(m, rb, hipHostRegisterMapped));
    printf("hipHostRegister %.1f GB (populated): %.3f s\n", rb / 1e9, now_s() - t);
    void* md = nullptr;
    CK(hipHostGetDevicePointer(&md, m, 0));
    printf("registered dev ptr == host ptr: %d\n", md == m);
    bw([&] { CK(hipMemcpyAsync(d, m, sz, hipMemcpyHostToDevice, s)); }, "sdma H2D 1GB from hipHostRegister'd", sz, 5);
    bw([&] { k_copy_chunked<<<256, 256, 0, s>>>((const u32x4*)md, (u32x4*)d, sz / 16, 4096); },
       "kernel H2D 1GB from hipHostRegister'd", sz, 5);
    t = now_s();
    CK(hipHostUnregister(m));
    printf("hipHostUnregister: %.3f s\n", now_s() - t);
    munmap(m, rb);
  }
  // VMM cost
  {
    hipMemAllocationProp prop = {};
    prop.type = hipMemAllocationTypePinned;
    prop.location.type = hipMemLocationTypeDevice;
    prop.location.id = 0;
    size_t gran = 0;
    hipError_t ge = hipMemGetAllocationGranularity(&gran, &prop, hipMemAllocationGranularityMinimum);
    printf("vmm granularity=%zu (err=%d)\n", gran, (int)ge);
    const int N = 256;
    void* va = nullptr;
    if (hipMemAddressReserve(&va, (size_t)N << 21, 0, nullptr, 0) == hipSuccess) {
      std::vector<hipMemGenericAllocationHandle_t> hs(N);
      double t = now_s();
      for (int i = 0; i < N; ++i) CK(hipMemCreate(&hs[i], 2 << 20, &prop, 0));
      double tc = now_s() - t;
      t = now_s();
      for (int i = 0; i < N; ++i) CK(hipMemMap((char*)va + ((size_t)i << 21), 2 << 20, 0, hs[i], 0));
      double tm = now_s() - t;
      hipMemAccessDesc ad = {};
      ad.location = prop.location;
      ad.flags = hipMemAccessFlagsProtReadWrite;
      t = now_s();
      for (int i = 0; i < N; ++i) CK(hipMemSetAccess((char*)va + ((size_t)i << 21), 2 << 20, &ad, 1));
      double ta = now_s() - t;
      t = now_s();
      for (int i = 0; i < N; ++i) CK(hipMemUnmap((char*)va + ((size_t)i << 21), 2 << 20));
      double tu = now_s() - t;
      printf("vmm per 2MB: create %.1f us map %.1f us setaccess %.1f us unmap %.1f us\n", tc / N * 1e6, tm / N * 1e6,
             ta / N * 1e6, tu / N * 1e6);
      for (int i = 0; i < N; ++i) hipMemRelease(hs[i]);
      hipMemAddressFree(va, (size_t)N << 21);
    } else {
      printf("vmm reserve failed\n");
    }
  }
  printf("probe done\n");
  return 0;
}
