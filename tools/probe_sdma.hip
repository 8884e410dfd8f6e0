// Copy-engine probe for the migration data plane (MI355X, gfx950).
//
// Measures, on one GPU:
//   1. host->HBM / HBM->host bandwidth of (a) the HIP runtime's hipMemcpyAsync,
//      (b) our CU copy kernel k_batch_copy (csrc/kernels/copy_kernels.hip) at
//      16 workgroups, (c) the SDMA engines driven directly through ROCr
//      (hsa_amd_memory_async_copy_on_engine), one engine and two in parallel;
//   2. interference: the time of an HBM-bound streaming-read kernel alone and
//      while each copy path streams host->HBM on another queue.
//
//   hipcc -O3 --offload-arch=gfx950 -I csrc/include tools/probe_sdma.hip -o build/probe_sdma -lhsa-runtime64
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <chrono>
#include <cstring>
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <vector>

#include "../csrc/kernels/copy_kernels.hip"

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                             \
    }                                                                      \
  } while (0)
#define HK(x)                                                              \
  do {                                                                     \
    hsa_status_t s_ = (x);                                                 \
    if (s_ != HSA_STATUS_SUCCESS) {                                        \
      fprintf(stderr, "%s:%d %s: hsa status 0x%x\n", __FILE__, __LINE__, #x, (unsigned)s_); \
      exit(1);                                                             \
    }                                                                      \
  } while (0)

static double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// HBM-bound victim: every wave streams 16 B/lane over a large buffer.
__global__ void __launch_bounds__(256) k_stream_read(const uint4* __restrict__ p, uint64_t n16, uint32_t* out) {
  uint32_t acc = 0;
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * 256) {
    uint4 v = p[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678u) out[0] = acc;  // keep the loads
}

struct Agents {
  hsa_agent_t gpu{}, cpu{};
  bool have_gpu = false, have_cpu = false;
};

static hsa_status_t find_agent(hsa_agent_t a, void* data) {
  auto* ag = (Agents*)data;
  hsa_device_type_t t;
  hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t);
  if (t == HSA_DEVICE_TYPE_GPU && !ag->have_gpu) {
    ag->gpu = a;
    ag->have_gpu = true;
  } else if (t == HSA_DEVICE_TYPE_CPU && !ag->have_cpu) {
    ag->cpu = a;
    ag->have_cpu = true;
  }
  return HSA_STATUS_SUCCESS;
}

int main(int argc, char** argv) {
  const size_t bytes = (argc > 1 ? strtoull(argv[1], nullptr, 0) : 1024) << 20;
  CK(hipSetDevice(0));
  void *dev = nullptr, *victim = nullptr, *host = nullptr;
  uint32_t* sink = nullptr;
  CK(hipMalloc(&dev, bytes));
  const size_t vbytes = 2ull << 30;  // 2 GB streaming-read victim (beyond the 256 MB Infinity Cache)
  CK(hipMalloc(&victim, vbytes));
  CK(hipMemset(victim, 1, vbytes));
  CK(hipMalloc(&sink, 64));
  CK(hipHostMalloc(&host, bytes, hipHostMallocMapped | hipHostMallocPortable));
  memset(host, 3, bytes);
  hipStream_t cs, ks;
  CK(hipStreamCreateWithFlags(&cs, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&ks, hipStreamNonBlocking));

  Agents ag;
  HK(hsa_iterate_agents(find_agent, &ag));
  uint32_t h2d_mask = 0, d2h_mask = 0;
  HK(hsa_amd_memory_copy_engine_status(ag.gpu, ag.cpu, &h2d_mask));
  HK(hsa_amd_memory_copy_engine_status(ag.cpu, ag.gpu, &d2h_mask));
  printf("sdma engines available: host->gpu mask 0x%x, gpu->host mask 0x%x\n", h2d_mask, d2h_mask);
  std::vector<uint32_t> engines;
  for (int i = 0; i < 16; ++i)
    if (h2d_mask & (1u << i)) engines.push_back(1u << i);

  // ---- copy paths
  auto sdma_copy = [&](void* dst, hsa_agent_t da, const void* src, hsa_agent_t sa, size_t n, int nengines,
                       bool wait) -> std::vector<hsa_signal_t> {
    std::vector<hsa_signal_t> sigs;
    size_t per = (n / nengines + 4095) & ~4095ull;
    for (int e = 0; e < nengines; ++e) {
      size_t off = per * e;
      if (off >= n) break;
      size_t len = std::min(per, n - off);
      hsa_signal_t s;
      HK(hsa_signal_create(1, 0, nullptr, &s));
      HK(hsa_amd_memory_async_copy_on_engine((char*)dst + off, da, (const char*)src + off, sa, len, 0, nullptr, s,
                                             (hsa_amd_sdma_engine_id_t)engines[e % engines.size()], true));
      sigs.push_back(s);
    }
    if (wait) {
      for (auto s : sigs) {
        hsa_signal_wait_scacquire(s, HSA_SIGNAL_CONDITION_LT, 1, UINT64_MAX, HSA_WAIT_STATE_ACTIVE);
        hsa_signal_destroy(s);
      }
      sigs.clear();
    }
    return sigs;
  };
  auto kernel_copy = [&](void* dst, const void* src, size_t n, hipStream_t s, uint32_t wgs) {
    ogkm::KInlineDescs inl;
    inl.d[0] = ogkm::KCopyDesc{(uint64_t)dst, (uint64_t)src, n};
    const uint32_t piece = 64 << 10;
    inl.piece_start[0] = 0;
    inl.piece_start[1] = (n + piece - 1) / piece;
    CK(ogkm::launch_batch_copy(nullptr, nullptr, &inl, 1, inl.piece_start[1], piece, wgs, s, true));
  };

  auto bw = [&](const char* name, auto&& fn) {
    fn();  // warm
    CK(hipDeviceSynchronize());
    double t0 = now();
    const int reps = 4;
    for (int r = 0; r < reps; ++r) fn();
    CK(hipDeviceSynchronize());
    double dt = now() - t0;
    printf("%-34s %7.2f GB/s\n", name, reps * bytes / dt / 1e9);
  };
  printf("== bandwidth (%zu MB per copy)\n", bytes >> 20);
  bw("h2d hipMemcpyAsync", [&] { CK(hipMemcpyAsync(dev, host, bytes, hipMemcpyHostToDevice, ks)); });
  bw("d2h hipMemcpyAsync", [&] { CK(hipMemcpyAsync(host, dev, bytes, hipMemcpyDeviceToHost, ks)); });
  bw("h2d k_batch_copy 16 WG", [&] { kernel_copy(dev, host, bytes, ks, 16); });
  bw("h2d k_batch_copy 32 WG", [&] { kernel_copy(dev, host, bytes, ks, 32); });
  bw("d2h k_batch_copy 16 WG", [&] { kernel_copy(host, dev, bytes, ks, 16); });
  for (int ne = 1; ne <= (int)std::min<size_t>(4, engines.size()); ++ne) {
    char nm[64];
    snprintf(nm, sizeof nm, "h2d sdma x%d", ne);
    bw(nm, [&] { sdma_copy(dev, ag.gpu, host, ag.cpu, bytes, ne, true); });
    snprintf(nm, sizeof nm, "d2h sdma x%d", ne);
    bw(nm, [&] { sdma_copy(host, ag.cpu, dev, ag.gpu, bytes, ne, true); });
  }

  // ---- interference: victim kernel time alone vs beside a running h2d copy
  auto victim_ms = [&](int reps) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    CK(hipEventRecord(a, cs));
    for (int r = 0; r < reps; ++r)
      hipLaunchKernelGGL(k_stream_read, dim3(2048), dim3(256), 0, cs, (const uint4*)victim, vbytes / 16, sink);
    CK(hipEventRecord(b, cs));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    CK(hipEventDestroy(a));
    CK(hipEventDestroy(b));
    return ms / reps;
  };
  victim_ms(3);
  float alone = victim_ms(20);
  printf("== interference: 2 GB streaming read, %.3f ms alone (%.0f GB/s)\n", alone, vbytes / alone / 1e6);
  auto beside = [&](const char* name, auto&& start_copy) {
    start_copy();
    float t = victim_ms(20);
    CK(hipDeviceSynchronize());
    printf("%-34s %7.3f ms (%.2fx)\n", name, t, t / alone);
  };
  const int nbig = 8;  // keep the copy running for the whole victim loop
  beside("beside hipMemcpyAsync h2d", [&] {
    for (int i = 0; i < nbig; ++i) CK(hipMemcpyAsync(dev, host, bytes, hipMemcpyHostToDevice, ks));
  });
  beside("beside k_batch_copy h2d 16 WG", [&] {
    for (int i = 0; i < nbig; ++i) kernel_copy(dev, host, bytes, ks, 16);
  });
  std::vector<hsa_signal_t> pend;
  beside("beside sdma h2d x2", [&] {
    for (int i = 0; i < nbig; ++i) {
      auto s = sdma_copy(dev, ag.gpu, host, ag.cpu, bytes, (int)std::min<size_t>(2, engines.size()), false);
      pend.insert(pend.end(), s.begin(), s.end());
    }
  });
  for (auto s : pend) {
    hsa_signal_wait_scacquire(s, HSA_SIGNAL_CONDITION_LT, 1, UINT64_MAX, HSA_WAIT_STATE_BLOCKED);
    hsa_signal_destroy(s);
  }
  CK(hipDeviceSynchronize());
  printf("done\n");
  return 0;
}
