// HBM <-> host-node (CXL pool stand-in) write/read paths, per NUMA node (MI355X).
//
// The emulated CXL pool of a multi-socket box is a NUMA node; for a GPU on
// socket S its pool is either on S ("local") or on the other socket ("remote").
// Round 2 measured HBM -> remote node at 12.8 GB/s through one SDMA engine.
// For every NUMA node with memory this probe measures, 1 GiB each way:
//   memcpy    hipMemcpyAsync (ROCclr blit / SDMA as the runtime chooses)
//   sdma1     one SDMA engine (hsa_amd_memory_async_copy_on_engine), per engine
//   sdmaN     64 MiB pieces round-robin over every engine of the direction's mask
//   cu<G>     a CU copy kernel (G workgroups) reading / writing the pinned pages
//   bounce    D2H into a staging ring on the GPU's own node (SDMA) + T CPU
//             threads copying each landed 64 MiB piece to the target node,
//             pipelined (H2D: the reverse)
//   cpu<T>    the CPU copy alone (GPU-node pinned -> target node), T threads
// Output: one JSON line per (node, path, direction).
//
//   hipcc -O3 --offload-arch=gfx950 tools/probe_cxl_paths.hip -o tools/bin/probe_cxl_paths -lhsa-runtime64 -lpthread
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <sys/mman.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <dirent.h>
#include <string>
#include <thread>
#include <vector>

#define CK(x)                                                                                  \
  do {                                                                                         \
    hipError_t e_ = (x);                                                                       \
    if (e_ != hipSuccess) {                                                                    \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));        \
      exit(1);                                                                                 \
    }                                                                                          \
  } while (0)

static double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static std::string read_line(const std::string& p) {
  FILE* f = fopen(p.c_str(), "r");
  if (!f) return "";
  char buf[256] = {0};
  if (!fgets(buf, sizeof buf, f)) buf[0] = 0;
  fclose(f);
  std::string s(buf);
  while (!s.empty() && (s.back() == '\n' || s.back() == ' ')) s.pop_back();
  return s;
}

static std::vector<int> memory_nodes() {
  std::vector<int> out;
  DIR* d = opendir("/sys/devices/system/node");
  if (!d) return out;
  while (dirent* e = readdir(d))
    if (!strncmp(e->d_name, "node", 4) && e->d_name[4] >= '0' && e->d_name[4] <= '9') out.push_back(atoi(e->d_name + 4));
  closedir(d);
  std::sort(out.begin(), out.end());
  return out;
}

// Page-aligned anonymous memory bound to `node`, populated there and registered with HIP.
static void* alloc_on_node(size_t bytes, int node) {
  void* p = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
  if (p == MAP_FAILED) return nullptr;
  unsigned long mask[4] = {0, 0, 0, 0};
  mask[node / 64] |= 1ul << (node % 64);
  long r = syscall(SYS_mbind, p, bytes, 2 /*MPOL_BIND*/, mask, 256, 0);
  if (r != 0) fprintf(stderr, "mbind node %d failed (errno %d)\n", node, errno);
  memset(p, 1, bytes);
  CK(hipHostRegister(p, bytes, hipHostRegisterMapped));
  return p;
}

static void free_on_node(void* p, size_t bytes) {
  (void)hipHostUnregister(p);
  munmap(p, bytes);
}

// The node a page actually landed on (get_mempolicy MPOL_F_NODE | MPOL_F_ADDR).
static int page_node(void* p) {
  int node = -1;
  if (syscall(SYS_get_mempolicy, &node, nullptr, 0, p, 3) != 0) return -1;
  return node;
}

__global__ void __launch_bounds__(256) k_copy16(uint4* __restrict__ dst, const uint4* __restrict__ src, uint64_t n16) {
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * 256) dst[i] = src[i];
}

struct Agents {
  std::vector<hsa_agent_t> gpus, cpus;
};

static hsa_status_t agent_cb(hsa_agent_t a, void* data) {
  auto* ag = (Agents*)data;
  hsa_device_type_t t;
  hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t);
  if (t == HSA_DEVICE_TYPE_GPU) ag->gpus.push_back(a);
  if (t == HSA_DEVICE_TYPE_CPU) ag->cpus.push_back(a);
  return HSA_STATUS_SUCCESS;
}

struct Sdma {
  hsa_agent_t gpu{}, cpu{};
  uint32_t h2d = 0, d2h = 0;
  hsa_signal_t sig{};
};

// Copy `bytes` in `piece`-sized pieces over the engines in `mask` (round-robin), wait.
static bool sdma_copy(Sdma& s, void* dst, bool dst_gpu, const void* src, size_t bytes, uint32_t mask, size_t piece) {
  std::vector<uint32_t> engs;
  for (int b = 0; b < 32; ++b)
    if ((mask >> b) & 1) engs.push_back(1u << b);
  if (engs.empty()) return false;
  size_t n = (bytes + piece - 1) / piece;
  hsa_signal_store_relaxed(s.sig, (hsa_signal_value_t)n);
  for (size_t i = 0; i < n; ++i) {
    size_t off = i * piece, len = std::min(piece, bytes - off);
    hsa_status_t st = hsa_amd_memory_async_copy_on_engine(
        (char*)dst + off, dst_gpu ? s.gpu : s.cpu, (const char*)src + off, dst_gpu ? s.cpu : s.gpu, len, 0, nullptr,
        s.sig, (hsa_amd_sdma_engine_id_t)engs[i % engs.size()], true);
    if (st != HSA_STATUS_SUCCESS) {
      fprintf(stderr, "sdma copy failed 0x%x\n", (unsigned)st);
      hsa_signal_subtract_relaxed(s.sig, (hsa_signal_value_t)(n - i));
      hsa_signal_wait_scacquire(s.sig, HSA_SIGNAL_CONDITION_EQ, 0, UINT64_MAX, HSA_WAIT_STATE_BLOCKED);
      return false;
    }
  }
  hsa_signal_wait_scacquire(s.sig, HSA_SIGNAL_CONDITION_EQ, 0, UINT64_MAX, HSA_WAIT_STATE_BLOCKED);
  return true;
}

static void par_memcpy(void* dst, const void* src, size_t bytes, int threads) {
  std::vector<std::thread> ts;
  size_t per = (bytes / threads + 4095) & ~(size_t)4095;
  for (int t = 0; t < threads; ++t) {
    size_t off = (size_t)t * per;
    if (off >= bytes) break;
    size_t len = std::min(per, bytes - off);
    ts.emplace_back([=] { memcpy((char*)dst + off, (const char*)src + off, len); });
  }
  for (auto& t : ts) t.join();
}

static void emit(int gnode, int node, const char* path, const char* dir, double gbps, const char* extra = "") {
  printf("{\"gpu_node\": %d, \"node\": %d, \"where\": \"%s\", \"path\": \"%s\", \"dir\": \"%s\", \"gbps\": %.2f%s}\n",
         gnode, node, node == gnode ? "local" : "remote", path, dir, gbps, extra);
  fflush(stdout);
}

int main(int argc, char** argv) {
  const size_t bytes = (size_t)(argc > 1 ? atoi(argv[1]) : 1024) << 20;
  const int iters = 3;
  const size_t piece = 64ull << 20;
  CK(hipSetDevice(0));
  char bus[64] = {0};
  CK(hipDeviceGetPCIBusId(bus, sizeof bus, 0));
  std::string bdf(bus);
  for (auto& c : bdf) c = (char)tolower(c);
  int gnode = atoi(read_line("/sys/bus/pci/devices/" + bdf + "/numa_node").c_str());
  if (gnode < 0) gnode = 0;
  std::vector<int> nodes = memory_nodes();
  printf("{\"probe\": \"cxl_paths\", \"gpu_bdf\": \"%s\", \"gpu_node\": %d, \"nodes\": %zu, \"bytes\": %zu}\n",
         bdf.c_str(), gnode, nodes.size(), bytes);

  Agents ag;
  hsa_init();
  hsa_iterate_agents(agent_cb, &ag);
  Sdma s;
  {
    unsigned dom = 0, b = 0, dv = 0, fn = 0;
    sscanf(bus, "%x:%x:%x.%x", &dom, &b, &dv, &fn);
    uint32_t want = (b << 8) | (dv << 3) | fn;
    for (auto g : ag.gpus) {
      uint32_t id = 0;
      hsa_agent_get_info(g, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_BDFID, &id);
      if (id == want) s.gpu = g;
    }
    if (!s.gpu.handle && !ag.gpus.empty()) s.gpu = ag.gpus[0];
    s.cpu = ag.cpus.empty() ? hsa_agent_t{0} : ag.cpus[0];
    hsa_amd_memory_copy_engine_status(s.gpu, s.cpu, &s.h2d);
    hsa_amd_memory_copy_engine_status(s.cpu, s.gpu, &s.d2h);
    hsa_signal_create(1, 0, nullptr, &s.sig);
    uint32_t ph = 0, pd = 0;
    hsa_amd_memory_get_preferred_copy_engine(s.gpu, s.cpu, &ph);
    hsa_amd_memory_get_preferred_copy_engine(s.cpu, s.gpu, &pd);
    printf("{\"cpu_agents\": %zu, \"sdma_h2d_mask\": %u, \"sdma_d2h_mask\": %u, \"preferred_h2d\": %u, "
           "\"preferred_d2h\": %u}\n", ag.cpus.size(), s.h2d, s.d2h, ph, pd);
  }

  void* dev = nullptr;
  CK(hipMalloc(&dev, bytes));
  CK(hipMemset(dev, 7, bytes));
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  // staging ring on the GPU's own node (the bounce path)
  const int nslots = 4;
  void* stage = alloc_on_node((size_t)nslots * piece, gnode);

  for (int node : nodes) {
    std::string mt = read_line("/sys/devices/system/node/node" + std::to_string(node) + "/meminfo");
    void* host = alloc_on_node(bytes, node);
    if (!host) continue;
    char extra[96];
    snprintf(extra, sizeof extra, ", \"page_node\": %d", page_node((char*)host + bytes / 2));
    void* hdev = nullptr;
    CK(hipHostGetDevicePointer(&hdev, host, 0));
    auto timed = [&](auto fn) {
      fn();
      double t0 = now();
      for (int i = 0; i < iters; ++i) fn();
      return (double)iters * bytes / (now() - t0) / 1e9;
    };
    // hipMemcpyAsync
    emit(gnode, node, "memcpy", "d2h", timed([&] {
      CK(hipMemcpyAsync(host, dev, bytes, hipMemcpyDeviceToHost, st));
      CK(hipStreamSynchronize(st));
    }), extra);
    emit(gnode, node, "memcpy", "h2d", timed([&] {
      CK(hipMemcpyAsync(dev, host, bytes, hipMemcpyHostToDevice, st));
      CK(hipStreamSynchronize(st));
    }), extra);
    // SDMA: each engine alone, then all engines
    for (int b = 0; b < 32; ++b) {
      char name[32];
      if ((s.d2h >> b) & 1) {
        snprintf(name, sizeof name, "sdma1_e%d", b);
        emit(gnode, node, name, "d2h", timed([&] { sdma_copy(s, host, false, dev, bytes, 1u << b, piece); }), extra);
      }
      if ((s.h2d >> b) & 1) {
        snprintf(name, sizeof name, "sdma1_e%d", b);
        emit(gnode, node, name, "h2d", timed([&] { sdma_copy(s, dev, true, host, bytes, 1u << b, piece); }), extra);
      }
    }
    emit(gnode, node, "sdmaN", "d2h", timed([&] { sdma_copy(s, host, false, dev, bytes, s.d2h, piece); }), extra);
    emit(gnode, node, "sdmaN", "h2d", timed([&] { sdma_copy(s, dev, true, host, bytes, s.h2d, piece); }), extra);
    // CU kernels through the mapped pinned pages
    for (int g : {32, 128, 512}) {
      char name[32];
      snprintf(name, sizeof name, "cu%d", g);
      emit(gnode, node, name, "d2h", timed([&] {
        hipLaunchKernelGGL(k_copy16, dim3(g), dim3(256), 0, st, (uint4*)hdev, (const uint4*)dev, bytes / 16);
        CK(hipStreamSynchronize(st));
      }), extra);
      emit(gnode, node, name, "h2d", timed([&] {
        hipLaunchKernelGGL(k_copy16, dim3(g), dim3(256), 0, st, (uint4*)dev, (const uint4*)hdev, bytes / 16);
        CK(hipStreamSynchronize(st));
      }), extra);
    }
    if (node != gnode && stage) {
      // CPU copies alone: GPU-node pinned staging -> target node
      for (int t : {4, 8, 16}) {
        char name[32];
        snprintf(name, sizeof name, "cpu%d", t);
        emit(gnode, node, name, "local_to_node", timed([&] {
          for (size_t off = 0; off < bytes; off += (size_t)nslots * piece)
            par_memcpy((char*)host + off, stage, std::min((size_t)nslots * piece, bytes - off), t);
        }), extra);
      }
      // pipelined bounce: SDMA piece i -> staging slot (i % nslots), CPU threads drain slot i - 1
      for (int t : {8, 16}) {
        char name[32];
        snprintf(name, sizeof name, "bounce_cpu%d", t);
        emit(gnode, node, name, "d2h", timed([&] {
          size_t n = bytes / piece;
          std::vector<hsa_signal_t> sg(nslots);
          for (auto& x : sg) hsa_signal_create(1, 0, nullptr, &x);
          uint32_t eng = s.d2h & (~s.d2h + 1);
          auto issue = [&](size_t i) {
            hsa_signal_store_relaxed(sg[i % nslots], 1);
            hsa_amd_memory_async_copy_on_engine((char*)stage + (i % nslots) * piece, s.cpu, (char*)dev + i * piece,
                                                s.gpu, piece, 0, nullptr, sg[i % nslots],
                                                (hsa_amd_sdma_engine_id_t)eng, true);
          };
          for (size_t i = 0; i < std::min(n, (size_t)nslots - 1); ++i) issue(i);
          for (size_t i = 0; i < n; ++i) {
            hsa_signal_wait_scacquire(sg[i % nslots], HSA_SIGNAL_CONDITION_EQ, 0, UINT64_MAX, HSA_WAIT_STATE_BLOCKED);
            if (i + nslots - 1 < n) issue(i + nslots - 1);
            par_memcpy((char*)host + i * piece, (char*)stage + (i % nslots) * piece, piece, t);
          }
          for (auto& x : sg) hsa_signal_destroy(x);
        }), extra);
        emit(gnode, node, name, "h2d", timed([&] {
          size_t n = bytes / piece;
          std::vector<hsa_signal_t> sg(nslots);
          for (auto& x : sg) hsa_signal_create(0, 0, nullptr, &x);
          uint32_t eng = s.h2d & (~s.h2d + 1);
          for (size_t i = 0; i < n; ++i) {
            // slot free once its previous H2D landed
            hsa_signal_wait_scacquire(sg[i % nslots], HSA_SIGNAL_CONDITION_EQ, 0, UINT64_MAX, HSA_WAIT_STATE_BLOCKED);
            par_memcpy((char*)stage + (i % nslots) * piece, (char*)host + i * piece, piece, t);
            hsa_signal_store_relaxed(sg[i % nslots], 1);
            hsa_amd_memory_async_copy_on_engine((char*)dev + i * piece, s.gpu, (char*)stage + (i % nslots) * piece,
                                                s.cpu, piece, 0, nullptr, sg[i % nslots],
                                                (hsa_amd_sdma_engine_id_t)eng, true);
          }
          for (auto& x : sg)
            hsa_signal_wait_scacquire(x, HSA_SIGNAL_CONDITION_EQ, 0, UINT64_MAX, HSA_WAIT_STATE_BLOCKED);
          for (auto& x : sg) hsa_signal_destroy(x);
        }), extra);
      }
    }
    free_on_node(host, bytes);
  }
  if (stage) free_on_node(stage, (size_t)nslots * piece);
  CK(hipFree(dev));
  return 0;
}
