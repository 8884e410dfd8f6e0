// HBM streaming-read ceiling for decode-GEMM-sized launches: what one launch
// that reads S bytes (MALL-cold: rotating over buffers totalling > 1 GB) can
// reach for a given wave count and loads-in-flight per lane. The decode GEMM's
// weight stream is this read plus MFMA work, so this is its speed-of-light at
// that decomposition.
//   hipcc --offload-arch=gfx950 -O3 tools/probe_hbm_read.hip -o build/probe_hbm_read
//   ./build/probe_hbm_read            -> one JSON line per (MB, waves, wg, unroll)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                         \
    }                                                                                  \
  } while (0)

// Each wave reads `per_wave` 1 KB blocks starting at wave * per_wave (lane l
// takes bytes 16 l .. 16 l + 15 of every block), UNR blocks in flight, and
// folds them into one word so the loads are live.
template <int UNR>
__global__ void __launch_bounds__(256) k_read(const u32x4_t* __restrict__ buf, uint64_t nblocks, uint32_t per_wave,
                                              uint32_t* sink) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t wave = (uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const uint64_t b0 = wave * per_wave;
  if (b0 >= nblocks) return;
  const uint64_t b1 = b0 + per_wave < nblocks ? b0 + per_wave : nblocks;
  u32x4_t acc = {0, 0, 0, 0};
  uint64_t b = b0;
  for (; b + UNR <= b1; b += UNR) {
    u32x4_t v[UNR];
#pragma unroll
    for (int u = 0; u < UNR; ++u) v[u] = __builtin_nontemporal_load(buf + (b + u) * 64 + lane);
#pragma unroll
    for (int u = 0; u < UNR; ++u) acc ^= v[u];
  }
  for (; b < b1; ++b) acc ^= __builtin_nontemporal_load(buf + b * 64 + lane);
  if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x9e3779b9u) sink[0] = 1;  // practically never
}

template <int UNR>
static void launch(const u32x4_t* p, uint64_t nblocks, uint32_t waves, uint32_t wg, uint32_t* sink, hipStream_t s) {
  const uint32_t per = (uint32_t)((nblocks + waves - 1) / waves);
  hipLaunchKernelGGL((k_read<UNR>), dim3((waves + wg - 1) / wg), dim3(64 * wg), 0, s, p, nblocks, per, sink);
}

int main() {
  const size_t total = (size_t)3 << 30;  // 3 GB of buffers
  char* base = nullptr;
  CK(hipMalloc(&base, total));
  CK(hipMemset(base, 1, total));
  uint32_t* sink = nullptr;
  CK(hipMalloc(&sink, 4));
  hipStream_t s;
  CK(hipStreamCreate(&s));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const size_t mbs[] = {32, 117, 470, 1024};
  const uint32_t wavesv[] = {256, 512, 768, 1024, 2048, 4096, 8192};
  const uint32_t wgs[] = {1, 4};
  const int unrs[] = {4, 8, 16};
  for (size_t mb : mbs) {
    const size_t bytes = mb << 20;
    const size_t nbuf = total / bytes;  // rotate: every launch reads a MALL-cold buffer
    const uint64_t nblocks = bytes / 1024;
    for (uint32_t waves : wavesv)
      for (uint32_t wg : wgs)
        for (int unr : unrs) {
          auto run = [&](size_t i) {
            const u32x4_t* p = reinterpret_cast<const u32x4_t*>(base + (i % nbuf) * bytes);
            if (unr == 4) launch<4>(p, nblocks, waves, wg, sink, s);
            else if (unr == 8) launch<8>(p, nblocks, waves, wg, sink, s);
            else launch<16>(p, nblocks, waves, wg, sink, s);
          };
          for (size_t i = 0; i < nbuf; ++i) run(i);
          CK(hipStreamSynchronize(s));
          const int it = 24;
          CK(hipEventRecord(e0, s));
          for (int i = 0; i < it; ++i) run(i);
          CK(hipEventRecord(e1, s));
          CK(hipEventSynchronize(e1));
          float ms = 0;
          CK(hipEventElapsedTime(&ms, e0, e1));
          const double us = 1e3 * ms / it;
          printf("{\"mb\": %zu, \"waves\": %u, \"wg_waves\": %u, \"unroll\": %d, \"us\": %.2f, \"gbps\": %.1f}\n", mb,
                 waves, wg, unr, us, bytes / us / 1e3);
          fflush(stdout);
        }
  }
  CK(hipGetLastError());
  return 0;
}
