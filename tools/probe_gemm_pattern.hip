// What costs the decode GEMM its streaming rate: the k_dgemm_pipe access
// pattern rebuilt step by step on MALL-cold weights, each variant one launch of
// `waves` one-wave workgroups over an [N, K] fragment-ordered bf16 matrix
// (unit = 4 row tiles x one K split, two register sets of 2 K steps):
//   w      weight fragments only (4 row-tile streams per wave), xor-folded
//   wx     + the 4 activation fragments per K step (L2-resident x)
//   wxm    + the 16 MFMAs per K step (= k_dgemm_pipe without the partial store)
//   wxms   + the f32 partial store (= k_dgemm_pipe)
//   xf*    the same with the activations stored in fragment order (16 x 32
//          tiles, 1 KB contiguous: one fully coalesced load per fragment)
//   hipcc --offload-arch=gfx950 -O3 tools/probe_gemm_pattern.hip -o build/probe_gemm_pattern
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                         \
    }                                                                                  \
  } while (0)

struct Args {
  const uint16_t* w;
  const uint16_t* x;
  float* part;
  uint32_t M, N, K, ksplit, klen, row_blocks;
  float magic;  // runtime value the folded result is compared with (keeps the loads live)
};

template <bool X, bool XF>
__device__ __forceinline__ void ld(u32x4_t (&wv)[2][4], u32x4_t (&xv)[2][4], const uint16_t* const (&wb)[4],
                                   const uint16_t* const (&xr)[4], uint32_t kst) {
#pragma unroll
  for (int u = 0; u < 2; ++u)
#pragma unroll
    for (int r = 0; r < 4; ++r)
      wv[u][r] = __builtin_nontemporal_load(reinterpret_cast<const u32x4_t*>(wb[r] + (uint64_t)(kst + u) * 512u));
  if (X) {
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
        xv[u][mt] = *reinterpret_cast<const u32x4_t*>(xr[mt] + (kst + u) * (XF ? 512u : 32u));
  }
}

template <bool X, bool MF>
__device__ __forceinline__ void use(f32x4_t (&acc)[4][4], u32x4_t& fold, const u32x4_t (&wv)[2][4],
                                    const u32x4_t (&xv)[2][4]) {
#pragma unroll
  for (int u = 0; u < 2; ++u)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      if (MF) {
#pragma unroll
        for (int mt = 0; mt < 4; ++mt)
          acc[r][mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, wv[u][r]),
                                                               __builtin_bit_cast(bf16x8_t, xv[u][mt]), acc[r][mt], 0,
                                                               0, 0);
      } else {
        fold ^= wv[u][r];
        if (X) fold ^= xv[u][r];
      }
    }
}

template <bool X, bool MF, bool ST, bool XF>
__global__ void __launch_bounds__(64) k_pat(Args a) {
  const uint32_t lane = threadIdx.x;
  const uint32_t unit = blockIdx.x;
  if (unit >= a.row_blocks * a.ksplit) return;
  const uint32_t rb = unit / a.ksplit, ks = unit - rb * a.ksplit;
  const uint32_t k_lo = ks * a.klen, k_hi = k_lo + a.klen < a.K ? k_lo + a.klen : a.K;
  const uint32_t kfr = a.K >> 5;
  const uint16_t* wb[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) wb[r] = a.w + (uint64_t)(rb * 4 + r) * kfr * 512u + lane * 8u;
  const uint16_t* xr[4];
#pragma unroll
  for (int mt = 0; mt < 4; ++mt)
    xr[mt] = XF ? a.x + (uint64_t)mt * kfr * 512u + lane * 8u
                : a.x + (uint64_t)(mt * 16 + (lane & 15u)) * a.K + 8u * (lane >> 4);
  f32x4_t acc[4][4];
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) acc[r][mt] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  u32x4_t fold = {0, 0, 0, 0};
  const uint32_t s0 = k_lo >> 5, nsteps = (k_hi - k_lo) >> 5, nbat = nsteps / 2;
  u32x4_t wA[2][4], xA[2][4], wB[2][4], xB[2][4];
  ld<X, XF>(wA, xA, wb, xr, s0);
  uint32_t b = 0;
  for (; b + 2 < nbat; b += 2) {
    ld<X, XF>(wB, xB, wb, xr, s0 + (b + 1) * 2);
    __builtin_amdgcn_sched_barrier(0);
    use<X, MF>(acc, fold, wA, xA);
    __builtin_amdgcn_sched_barrier(0);
    ld<X, XF>(wA, xA, wb, xr, s0 + (b + 2) * 2);
    __builtin_amdgcn_sched_barrier(0);
    use<X, MF>(acc, fold, wB, xB);
    __builtin_amdgcn_sched_barrier(0);
  }
  if (b + 1 < nbat) {
    ld<X, XF>(wB, xB, wb, xr, s0 + (b + 1) * 2);
    use<X, MF>(acc, fold, wA, xA);
    use<X, MF>(acc, fold, wB, xB);
  } else {
    use<X, MF>(acc, fold, wA, xA);
  }
  if (ST) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const uint32_t n = (rb * 4 + r) * 16u + 4u * (lane >> 4);
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) {
        const uint32_t m = mt * 16 + (lane & 15u);
        *reinterpret_cast<f32x4_t*>(a.part + ((uint64_t)ks * a.M + m) * a.N + n) = acc[r][mt];
      }
    }
  } else {
    float s = __uint_as_float(fold.x ^ fold.y ^ fold.z ^ fold.w);
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) s += acc[r][mt].x + acc[r][mt].y + acc[r][mt].z + acc[r][mt].w;
    if (s == a.magic) a.part[lane] = s;  // keep the work live
  }
}

int main() {
  const size_t total = (size_t)3 << 30;
  char* base = nullptr;
  CK(hipMalloc(&base, total));
  CK(hipMemset(base, 0, total));
  uint16_t* x = nullptr;
  CK(hipMalloc(&x, 64 * 28672 * 2));
  CK(hipMemset(x, 0, 64 * 28672 * 2));
  float* part = nullptr;
  CK(hipMalloc(&part, (size_t)256 << 20));
  hipStream_t s;
  CK(hipStreamCreate(&s));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const uint32_t shapes[][2] = {{4096, 4096}, {14336, 4096}, {4096, 14336}, {57344, 8192}};
  const uint32_t unitsv[] = {512, 768, 1024, 2048};
  const char* names[] = {"w", "wx", "wxm", "wxms", "wxf", "wxfm", "wxfms"};
  for (auto& sh : shapes) {
    const uint32_t N = sh[0], K = sh[1];
    const size_t bytes = (size_t)N * K * 2;
    const size_t nbuf = total / bytes;
    for (uint32_t target : unitsv) {
      const uint32_t rb = N / 64;
      uint32_t ksp = rb >= target ? 1 : (target + rb - 1) / rb;
      const uint32_t ksteps = K / 32;
      if (ksp > ksteps / 4) ksp = ksteps / 4;
      const uint32_t steps = (ksteps + ksp - 1) / ksp;
      Args a{nullptr, x, part, 64, N, K, (K + steps * 32 - 1) / (steps * 32), steps * 32, rb, 12345.678f};
      if ((size_t)a.ksplit * 64 * N * 4 > ((size_t)256 << 20)) continue;
      for (int v = 0; v < 7; ++v) {
        auto run = [&](size_t i) {
          Args b = a;
          b.w = reinterpret_cast<const uint16_t*>(base + (i % nbuf) * bytes);
          const dim3 g(rb * a.ksplit), blk(64);
          if (v == 0) hipLaunchKernelGGL((k_pat<false, false, false, false>), g, blk, 0, s, b);
          else if (v == 1) hipLaunchKernelGGL((k_pat<true, false, false, false>), g, blk, 0, s, b);
          else if (v == 2) hipLaunchKernelGGL((k_pat<true, true, false, false>), g, blk, 0, s, b);
          else if (v == 3) hipLaunchKernelGGL((k_pat<true, true, true, false>), g, blk, 0, s, b);
          else if (v == 4) hipLaunchKernelGGL((k_pat<true, false, false, true>), g, blk, 0, s, b);
          else if (v == 5) hipLaunchKernelGGL((k_pat<true, true, false, true>), g, blk, 0, s, b);
          else hipLaunchKernelGGL((k_pat<true, true, true, true>), g, blk, 0, s, b);
        };
        for (size_t i = 0; i < nbuf + 2; ++i) run(i);
        CK(hipStreamSynchronize(s));
        const int it = 24;
        CK(hipEventRecord(e0, s));
        for (int i = 0; i < it; ++i) run(i);
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        const double us = 1e3 * ms / it;
        printf("{\"N\": %u, \"K\": %u, \"units\": %u, \"ksplit\": %u, \"variant\": \"%s\", \"us\": %.2f, \"gbps\": %.1f}\n",
               N, K, rb * a.ksplit, a.ksplit, names[v], us, bytes / us / 1e3);
        fflush(stdout);
      }
    }
  }
  CK(hipGetLastError());
  return 0;
}
