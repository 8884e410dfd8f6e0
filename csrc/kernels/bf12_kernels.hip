// Fused H2D copy + BF12 decode (see ogkm/codec.hpp for the format).
//
// One work item = one 32768-value tile (64 KB of bf16 output) of one block. A
// workgroup of 256 threads (4 waves):
//   1. streams the tile's packed planes straight from pinned host / CXL memory
//      (16-B sign|mantissa loads + 8-B exponent-code loads per lane, non-temporal:
//      48 KB cross PCIe instead of 64 KB),
//   2. rebuilds the bf16 words into an LDS staging tile (64 KB),
//   3. patches the tile's escaped values into LDS,
//   4. writes the finished tile to HBM with 16-B non-temporal stores.
// The kernel is PCIe-bound like the plain copy kernel; LDS staging keeps the HBM
// write pass fully coalesced and writes every output byte exactly once.
#include <hip/hip_runtime.h>

#include "ogkm/codec.hpp"
#include "ogkm/kernels.hpp"

namespace ogkm {

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

constexpr int kDecThreads = 256;

// 4 values: sign|mantissa bytes in `s` (one per byte), 4 codes in the low 16
// bits of `c` (one nibble each) -> two u32 words of packed bf16 pairs.
__device__ __forceinline__ u32x2 dec4(uint32_t s, uint32_t c, uint32_t base) {
  u32x2 r;
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    uint32_t w = 0;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      int k = 2 * p + q;
      uint32_t sm = (s >> (8 * k)) & 0xFF;
      uint32_t e = (base + ((c >> (4 * k)) & 0xF)) & 0xFF;
      uint32_t v = ((sm & 0x80) << 8) | (e << 7) | (sm & 0x7F);
      w |= v << (16 * q);
    }
    r[p] = w;
  }
  return r;
}

__global__ void __launch_bounds__(kDecThreads)
    k_bf12_decode(KBf12Descs inl, uint32_t n, uint64_t total_items) {
  __shared__ u32x4 tile[kBf12Tile * 2 / 16];  // 64 KB staging tile
  __shared__ uint32_t s_desc, s_base, s_e0, s_e1;
  uint32_t hint = 0;
  for (uint64_t item = blockIdx.x; item < total_items; item += gridDim.x) {
    if (threadIdx.x == 0) {
      uint32_t i = hint;
      while (i + 1 < n && inl.item_start[i + 1] <= item) ++i;
      if (inl.item_start[i] > item) {
        i = 0;
        while (i + 1 < n && inl.item_start[i + 1] <= item) ++i;
      }
      s_desc = i;
      const Bf12Header* h = reinterpret_cast<const Bf12Header*>(inl.d[i].src);
      uint32_t t = (uint32_t)(item - inl.item_start[i]);
      s_base = __builtin_nontemporal_load(&h->base);
      s_e0 = __builtin_nontemporal_load(&h->exc_off[t]);
      s_e1 = __builtin_nontemporal_load(&h->exc_off[t + 1]);
    }
    __syncthreads();
    const uint32_t di = s_desc;
    hint = di;
    const KBf12Desc d = inl.d[di];
    const uint32_t t = (uint32_t)(item - inl.item_start[di]);
    const uint32_t lo = t * kBf12Tile;
    const uint32_t cnt = d.n_values - lo < kBf12Tile ? d.n_values - lo : kBf12Tile;
    const uint32_t base = s_base;
    const uint8_t* src = reinterpret_cast<const uint8_t*>(d.src);
    // 8 values per lane-group: 8 B of sign|mantissa + 4 B of codes -> 16 B of bf16,
    // so consecutive lanes write consecutive 16-B LDS slots (conflict-free).
    const u32x2* sm8 = reinterpret_cast<const u32x2*>(src + kBf12HeaderBytes + lo);
    const uint32_t* cd4 = reinterpret_cast<const uint32_t*>(src + kBf12HeaderBytes + d.n_values + lo / 2);
    const uint32_t groups = cnt / 8;  // <= 4096 -> 16 per thread
    const Bf12Exception* exc =
        reinterpret_cast<const Bf12Exception*>(src + kBf12HeaderBytes + d.n_values + d.n_values / 2);
    const uint32_t e0 = s_e0, e1 = s_e1;
    // 1: issue every load of the tile (and this lane's first exception) before
    //    using any of it: 48 KB per workgroup in flight across PCIe.
    constexpr int kPer = kBf12Tile / 8 / kDecThreads;  // 16
    u32x2 s[kPer];
    uint32_t c[kPer];
#pragma unroll
    for (int u = 0; u < kPer; ++u) {
      uint32_t g = threadIdx.x + u * kDecThreads;
      if (g < groups) {
        s[u] = __builtin_nontemporal_load(sm8 + g);
        c[u] = __builtin_nontemporal_load(cd4 + g);
      }
    }
    const bool has_ex = e0 + threadIdx.x < e1;
    Bf12Exception ex0 = {0, 0, 0};
    if (has_ex) ex0 = exc[e0 + threadIdx.x];
    // 2: rebuild bf16 words into the LDS staging tile.
#pragma unroll
    for (int u = 0; u < kPer; ++u) {
      uint32_t g = threadIdx.x + u * kDecThreads;
      if (g < groups) {
        u32x2 a0 = dec4(s[u][0], c[u], base), a1 = dec4(s[u][1], c[u] >> 16, base);
        tile[g] = u32x4{a0[0], a0[1], a1[0], a1[1]};
      }
    }
    __syncthreads();
    // 3: patch escaped values (rare) in LDS.
    uint16_t* t16 = reinterpret_cast<uint16_t*>(tile);
    if (has_ex) t16[ex0.index - lo] = ex0.bits;
    for (uint32_t k = e0 + threadIdx.x + kDecThreads; k < e1; k += kDecThreads) {
      Bf12Exception ex = exc[k];
      t16[ex.index - lo] = ex.bits;
    }
    __syncthreads();
    // 4: coalesced write of the finished tile to HBM.
    u32x4* dst = reinterpret_cast<u32x4*>(d.dst + (uint64_t)lo * 2);
    for (uint32_t q = threadIdx.x; q < cnt / 8; q += kDecThreads) __builtin_nontemporal_store(tile[q], dst + q);
    __syncthreads();
  }
}

hipError_t launch_bf12_decode(const KBf12Descs& inl, uint32_t n, uint32_t workgroups, hipStream_t s) {
  uint64_t total = inl.item_start[n];
  if (n == 0 || total == 0) return hipSuccess;
  uint32_t grid = (uint32_t)(total < workgroups ? total : workgroups);
  hipLaunchKernelGGL(k_bf12_decode, dim3(grid), dim3(kDecThreads), 0, s, inl, n, total);
  return hipGetLastError();
}


// ---------------------------------------------------------------------------
// BF11 tile decode (codec.hpp): one 32768-value tile of a BF11 block, HBM ->
// HBM. Each wave owns 16 of the tile's 64 wave groups (512 values; 8 per lane).
// Phase 1 issues every sign|mantissa (8 B) and primary-code (2 B) load; phase 2
// turns each lane's escape count into its first secondary nibble with a wave
// prefix count (4 ballots + mbcnt - no LDS, no barrier) and issues the nibble
// loads; phase 3 rebuilds the bf16 words and stores 16 B per lane.
__device__ __forceinline__ uint32_t mbcnt64(uint64_t m) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// Escapes before this lane in the wave, for per-lane counts 0..8.
__device__ __forceinline__ uint32_t wave_excl_prefix8(uint32_t cnt) {
  const uint64_t b0 = __ballot(cnt & 1u), b1 = __ballot(cnt & 2u), b2 = __ballot(cnt & 4u), b3 = __ballot(cnt & 8u);
  return mbcnt64(b0) + 2u * mbcnt64(b1) + 4u * mbcnt64(b2) + 8u * mbcnt64(b3);
}

__device__ __forceinline__ uint32_t bf11_word(uint32_t sm, uint32_t pcv, uint32_t& nibs, uint32_t prim,
                                              uint32_t sbase, int k) {
  const uint32_t c = (pcv >> (2 * k)) & 3u;
  const bool esc = c == 3u;
  const uint32_t e = esc ? ((sbase + (nibs & 15u)) & 0xFFu) : ((prim >> (8u * c)) & 0xFFu);
  nibs = esc ? nibs >> 4 : nibs;
  const uint32_t b = (sm >> (8 * (k & 3))) & 0xFFu;
  return ((b & 0x80u) << 8) | (e << 7) | (b & 0x7Fu);
}

__device__ __forceinline__ void bf11_decode_tile(const uint8_t* __restrict__ blk, uint16_t* __restrict__ out,
                                                 uint32_t t) {
  const Bf11Header* h = reinterpret_cast<const Bf11Header*>(blk);
  const uint32_t n = h->n_values;
  const uint32_t prim = h->prim, sbase = h->sec_base;
  const uint8_t* sm_plane = blk + kBf11HeaderBytes;
  const uint16_t* pc_plane = reinterpret_cast<const uint16_t*>(blk + h->off_prim);
  const uint32_t* wg_plane = reinterpret_cast<const uint32_t*>(blk + h->off_wg);
  const uint32_t* sec32 = reinterpret_cast<const uint32_t*>(blk + h->off_sec);
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  constexpr int kPer = kBf12Tile / kBf11Group / (kDecThreads / 64);  // 16 groups per wave
  u32x2 smv[kPer];
  uint32_t pcv[kPer];
  uint32_t valid = 0;
#pragma unroll
  for (int u = 0; u < kPer; ++u) {
    const uint32_t g = t * (kBf12Tile / kBf11Group) + (uint32_t)u * (kDecThreads / 64) + wave;
    const uint32_t v0 = g * kBf11Group + lane * 8u;
    pcv[u] = 0;
    if (v0 < n) {
      smv[u] = __builtin_nontemporal_load(reinterpret_cast<const u32x2*>(sm_plane + v0));
      pcv[u] = __builtin_nontemporal_load(pc_plane + (v0 >> 3));
      valid |= 1u << u;
    }
  }
  uint32_t nib[kPer];
#pragma unroll
  for (int u = 0; u < kPer; ++u) {
    const uint32_t g = t * (kBf12Tile / kBf11Group) + (uint32_t)u * (kDecThreads / 64) + wave;
    const uint32_t escm = pcv[u] & (pcv[u] >> 1) & 0x5555u;
    const uint32_t pre = wave_excl_prefix8((uint32_t)__builtin_popcount(escm));  // every lane joins
    nib[u] = 0;
    if ((valid >> u) & 1u) {
      const uint32_t idx = wg_plane[g] + pre;
      if (escm) {
        const uint32_t q = idx >> 3, sh = (idx & 7u) * 4u;
        const uint64_t w = ((uint64_t)sec32[q + 1] << 32) | sec32[q];
        nib[u] = (uint32_t)(w >> sh);
      }
    }
  }
#pragma unroll
  for (int u = 0; u < kPer; ++u) {
    if ((valid >> u) & 1u) {
      const uint32_t g = t * (kBf12Tile / kBf11Group) + (uint32_t)u * (kDecThreads / 64) + wave;
      const uint32_t v0 = g * kBf11Group + lane * 8u;
      uint32_t nb = nib[u];
      u32x4 o;
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        const uint32_t sm = smv[u][p >> 1];
        const uint32_t lo = bf11_word(sm, pcv[u], nb, prim, sbase, 2 * p);
        const uint32_t hi = bf11_word(sm, pcv[u], nb, prim, sbase, 2 * p + 1);
        o[p] = lo | (hi << 16);
      }
      __builtin_nontemporal_store(o, reinterpret_cast<u32x4*>(out + v0));
    }
  }
  const uint32_t e0 = h->exc_off[t], e1 = h->exc_off[t + 1];
  if (e1 > e0) {  // uniform: only tiles with exceptions pay the barrier
    __syncthreads();
    const Bf12Exception* exc = reinterpret_cast<const Bf12Exception*>(blk + h->off_exc);
    for (uint32_t k = e0 + threadIdx.x; k < e1; k += kDecThreads) {
      Bf12Exception ex = exc[k];
      out[ex.index] = ex.bits;
    }
  }
}

// ---------------------------------------------------------------------------
// HBM-resident streams: unpack a packed tensor (codec.hpp "BFS1") into a bf16
// staging buffer right before use. Both sides are HBM, so there is no PCIe
// latency to hide and no need for LDS: every lane decodes 16 groups of 8 values
// straight from registers into coalesced 16-B stores (consecutive lanes ->
// consecutive 16 B), then, after a workgroup barrier, the tile's rare escaped
// values are patched in place. No LDS means many workgroups per CU; the grid is
// one item per tile (a 70B layer is ~27k items, >> 256 CUs).
__global__ void __launch_bounds__(kDecThreads)
    k_bf12_unpack(const uint8_t* __restrict__ stream, uint8_t* __restrict__ out, uint64_t dst_stride,
                  uint32_t tile_shift, uint64_t total_items, uint32_t row_shift, uint32_t chunk_values) {
  const Bf12StreamChunk* table = reinterpret_cast<const Bf12StreamChunk*>(stream + sizeof(Bf12StreamHeader));
  for (uint64_t item = blockIdx.x; item < total_items; item += gridDim.x) {
    const uint64_t c = item >> tile_shift;
    const uint32_t t = (uint32_t)(item & ((1u << tile_shift) - 1));
    const Bf12StreamChunk ch = table[c];  // uniform: scalar loads
    const uint32_t lo = t * kBf12Tile;
    if (lo >= ch.n_values) continue;     // uniform across the workgroup
    const uint32_t cnt = ch.n_values - lo < kBf12Tile ? ch.n_values - lo : kBf12Tile;
    const uint8_t* blk = stream + ch.offset;
    const uint64_t doff = (c >> row_shift) * dst_stride + (c & ((1ull << row_shift) - 1)) * chunk_values;
    u32x4* dst = reinterpret_cast<u32x4*>(out + (doff + lo) * 2);
    if (!ch.encoded) {  // raw chunk: plain tile copy (cnt may have an odd tail)
      const u32x4* src = reinterpret_cast<const u32x4*>(blk + (uint64_t)lo * 2);
      for (uint32_t q = threadIdx.x; q < cnt / 8; q += kDecThreads) __builtin_nontemporal_store(src[q], dst + q);
      const uint16_t* s16 = reinterpret_cast<const uint16_t*>(blk) + lo;
      uint16_t* d16 = reinterpret_cast<uint16_t*>(out) + doff + lo;
      for (uint32_t k = (cnt & ~7u) + threadIdx.x; k < cnt; k += kDecThreads) d16[k] = s16[k];
      continue;
    }
    if (ch.encoded == 2) {
      bf11_decode_tile(blk, reinterpret_cast<uint16_t*>(out) + doff, t);
      continue;
    }
    const Bf12Header* h = reinterpret_cast<const Bf12Header*>(blk);
    const uint32_t n = ch.n_values;
    const uint32_t base = h->base;
    const uint32_t e0 = h->exc_off[t], e1 = h->exc_off[t + 1];
    const u32x2* sm8 = reinterpret_cast<const u32x2*>(blk + kBf12HeaderBytes + lo);
    const uint32_t* cd4 = reinterpret_cast<const uint32_t*>(blk + kBf12HeaderBytes + n + lo / 2);
    const uint32_t groups = cnt / 8;
    constexpr int kPer = kBf12Tile / 8 / kDecThreads;  // 16
    u32x2 sv[kPer];
    uint32_t cv[kPer];
#pragma unroll
    for (int u = 0; u < kPer; ++u) {
      uint32_t g = threadIdx.x + u * kDecThreads;
      if (g < groups) {
        sv[u] = __builtin_nontemporal_load(sm8 + g);
        cv[u] = __builtin_nontemporal_load(cd4 + g);
      }
    }
#pragma unroll
    for (int u = 0; u < kPer; ++u) {
      uint32_t g = threadIdx.x + u * kDecThreads;
      if (g < groups) {
        u32x2 a0 = dec4(sv[u][0], cv[u], base), a1 = dec4(sv[u][1], cv[u] >> 16, base);
        dst[g] = u32x4{a0[0], a0[1], a1[0], a1[1]};
      }
    }
    if (e1 > e0) {  // uniform branch: only tiles with escapes pay the barrier
      __syncthreads();  // workgroup-scope ordering: the patch lands after the bulk store
      const Bf12Exception* exc =
          reinterpret_cast<const Bf12Exception*>(blk + kBf12HeaderBytes + n + n / 2);
      uint16_t* d16 = reinterpret_cast<uint16_t*>(out) + doff;
      for (uint32_t k = e0 + threadIdx.x; k < e1; k += kDecThreads) {
        Bf12Exception ex = exc[k];
        d16[ex.index] = ex.bits;
      }
    }
  }
}

hipError_t launch_bf12_unpack(const void* stream, void* dst, uint32_t nchunks, uint32_t chunk_values,
                              uint32_t workgroups, hipStream_t s, uint64_t dst_stride, uint32_t row_shift) {
  if (nchunks == 0) return hipSuccess;
  if (chunk_values < 8192 || (chunk_values & (chunk_values - 1)) || chunk_values > kBf12Tile * kBf12MaxTiles)
    return hipErrorInvalidValue;
  uint32_t shift = 0;
  while ((kBf12Tile << shift) < chunk_values) ++shift;  // tiles per chunk = 1 << shift
  uint64_t total = (uint64_t)nchunks << shift;
  uint64_t grid = workgroups && workgroups < total ? workgroups : total;
  hipLaunchKernelGGL(k_bf12_unpack, dim3((uint32_t)grid), dim3(kDecThreads), 0, s, (const uint8_t*)stream,
                     (uint8_t*)dst, dst_stride ? dst_stride : (uint64_t)chunk_values, shift, total, row_shift,
                     chunk_values);
  return hipGetLastError();
}

}  // namespace ogkm
