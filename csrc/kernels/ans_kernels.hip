// k_ans_unpack: HBM -> HBM unpack of an ANS stream (codec.hpp "ANS1" chunks,
// interleaved rANS over the exponents, raw sign|mantissa plane) into bf16.
//
// Work item = 4 consecutive 32 Ki-value segments of one chunk, one per wave of
// a 256-thread workgroup. The workgroup first expands the chunk's 256-entry
// frequency table into a 4096-slot decode table in LDS (16 KB: slot ->
// exponent | freq << 8 | (slot - cum) << 20; one wave-scan for the cumulative
// counts, 16 slots per thread). Then every lane runs its own rANS state:
//   slot lookup (LDS) -> state update -> renormalise if below 2^16.
// Renormalisation words of a segment are consumed in (step, lane) order: a
// ballot gives each needing lane its rank, and the word is fetched from a
// 3-register window of the segment's word stream (192 words in use + 128
// prefetched) with ds_bpermute - no LDS staging of the stream, so the table is
// the only LDS a workgroup holds and many workgroups share a CU to hide the
// serial per-lane dependency. Every 8 steps a lane owns 8 consecutive values
// and writes one coalesced 16-B store (1 KB per wave).
#include <hip/hip_runtime.h>

#include "ogkm/codec.hpp"
#include "ogkm/kernels.hpp"

namespace ogkm {

namespace {

typedef unsigned int au32x2 __attribute__((ext_vector_type(2)));
typedef unsigned int au32x4 __attribute__((ext_vector_type(4)));

constexpr int kAnsThreads = 256;
constexpr uint32_t kAnsSegsPerItem = kAnsThreads / 64;
constexpr uint32_t kAnsSlots = 1u << kAnsPrecBits;

__device__ __forceinline__ uint32_t ans_mbcnt(uint64_t m) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

__device__ __forceinline__ uint32_t ans_bperm(uint32_t lane, uint32_t v) {
  return (uint32_t)__builtin_amdgcn_ds_bpermute((int)(lane << 2), (int)v);
}

}  // namespace

__device__ __forceinline__ void ans_decode_seg(const uint8_t* __restrict__ blk, uint32_t n_values, uint32_t seg,
                                               uint16_t* __restrict__ dst, const uint32_t* tab);

// Work item `sub` (4 segments, one per wave) of the ANS1 chunk at `blk`, whose
// values land at dst[0, n_values). Called by the whole workgroup (barriers).
// err (host-coherent, may be null): {count, tag, chunk, freq sum} of corrupt
// ANS chunks - a frequency table that does not sum to 2^kAnsPrecBits (data that
// is not a valid stream: a race or a wrong pointer upstream). Such a chunk is
// zero-filled and reported instead of being decoded.
__device__ __forceinline__ void ans_decode_item(const uint8_t* __restrict__ blk, uint32_t n_values, uint32_t sub,
                                                uint16_t* __restrict__ dst, uint32_t* tab, uint32_t* cum,
                                                uint32_t* wsum, uint64_t* __restrict__ err, uint64_t tag,
                                                uint64_t c) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t v_lo = sub * kAnsSegsPerItem * kAnsSegValues;
  if (v_lo >= n_values) return;  // uniform across the workgroup
  const AnsHeader* h = reinterpret_cast<const AnsHeader*>(blk);
  __syncthreads();  // the previous item's table readers are done
  // cumulative frequencies: thread t owns symbol t (blockDim == 256 symbols)
  uint32_t s = h->freq[threadIdx.x];
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(s, d, 64);
    if (lane >= (uint32_t)d) s += y;
  }
  if (lane == 63u) wsum[wave] = s;
  __syncthreads();
  uint32_t add = 0;
  for (uint32_t w = 0; w < wave; ++w) add += wsum[w];
  cum[threadIdx.x + 1] = s + add;
  if (threadIdx.x == 0) cum[0] = 0;
  __syncthreads();
  if (cum[256] != kAnsSlots) {  // not an ANS chunk: report + zero-fill (workgroup-uniform)
    if (threadIdx.x == 0 && err) {
      if (__hip_atomic_fetch_add(err, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) == 0) {
        __hip_atomic_store(err + 1, tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(err + 2, c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(err + 3, (uint64_t)cum[256], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
    }
    const uint32_t v_hi = n_values - v_lo < kAnsSegsPerItem * kAnsSegValues
                              ? n_values : v_lo + kAnsSegsPerItem * kAnsSegValues;
    for (uint32_t k = v_lo + threadIdx.x; k < v_hi; k += kAnsThreads) dst[k] = 0;
    return;
  }
  {  // decode table: thread t fills slots [16 t, 16 t + 16)
    const uint32_t k0 = threadIdx.x * (kAnsSlots / kAnsThreads);
    uint32_t lo = 0, hi = 256;
    while (hi - lo > 1) {
      const uint32_t mid = (lo + hi) >> 1;
      if (cum[mid] <= k0) lo = mid; else hi = mid;
    }
    uint32_t sym = lo;
    for (uint32_t k = k0; k < k0 + kAnsSlots / kAnsThreads; ++k) {
      while (sym < 255u && cum[sym + 1] <= k) ++sym;
      tab[k] = sym | ((cum[sym + 1] - cum[sym]) << 8) | ((k - cum[sym]) << 20);
    }
  }
  __syncthreads();
  const uint32_t seg = sub * kAnsSegsPerItem + wave;
  if (seg >= h->n_seg) return;  // wave-uniform (the next barrier is at the next item's start)
  ans_decode_seg(blk, n_values, seg, dst, tab);
}

// One wave decodes segment `seg` of the ANS1 chunk at `blk` (its decode table
// already in `tab`).
__device__ __forceinline__ void ans_decode_seg(const uint8_t* __restrict__ blk, uint32_t n_values, uint32_t seg,
                                               uint16_t* __restrict__ dst, const uint32_t* tab) {
  const uint32_t lane = threadIdx.x & 63u;
  const AnsHeader* h = reinterpret_cast<const AnsHeader*>(blk);
  const uint32_t* dir = reinterpret_cast<const uint32_t*>(blk + h->off_dir);
  const uint32_t off = dir[seg], end = dir[seg + 1];
  const uint32_t npairs = (end - off - 256u) / 4u;  // word pairs (the encoder pads to an even count)
  uint32_t x = reinterpret_cast<const uint32_t*>(blk + off)[lane];
  const uint32_t* wsrc = reinterpret_cast<const uint32_t*>(blk + off + 256u);
  // word window: W0 = words [wb, wb + 128), W1 = the next 128, W2 = prefetch
  uint32_t W0 = lane < npairs ? wsrc[lane] : 0u;
  uint32_t W1 = 64u + lane < npairs ? wsrc[64u + lane] : 0u;
  uint32_t W2 = 128u + lane < npairs ? wsrc[128u + lane] : 0u;
  uint32_t wb = 0, wp = 0;
  const uint32_t base = seg * kAnsSegValues;
  const uint32_t nv = n_values - base < kAnsSegValues ? n_values - base : kAnsSegValues;
  const uint32_t groups = nv / 512u;
  const uint8_t* smp = blk + kAnsHeaderBytes;
  au32x2 smn = __builtin_nontemporal_load(reinterpret_cast<const au32x2*>(smp + base + lane * 8u));
  for (uint32_t g = 0; g < groups; ++g) {
    const uint32_t v0 = base + (g * 64u + lane) * 8u;
    const au32x2 sm = smn;
    if (g + 1 < groups) smn = __builtin_nontemporal_load(reinterpret_cast<const au32x2*>(smp + v0 + 512u));
    au32x4 o = {0u, 0u, 0u, 0u};
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const uint32_t t = tab[x & (kAnsSlots - 1u)];
      x = ((t >> 8) & 0xFFFu) * (x >> kAnsPrecBits) + (t >> 20);
      const bool need = x < kAnsLowBound;
      const uint64_t m = __ballot(need);
      if (m) {  // wave-uniform
        const uint32_t rel = wp - wb + ans_mbcnt(m);  // < 192
        const uint32_t a = ans_bperm((rel >> 1) & 63u, W0), b = ans_bperm((rel >> 1) & 63u, W1);
        const uint32_t pr = rel < 128u ? a : b;
        const uint32_t word = (rel & 1u) ? (pr >> 16) : (pr & 0xFFFFu);
        if (need) x = (x << 16) | word;
        wp += (uint32_t)__builtin_popcountll(m);
        if (wp - wb >= 128u) {
          W0 = W1;
          W1 = W2;
          wb += 128u;
          const uint32_t q = (wb + 256u) / 2u + lane;
          W2 = q < npairs ? wsrc[q] : 0u;
        }
      }
      const uint32_t byte = (sm[j >> 2] >> (8 * (j & 3))) & 0xFFu;
      const uint32_t val = ((byte & 0x80u) << 8) | ((t & 0xFFu) << 7) | (byte & 0x7Fu);
      o[j >> 1] |= val << (16 * (j & 1));
    }
    __builtin_nontemporal_store(o, reinterpret_cast<au32x4*>(dst + v0));
  }
}

__global__ void __launch_bounds__(kAnsThreads)
    k_ans_unpack(const uint8_t* __restrict__ stream, uint16_t* __restrict__ out, uint64_t dst_stride,
                 uint32_t items_per_chunk, uint64_t total_items, uint64_t* __restrict__ err, uint32_t row_shift,
                 uint32_t chunk_values) {
  __shared__ uint32_t tab[kAnsSlots];
  __shared__ uint32_t cum[257];
  __shared__ uint32_t wsum[kAnsSegsPerItem];
  const Bf12StreamChunk* table = reinterpret_cast<const Bf12StreamChunk*>(stream + sizeof(Bf12StreamHeader));
  for (uint64_t item = blockIdx.x; item < total_items; item += gridDim.x) {
    const uint64_t c = item / items_per_chunk;
    const uint32_t sub = (uint32_t)(item - c * items_per_chunk);
    const Bf12StreamChunk ch = table[c];  // uniform: scalar loads
    const uint8_t* blk = stream + ch.offset;
    uint16_t* dst = out + (c >> row_shift) * dst_stride + (c & ((1ull << row_shift) - 1)) * chunk_values;
    const uint32_t v_lo = sub * kAnsSegsPerItem * kAnsSegValues;
    if (v_lo >= ch.n_values) continue;  // uniform across the workgroup
    if (ch.encoded != 3) {              // raw chunk: plain copy of this item's range
      const uint32_t v_hi = ch.n_values - v_lo < kAnsSegsPerItem * kAnsSegValues
                                ? ch.n_values : v_lo + kAnsSegsPerItem * kAnsSegValues;
      const uint16_t* src = reinterpret_cast<const uint16_t*>(blk);
      const uint32_t g_lo = v_lo / 8, g_hi = v_hi / 8;
      for (uint32_t g = g_lo + threadIdx.x; g < g_hi; g += kAnsThreads)
        __builtin_nontemporal_store(__builtin_nontemporal_load(reinterpret_cast<const au32x4*>(src) + g),
                                    reinterpret_cast<au32x4*>(dst) + g);
      for (uint32_t k = g_hi * 8 + threadIdx.x; k < v_hi; k += kAnsThreads) dst[k] = src[k];
      continue;
    }
    ans_decode_item(blk, ch.n_values, sub, dst, tab, cum, wsum, err, (uint64_t)stream, c);
  }
}

// Packed host copies of the runtime (ring op DECODE_ANS): one ANS1 chunk per
// 2 MB block, staged in HBM by the engines; block k's items are
// [item_start[k], item_start[k + 1]). A block whose header does not match
// (magic / value count) is reported and zero-filled like a bad table.
__global__ void __launch_bounds__(kAnsThreads)
    k_ans_blocks(const KAnsBlocks b, uint32_t n, uint64_t* __restrict__ err) {
  __shared__ uint32_t tab[kAnsSlots];
  __shared__ uint32_t cum[257];
  __shared__ uint32_t wsum[kAnsSegsPerItem];
  const uint32_t total = b.item_start[n];
  for (uint32_t item = blockIdx.x; item < total; item += gridDim.x) {
    uint32_t k = 0;
    while (k + 1 < n && b.item_start[k + 1] <= item) ++k;  // uniform scan (n <= 64)
    const uint8_t* blk = reinterpret_cast<const uint8_t*>(b.src[k]);
    uint16_t* dst = reinterpret_cast<uint16_t*>(b.dst[k]);
    const uint32_t nv = b.n_values[k];
    const AnsHeader* h = reinterpret_cast<const AnsHeader*>(blk);
    if (h->magic != kAnsMagic || h->n_values != nv) {  // uniform
      const uint32_t sub = item - b.item_start[k];
      if (threadIdx.x == 0 && err && __hip_atomic_fetch_add(err, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) == 0) {
        __hip_atomic_store(err + 1, b.src[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(err + 2, (uint64_t)k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(err + 3, (uint64_t)h->magic, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
      const uint32_t v_lo = sub * kAnsSegsPerItem * kAnsSegValues;
      const uint32_t v_hi = nv - v_lo < kAnsSegsPerItem * kAnsSegValues ? nv : v_lo + kAnsSegsPerItem * kAnsSegValues;
      for (uint32_t v = v_lo + threadIdx.x; v < v_hi; v += kAnsThreads) dst[v] = 0;
      continue;
    }
    ans_decode_item(blk, nv, item - b.item_start[k], dst, tab, cum, wsum, err, b.src[k], k);
  }
}

// Segmented packed host copies (Residency fmt 3, ring DECODE_SEGS): many small
// ANS1 chunks of ONE 32 Ki-value segment each. One wave per chunk - its own
// decode table in its own 16 KB of LDS, built by the wave alone (no
// workgroup barrier) - so all four waves of a workgroup decode; with the block
// kernel's 4-segment items three of them would idle on such chunks.
__global__ void __launch_bounds__(kAnsThreads)
    k_ans_segs(const KAnsSegs d, uint32_t n, uint64_t* __restrict__ err) {
  __shared__ uint32_t tabs[kAnsSegsPerItem][kAnsSlots];
  __shared__ uint32_t cums[kAnsSegsPerItem][257];
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t k = blockIdx.x * kAnsSegsPerItem + wave;
  if (k >= n) return;  // wave-uniform; no workgroup barrier below
  const uint8_t* blk = reinterpret_cast<const uint8_t*>(d.src[k]);
  uint16_t* dst = reinterpret_cast<uint16_t*>(d.dst[k]);
  const AnsHeader* h = reinterpret_cast<const AnsHeader*>(blk);
  uint32_t* tab = tabs[wave];
  uint32_t* cum = cums[wave];
  // cumulative frequencies: lane owns symbols 4 lane .. 4 lane + 3
  uint32_t f[4], t = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    f[j] = h->freq[4 * lane + j];
    t += f[j];
  }
  uint32_t inc = t;
#pragma unroll
  for (int s = 1; s < 64; s <<= 1) {
    const uint32_t y = __shfl_up(inc, s, 64);
    if (lane >= (uint32_t)s) inc += y;
  }
  uint32_t c = inc - t;  // exclusive prefix
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    cum[4 * lane + j] = c;
    c += f[j];
  }
  if (lane == 63u) cum[256] = c;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  const bool bad = h->magic != kAnsMagic || h->n_values != kAnsSegValues || h->n_seg != 1 || cum[256] != kAnsSlots;
  if (bad) {  // wave-uniform: report + zero-fill the segment
    if (lane == 0 && err && __hip_atomic_fetch_add(err, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) == 0) {
      __hip_atomic_store(err + 1, d.src[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      __hip_atomic_store(err + 2, (uint64_t)k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      __hip_atomic_store(err + 3, (uint64_t)h->magic, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    for (uint32_t g = lane; g < kAnsSegValues / 8; g += 64)
      reinterpret_cast<au32x4*>(dst)[g] = au32x4{0u, 0u, 0u, 0u};
    return;
  }
  {  // decode table: lane fills slots [64 lane, 64 lane + 64)
    const uint32_t k0 = lane * (kAnsSlots / 64);
    uint32_t lo = 0, hi = 256;
    while (hi - lo > 1) {
      const uint32_t mid = (lo + hi) >> 1;
      if (cum[mid] <= k0) lo = mid; else hi = mid;
    }
    uint32_t sym = lo;
    for (uint32_t q = k0; q < k0 + kAnsSlots / 64; ++q) {
      while (sym < 255u && cum[sym + 1] <= q) ++sym;
      tab[q] = sym | ((cum[sym + 1] - cum[sym]) << 8) | ((q - cum[sym]) << 20);
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  ans_decode_seg(blk, kAnsSegValues, 0, dst, tab);
}

hipError_t launch_ans_segs(const KAnsSegs& d, uint32_t n, hipStream_t s, uint64_t* err) {
  if (n == 0) return hipSuccess;
  if (n > (uint32_t)kAnsInlineSegs) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_ans_segs, dim3((n + kAnsSegsPerItem - 1) / kAnsSegsPerItem), dim3(kAnsThreads), 0, s, d, n,
                     err);
  return hipGetLastError();
}

hipError_t launch_ans_unpack(const void* stream, void* dst, uint32_t nchunks, uint32_t chunk_values,
                             uint32_t workgroups, hipStream_t s, uint64_t dst_stride, uint64_t* err,
                             uint32_t row_shift) {
  if (nchunks == 0) return hipSuccess;
  if (chunk_values < 8192 || (chunk_values & (chunk_values - 1)) || chunk_values > (1u << 20))
    return hipErrorInvalidValue;
  const uint32_t segs = (chunk_values + kAnsSegValues - 1) / kAnsSegValues;
  const uint32_t per_chunk = (segs + kAnsSegsPerItem - 1) / kAnsSegsPerItem;
  const uint64_t total = (uint64_t)nchunks * per_chunk;
  const uint64_t grid = workgroups && workgroups < total ? workgroups : total;
  hipLaunchKernelGGL(k_ans_unpack, dim3((uint32_t)grid), dim3(kAnsThreads), 0, s, (const uint8_t*)stream,
                     (uint16_t*)dst, dst_stride ? dst_stride : (uint64_t)chunk_values, per_chunk, total, err, row_shift,
                     chunk_values);
  return hipGetLastError();
}

hipError_t launch_ans_blocks(const KAnsBlocks& b, uint32_t n, hipStream_t s, uint64_t* err) {
  if (n == 0) return hipSuccess;
  if (n > (uint32_t)kAnsInlineBlocks) return hipErrorInvalidValue;
  const uint32_t total = b.item_start[n];
  if (total == 0) return hipSuccess;
  hipLaunchKernelGGL(k_ans_blocks, dim3(total), dim3(kAnsThreads), 0, s, b, n, err);
  return hipGetLastError();
}

}  // namespace ogkm
