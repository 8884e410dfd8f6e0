// Decode GEMM: Y[M, N] = X[M, K] . W[N, K]^T for small M (decode batches),
// weight-streaming on the MFMA cores, with the weight read straight from the
// tier format it rests in:
//   * raw bf16 in "fragment order" (see below), or
//   * a BF11/raw packed stream (codec.hpp) - decoded in registers, so the
//     packed bytes are the only weight bytes that cross HBM (no bf16 staging).
//
// Fragment order. W is stored as 16x32 tiles, tile (rt, ks) at index
// rt * (K/32) + ks, each 512 values = 1 KB of bf16 laid out lane-major: lane l
// owns 8 consecutive values = W[16 rt + (l & 15)][32 ks + 8 (l >> 4) + j]. That
// is exactly the A-operand fragment of v_mfma_f32_16x16x32_bf16, so one
// 16-byte load per lane fetches a whole fragment (one fully coalesced 1 KB
// wave access), and it is exactly one BF11 wave group (512 values; 8 per
// lane), so the packed decoder hands each lane its fragment with no shuffle.
//
// Work split. One wave = one unit = 64 rows (4 row tiles) x a K range (split-K
// when N is small so the grid has >> 256 CUs' worth of waves). A wave keeps
// 4 (row tiles) x 4 (16-column M tiles) f32x4 accumulators; per 32-wide K step
// it loads 4 weight fragments + 4 activation fragments and issues 16 MFMAs.
// Partials go to an f32 [ksplit][M][N] slab; k_dgemm_reduce sums the splits and
// applies the fused epilogue (store / + residual / SiLU(gate) * up).
#include <hip/hip_runtime.h>

#include "ogkm/codec.hpp"
#include "ogkm/kernels.hpp"

namespace ogkm {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2_t __attribute__((ext_vector_type(2)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));

constexpr int kRowTiles = 4;   // row tiles (16 rows) per wave
constexpr int kMTiles = 4;     // 16-column tiles of M per block (M block = 64)

__device__ __forceinline__ uint32_t dg_mbcnt(uint64_t m) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

__device__ __forceinline__ uint32_t dg_prefix8(uint32_t cnt) {
  const uint64_t b0 = __ballot(cnt & 1u), b1 = __ballot(cnt & 2u), b2 = __ballot(cnt & 4u), b3 = __ballot(cnt & 8u);
  return dg_mbcnt(b0) + 2u * dg_mbcnt(b1) + 4u * dg_mbcnt(b2) + 8u * dg_mbcnt(b3);
}

// One BF11 wave group (or raw span) of a packed stream -> this lane's 8 bf16.
// `g` is the wave-uniform value index of the fragment inside the stream.
struct PackedStream {
  const uint8_t* base;
  uint32_t chunk_shift;  // log2(chunk_values)
};

__device__ __forceinline__ u32x4_t load_packed_frag(const PackedStream& ps, uint64_t g, uint32_t lane) {
  const Bf12StreamChunk* table = reinterpret_cast<const Bf12StreamChunk*>(ps.base + sizeof(Bf12StreamHeader));
  const uint64_t c = g >> ps.chunk_shift;
  const uint32_t v = (uint32_t)(g & ((1ull << ps.chunk_shift) - 1));
  const Bf12StreamChunk ch = table[c];
  const uint8_t* blk = ps.base + ch.offset;
  if (ch.encoded != 2) {  // raw bf16 chunk (the packer never emits BF12 for GEMM weights)
    return __builtin_nontemporal_load(reinterpret_cast<const u32x4_t*>(blk + ((uint64_t)v + lane * 8u) * 2));
  }
  const Bf11Header* h = reinterpret_cast<const Bf11Header*>(blk);
  const uint32_t v0 = v + lane * 8u;
  const u32x2_t sm = __builtin_nontemporal_load(reinterpret_cast<const u32x2_t*>(blk + kBf11HeaderBytes + v0));
  const uint32_t pcv = __builtin_nontemporal_load(reinterpret_cast<const uint16_t*>(blk + h->off_prim) + (v0 >> 3));
  const uint32_t escm = pcv & (pcv >> 1) & 0x5555u;
  const uint32_t pre = dg_prefix8((uint32_t)__builtin_popcount(escm));
  const uint32_t t = v >> 15;
  uint32_t nibs = 0;
  if (escm) {
    const uint32_t idx = reinterpret_cast<const uint32_t*>(blk + h->off_wg)[v >> 9] + pre;
    const uint32_t* sec32 = reinterpret_cast<const uint32_t*>(blk + h->off_sec);
    const uint32_t q = idx >> 3, sh = (idx & 7u) * 4u;
    const uint64_t w = ((uint64_t)sec32[q + 1] << 32) | sec32[q];
    nibs = (uint32_t)(w >> sh);
  }
  const uint32_t prim = h->prim, sbase = h->sec_base;
  uint32_t exc_lanes = 0;  // bit j: value j is an exception (secondary code 15)
  u32x4_t o;
  uint32_t nb = nibs;
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    uint32_t w2 = 0;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int k = 2 * p + q;
      const uint32_t c2 = (pcv >> (2 * k)) & 3u;
      const bool esc = c2 == 3u;
      const uint32_t sc = nb & 15u;
      exc_lanes |= (esc && sc == 15u) ? (1u << k) : 0u;
      const uint32_t e = esc ? ((sbase + sc) & 0xFFu) : ((prim >> (8u * c2)) & 0xFFu);
      nb = esc ? nb >> 4 : nb;
      const uint32_t b = (sm[p >> 1] >> (8 * (k & 3))) & 0xFFu;
      w2 |= (((b & 0x80u) << 8) | (e << 7) | (b & 0x7Fu)) << (16 * q);
    }
    o[p] = w2;
  }
  if (exc_lanes) {  // rare: exact bits from the tile's sorted exception list
    const Bf12Exception* exc = reinterpret_cast<const Bf12Exception*>(blk + h->off_exc);
    const uint32_t e0 = h->exc_off[t], e1 = h->exc_off[t + 1];
    for (int k = 0; k < 8; ++k) {
      if (!((exc_lanes >> k) & 1u)) continue;
      const uint32_t want = v0 + (uint32_t)k;
      uint32_t lo = e0, hi = e1;
      while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (exc[mid].index < want) lo = mid + 1; else hi = mid;
      }
      const uint32_t bits = (lo < e1 && exc[lo].index == want) ? exc[lo].bits : 0u;
      const uint32_t sh = 16u * (k & 1);
      o[k >> 1] = (o[k >> 1] & ~(0xFFFFu << sh)) | (bits << sh);
    }
  }
  return o;
}

// Weight loader modes. RAW: bf16 fragments. PACKED: generic packed stream
// (BF11 or raw chunks), one fragment at a time. PACKED_BF11: every chunk the
// wave touches is BF11 (checked on the host) - the K loop is unrolled U steps
// and split into phases so each wave keeps 4U fragments' loads in flight:
//   P1  sign|mantissa (8 B) + primary codes (2 B) of all 4U fragments, X fragments
//   P2  escape prefix counts (ballots) -> secondary-nibble loads (8 B)
//   P3  rebuild bf16 fragments in registers -> 16 U MFMAs.
enum : int { MODE_RAW = 0, MODE_PACKED = 1, MODE_PACKED_BF11 = 2 };

// Rebuild one lane's 8 bf16 of a BF11 wave group. No serial dependency
// between values: value k's secondary nibble is found by the rank of its escape
// bit (popcount of the lower escape bits), the primary exponents of 4 values
// come out of one byte permute of `prim`, and sign|mantissa bytes are spread
// into bf16 halves by byte permutes.
__device__ __forceinline__ uint32_t code_sel4(uint32_t x) {  // 4 two-bit codes -> 4 selector bytes
  return (x & 3u) | ((x & 0xCu) << 6) | ((x & 0x30u) << 12) | ((x & 0xC0u) << 18);
}

__device__ __forceinline__ u32x4_t bf11_frag_words(u32x2_t sm, uint32_t pcv, uint32_t nibs, uint32_t prim,
                                                  uint32_t sbase, uint32_t* exc_mask) {
  const uint32_t escm = pcv & (pcv >> 1) & 0x5555u;  // bit 2k: value k escaped
  const uint32_t pe[2] = {__builtin_amdgcn_perm(0u, prim, code_sel4(pcv & 0xFFu)),
                          __builtin_amdgcn_perm(0u, prim, code_sel4(pcv >> 8))};
  uint32_t e[8];
  uint32_t em = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const uint32_t rank = (uint32_t)__builtin_popcount(escm & ((1u << (2 * k)) - 1u));
    const uint32_t sc = (nibs >> (4u * rank)) & 15u;
    const bool esc = (escm >> (2 * k)) & 1u;
    em |= (esc && sc == 15u) ? (1u << k) : 0u;
    e[k] = esc ? ((sbase + sc) & 0xFFu) : ((pe[k >> 2] >> (8 * (k & 3))) & 0xFFu);
  }
  u32x4_t o;
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const uint32_t w = sm[p >> 1];
    // bytes (2p & 3) and (2p & 3) + 1 of w into the low bytes of the two halves
    const uint32_t sel = (p & 1) ? 0x0C030C02u : 0x0C010C00u;
    const uint32_t x = __builtin_amdgcn_perm(0u, w, sel);
    const uint32_t t = ((x << 8) & 0x80008000u) | (x & 0x007F007Fu);
    o[p] = t | (e[2 * p] << 7) | (e[2 * p + 1] << 23);
  }
  *exc_mask = em;
  return o;
}

__device__ __noinline__ u32x4_t bf11_patch_exceptions(const uint8_t* blk, uint32_t v0, uint32_t em, u32x4_t o) {
  const Bf11Header* h = reinterpret_cast<const Bf11Header*>(blk);
  const Bf12Exception* exc = reinterpret_cast<const Bf12Exception*>(blk + h->off_exc);
  const uint32_t t = v0 >> 15;
  const uint32_t e0 = h->exc_off[t], e1 = h->exc_off[t + 1];
  for (int k = 0; k < 8; ++k) {
    if (!((em >> k) & 1u)) continue;
    const uint32_t want = v0 + (uint32_t)k;
    uint32_t lo = e0, hi = e1;
    while (lo < hi) {
      const uint32_t mid = (lo + hi) >> 1;
      if (exc[mid].index < want) lo = mid + 1; else hi = mid;
    }
    const uint32_t bits = (lo < e1 && exc[lo].index == want) ? exc[lo].bits : 0u;
    const uint32_t sh = 16u * (k & 1);
    o[k >> 1] = (o[k >> 1] & ~(0xFFFFu << sh)) | (bits << sh);
  }
  return o;
}

template <int kMode, int U>
__global__ void __launch_bounds__(256) k_dgemm(DGemmArgs a) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t unit = blockIdx.x * (blockDim.x >> 6) + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (unit >= a.row_blocks * a.ksplit) return;  // wave-uniform exit
  const uint32_t rb = unit / a.ksplit, ks = unit - rb * a.ksplit;
  const uint32_t k_lo = ks * a.klen;
  const uint32_t k_hi = k_lo + a.klen < a.K ? k_lo + a.klen : a.K;
  const uint32_t n_tiles = a.N >> 4;
  const uint32_t rt0 = rb * kRowTiles;
  const uint32_t nrt = n_tiles - rt0 < (uint32_t)kRowTiles ? n_tiles - rt0 : (uint32_t)kRowTiles;
  const uint32_t kfr = a.K >> 5;
  const uint32_t m_base = blockIdx.y * (kMTiles * 16);
  const uint32_t h = lane >> 4;
  PackedStream ps{a.w, a.chunk_shift};
  const Bf12StreamChunk* table = reinterpret_cast<const Bf12StreamChunk*>(a.w + sizeof(Bf12StreamHeader));
  const uint64_t cmask = (1ull << a.chunk_shift) - 1;

  const uint16_t* xrow[kMTiles];  // this lane's activation fragment at K step 0; + step * xstep per step
  bool mval[kMTiles];
  const uint32_t xstep = a.x_frag ? 512u : 32u;
#pragma unroll
  for (int mt = 0; mt < kMTiles; ++mt) {
    const uint32_t m = m_base + mt * 16 + (lane & 15u);
    mval[mt] = m < a.M;
    xrow[mt] = a.x_frag ? a.x + (uint64_t)(m_base / 16 + mt) * kfr * 512u + lane * 8u
                        : a.x + (uint64_t)(mval[mt] ? m : 0) * a.ldx + 8u * h;
  }
  f32x4_t acc[kRowTiles][kMTiles];
#pragma unroll
  for (int r = 0; r < kRowTiles; ++r)
#pragma unroll
    for (int mt = 0; mt < kMTiles; ++mt) acc[r][mt] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  uint32_t k = k_lo;
  if constexpr (kMode == MODE_PACKED_BF11 || kMode == MODE_RAW) {
    for (; k + 32 * U <= k_hi; k += 32 * U) {
      const uint32_t kst = k >> 5;
      u32x4_t xb[U][kMTiles];
      if constexpr (kMode == MODE_RAW) {
        u32x4_t wa[U][kRowTiles];
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
          for (int r = 0; r < kRowTiles; ++r)
            wa[u][r] = (uint32_t)r < nrt
                           ? __builtin_nontemporal_load(reinterpret_cast<const u32x4_t*>(
                                 a.w + (a.w_off + ((uint64_t)(rt0 + r) * kfr + kst + u) * 512u + lane * 8u) * 2))
                           : u32x4_t{0, 0, 0, 0};
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
          for (int mt = 0; mt < kMTiles; ++mt)
            xb[u][mt] = mval[mt] ? *reinterpret_cast<const u32x4_t*>(xrow[mt] + ((k >> 5) + u) * xstep)
                                 : u32x4_t{0, 0, 0, 0};
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
          for (int r = 0; r < kRowTiles; ++r)
            if ((uint32_t)r < nrt) {
#pragma unroll
              for (int mt = 0; mt < kMTiles; ++mt)
                acc[r][mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, wa[u][r]),
                                                                     __builtin_bit_cast(bf16x8_t, xb[u][mt]),
                                                                     acc[r][mt], 0, 0, 0);
            }
      } else {
        // P1: primary planes of every fragment of the block
        u32x2_t smv[U][kRowTiles];
        uint32_t pcv[U][kRowTiles];
        const uint8_t* blks[U][kRowTiles];
        uint32_t vv[U][kRowTiles], nv[U][kRowTiles];
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
          for (int r = 0; r < kRowTiles; ++r) {
            pcv[u][r] = 0;
            if ((uint32_t)r < nrt) {
              const uint64_t g = a.w_off + ((uint64_t)(rt0 + r) * kfr + kst + u) * 512u;
              const Bf12StreamChunk ch = table[g >> a.chunk_shift];
              const uint8_t* blk = a.w + ch.offset;
              const uint32_t v = (uint32_t)(g & cmask);
              blks[u][r] = blk;
              vv[u][r] = v;
              nv[u][r] = ch.n_values;
              const uint32_t v0 = v + lane * 8u;
              smv[u][r] = __builtin_nontemporal_load(reinterpret_cast<const u32x2_t*>(blk + kBf11HeaderBytes + v0));
              pcv[u][r] = __builtin_nontemporal_load(
                  reinterpret_cast<const uint16_t*>(blk + bf11_layout(ch.n_values).off_prim) + (v0 >> 3));
            }
          }
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
          for (int mt = 0; mt < kMTiles; ++mt)
            xb[u][mt] = mval[mt] ? *reinterpret_cast<const u32x4_t*>(xrow[mt] + ((k >> 5) + u) * xstep)
                                 : u32x4_t{0, 0, 0, 0};
        // P2: escape prefixes -> secondary nibbles
        u32x2_t sec[U][kRowTiles];
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
          for (int r = 0; r < kRowTiles; ++r) {
            sec[u][r] = u32x2_t{0, 0};
            if ((uint32_t)r < nrt) {
              const uint32_t escm = pcv[u][r] & (pcv[u][r] >> 1) & 0x5555u;
              const uint32_t pre = dg_prefix8((uint32_t)__builtin_popcount(escm));
              const Bf11Layout lay = bf11_layout(nv[u][r]);
              const uint32_t v = vv[u][r];
              const uint32_t idx = reinterpret_cast<const uint32_t*>(blks[u][r] + lay.off_wg)[v >> 9] + pre;
              if (escm) {
                const uint32_t* sec32 = reinterpret_cast<const uint32_t*>(blks[u][r] + lay.off_sec) + (idx >> 3);
                sec[u][r] = u32x2_t{sec32[0], sec32[1]};
              }
              vv[u][r] = (idx & 7u) * 4u;  // reuse: nibble shift
            }
          }
        // P3: decode + MFMA
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
          for (int r = 0; r < kRowTiles; ++r) {
            if ((uint32_t)r < nrt) {
              const Bf11Header* hd = reinterpret_cast<const Bf11Header*>(blks[u][r]);
              const uint64_t w64 = ((uint64_t)sec[u][r][1] << 32) | sec[u][r][0];
              uint32_t em;
              u32x4_t wa = bf11_frag_words(smv[u][r], pcv[u][r], (uint32_t)(w64 >> vv[u][r]), hd->prim,
                                           hd->sec_base, &em);
              if (em) {
                const uint64_t g = a.w_off + ((uint64_t)(rt0 + r) * kfr + kst + u) * 512u;
                wa = bf11_patch_exceptions(blks[u][r], (uint32_t)(g & cmask) + lane * 8u, em, wa);
              }
#pragma unroll
              for (int mt = 0; mt < kMTiles; ++mt)
                acc[r][mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, wa),
                                                                     __builtin_bit_cast(bf16x8_t, xb[u][mt]),
                                                                     acc[r][mt], 0, 0, 0);
            }
          }
      }
    }
  }
  // tail (and the generic packed mode): one K step at a time
  for (; k < k_hi; k += 32) {
    const uint32_t kst = k >> 5;
    u32x4_t wa[kRowTiles];
#pragma unroll
    for (int r = 0; r < kRowTiles; ++r) {
      if ((uint32_t)r < nrt) {
        const uint64_t frag = (uint64_t)(rt0 + r) * kfr + kst;
        if constexpr (kMode != MODE_RAW) {
          wa[r] = load_packed_frag(ps, a.w_off + frag * 512u, lane);
        } else {
          wa[r] = __builtin_nontemporal_load(
              reinterpret_cast<const u32x4_t*>(a.w + (a.w_off + frag * 512u + lane * 8u) * 2));
        }
      } else {
        wa[r] = u32x4_t{0, 0, 0, 0};
      }
    }
    u32x4_t xb[kMTiles];
#pragma unroll
    for (int mt = 0; mt < kMTiles; ++mt)
      xb[mt] = mval[mt] ? *reinterpret_cast<const u32x4_t*>(xrow[mt] + (k >> 5) * xstep) : u32x4_t{0, 0, 0, 0};
#pragma unroll
    for (int r = 0; r < kRowTiles; ++r) {
      if ((uint32_t)r < nrt) {
#pragma unroll
        for (int mt = 0; mt < kMTiles; ++mt)
          acc[r][mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, wa[r]),
                                                               __builtin_bit_cast(bf16x8_t, xb[mt]), acc[r][mt], 0,
                                                               0, 0);
      }
    }
  }
  // D layout (16x16x32): col = lane & 15 -> m, row = 4 (lane >> 4) + reg -> n.
#pragma unroll
  for (int r = 0; r < kRowTiles; ++r) {
    if ((uint32_t)r >= nrt) continue;
    const uint32_t n = (rt0 + r) * 16u + 4u * h;
#pragma unroll
    for (int mt = 0; mt < kMTiles; ++mt) {
      const uint32_t m = m_base + mt * 16 + (lane & 15u);
      if (m < a.M) *reinterpret_cast<f32x4_t*>(a.part + ((uint64_t)ks * a.M + m) * a.N + n) = acc[r][mt];
    }
  }
}

__device__ __forceinline__ uint16_t f32_to_bf16_rne(float f) {
  uint32_t u = __float_as_uint(f);
  if ((u & 0x7F800000u) == 0x7F800000u && (u & 0x7FFFFFu)) return (uint16_t)((u >> 16) | 0x40u);  // quiet NaN
  u += 0x7FFFu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}
__device__ __forceinline__ float bf16_to_f32(uint16_t b) { return __uint_as_float((uint32_t)b << 16); }

// Split-K sum + epilogue of 4 consecutive output columns (n .. n + 3) of row m.
__device__ __forceinline__ void dg_reduce_quad(const DGemmReduceArgs& a, uint32_t m, uint32_t n) {
  const uint32_t nout = a.epi == DGEMM_EPI_SILU_MUL ? a.N / 2 : a.N;
  f32x4_t s = {0.f, 0.f, 0.f, 0.f}, u = {0.f, 0.f, 0.f, 0.f};
  // Batches of 8 split rows: all loads of a batch are issued before the first
  // add (8 requests in flight per lane instead of one dependent load per split;
  // the wd shapes run 64 splits). Summation order is unchanged (k ascending).
  constexpr uint32_t kB = 8;
  uint32_t k = 0;
  for (; k + kB <= a.ksplit; k += kB) {
    f32x4_t v[kB], w[kB];
#pragma unroll
    for (uint32_t j = 0; j < kB; ++j) {
      const float* row = a.part + ((uint64_t)(k + j) * a.M + m) * a.N;
      v[j] = *reinterpret_cast<const f32x4_t*>(row + n);
      if (a.epi == DGEMM_EPI_SILU_MUL) w[j] = *reinterpret_cast<const f32x4_t*>(row + nout + n);
    }
#pragma unroll
    for (uint32_t j = 0; j < kB; ++j) {
      s += v[j];
      if (a.epi == DGEMM_EPI_SILU_MUL) u += w[j];
    }
  }
  for (; k < a.ksplit; ++k) {
    const float* row = a.part + ((uint64_t)k * a.M + m) * a.N;
    s += *reinterpret_cast<const f32x4_t*>(row + n);
    if (a.epi == DGEMM_EPI_SILU_MUL) u += *reinterpret_cast<const f32x4_t*>(row + nout + n);
  }
  uint16_t o[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    float y = s[j];
    if (a.epi == DGEMM_EPI_RESID) {
      y = bf16_to_f32(f32_to_bf16_rne(y)) + bf16_to_f32(a.resid[(uint64_t)m * a.ldr + n + j]);
    } else if (a.epi == DGEMM_EPI_SILU_MUL) {
      const float g = bf16_to_f32(f32_to_bf16_rne(y)), up = bf16_to_f32(f32_to_bf16_rne(u[j]));
      y = g / (1.f + __expf(-g)) * up;
    }
    o[j] = f32_to_bf16_rne(y);
  }
  uint16_t* dst = a.out_frag ? a.out + frag_index(m, a.out_col0 + n, a.out_cols) : a.out + (uint64_t)m * a.ldo + n;
  *reinterpret_cast<u32x2_t*>(dst) = u32x2_t{(uint32_t)o[0] | ((uint32_t)o[1] << 16), (uint32_t)o[2] | ((uint32_t)o[3] << 16)};
}

// One thread = 4 consecutive output columns of one row.
__global__ void __launch_bounds__(256) k_dgemm_reduce(DGemmReduceArgs a) {
  const uint32_t nout = a.epi == DGEMM_EPI_SILU_MUL ? a.N / 2 : a.N;
  const uint32_t q = nout / 4;
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (uint64_t)a.M * q) return;
  const uint32_t m = (uint32_t)(i / q), n = (uint32_t)(i - (uint64_t)m * q) * 4u;
  dg_reduce_quad(a, m, n);
}

// DGemmArgs::direct (one K split, STORE / RESID): the epilogue straight from
// the accumulators - no partial slab, no reduce. Same arithmetic as
// k_dgemm_reduce with one split (0 + x == x: the accumulator is never -0).
__device__ __forceinline__ void dg_store_direct(const DGemmReduceArgs& r, uint32_t m, uint32_t n, f32x4_t v) {
  uint16_t o[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    float y = v[e];
    if (r.epi == DGEMM_EPI_RESID) y = bf16_to_f32(f32_to_bf16_rne(y)) + bf16_to_f32(r.resid[(uint64_t)m * r.ldr + n + e]);
    o[e] = f32_to_bf16_rne(y);
  }
  uint16_t* dst = r.out_frag ? r.out + frag_index(m, r.out_col0 + n, r.out_cols) : r.out + (uint64_t)m * r.ldo + n;
  *reinterpret_cast<u32x2_t*>(dst) = u32x2_t{(uint32_t)o[0] | ((uint32_t)o[1] << 16), (uint32_t)o[2] | ((uint32_t)o[3] << 16)};
}

// In-kernel split-K fixup (DGemmArgs::fix_cnt), called by every wave of
// k_dgemm_pipe / k_dgemm_lring after its partial stores (the counter form of
// cdna_hip_programming.md's in-launch split-K reduction): the agent-scope
// release fence writes this wave's partials back from its XCD's L2 before its
// arrival is counted; the group's last arrival fences acquire (so it reads the
// other XCDs' partials, not stale lines), resets the counter for the next
// launch and writes the group's 64 output columns x (up to) 64 rows - 8 quads
// per lane per batch with every split load issued before the first add (the
// reducer is one wave: its loads in flight set its speed). Summation order
// is k ascending, as in k_dgemm_reduce: the output is bit-identical.
__device__ __forceinline__ void dg_fixup(const DGemmArgs& a, uint32_t rb, uint32_t lane) {
  const bool silu = a.fix.epi == DGEMM_EPI_SILU_MUL;
  const uint32_t groups = silu ? a.row_blocks / 2 : a.row_blocks;
  const uint32_t g = rb < groups ? rb : rb - groups;
  uint32_t* cnt = a.fix_cnt + (uint64_t)blockIdx.y * a.row_blocks + g;
  const uint32_t arrivals = silu ? 2u * a.ksplit : a.ksplit;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the fence's own wait can be dropped (guide, Pitfall 12)
  uint32_t old = 0;
  if (lane == 0) old = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  old = __builtin_amdgcn_readfirstlane(old);
  if (old + 1u != arrivals) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (lane == 0) __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const DGemmReduceArgs& r = a.fix;
  const uint32_t nout = silu ? r.N / 2 : r.N;
  const uint32_t n0 = g * 64u, m0 = blockIdx.y * 64u;
  const uint32_t items = (r.M - m0 < 64u ? r.M - m0 : 64u) * 16u;
  constexpr int kQ = 8;
  for (uint32_t i0 = 0; i0 < items; i0 += 64u * kQ) {
    uint32_t mm[kQ], nn[kQ];
    bool ok[kQ];
    f32x4_t s[kQ], u[kQ];
#pragma unroll
    for (int j = 0; j < kQ; ++j) {
      const uint32_t i = i0 + j * 64u + lane;
      mm[j] = m0 + (i >> 4);
      nn[j] = n0 + (i & 15u) * 4u;
      ok[j] = i < items && nn[j] < nout;
      s[j] = u[j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    }
    for (uint32_t k = 0; k < r.ksplit; ++k) {
      f32x4_t v[kQ], w[kQ];
#pragma unroll
      for (int j = 0; j < kQ; ++j) {
        const float* row = r.part + ((uint64_t)k * r.M + (ok[j] ? mm[j] : m0)) * r.N;
        v[j] = *reinterpret_cast<const f32x4_t*>(row + (ok[j] ? nn[j] : 0u));
        if (silu) w[j] = *reinterpret_cast<const f32x4_t*>(row + nout + (ok[j] ? nn[j] : 0u));
      }
#pragma unroll
      for (int j = 0; j < kQ; ++j) {
        s[j] += v[j];
        if (silu) u[j] += w[j];
      }
    }
#pragma unroll
    for (int j = 0; j < kQ; ++j) {
      if (!ok[j]) continue;
      uint16_t o[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float y = s[j][e];
        if (r.epi == DGEMM_EPI_RESID) {
          y = bf16_to_f32(f32_to_bf16_rne(y)) + bf16_to_f32(r.resid[(uint64_t)mm[j] * r.ldr + nn[j] + e]);
        } else if (silu) {
          const float gt = bf16_to_f32(f32_to_bf16_rne(y)), up = bf16_to_f32(f32_to_bf16_rne(u[j][e]));
          y = gt / (1.f + __expf(-gt)) * up;
        }
        o[e] = f32_to_bf16_rne(y);
      }
      uint16_t* dst = r.out_frag ? r.out + frag_index(mm[j], r.out_col0 + nn[j], r.out_cols)
                                 : r.out + (uint64_t)mm[j] * r.ldo + nn[j];
      *reinterpret_cast<u32x2_t*>(dst) =
          u32x2_t{(uint32_t)o[0] | ((uint32_t)o[1] << 16), (uint32_t)o[2] | ((uint32_t)o[3] << 16)};
    }
  }
}

// Raw-weight variant with the activations shared through LDS: a workgroup's 4
// waves take 4 consecutive row tiles (one each) over the same K range; per K
// step each wave loads ONE of the 4 activation fragments (M tiles) and
// publishes it in LDS, so the VMEM instructions per weight byte match the
// 4-row-tile kernel while the wave count per K split is 4x higher - i.e. the
// same occupancy with 4x fewer split-K partials (ksplit x M x N x 4 B of f32,
// written and re-read by the reduce: up to 40% extra HBM traffic at 8B shapes).
template <int U>
__global__ void __launch_bounds__(256) k_dgemm_lds(DGemmArgs a) {
  __shared__ u32x4_t xs[U][kMTiles][64];
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t unit = blockIdx.x;  // row block * ksplit + k split (block-uniform)
  if (unit >= a.row_blocks * a.ksplit) return;
  const uint32_t rb = unit / a.ksplit, ks = unit - rb * a.ksplit;
  const uint32_t rt = rb * 4u + wave;
  const bool has_rt = rt < (a.N >> 4);  // wave-uniform; every wave still takes part in the x exchange
  const uint32_t k_lo = ks * a.klen;
  const uint32_t k_hi = k_lo + a.klen < a.K ? k_lo + a.klen : a.K;
  const uint32_t kfr = a.K >> 5;
  const uint32_t m_base = blockIdx.y * (kMTiles * 16);
  const uint32_t h = lane >> 4;
  const uint32_t mx = m_base + wave * 16 + (lane & 15u);  // the activation row this wave fetches
  const bool mxv = mx < a.M;
  const uint32_t xstep = a.x_frag ? 512u : 32u;
  const uint16_t* xr = a.x_frag ? a.x + (uint64_t)(mx >> 4) * kfr * 512u + lane * 8u
                                : a.x + (uint64_t)(mxv ? mx : 0) * a.ldx + 8u * h;
  const uint16_t* wrow =
      reinterpret_cast<const uint16_t*>(a.w) + a.w_off + (uint64_t)(has_rt ? rt : 0) * kfr * 512u + lane * 8u;
  f32x4_t acc[kMTiles];
#pragma unroll
  for (int mt = 0; mt < kMTiles; ++mt) acc[mt] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  uint32_t k = k_lo;
  for (; k + 32 * U <= k_hi; k += 32 * U) {
    const uint32_t kst = k >> 5;
    u32x4_t wa[U], xv[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
      wa[u] = has_rt ? __builtin_nontemporal_load(reinterpret_cast<const u32x4_t*>(wrow + (uint64_t)(kst + u) * 512u))
                     : u32x4_t{0, 0, 0, 0};
#pragma unroll
    for (int u = 0; u < U; ++u)
      xv[u] = mxv ? *reinterpret_cast<const u32x4_t*>(xr + ((k >> 5) + u) * xstep) : u32x4_t{0, 0, 0, 0};
    __syncthreads();  // the previous block's LDS reads are done
#pragma unroll
    for (int u = 0; u < U; ++u) xs[u][wave][lane] = xv[u];
    __syncthreads();
    if (has_rt) {
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int mt = 0; mt < kMTiles; ++mt)
          acc[mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, wa[u]),
                                                            __builtin_bit_cast(bf16x8_t, xs[u][mt][lane]), acc[mt],
                                                            0, 0, 0);
    }
  }
  for (; k < k_hi; k += 32) {
    const u32x4_t wa = has_rt ? __builtin_nontemporal_load(
                                    reinterpret_cast<const u32x4_t*>(wrow + (uint64_t)(k >> 5) * 512u))
                              : u32x4_t{0, 0, 0, 0};
    const u32x4_t xv = mxv ? *reinterpret_cast<const u32x4_t*>(xr + (k >> 5) * xstep) : u32x4_t{0, 0, 0, 0};
    __syncthreads();
    xs[0][wave][lane] = xv;
    __syncthreads();
    if (has_rt) {
#pragma unroll
      for (int mt = 0; mt < kMTiles; ++mt)
        acc[mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, wa),
                                                          __builtin_bit_cast(bf16x8_t, xs[0][mt][lane]), acc[mt], 0,
                                                          0, 0);
    }
  }
  if (!has_rt) return;
  // D layout (16x16x32): col = lane & 15 -> m, row = 4 (lane >> 4) + reg -> n.
  const uint32_t n = rt * 16u + 4u * h;
#pragma unroll
  for (int mt = 0; mt < kMTiles; ++mt) {
    const uint32_t m = m_base + mt * 16 + (lane & 15u);
    if (m < a.M) *reinterpret_cast<f32x4_t*>(a.part + ((uint64_t)ks * a.M + m) * a.N + n) = acc[mt];
  }
}

// ------------------------------------------------------------------ pipelined raw split-K
// Shared by k_dgemm_pipe: one batch of U K steps (4 weight + 4 activation
// fragments each) and its 16 U MFMAs.
template <int U>
__device__ __forceinline__ void dgf_load(u32x4_t (&wv)[U][4], u32x4_t (&xv)[U][4], const uint16_t* const (&wb)[4],
                                         const uint16_t* const (&xr)[4], uint32_t kst, uint32_t xstep) {
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int r = 0; r < 4; ++r)
      wv[u][r] = __builtin_nontemporal_load(reinterpret_cast<const u32x4_t*>(wb[r] + (uint64_t)(kst + u) * 512u));
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) xv[u][mt] = *reinterpret_cast<const u32x4_t*>(xr[mt] + (kst + u) * xstep);
}

template <int U>
__device__ __forceinline__ void dgf_mfma(f32x4_t (&acc)[4][4], const u32x4_t (&wv)[U][4], const u32x4_t (&xv)[U][4]) {
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
        acc[r][mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, wv[u][r]),
                                                             __builtin_bit_cast(bf16x8_t, xv[u][mt]), acc[r][mt], 0,
                                                             0, 0);
}

// k_dgemm_pipe: raw-weight split-K unit per wave (one row block = 4 row tiles x
// one K split, f32 partials for k_dgemm_reduce - the k_dgemm<RAW> contract) with
// a software-pipelined main loop: two register sets of U K steps, batch b+1's
// loads issued before batch b's MFMAs (sched_barrier-pinned), and every load
// unconditional (row-tile / M-row indices clamped to valid memory; clamped
// lanes' outputs are never stored).
template <int U>
__global__ void __launch_bounds__(256, 2) k_dgemm_pipe(DGemmArgs a) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t unit = blockIdx.x * (blockDim.x >> 6) + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (unit >= a.row_blocks * a.ksplit) return;  // wave-uniform exit (no barriers in this kernel)
  const uint32_t rb = unit / a.ksplit, ks = unit - rb * a.ksplit;
  const uint32_t k_lo = ks * a.klen;
  const uint32_t k_hi = k_lo + a.klen < a.K ? k_lo + a.klen : a.K;
  const uint32_t ntiles = a.N >> 4, kfr = a.K >> 5;
  const uint16_t* w = reinterpret_cast<const uint16_t*>(a.w) + a.w_off;
  const uint16_t* wb[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const uint32_t t = rb * 4 + r;
    wb[r] = w + (uint64_t)(t < ntiles ? t : ntiles - 1) * kfr * 512u + lane * 8u;
  }
  const uint32_t m_base = blockIdx.y * 64u;
  const uint16_t* xr[4];
  const uint32_t xstep = a.x_frag ? 512u : 32u;  // elements per K step of this lane's activation fragment
#pragma unroll
  for (int mt = 0; mt < 4; ++mt) {
    const uint32_t m = m_base + mt * 16 + (lane & 15u), mc = m < a.M ? m : a.M - 1;
    xr[mt] = a.x_frag ? a.x + (uint64_t)(mc >> 4) * kfr * 512u + (mc & 15u) * 8u + (lane >> 4) * 128u
                      : a.x + (uint64_t)mc * a.ldx + 8u * (lane >> 4);
  }
  f32x4_t acc[4][4];
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) acc[r][mt] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  const uint32_t s0 = k_lo >> 5, nsteps = k_hi > k_lo ? (k_hi - k_lo) >> 5 : 0;
  const uint32_t nbat = nsteps / U;
  if (nbat) {
    u32x4_t wA[U][4], xA[U][4], wB[U][4], xB[U][4];
    dgf_load<U>(wA, xA, wb, xr, s0, xstep);
    uint32_t b = 0;
    for (; b + 2 < nbat; b += 2) {
      dgf_load<U>(wB, xB, wb, xr, s0 + (b + 1) * U, xstep);
      __builtin_amdgcn_sched_barrier(0);
      dgf_mfma<U>(acc, wA, xA);
      __builtin_amdgcn_sched_barrier(0);
      dgf_load<U>(wA, xA, wb, xr, s0 + (b + 2) * U, xstep);
      __builtin_amdgcn_sched_barrier(0);
      dgf_mfma<U>(acc, wB, xB);
      __builtin_amdgcn_sched_barrier(0);
    }
    if (b + 1 < nbat) {
      dgf_load<U>(wB, xB, wb, xr, s0 + (b + 1) * U, xstep);
      __builtin_amdgcn_sched_barrier(0);
      dgf_mfma<U>(acc, wA, xA);
      dgf_mfma<U>(acc, wB, xB);
    } else {
      dgf_mfma<U>(acc, wA, xA);
    }
  }
  for (uint32_t st = nbat * U; st < nsteps; ++st) {
    u32x4_t w1[1][4], x1[1][4];
    dgf_load<1>(w1, x1, wb, xr, s0 + st, xstep);
    dgf_mfma<1>(acc, w1, x1);
  }
  // D layout (16x16x32): col = lane & 15 -> m, row = 4 (lane >> 4) + reg -> n.
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    if (rb * 4 + r >= ntiles) continue;
    const uint32_t n = (rb * 4 + r) * 16u + 4u * (lane >> 4);
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
      const uint32_t m = m_base + mt * 16 + (lane & 15u);
      if (m >= a.M) continue;
      if (a.direct)
        dg_store_direct(a.fix, m, n, acc[r][mt]);
      else
        *reinterpret_cast<f32x4_t*>(a.part + ((uint64_t)ks * a.M + m) * a.N + n) = acc[r][mt];
    }
  }
  if (a.fix_cnt) dg_fixup(a, rb, lane);
}

// k_dgemm_lring: the same split-K unit (4 row tiles x one K range, one wave per
// workgroup) with its operands staged through an LDS ring instead of VGPRs.
// Every K step's 4 weight + 4 activation fragments (8 x 1 KB, lane-linear -
// exactly the layout global_load_lds writes) go global -> LDS with no VGPR
// round trip, so D steps (D x 4 KB of weights) stay in flight per wave at ~60
// VGPRs (a register ring of 3+ K steps runs out of registers: the compiler
// shuffles it through AGPRs).
// Consumption waits on vmcnt by hand (loads retire in order: (D-1) x 8 newer
// ones may stay outstanding) and reads the slot with ds_read_b128 in inline
// asm, so the compiler's conservative LDS-DMA wait (vmcnt(0) before any LDS
// read) never drains the ring. Summation order = k_dgemm_pipe's.
template <int N>
__device__ __forceinline__ void dg_wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

template <int D>
__device__ __forceinline__ void lring_issue(u32x4_t (&ring)[D][8][64], uint32_t slot, uint32_t st,
                                            const uint16_t* const (&wb)[4], const uint16_t* const (&xr)[4],
                                            uint32_t xstep) {
#pragma unroll
  for (int r = 0; r < 4; ++r)
    __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(wb[r] + (uint64_t)st * 512u), &ring[slot][r][0],
                                     16, 0, 0);
#pragma unroll
  for (int mt = 0; mt < 4; ++mt)
    __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(xr[mt] + st * xstep), &ring[slot][4 + mt][0], 16,
                                     0, 0);
}

template <int D>
__global__ void __launch_bounds__(64) k_dgemm_lring(DGemmArgs a) {
  static_assert((D - 1) * 8 <= 63, "vmcnt range");
  __shared__ u32x4_t ring[D][8][64];  // slot, fragment (w rt 0-3, x mt 0-3), lane
  const uint32_t lane = threadIdx.x;
  const uint32_t unit = blockIdx.x;
  if (unit >= a.row_blocks * a.ksplit) return;
  const uint32_t rb = unit / a.ksplit, ks = unit - rb * a.ksplit;
  const uint32_t k_lo = ks * a.klen;
  const uint32_t k_hi = k_lo + a.klen < a.K ? k_lo + a.klen : a.K;
  const uint32_t ntiles = a.N >> 4, kfr = a.K >> 5;
  const uint16_t* w = reinterpret_cast<const uint16_t*>(a.w) + a.w_off;
  const uint16_t* wb[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const uint32_t t = rb * 4 + r;
    wb[r] = w + (uint64_t)(t < ntiles ? t : ntiles - 1) * kfr * 512u + lane * 8u;
  }
  const uint32_t m_base = blockIdx.y * 64u;
  const uint16_t* xr[4];
  const uint32_t xstep = a.x_frag ? 512u : 32u;  // elements per K step of this lane's activation fragment
#pragma unroll
  for (int mt = 0; mt < 4; ++mt) {
    const uint32_t m = m_base + mt * 16 + (lane & 15u), mc = m < a.M ? m : a.M - 1;
    xr[mt] = a.x_frag ? a.x + (uint64_t)(mc >> 4) * kfr * 512u + (mc & 15u) * 8u + (lane >> 4) * 128u
                      : a.x + (uint64_t)mc * a.ldx + 8u * (lane >> 4);
  }
  f32x4_t acc[4][4];
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) acc[r][mt] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  const uint32_t s0 = k_lo >> 5, nsteps = k_hi > k_lo ? (k_hi - k_lo) >> 5 : 0;

#pragma unroll
  for (int d = 0; d < D; ++d)
    if ((uint32_t)d < nsteps) lring_issue<D>(ring, d, s0 + d, wb, xr, xstep);
  // LDS byte address of this lane's 16 B in slot 0, fragment 0
  const uint32_t lbase = (uint32_t)(uintptr_t)&ring[0][0][lane];
  uint32_t slot = 0;
  for (uint32_t st = 0; st < nsteps; ++st) {
    if (st + D <= nsteps)
      dg_wait_vm<(D - 1) * 8>();
    else
      dg_wait_vm<0>();
    const uint32_t la = lbase + slot * (8u * 1024u);
    u32x4_t f0, f1, f2, f3, f4, f5, f6, f7;
    asm volatile(
        "ds_read_b128 %0, %8\n"
        "ds_read_b128 %1, %8 offset:1024\n"
        "ds_read_b128 %2, %8 offset:2048\n"
        "ds_read_b128 %3, %8 offset:3072\n"
        "ds_read_b128 %4, %8 offset:4096\n"
        "ds_read_b128 %5, %8 offset:5120\n"
        "ds_read_b128 %6, %8 offset:6144\n"
        "ds_read_b128 %7, %8 offset:7168\n"
        "s_waitcnt lgkmcnt(0)"
        : "=&v"(f0), "=&v"(f1), "=&v"(f2), "=&v"(f3), "=&v"(f4), "=&v"(f5), "=&v"(f6), "=&v"(f7)
        : "v"(la)
        : "memory");
    if (st + D < nsteps) lring_issue<D>(ring, slot, s0 + st + D, wb, xr, xstep);
    const u32x4_t wf[4] = {f0, f1, f2, f3}, xf[4] = {f4, f5, f6, f7};
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
        acc[r][mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, wf[r]),
                                                             __builtin_bit_cast(bf16x8_t, xf[mt]), acc[r][mt], 0, 0,
                                                             0);
    slot = slot + 1 == (uint32_t)D ? 0 : slot + 1;
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    if (rb * 4 + r >= ntiles) continue;
    const uint32_t n = (rb * 4 + r) * 16u + 4u * (lane >> 4);
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
      const uint32_t m = m_base + mt * 16 + (lane & 15u);
      if (m >= a.M) continue;
      if (a.direct)
        dg_store_direct(a.fix, m, n, acc[r][mt]);
      else
        *reinterpret_cast<f32x4_t*>(a.part + ((uint64_t)ks * a.M + m) * a.N + n) = acc[r][mt];
    }
  }
  if (a.fix_cnt) dg_fixup(a, rb, lane);
}

hipError_t launch_dgemm(const DGemmArgs& a, int mode, hipStream_t s) {
  if (a.N % 16 || a.K % 32 || a.klen % 32 || !a.ksplit || a.row_blocks != (a.N / 16 + kRowTiles - 1) / kRowTiles)
    return hipErrorInvalidValue;
  if ((a.fix_cnt || a.direct) && !dgemm_fixup_ok(a, mode)) return hipErrorInvalidValue;
  if (a.direct && (a.fix_cnt || a.ksplit != 1 || a.fix.epi == DGEMM_EPI_SILU_MUL)) return hipErrorInvalidValue;
  const uint32_t units = a.row_blocks * a.ksplit;
  if (mode == DGEMM_W_RAW && a.lds_x) {
    dim3 grid(units, (a.M + kMTiles * 16 - 1) / (kMTiles * 16));
    if (a.unroll == 2)
      hipLaunchKernelGGL((k_dgemm_lds<2>), grid, dim3(256), 0, s, a);
    else if (a.unroll == 8)
      hipLaunchKernelGGL((k_dgemm_lds<8>), grid, dim3(256), 0, s, a);
    else
      hipLaunchKernelGGL((k_dgemm_lds<4>), grid, dim3(256), 0, s, a);
    return hipGetLastError();
  }
  // One-wave workgroups (wg_waves 1) spread a GEMM's units over every CU (with
  // 4-wave workgroups, 768 units occupy only 192 of the 256 CUs).
  if (mode == DGEMM_W_RAW && a.unroll == 1 && a.depth >= 30) {  // LDS ring: depth = 10 x slots
    dim3 grid(units, (a.M + kMTiles * 16 - 1) / (kMTiles * 16));
    switch (a.depth) {
      case 30: hipLaunchKernelGGL((k_dgemm_lring<3>), grid, dim3(64), 0, s, a); break;
      case 40: hipLaunchKernelGGL((k_dgemm_lring<4>), grid, dim3(64), 0, s, a); break;
      case 50: hipLaunchKernelGGL((k_dgemm_lring<5>), grid, dim3(64), 0, s, a); break;
      case 60: hipLaunchKernelGGL((k_dgemm_lring<6>), grid, dim3(64), 0, s, a); break;
      case 70: hipLaunchKernelGGL((k_dgemm_lring<7>), grid, dim3(64), 0, s, a); break;
      default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
  }
  const uint32_t ww = a.wg_waves == 1 ? 1u : 4u;
  dim3 grid((units + ww - 1) / ww, (a.M + kMTiles * 16 - 1) / (kMTiles * 16));
  const dim3 block(64 * ww);
  switch (mode) {
    case DGEMM_W_RAW:
      if (a.unroll == 4)
        hipLaunchKernelGGL((k_dgemm<MODE_RAW, 4>), grid, block, 0, s, a);
      else if (a.unroll == 1)  // unroll 1 = the pipelined raw kernel (k_dgemm_pipe, two sets of U = 2)
        hipLaunchKernelGGL((k_dgemm_pipe<2>), grid, block, 0, s, a);
      else
        hipLaunchKernelGGL((k_dgemm<MODE_RAW, 2>), grid, block, 0, s, a);
      break;
    case DGEMM_W_PACKED:
      hipLaunchKernelGGL((k_dgemm<MODE_PACKED, 1>), grid, block, 0, s, a);
      break;
    case DGEMM_W_PACKED_BF11:
      if (a.unroll == 4)
        hipLaunchKernelGGL((k_dgemm<MODE_PACKED_BF11, 4>), grid, block, 0, s, a);
      else if (a.unroll == 1)
        hipLaunchKernelGGL((k_dgemm<MODE_PACKED_BF11, 1>), grid, block, 0, s, a);
      else
        hipLaunchKernelGGL((k_dgemm<MODE_PACKED_BF11, 2>), grid, block, 0, s, a);
      break;
    default:
      return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_dgemm_reduce(const DGemmReduceArgs& a, hipStream_t s) {
  const uint32_t nout = a.epi == DGEMM_EPI_SILU_MUL ? a.N / 2 : a.N;
  if (nout % 4) return hipErrorInvalidValue;
  const uint64_t threads = (uint64_t)a.M * (nout / 4);
  if (!threads) return hipSuccess;
  hipLaunchKernelGGL(k_dgemm_reduce, dim3((uint32_t)((threads + 255) / 256)), dim3(256), 0, s, a);
  return hipGetLastError();
}

}  // namespace ogkm
