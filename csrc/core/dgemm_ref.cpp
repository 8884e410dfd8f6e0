// CPU reference of the decode GEMM (csrc/kernels/decode_gemm.hip) for the fake
// backend and tests: same fragment order, same packed-stream decode (one BF11
// wave group per fragment, exceptions included), same split-K partial layout
// and epilogues, f32 accumulation.
#include <cmath>
#include <cstring>
#include <vector>

#include "ogkm/codec.hpp"
#include "ogkm/dgemm.hpp"

namespace ogkm {

static inline float bf2f(uint16_t b) {
  uint32_t u = (uint32_t)b << 16;
  float f;
  memcpy(&f, &u, 4);
  return f;
}
static inline uint16_t f2bf(float f) {
  uint32_t u;
  memcpy(&u, &f, 4);
  if ((u & 0x7F800000u) == 0x7F800000u && (u & 0x7FFFFFu)) return (uint16_t)((u >> 16) | 0x40u);
  u += 0x7FFFu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}

// 512 values of fragment starting at stream value index g.
static void packed_fragment(const uint8_t* base, uint32_t chunk_shift, uint64_t g, uint16_t* out) {
  const Bf12StreamChunk* table = reinterpret_cast<const Bf12StreamChunk*>(base + sizeof(Bf12StreamHeader));
  const uint64_t c = g >> chunk_shift;
  const uint32_t v = (uint32_t)(g & ((1ull << chunk_shift) - 1));
  const Bf12StreamChunk& ch = table[c];
  const uint8_t* blk = base + ch.offset;
  if (ch.encoded == 2) {
    bf11_decode_group(blk, v, out);
  } else if (ch.encoded == 1) {
    std::vector<uint16_t> tmp(ch.n_values);
    bf12_decode(blk, tmp.data(), ch.n_values);
    memcpy(out, tmp.data() + v, 1024);
  } else {
    memcpy(out, blk + (uint64_t)v * 2, 1024);
  }
}

void dgemm_cpu(const DGemmArgs& a, bool packed) {
  const uint32_t kfr = a.K / 32, ntiles = a.N / 16;
  std::vector<uint16_t> frag(512);
  std::vector<float> w(16 * 32);
  for (uint32_t ks = 0; ks < a.ksplit; ++ks) {
    for (uint32_t m = 0; m < a.M; ++m) memset(a.part + ((uint64_t)ks * a.M + m) * a.N, 0, (size_t)a.N * 4);
    const uint32_t k_lo = ks * a.klen, k_hi = std::min(a.K, k_lo + a.klen);
    for (uint32_t rt = 0; rt < ntiles; ++rt) {
      for (uint32_t k = k_lo; k < k_hi; k += 32) {
        const uint64_t fi = (uint64_t)rt * kfr + (k >> 5);
        if (packed) {
          packed_fragment(a.w, a.chunk_shift, a.w_off + fi * 512, frag.data());
        } else {
          memcpy(frag.data(), a.w + (a.w_off + fi * 512) * 2, 1024);
        }
        for (uint32_t l = 0; l < 64; ++l)
          for (uint32_t j = 0; j < 8; ++j) w[(l & 15) * 32 + 8 * (l >> 4) + j] = bf2f(frag[l * 8 + j]);
        for (uint32_t m = 0; m < a.M; ++m) {
          const uint16_t* xr = a.x + (uint64_t)m * a.ldx + k;
          float* pr = a.part + ((uint64_t)ks * a.M + m) * a.N + rt * 16;
          for (uint32_t r = 0; r < 16; ++r) {
            float s = 0.f;
            for (uint32_t kk = 0; kk < 32; ++kk) s += w[r * 32 + kk] * bf2f(xr[kk]);
            pr[r] += s;
          }
        }
      }
    }
  }
}

void dgemm_reduce_cpu(const DGemmReduceArgs& a) {
  const uint32_t nout = a.epi == DGEMM_EPI_SILU_MUL ? a.N / 2 : a.N;
  for (uint32_t m = 0; m < a.M; ++m) {
    for (uint32_t n = 0; n < nout; ++n) {
      float s = 0.f, u = 0.f;
      for (uint32_t k = 0; k < a.ksplit; ++k) {
        const float* row = a.part + ((uint64_t)k * a.M + m) * a.N;
        s += row[n];
        if (a.epi == DGEMM_EPI_SILU_MUL) u += row[nout + n];
      }
      float y = s;
      if (a.epi == DGEMM_EPI_RESID) {
        y = bf2f(f2bf(y)) + bf2f(a.resid[(uint64_t)m * a.ldr + n]);
      } else if (a.epi == DGEMM_EPI_SILU_MUL) {
        const float g = bf2f(f2bf(y)), up = bf2f(f2bf(u));
        y = g / (1.f + std::exp(-g)) * up;
      }
      a.out[(uint64_t)m * a.ldo + n] = f2bf(y);
    }
  }
}

}  // namespace ogkm
