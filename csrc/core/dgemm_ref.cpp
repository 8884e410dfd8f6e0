// CPU reference of the decode GEMM (csrc/kernels/decode_gemm.hip) for the fake
// backend and tests: same fragment order, same packed-stream decode (one BF11
// wave group per fragment, exceptions included), same split-K partial layout
// and epilogues, f32 accumulation.
#include <algorithm>
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
          float xv[32];
          for (uint32_t kk = 0; kk < 32; ++kk)
            xv[kk] = bf2f(a.x_frag ? a.x[frag_index(m, k + kk, a.K)] : a.x[(uint64_t)m * a.ldx + k + kk]);
          float* pr = a.part + ((uint64_t)ks * a.M + m) * a.N + rt * 16;
          for (uint32_t r = 0; r < 16; ++r) {
            float s = 0.f;
            for (uint32_t kk = 0; kk < 32; ++kk) s += w[r * 32 + kk] * xv[kk];
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
      a.out[a.out_frag ? frag_index(m, a.out_col0 + n, a.out_cols) : (uint64_t)m * a.ldo + n] = f2bf(y);
    }
  }
}

void rmsnorm_cpu(const ResidNormArgs& a) {
  for (uint32_t r = 0; r < a.rows; ++r) {
    uint16_t* xr = a.x + (uint64_t)r * a.ldx;
    if (a.part) {  // the RESID epilogue of the deferred GEMM (k_dgemm_reduce order: k ascending)
      for (uint32_t i = 0; i < a.dim; ++i) {
        float s = 0.f;
        for (uint32_t k = 0; k < a.ksplit; ++k) s += a.part[((uint64_t)k * a.rows + r) * a.dim + i];
        xr[i] = f2bf(bf2f(f2bf(s)) + bf2f(xr[i]));
      }
    }
    float ss = 0.f;
    for (uint32_t i = 0; i < a.dim; ++i) ss += bf2f(xr[i]) * bf2f(xr[i]);
    const float inv = 1.f / std::sqrt(ss / (float)a.dim + a.eps);
    for (uint32_t i = 0; i < a.dim; ++i)
      a.y[a.y_frag ? frag_index(r, i, a.dim) : (uint64_t)r * a.ldy + i] =
          f2bf(bf2f(f2bf(bf2f(xr[i]) * inv)) * bf2f(a.w[i]));
  }
}

void rope_kv_cpu(const RopeKvArgs& a) {
  const uint32_t half = a.hd / 2, heads = a.hq + 2 * a.hkv;
  for (uint32_t b = 0; b < a.B; ++b)
    for (uint32_t hh = 0; hh < heads; ++hh)
      for (uint32_t i = 0; i < half; ++i) {
        float x1, x2;
        if (a.part) {  // deferred qkv GEMM: its store epilogue, here
          const uint32_t n = heads * a.hd, c1 = hh * a.hd + i;
          float s1 = 0.f, s2 = 0.f;
          for (uint32_t k = 0; k < a.ksplit; ++k) {
            s1 += a.part[((uint64_t)k * a.B + b) * n + c1];
            s2 += a.part[((uint64_t)k * a.B + b) * n + c1 + half];
          }
          x1 = bf2f(f2bf(s1));
          x2 = bf2f(f2bf(s2));
        } else {
          const uint16_t* src = a.qkv + (uint64_t)b * a.ldqkv + (uint64_t)hh * a.hd;
          x1 = bf2f(src[i]);
          x2 = bf2f(src[i + half]);
        }
        if (hh < a.hq + a.hkv) {
          const float c = a.cos[i], s = a.sin[i];
          const float r1 = x1 * c - x2 * s, r2 = x2 * c + x1 * s;
          x1 = r1;
          x2 = r2;
        }
        const uint16_t o1 = f2bf(x1), o2 = f2bf(x2);
        if (hh < a.hq) {
          uint16_t* q = a.q_out + ((uint64_t)b * a.hq + hh) * a.hd;
          q[i] = o1;
          q[i + half] = o2;
          continue;
        }
        const uint32_t kv = hh < a.hq + a.hkv ? 0u : 1u;
        const uint32_t h = hh - a.hq - kv * a.hkv;
        uint16_t* c = a.cache + ((((uint64_t)kv * a.B + b) * a.hkv + h) * a.T + a.pos) * a.hd;
        c[i] = o1;
        c[i + half] = o2;
        if (a.tail) {
          uint16_t* t = a.tail + ((((uint64_t)kv * a.B + b) * a.hkv + h) * a.tail_T + a.tail_pos) * a.hd;
          t[i] = o1;
          t[i + half] = o2;
        }
      }
}

void attn_decode_cpu(const AttnArgs& a) {
  const uint32_t g = a.hq / a.hkv;
  std::vector<float> sc(a.len), o(a.hd);
  for (uint32_t b = 0; b < a.B; ++b)
    for (uint32_t qh = 0; qh < a.hq; ++qh) {
      const uint32_t kvh = qh / g;
      const uint16_t* q = a.q + ((uint64_t)b * a.hq + qh) * a.hd;
      const uint16_t* kb = a.cache + (((uint64_t)0 * a.B + b) * a.hkv + kvh) * (uint64_t)a.T * a.hd;
      const uint16_t* vb = a.cache + (((uint64_t)1 * a.B + b) * a.hkv + kvh) * (uint64_t)a.T * a.hd;
      float m = -INFINITY;
      for (uint32_t t = 0; t < a.len; ++t) {
        float s = 0.f;
        for (uint32_t d = 0; d < a.hd; ++d) s += bf2f(q[d]) * a.scale * bf2f(kb[(uint64_t)t * a.hd + d]);
        sc[t] = s;
        m = std::max(m, s);
      }
      float l = 0.f;
      for (uint32_t t = 0; t < a.len; ++t) {
        sc[t] = std::exp(sc[t] - m);
        l += sc[t];
      }
      std::fill(o.begin(), o.end(), 0.f);
      for (uint32_t t = 0; t < a.len; ++t)
        for (uint32_t d = 0; d < a.hd; ++d) o[d] += sc[t] * bf2f(vb[(uint64_t)t * a.hd + d]);
      for (uint32_t d = 0; d < a.hd; ++d)
        a.out[a.out_frag ? frag_index(b, qh * a.hd + d, a.hq * a.hd) : ((uint64_t)b * a.hq + qh) * a.hd + d] =
            f2bf(o[d] / l);
    }
}

}  // namespace ogkm
