// BF12 host-side codec (reference implementation; the GPU decoder in
// csrc/kernels/bf12_kernels.hip must produce bit-identical output).
#include "ogkm/codec.hpp"

#include <algorithm>
#include <cstring>
#include <thread>
#include <vector>

namespace ogkm {

bool block_decode(uint8_t fmt, const uint8_t* in, uint16_t* out, uint32_t n_values) {
  if (fmt == 1) return bf12_decode(in, out, n_values);
  if (fmt == 2) return ans_decode(in, out, n_values);
  return false;
}

uint64_t bf12_encode(const uint16_t* in, uint32_t n, uint8_t* out, uint64_t cap) {
  if (n == 0 || (n & 1) || n > kBf12Tile * kBf12MaxTiles) return 0;
  // 1) exponent histogram -> base maximising the values covered by codes 0..14
  uint32_t hist[256] = {0};
  for (uint32_t i = 0; i < n; ++i) hist[(in[i] >> 7) & 0xFF]++;
  uint32_t best = 0, best_cnt = 0, win = 0;
  for (uint32_t e = 0; e < 15; ++e) win += hist[e];
  best_cnt = win;
  for (uint32_t b = 1; b + 15 <= 256; ++b) {
    win += hist[b + 14] - hist[b - 1];
    if (win > best_cnt) {
      best_cnt = win;
      best = b;
    }
  }
  uint32_t n_exc = n - best_cnt;
  uint64_t need = bf12_encoded_bytes(n, n_exc);
  if (need > cap) return 0;
  // 2) planes + per-tile exception lists
  Bf12Header h;
  memset(&h, 0, sizeof h);
  h.magic = kBf12Magic;
  h.base = best;
  h.n_values = n;
  h.n_exc = n_exc;
  uint8_t* sm = out + kBf12HeaderBytes;
  uint8_t* codes = sm + n;
  Bf12Exception* exc = reinterpret_cast<Bf12Exception*>(codes + n / 2);
  uint32_t ntiles = (n + kBf12Tile - 1) / kBf12Tile;
  uint32_t e_out = 0;
  for (uint32_t t = 0; t < ntiles; ++t) {
    h.exc_off[t] = e_out;
    uint32_t lo = t * kBf12Tile, hi = lo + kBf12Tile < n ? lo + kBf12Tile : n;
    for (uint32_t i = lo; i < hi; i += 2) {
      uint8_t nib[2];
      for (int k = 0; k < 2; ++k) {
        uint16_t v = in[i + k];
        uint32_t e = (v >> 7) & 0xFF;
        sm[i + k] = (uint8_t)(((v >> 8) & 0x80) | (v & 0x7F));
        uint32_t c = e - best;
        if (e < best || c >= 15) {
          c = 15;
          exc[e_out++] = Bf12Exception{i + k, v, 0};
        }
        nib[k] = (uint8_t)c;
      }
      codes[i >> 1] = (uint8_t)(nib[0] | (nib[1] << 4));
    }
  }
  for (uint32_t t = ntiles; t <= kBf12MaxTiles; ++t) h.exc_off[t] = e_out;
  memcpy(out, &h, sizeof h);
  return need;
}

bool bf12_decode(const uint8_t* in, uint16_t* out, uint32_t n) {
  Bf12Header h;
  memcpy(&h, in, sizeof h);
  if (h.magic != kBf12Magic || h.n_values != n) return false;
  const uint8_t* sm = in + kBf12HeaderBytes;
  const uint8_t* codes = sm + n;
  const Bf12Exception* exc = reinterpret_cast<const Bf12Exception*>(codes + n / 2);
  for (uint32_t i = 0; i < n; ++i) {
    uint32_t c = (codes[i >> 1] >> ((i & 1) * 4)) & 0xF;
    uint32_t s = sm[i];
    out[i] = (uint16_t)(((s & 0x80) << 8) | (((h.base + c) & 0xFF) << 7) | (s & 0x7F));
  }
  for (uint32_t k = 0; k < h.n_exc; ++k) out[exc[k].index] = exc[k].bits;
  return true;
}


// ---------------------------------------------------------------------------
// BF11 (two-level exponent code)

static inline uint64_t al8(uint64_t x) { return (x + 7) & ~7ull; }

uint64_t bf11_encode(const uint16_t* in, uint32_t n, uint8_t* out, uint64_t cap) {
  if (n == 0 || (n & 7) || n > kBf12Tile * kBf12MaxTiles) return 0;
  uint32_t hist[256] = {0};
  for (uint32_t i = 0; i < n; ++i) hist[(in[i] >> 7) & 0xFF]++;
  // primary: the three most frequent exponents
  uint8_t prim[3] = {0, 0, 0};
  bool taken[256] = {false};
  for (int k = 0; k < 3; ++k) {
    uint32_t best = 0, cnt = 0;
    bool any = false;
    for (uint32_t e = 0; e < 256; ++e)
      if (!taken[e] && (!any || hist[e] > cnt)) {
        best = e;
        cnt = hist[e];
        any = true;
      }
    prim[k] = (uint8_t)best;
    taken[best] = true;
  }
  int8_t pcode[256];
  for (int e = 0; e < 256; ++e) pcode[e] = -1;
  for (int k = 0; k < 3; ++k) pcode[prim[k]] = (int8_t)k;
  // secondary window: 15 consecutive exponents covering most escaped values
  uint32_t rest[256];
  for (int e = 0; e < 256; ++e) rest[e] = pcode[e] >= 0 ? 0 : hist[e];
  uint32_t sbase = 0, win = 0, best_win;
  for (uint32_t e = 0; e < 15; ++e) win += rest[e];
  best_win = win;
  for (uint32_t b = 1; b + 15 <= 256; ++b) {
    win += rest[b + 14] - rest[b - 1];
    if (win > best_win) {
      best_win = win;
      sbase = b;
    }
  }
  uint32_t n_sec = 0;
  for (int e = 0; e < 256; ++e) n_sec += rest[e];
  uint32_t n_exc = n_sec - best_win;
  const uint32_t ngroups = (n + kBf11Group - 1) / kBf11Group;
  Bf11Header h;
  memset(&h, 0, sizeof h);
  h.magic = kBf11Magic;
  h.n_values = n;
  h.n_exc = n_exc;
  h.prim = prim[0] | (prim[1] << 8) | (prim[2] << 16);
  h.sec_base = sbase;
  h.n_sec = n_sec;
  const Bf11Layout lay = bf11_layout(n);
  h.off_prim = lay.off_prim;
  h.off_wg = lay.off_wg;
  h.off_sec = lay.off_sec;
  (void)ngroups;
  h.off_exc = (uint32_t)al8(h.off_sec + (n_sec + 1) / 2 + 8);
  const uint64_t need = (uint64_t)h.off_exc + (uint64_t)n_exc * sizeof(Bf12Exception);
  if (need > cap) return 0;
  uint8_t* sm = out + kBf11HeaderBytes;
  uint8_t* pc = out + h.off_prim;
  uint32_t* wg = reinterpret_cast<uint32_t*>(out + h.off_wg);
  uint8_t* sec = out + h.off_sec;
  Bf12Exception* exc = reinterpret_cast<Bf12Exception*>(out + h.off_exc);
  memset(pc, 0, n / 4);
  memset(sec, 0, h.off_exc - h.off_sec);
  uint32_t nib = 0, e_out = 0;
  const uint32_t ntiles = (n + kBf12Tile - 1) / kBf12Tile;
  for (uint32_t i = 0; i < n; ++i) {
    if (i % kBf12Tile == 0) {
      h.exc_off[i / kBf12Tile] = e_out;
      h.sec_tile[i / kBf12Tile] = nib;
    }
    if (i % kBf11Group == 0) wg[i / kBf11Group] = nib;
    const uint16_t v = in[i];
    const uint32_t e = (v >> 7) & 0xFF;
    sm[i] = (uint8_t)(((v >> 8) & 0x80) | (v & 0x7F));
    uint32_t c = pcode[e] >= 0 ? (uint32_t)pcode[e] : 3u;
    pc[i >> 2] |= (uint8_t)(c << (2 * (i & 3)));
    if (c == 3) {
      uint32_t sc = e - sbase;
      if (e < sbase || sc >= 15) {
        sc = 15;
        exc[e_out++] = Bf12Exception{i, v, 0};
      }
      sec[nib >> 1] |= (uint8_t)(sc << (4 * (nib & 1)));
      ++nib;
    }
  }
  for (uint32_t t = ntiles; t <= kBf12MaxTiles; ++t) {
    h.exc_off[t] = e_out;
    h.sec_tile[t] = nib;
  }
  memcpy(out, &h, sizeof h);
  return need;
}

bool bf11_decode(const uint8_t* in, uint16_t* out, uint32_t n) {
  Bf11Header h;
  memcpy(&h, in, sizeof h);
  if (h.magic != kBf11Magic || h.n_values != n) return false;
  const uint8_t* sm = in + kBf11HeaderBytes;
  const uint8_t* pc = in + h.off_prim;
  const uint8_t* sec = in + h.off_sec;
  const Bf12Exception* exc = reinterpret_cast<const Bf12Exception*>(in + h.off_exc);
  uint32_t nib = 0;
  for (uint32_t i = 0; i < n; ++i) {
    uint32_t c = (pc[i >> 2] >> (2 * (i & 3))) & 3;
    uint32_t e;
    if (c < 3) {
      e = (h.prim >> (8 * c)) & 0xFF;
    } else {
      e = (h.sec_base + ((sec[nib >> 1] >> (4 * (nib & 1))) & 0xF)) & 0xFF;
      ++nib;
    }
    uint32_t s = sm[i];
    out[i] = (uint16_t)(((s & 0x80) << 8) | (e << 7) | (s & 0x7F));
  }
  if (nib != h.n_sec) return false;
  for (uint32_t k = 0; k < h.n_exc; ++k) out[exc[k].index] = exc[k].bits;
  return true;
}

void bf11_decode_group(const uint8_t* in, uint32_t v, uint16_t* out) {
  Bf11Header h;
  memcpy(&h, in, sizeof h);
  const uint8_t* sm = in + kBf11HeaderBytes;
  const uint8_t* pc = in + h.off_prim;
  const uint8_t* sec = in + h.off_sec;
  uint32_t nib;
  memcpy(&nib, in + h.off_wg + 4ull * (v / kBf11Group), 4);
  const uint32_t cnt = std::min<uint32_t>(kBf11Group, h.n_values - v);
  for (uint32_t k = 0; k < cnt; ++k) {
    const uint32_t i = v + k;
    const uint32_t c = (pc[i >> 2] >> (2 * (i & 3))) & 3;
    uint32_t e;
    bool exc = false;
    if (c < 3) {
      e = (h.prim >> (8 * c)) & 0xFF;
    } else {
      const uint32_t sc = (sec[nib >> 1] >> (4 * (nib & 1))) & 0xF;
      exc = sc == 15;
      e = (h.sec_base + sc) & 0xFF;
      ++nib;
    }
    const uint32_t s = sm[i];
    out[k] = (uint16_t)(((s & 0x80) << 8) | (e << 7) | (s & 0x7F));
    if (exc) {
      const Bf12Exception* ex = reinterpret_cast<const Bf12Exception*>(in + h.off_exc);
      const uint32_t t = i / kBf12Tile;
      for (uint32_t q = h.exc_off[t]; q < h.exc_off[t + 1]; ++q)
        if (ex[q].index == i) out[k] = ex[q].bits;
    }
  }
}

uint64_t bf12_pack(const uint16_t* in, uint64_t n, uint32_t chunk_values, uint8_t* out, uint64_t cap,
                   unsigned threads, PackFormat fmt) {
  if (!n || chunk_values < 8192 || (chunk_values & (chunk_values - 1)) || chunk_values > kBf12Tile * kBf12MaxTiles)
    return 0;
  if (cap < bf12_pack_bound(n, chunk_values)) return 0;
  const uint64_t nch = (n + chunk_values - 1) / chunk_values;
  const uint64_t head = bf12_stream_head_bytes(nch);
  const uint64_t slot = (uint64_t)chunk_values * 2 + 512;  // worst case per chunk
  std::vector<Bf12StreamChunk> table(nch);
  std::vector<uint64_t> bytes(nch);
  // 1) every chunk encodes into its worst-case slot, in parallel
  auto work = [&](uint64_t c0, uint64_t c1) {
    for (uint64_t c = c0; c < c1; ++c) {
      uint64_t lo = c * chunk_values;
      uint32_t cnt = (uint32_t)std::min<uint64_t>(chunk_values, n - lo);
      uint8_t* dst = out + head + c * slot;
      uint64_t e = 0;
      uint32_t kind = 0;
      if (fmt == PackFormat::ANS) {
        e = cnt % 512 == 0 ? ans_encode(in + lo, cnt, dst, (uint64_t)cnt * 2) : 0;
        kind = e ? 3 : 0;
      } else if (cnt % 8 == 0 && fmt == PackFormat::BF11_STRICT) {
        e = bf11_encode(in + lo, cnt, dst, (uint64_t)cnt * 2);
        kind = e ? 2 : 0;
      } else if (cnt % 8 == 0 && fmt == PackFormat::BF11) {
        e = bf11_encode(in + lo, cnt, dst, (uint64_t)cnt * 2);
        kind = e ? 2 : 0;
        // BF11 wins for weight-like data; keep BF12 where it is smaller
        // (e.g. flat exponent histograms that escape most values).
        if (e && e > (uint64_t)cnt * 3 / 2 + kBf12HeaderBytes) {
          uint64_t e12 = bf12_encode(in + lo, cnt, dst, e);
          if (e12) {
            e = e12;
            kind = 1;
          } else {
            e = bf11_encode(in + lo, cnt, dst, (uint64_t)cnt * 2);
          }
        }
      }
      if (!e && cnt % 8 == 0 && fmt != PackFormat::BF11_STRICT && fmt != PackFormat::ANS) {
        e = bf12_encode(in + lo, cnt, dst, (uint64_t)cnt * 2);
        kind = e ? 1 : 0;
      }
      table[c].n_values = cnt;
      table[c].encoded = kind;
      if (!e) {
        memcpy(dst, in + lo, (size_t)cnt * 2);
        e = (uint64_t)cnt * 2;
      }
      bytes[c] = e;
    }
  };
  threads = std::max(1u, std::min<unsigned>(threads, (unsigned)nch));
  std::vector<std::thread> th;
  uint64_t per = (nch + threads - 1) / threads;
  for (unsigned k = 0; k < threads; ++k) {
    uint64_t c0 = k * per, c1 = std::min(nch, c0 + per);
    if (c0 < c1) th.emplace_back(work, c0, c1);
  }
  for (auto& x : th) x.join();
  // 2) compact left (destinations never pass their sources)
  uint64_t off = head;
  for (uint64_t c = 0; c < nch; ++c) {
    uint64_t from = head + c * slot;
    if (off != from) memmove(out + off, out + from, bytes[c]);
    table[c].offset = off;
    off = (off + bytes[c] + 255) & ~255ull;
  }
  Bf12StreamHeader h{kBf12StreamMagic, (uint32_t)nch, chunk_values, (uint32_t)fmt, n, off};
  memset(out, 0, head);
  memcpy(out, &h, sizeof h);
  memcpy(out + sizeof h, table.data(), nch * sizeof(Bf12StreamChunk));
  return off;
}

bool bf12_unpack(const uint8_t* stream, uint16_t* out, uint64_t n, uint64_t dst_stride, uint32_t row_shift) {
  Bf12StreamHeader h;
  memcpy(&h, stream, sizeof h);
  if (h.magic != kBf12StreamMagic || h.n_values != n) return false;
  const Bf12StreamChunk* t = reinterpret_cast<const Bf12StreamChunk*>(stream + sizeof h);
  for (uint32_t c = 0; c < h.nchunks; ++c) {
    const uint64_t stride = dst_stride ? dst_stride : h.chunk_values;
    uint16_t* dst = out + ((uint64_t)c >> row_shift) * stride + ((uint64_t)c & ((1ull << row_shift) - 1)) * h.chunk_values;
    if (t[c].encoded == 3) {
      if (!ans_decode(stream + t[c].offset, dst, t[c].n_values)) return false;
    } else if (t[c].encoded == 2) {
      if (!bf11_decode(stream + t[c].offset, dst, t[c].n_values)) return false;
    } else if (t[c].encoded == 1) {
      if (!bf12_decode(stream + t[c].offset, dst, t[c].n_values)) return false;
    } else {
      memcpy(dst, stream + t[c].offset, (size_t)t[c].n_values * 2);
    }
  }
  return true;
}

}  // namespace ogkm
