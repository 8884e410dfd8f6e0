// ANS1 chunk codec (CPU encoder + reference decoder). Format: codec.hpp.
//
// The encoder runs each segment's (step, lane) sequence backwards, pushing
// renormalisation words; reversing the word list yields exactly the order in
// which the wave-parallel decoder (csrc/kernels/ans_kernels.hip) consumes them:
// step by step, lanes in ascending order within a step.
#include <algorithm>
#include <cstring>
#include <vector>

#include "ogkm/codec.hpp"

namespace ogkm {

namespace {

constexpr uint32_t kM = 1u << kAnsPrecBits;

inline uint32_t seg_value(uint32_t t, uint32_t lane) { return ((t >> 3) * 64u + lane) * 8u + (t & 7u); }

// Exponent histogram -> frequencies summing to 2^12, every present symbol >= 1,
// at least two symbols (so every frequency fits 12 bits).
void normalise(const uint32_t* cnt, uint32_t n, uint16_t* freq) {
  int64_t sum = 0;
  int present = 0, top = -1;
  for (int s = 0; s < 256; ++s) {
    freq[s] = 0;
    if (!cnt[s]) continue;
    ++present;
    uint32_t f = (uint32_t)(((uint64_t)cnt[s] * kM + n / 2) / n);
    freq[s] = (uint16_t)std::max<uint32_t>(1u, f);
    sum += freq[s];
    if (top < 0 || cnt[s] > cnt[top]) top = s;
  }
  if (present == 1) {  // a second (unused) symbol keeps the top frequency < 2^12
    freq[top ^ 1] = 1;
    sum += 1;
  }
  int64_t diff = (int64_t)kM - sum;
  if (diff >= 0 || freq[top] + diff >= 1) {
    freq[top] = (uint16_t)(freq[top] + diff);
    return;
  }
  // Too many rare symbols rounded up: take the excess from the largest ones.
  while (diff < 0) {
    int best = -1;
    for (int s = 0; s < 256; ++s)
      if (freq[s] > 1 && (best < 0 || freq[s] > freq[best])) best = s;
    --freq[best];
    ++diff;
  }
}

}  // namespace

uint64_t ans_encode(const uint16_t* in, uint32_t n, uint8_t* out, uint64_t cap) {
  if (!n || n % 512 || n > (1u << 20)) return 0;
  const uint32_t n_seg = (n + kAnsSegValues - 1) / kAnsSegValues;
  const uint32_t off_dir = (kAnsHeaderBytes + n + 3u) & ~3u;
  uint64_t pos = off_dir + 4ull * (n_seg + 1);
  if (pos > cap) return 0;
  uint32_t cnt[256] = {0};
  for (uint32_t i = 0; i < n; ++i) cnt[(in[i] >> 7) & 0xFF]++;
  AnsHeader h;
  memset(&h, 0, sizeof h);
  h.magic = kAnsMagic;
  h.n_values = n;
  h.n_seg = n_seg;
  h.off_dir = off_dir;
  normalise(cnt, n, h.freq);
  uint32_t cum[257];
  cum[0] = 0;
  for (int s = 0; s < 256; ++s) cum[s + 1] = cum[s] + h.freq[s];
  // Division-free state update: x / f by a 64-bit reciprocal (exact for every
  // 32-bit x and f >= 2: q = (ceil(2^64 / f) * x) >> 64); f == 1 is x itself.
  struct Sym {
    uint64_t rcp;
    uint32_t f, x_max, cum;
  } sy[256];
  for (int s = 0; s < 256; ++s) {
    const uint32_t f = h.freq[s];
    sy[s].f = f;
    sy[s].x_max = f << (32 - kAnsPrecBits);  // x_max = ((L >> prec) << 16) * f
    sy[s].cum = cum[s];
    sy[s].rcp = f > 1 ? ~0ull / f + 1 : 0;
  }
  uint8_t* sm = out + kAnsHeaderBytes;
  for (uint32_t i = 0; i < n; ++i) sm[i] = (uint8_t)(((in[i] >> 8) & 0x80u) | (in[i] & 0x7Fu));
  std::vector<uint32_t> dir(n_seg + 1);
  // Renormalisation words are written back to front (the decoder consumes them
  // in the reverse of the encoding order): at most one per value.
  std::vector<uint16_t> wbuf(kAnsSegValues + 1);
  for (uint32_t s = 0; s < n_seg; ++s) {
    const uint32_t base = s * kAnsSegValues;
    const uint32_t steps = std::min(kAnsSegValues, n - base) / 64u;
    uint32_t x[64];
    for (auto& v : x) v = kAnsLowBound;
    uint16_t* const wend = wbuf.data() + wbuf.size();  // (w[-1] stays inside: one spare slot)
    uint16_t* w = wend;
    for (uint32_t t = steps; t-- > 0;) {
      const uint16_t* row = in + base + (t >> 3) * 512u + (t & 7u);  // value (t/8*64 + l)*8 + t%8
      for (uint32_t l = 64; l-- > 0;) {
        const Sym& y = sy[(row[l * 8u] >> 7) & 0xFF];
        uint32_t v = x[l];
        // branch-free renormalisation (the branch is a coin flip ~1 value in 6)
        const uint32_t r = v >= y.x_max;
        w[-1] = (uint16_t)(v & 0xFFFFu);
        w -= r;
        v = r ? v >> 16 : v;
        const uint32_t q = y.rcp ? (uint32_t)(((unsigned __int128)y.rcp * v) >> 64) : v;
        x[l] = (q << kAnsPrecBits) + (v - q * y.f) + y.cum;
      }
    }
    const uint64_t nw = (uint64_t)(wend - w);
    dir[s] = (uint32_t)pos;
    const uint64_t bytes = 256 + ((nw * 2 + 3) & ~3ull);
    if (pos + bytes > cap) return 0;
    memcpy(out + pos, x, 256);
    if (nw) memcpy(out + pos + 256, w, nw * 2);
    if (nw & 1) memset(out + pos + 256 + nw * 2, 0, 2);
    pos += bytes;
  }
  dir[n_seg] = (uint32_t)pos;
  memcpy(out, &h, sizeof h);
  memset(out + kAnsHeaderBytes + n, 0, off_dir - kAnsHeaderBytes - n);
  memcpy(out + off_dir, dir.data(), 4ull * (n_seg + 1));
  return pos;
}

bool ans_decode(const uint8_t* in, uint16_t* out, uint32_t n) {
  AnsHeader h;
  memcpy(&h, in, sizeof h);
  if (h.magic != kAnsMagic || h.n_values != n || n % 512) return false;
  uint32_t cum[257];
  cum[0] = 0;
  for (int s = 0; s < 256; ++s) cum[s + 1] = cum[s] + h.freq[s];
  if (cum[256] != kM) return false;
  std::vector<uint8_t> slot_sym(kM);
  for (int s = 0; s < 256; ++s)
    for (uint32_t k = cum[s]; k < cum[s + 1]; ++k) slot_sym[k] = (uint8_t)s;
  const uint8_t* sm = in + kAnsHeaderBytes;
  const uint32_t* dir = reinterpret_cast<const uint32_t*>(in + h.off_dir);
  for (uint32_t s = 0; s < h.n_seg; ++s) {
    const uint32_t base = s * kAnsSegValues;
    const uint32_t steps = std::min(kAnsSegValues, n - base) / 64u;
    uint32_t x[64];
    memcpy(x, in + dir[s], 256);
    const uint16_t* w = reinterpret_cast<const uint16_t*>(in + dir[s] + 256);
    const uint64_t nw = (dir[s + 1] - dir[s] - 256) / 2;
    uint64_t wp = 0;
    for (uint32_t t = 0; t < steps; ++t) {
      for (uint32_t l = 0; l < 64; ++l) {
        const uint32_t slot = x[l] & (kM - 1);
        const uint32_t sym = slot_sym[slot];
        x[l] = h.freq[sym] * (x[l] >> kAnsPrecBits) + slot - cum[sym];
        if (x[l] < kAnsLowBound) {
          if (wp >= nw) return false;
          x[l] = (x[l] << 16) | w[wp++];
        }
        const uint32_t v = base + seg_value(t, l);
        const uint32_t b = sm[v];
        out[v] = (uint16_t)(((b & 0x80u) << 8) | (sym << 7) | (b & 0x7Fu));
      }
    }
    for (uint32_t l = 0; l < 64; ++l)
      if (x[l] != kAnsLowBound) return false;  // every lane must end where the encoder began
  }
  return true;
}

}  // namespace ogkm
